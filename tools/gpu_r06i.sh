#!/bin/bash
# Round-6: the demoted kernel's register budget (256 VGPRs: co-resident with the stage kernels) on
# configs[4] and on the unlocked streams it exists for.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked or long_hash" > "$out/dem_tests.log" 2>&1 || { echo "demotion tests failed"; tail -30 "$out/dem_tests.log"; exit 1; }
tail -1 "$out/dem_tests.log"
for rep in 1 2; do
  for spec in new= w2=$A/build_ab_W2/libfmrx.so nodl=$A/build_ab_NO_DEMOTED_LAUNCH/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json")"
  done
done
for spec in new= w2=$A/build_ab_W2/libfmrx.so; do
  name=${spec%%=*}; path=${spec#*=}
  FMRX_LIB_PATH=$path timeout -k 10 300 python -u tools/bench_unlocked.py --only unlocked_m0_rand_80s unlocked_m2_synth_170b \
      --out "$out/unlocked_$name.json" > "$out/unlocked_$name.log" 2>&1 || { echo "unlocked $name failed"; tail -5 "$out/unlocked_$name.log"; exit 1; }
done
python - "$out" <<'PY'
import json, sys
for n in ("new", "w2"):
    d = json.load(open(f"{sys.argv[1]}/unlocked_{n}.json"))
    print(n, {k: (v["seconds"]["median"], v["ns_per_pll_step"], v["bit_exact_pcm"]) for k, v in d.items() if isinstance(v, dict)})
PY
