#!/bin/bash
# Round-6: the demoted kernel's helpers inlined (no scratch beyond the runners' 16 B) on configs[4]
# and on the unlocked streams.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked or pll" > "$out/dem_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/dem_tests.log"; exit 1; }
tail -1 "$out/dem_tests.log"
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
for rep in 1 2; do
  for spec in new= inl=$A/build_ab_INL/libfmrx.so nodl=$A/build_ab_NO_DEMOTED_LAUNCH/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json" | cut -c1-300)"
  done
done
FMRX_LIB_PATH=$A/build_ab_INL/libfmrx.so timeout -k 10 400 python -u tools/bench_unlocked.py --out "$out/unlocked_inl.json" > "$out/unlocked_inl.log" 2>&1 || { echo "unlocked failed"; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/unlocked_inl.json"))
print("inl", {k: (v["seconds"]["median"], v["ns_per_pll_step"], v["bit_exact_pcm"], v["bit_exact_pll_state"]) for k, v in d.items() if isinstance(v, dict)})
PY
