#!/bin/bash
# Round-6: the chain-side demotion without peeled loops, the demoted kernel's helpers inlined --
# PLL / demotion / seam tests, the locked 72 s A/B and configs[4] against the pre-round library,
# the unlocked streams.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked or pll" > "$out/dem_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/dem_tests.log"; exit 1; }
tail -1 "$out/dem_tests.log"
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
for rep in 1 2; do
  for spec in new= head=$A/build_ab_head/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cut -c1-200 "$out/${name}_$rep.json")"
  done
done
timeout -k 10 400 python -u tools/bench_unlocked.py --out "$out/unlocked.json" > "$out/unlocked.log" 2>&1 || { echo "unlocked failed"; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/unlocked.json"))
print({k: (v["seconds"]["median"], v["ns_per_pll_step"], v["bit_exact_pcm"], v["bit_exact_pll_state"]) for k, v in d.items() if isinstance(v, dict)})
for f in ("new_1", "new_2", "head_1", "head_2"):
    pass
PY
python - "$out" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/ab/*.json")):
    d = json.load(open(f))["m0_rf51_synth_72s"]
    print(f.split("/")[-1], d["seconds"]["median"], {k.replace("runner_", ""): v.get("ns_per_step") for k, v in d["regimes"].items()})
PY
