#!/bin/bash
# Round-6: the range test only on the demotion path.  PLL / demotion tests, the locked 72 s A/B against
# the no-demotion build and the pre-round library.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "pll or demotion or unlocked or redo" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
tools/gpu_r06_ab2.sh "$out/ab" new= nodem=$A/build_ab_nodem/libfmrx.so head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
python - "$out" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/ab/*.json")):
    d = json.load(open(f))["m0_rf51_synth_72s"]
    print(f.split("/")[-1], d["seconds"]["median"], {k.replace("runner_", ""): v.get("ns_per_step") for k, v in d["regimes"].items()})
PY
