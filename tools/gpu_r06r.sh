#!/bin/bash
# Round-6: short calls below 2^17 through the demoted kernel (one launch).  PLL / seam / split tests,
# the seam in the lane regime, bench_seam.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "pll or seam or split or two_context or stereo or unlocked or long_hash or rds" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 120 python -u tools/seam_profile.py --blocks 150 --warmup 20 > "$out/seam_py_lane.json" 2>&1 || { echo "seam lane failed"; exit 1; }
echo "lane $(cat "$out/seam_py_lane.json")"
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/seam.json"))
print("py", d["serial"]["x_realtime"], d["two_threads"]["x_realtime"], "native", d["native"]["serial"]["x_realtime"], d["native"]["two_threads"]["x_realtime"], "cli16", d["cli"]["default_batch_16"]["x_realtime"], d["seam_pcm_equals_cli_prefix"])
PY
