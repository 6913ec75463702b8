#!/bin/bash
# Round-6: short calls past 2^22 on a 128-step three-candidate form.  PLL / seam / long-run tests,
# the seam per regime (the stick included), bench_seam.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "pll or seam or thread_split or two_context or long_hash or unlocked or stereo_call or pipelined" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for sb in 0 1500 8000 26300; do
  timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 --start-block $sb > "$out/seam_py_$sb.json" 2>&1 || { echo "seam $sb failed"; exit 1; }
  echo "$sb $(cat "$out/seam_py_$sb.json")"
done
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/seam.json"))
print("py", d["serial"]["x_realtime"], d["two_threads"]["x_realtime"], "native", d["native"]["serial"]["x_realtime"], d["native"]["two_threads"]["x_realtime"], "cli16", d["cli"]["default_batch_16"]["x_realtime"], d["seam_pcm_equals_cli_prefix"])
PY
echo done
