#!/bin/bash
# Round-6: short calls on the long forms when they hold two intervals.  The -m gpu suite, the seam
# (Python + C++), its trace in the 2^22 regime, the locked 72 s A/B.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(f"{sys.argv[1]}/seam.json"))
print("py", d["serial"]["x_realtime"], d["two_threads"]["x_realtime"], "native", d["native"]["serial"]["x_realtime"], d["native"]["two_threads"]["x_realtime"], d["seam_pcm_equals_cli_prefix"])
PY
for sb in 0 1500 8000; do
  timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 --start-block $sb > "$out/seam_py_$sb.json" 2>&1 || { echo "seam $sb failed"; exit 1; }
  echo "$sb $(cat "$out/seam_py_$sb.json")"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 --start-block 8000 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
echo done
