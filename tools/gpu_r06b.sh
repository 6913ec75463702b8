#!/bin/bash
# Round-6 GPU iteration: the -m gpu suite, the locked-stream A/B against the pre-round library, the
# per-block seam (Python timing + a kernel/copy trace).  arg: output dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
if [ -e software-defined-radio-course-project_amd/build_ab_head/libfmrx.so ]; then
  tools/gpu_r06_ab.sh "$out/ab" new= head=software-defined-radio-course-project_amd/build_ab_head/libfmrx.so || exit 1
fi
timeout -k 10 300 python -u tools/seam_profile.py --blocks 1500 > "$out/seam_py.json" 2>&1 || { echo "seam failed"; exit 1; }
cat "$out/seam_py.json"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
echo done
