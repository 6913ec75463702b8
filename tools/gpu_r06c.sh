#!/bin/bash
# Round-6 seam iteration: the -m gpu suite, the locked-stream A/B against the pre-round library,
# the per-block seam under each RF staging variant (Python timing), bench_seam, a kernel / copy /
# HIP-API trace of the seam, and the unlocked-loop timings.  arg: output dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
if [ -e software-defined-radio-course-project_amd/build_ab_head/libfmrx.so ]; then
  tools/gpu_r06_ab.sh "$out/ab" new= head=software-defined-radio-course-project_amd/build_ab_head/libfmrx.so || exit 1
fi
for v in "base" "FMRX_SEAM_RF_ZC=1" "FMRX_SEAM_RF_DMAOUT=1" "FMRX_SEAM_RF_ZC=1 FMRX_SEAM_RF_DMAOUT=1"; do
  env_args=""; [ "$v" != base ] && env_args="$v"
  env $env_args timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 > "$out/seam_py_${v// /_}.json" 2>&1 || { echo "seam $v failed"; exit 1; }
  echo "$v $(cat "$out/seam_py_${v// /_}.json")"
done
timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 --start-block 1500 > "$out/seam_py_late.json" 2>&1 || { echo "seam late failed"; exit 1; }
echo "late $(cat "$out/seam_py_late.json")"
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
cat "$out/seam.json"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
timeout -k 10 400 python -u tools/bench_unlocked.py --out "$out/unlocked.json" > "$out/unlocked.log" 2>&1 || { echo "unlocked failed"; exit 1; }
echo done
