#!/bin/bash
# Round-6 GPU session: the -m gpu suite, the default bench line, the locked-stream A/B against the
# pre-round library and the unlocked-loop timings (with the reference CPU path on the same bytes).
# arg: output dir.  Every GPU step under its own time limit; the first failure ends the script.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
if [ -e software-defined-radio-course-project_amd/build_ab_head/libfmrx.so ]; then
  tools/gpu_r06_ab.sh "$out/ab" new= head=software-defined-radio-course-project_amd/build_ab_head/libfmrx.so || exit 1
fi
timeout -k 10 400 python -u tools/bench_unlocked.py --cpu --out "$out/unlocked.json" > "$out/unlocked.log" 2>&1 || { echo "unlocked failed"; exit 1; }

# the per-block seam: host timing, then the same under a kernel + copy trace
timeout -k 10 300 python -u tools/bench_seam.py --blocks 2000 > "$out/seam.json" 2> "$out/seam.err" || { echo "seam failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
echo seam-done
