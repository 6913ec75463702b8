#!/bin/bash
# Round-6 iteration: the demotion decision at the interval's start.  Demotion + seam tests, the
# -m gpu suite, the locked-stream A/B, one 10 s stream, bench_seam, a seam trace (2^22 regime),
# the default bench line.  arg: output dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked" > "$out/dem_tests.log" 2>&1 || { echo "demotion tests failed"; tail -30 "$out/dem_tests.log"; exit 1; }
tail -1 "$out/dem_tests.log"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
A=software-defined-radio-course-project_amd
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
timeout -k 10 200 python -u tools/bench_stereo.py --seconds 10 --streams 1 256 > "$out/st10.json" 2> "$out/st10.err" || { echo "st10 failed"; exit 1; }
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
cat "$out/seam.json"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 --start-block 8000 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
echo done
