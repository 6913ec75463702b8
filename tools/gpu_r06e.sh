#!/bin/bash
# Round-6 iteration: chain-side pll_demote in the index / count runners.  Demotion + seam tests
# first, the -m gpu suite, the locked-stream A/B (pre-round library, no-demotion build), the
# unlocked-loop timings, the seam.  arg: output dir.
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
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so nodem=$A/build_ab_nodem/libfmrx.so || { echo "ab failed"; exit 1; }
timeout -k 10 400 python -u tools/bench_unlocked.py --out "$out/unlocked.json" > "$out/unlocked.log" 2>&1 || { echo "unlocked failed"; exit 1; }
timeout -k 10 200 python -u tools/bench_stereo.py --seconds 10 --streams 1 256 > "$out/st10.json" 2> "$out/st10.err" || { echo "st10 failed"; exit 1; }
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
cat "$out/seam.json"
echo done
