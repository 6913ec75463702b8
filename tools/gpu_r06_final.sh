#!/bin/bash
# Round-6 record session: the -m gpu suite, smoke, the default bench line, the bench under a kernel
# trace (profile of record), the seam (Python + C++ legs, CLI), the unlocked streams with the
# reference CPU path, one 10 s stream.  Every GPU step under its own limit; the first failure ends it.
set -o pipefail
out=${1:-gpurun_out/r06final}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
cut -c1-400 "$out/bench.json"
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
timeout -k 10 200 python -u tools/bench_stereo.py --seconds 10 --streams 1 > "$out/st10.json" 2> "$out/st10.err" || { echo "st10 failed"; exit 1; }
timeout -k 10 500 python -u tools/bench_unlocked.py --cpu --out "$out/unlocked.json" > "$out/unlocked.log" 2>&1 || { echo "unlocked failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 --start-block 8000 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python3 bench.py > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { echo "bench prof failed"; exit 1; }
echo done
