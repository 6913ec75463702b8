#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests, configs[2] and configs[4] (256 stereo streams x 60 s) with their kernel traces.
set -o pipefail
OUT=gpurun_out/${1:-r03_prep}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pll or stereo or bench_config or many_streams" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o c4 -- python3 tools/bench_stereo.py --streams 256 --seconds 60 > $OUT/c4.json 2>&1 || { tail $OUT/c4.json; exit 2; }
grep '^{' $OUT/c4.json
timeout -k 10 300 python3 tools/bench_stereo.py --streams 256 --seconds 60 > $OUT/c4_plain.json 2>&1 || { tail $OUT/c4_plain.json; exit 3; }
grep '^{' $OUT/c4_plain.json
timeout -k 10 300 python3 tools/bench_stereo.py --gib > $OUT/c2.json 2>&1 || { tail $OUT/c2.json; exit 4; }
grep '^{' $OUT/c2.json
