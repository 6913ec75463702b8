#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the whole GPU suite, a kernel trace of configs[2], the stereo stream sweep.
set -o pipefail
OUT=gpurun_out/r03_pred
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_gib -o run --output-format csv -- \
    python3 tools/bench_stereo.py --gib > $OUT/kt_gib.log 2>&1 || { tail $OUT/kt_gib.log; exit 2; }
grep -h "^{" $OUT/kt_gib.log
FMRX_PLL_PRED=0 timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/gib_nopred.json 2>&1 || exit 3
cat $OUT/gib_nopred.json
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 --seconds 30 > $OUT/streams_30s.json 2>&1 || exit 4
cat $OUT/streams_30s.json
