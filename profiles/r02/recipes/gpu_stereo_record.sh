#!/bin/bash
# Stereo records: configs[2] (SAT on and off), stereo streams, the CLI, kernel trace of configs[2].
set -o pipefail
TAG=${1:-stereo_record}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib.json 2> $OUT/err.log || exit 1
FMRX_PLL_SAT=0 timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib_nosat.json 2>> $OUT/err.log || exit 2
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/bench_stereo.json 2>> $OUT/err.log || exit 3
timeout -k 10 300 python tools/bench_cli.py > $OUT/bench_cli.json 2>> $OUT/err.log || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_gib -o run --output-format csv -- \
    python3 tools/bench_stereo.py --gib > $OUT/kt_gib.log 2>&1 || exit 5
echo done
