#!/bin/bash
# Stereo records after the saturated-segment runner: GPU tests, stereo streams, configs[2]
# (1 GiB, SAT on and off), RDS, config-5 share, CLI, kernel trace of configs[2].
set -o pipefail
TAG=${1:-r02g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/bench_stereo.json 2> $OUT/bench_stereo.err || exit 3
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib.json 2> $OUT/bench_stereo_gib.err || exit 4
FMRX_PLL_SAT=0 timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib_nosat.json 2>> $OUT/bench_stereo_gib.err || exit 5
timeout -k 10 300 python tools/bench_rds.py --streams 1,256 > $OUT/bench_rds.json 2> $OUT/bench_rds.err || exit 6
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/bench_streams.py --streams 32 --seconds 10 --check > $OUT/bench_streams32.json 2> $OUT/bench_streams32.err || exit 7
timeout -k 10 300 python tools/bench_cli.py > $OUT/bench_cli.json 2> $OUT/bench_cli.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_gib -o run --output-format csv -- \
    python3 tools/bench_stereo.py --gib > $OUT/kt_gib.log 2>&1 || exit 9
echo done
