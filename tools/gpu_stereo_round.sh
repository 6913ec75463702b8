#!/bin/bash
# One GPU session for the stereo/RDS engine: full GPU test suite, the bench line, stereo
# (streams and BASELINE configs[2]) and RDS benches, config-5 per-GPU share through the
# distributed runner, the CLI against the reference's `project`, and kernel-trace profiles of
# the stereo bench at 1 and 256 streams.
# Usage (on the GPU box via gpurun): bash tools/gpu_stereo_round.sh <tag>
set -o pipefail
TAG=${1:-stereo}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 2
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/bench_stereo.json 2> $OUT/bench_stereo.err || exit 3
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib.json 2> $OUT/bench_stereo_gib.err || exit 4
timeout -k 10 300 python tools/bench_rds.py --streams 1,256 > $OUT/bench_rds.json 2> $OUT/bench_rds.err || exit 5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/bench_streams.py --streams 32 --seconds 10 --check > $OUT/bench_streams32.json 2> $OUT/bench_streams32.err || exit 6
timeout -k 10 300 python tools/bench_cli.py > $OUT/bench_cli.json 2> $OUT/bench_cli.err || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_stereo1 -o run --output-format csv -- \
    python3 tools/bench_stereo.py --streams 1 > $OUT/kt_stereo1.log 2>&1 || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_stereo256 -o run --output-format csv -- \
    python3 tools/bench_stereo.py --streams 256 > $OUT/kt_stereo256.log 2>&1 || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_stereo2048 -o run --output-format csv -- \
    python3 tools/bench_stereo.py --streams 2048 > $OUT/kt_stereo2048.log 2>&1 || exit 10
echo done
