#!/bin/bash
# Round-2 session of record: GPU tests, bench + kernel trace + PMC passes (tools/gpu_bench_prof.sh),
# clock stamps (steady state, default split and equal shares; after idle), stereo benches.
set -o pipefail
TAG=${1:-r02c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
bash tools/gpu_bench_prof.sh $TAG || exit 2
timeout -k 10 120 python tools/mono_stamps.py > $OUT/stamps_steady.json 2> $OUT/stamps.err || exit 3
FMRX_MONO_SPLIT=0 timeout -k 10 120 python tools/mono_stamps.py > $OUT/stamps_steady_equal.json 2>> $OUT/stamps.err || exit 4
timeout -k 10 120 python tools/mono_stamps.py --idle > $OUT/stamps_idle.json 2>> $OUT/stamps.err || exit 5
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/bench_stereo.json 2> $OUT/bench_stereo.err || exit 6
timeout -k 10 300 python tools/bench_modes.py > $OUT/bench_modes.json 2> $OUT/bench_modes.err || exit 7
echo done
