#!/bin/bash
# Sweep of the first-dispatched wave's share (FMRX_MONO_SPLIT, 1/1024) of the fused mono kernel,
# parity subset first.  Usage (gpurun): bash tools/gpu_split_sweep.sh <tag> [shares...]
set -o pipefail
TAG=${1:-split}
shift
LIST=${@:-0 560 600 640 680}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mono or polyphase or rf_block or time_shard or window" > $OUT/pytest.log 2>&1 || exit 1
for r in 1 2; do
for sh in $LIST; do
  FMRX_MONO_SPLIT=$sh timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > $OUT/bench_${sh}_$r.json 2>/dev/null || exit 2
done
done
FMRX_MONO_SPLIT=600 timeout -k 10 120 python tools/mono_stamps.py > $OUT/stamps_600.json 2> $OUT/stamps.err || exit 3
echo ok
