#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests and stereo throughput at 1 / 32 / 256 / 1,024 / 2,048 streams x 10 s
# (the two-wave runner only where each of its waves gets a SIMD).
set -o pipefail
OUT=gpurun_out/r03_streams2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "predicted or saturated or speculation or pipe or long_hash or bench_config or trig_hint or many_streams" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/streams.json 2>&1 || { tail $OUT/streams.json; exit 2; }
cat $OUT/streams.json
