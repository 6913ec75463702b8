#!/bin/bash
# Saturated runner change: PLL runner tests, configs[2] three times.
set -o pipefail
OUT=gpurun_out/${1:-sat4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "saturated or speculation or pll_primitive or long_hash" > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python tools/bench_stereo.py --gib >> $OUT/gib.json 2>> $OUT/bench.err || exit 2
done
echo done
