#!/bin/bash
# Runner changes: PLL/stereo GPU tests, configs[2] twice, stereo streams 1..2048.
set -o pipefail
OUT=gpurun_out/${1:-sat3}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "stereo or pll or rds or cli or smoke" > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python tools/bench_stereo.py --gib >> $OUT/gib.json 2>> $OUT/bench.err || exit 2
done
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/streams.json 2>> $OUT/bench.err || exit 3
echo done
