#!/bin/bash
# A/B of the speculative PLL runners (FMRX_PLL_RUNNER: 1 lane roles, 2 lane form without the
# offset lane, 0 the previous form): stereo/PLL/RDS parity first, then stereo benches.
set -o pipefail
OUT=gpurun_out/${1:-runner_ab}
RUNNERS=${2:-"1 0"}
STREAMS=${3:-"1 32 256 1024 2048"}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "stereo or pll or rds or smoke or cli" > $OUT/pytest.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for r in $RUNNERS; do
    FMRX_PLL_RUNNER=$r timeout -k 10 200 python tools/bench_stereo.py --streams $STREAMS \
        > $OUT/bench_r$r.$rep.json 2>> $OUT/bench.err || exit 2
  done
done
echo done
