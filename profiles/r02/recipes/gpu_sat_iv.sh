#!/bin/bash
# Interval form of the saturated runner (FMRX_PLL_SAT_IV=1) against the committed form (0): the
# whole GPU suite with the interval form selected, then configs[2] (1 GiB stereo, bit-exact vs
# the reference build) alternating the two forms.  Kept as the recipe of
# profiles/r02/sat/interval/; the interval form was removed after this A/B, so today
# FMRX_PLL_SAT_IV selects nothing.
set -o pipefail
OUT=gpurun_out/${1:-sat_iv}
mkdir -p $OUT
FMRX_PLL_SAT_IV=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_iv.log 2>&1 || exit 1
for iv in 1 0 1 0; do
  FMRX_PLL_SAT_IV=$iv timeout -k 10 200 python tools/bench_stereo.py --gib >> $OUT/gib_iv$iv.json 2>> $OUT/bench.err || exit 2
done
echo done
