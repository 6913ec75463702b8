#!/bin/bash
# Step-parallel saturated runner (FMRX_PLL_SAT=1) vs the per-step form (2): PLL runner tests
# with the speculation counters, then configs[2] (1 GiB stereo) under each form.  (Kept as the
# recipe of profiles/r02/sat/gib_*; the per-step form was removed after this A/B, so today both
# values select pll_sat_kernel.)
set -o pipefail
OUT=gpurun_out/${1:-sat2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "saturated or speculation or pll_primitive" > $OUT/pytest.log 2>&1 || exit 1
for sat in 1 2 1 2; do
  FMRX_PLL_SAT=$sat timeout -k 10 200 python tools/bench_stereo.py --gib >> $OUT/gib_sat$sat.json 2>> $OUT/bench.err || exit 2
done
echo done
