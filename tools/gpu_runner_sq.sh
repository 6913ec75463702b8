#!/bin/bash
# SQ + GRBM counter passes of the speculative PLL runner at 1 and 1,024 streams, both runner
# forms (FMRX_PLL_RUNNER=1 lane roles, 0 the previous one): issue, waits and the clock.
set -o pipefail
OUT=gpurun_out/${1:-runner_sq}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for ns in 1 1024; do
  for r in 1 0; do
    for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
               "GRBM_GUI_ACTIVE GRBM_COUNT"; do
      i=$((i+1))
      echo "pass $i ns=$ns runner=$r $grp" >> $OUT/passes.txt
      FMRX_PLL_RUNNER=$r timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
          python3 tools/bench_stereo.py --streams $ns --seconds 4 > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 1; }
    done
  done
done
echo done
