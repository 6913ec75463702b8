#!/bin/bash
# SQ + GRBM counter passes of the speculative PLL runner at 1 and 1,024 streams, runner forms
# given by FMRX_PLL_RUNNER values (default "1 0": lane roles, the previous form).
set -o pipefail
OUT=gpurun_out/${1:-runner_sq}
RUNNERS=${2:-"1 0"}
STREAMS=${3:-"1 1024"}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for ns in $STREAMS; do
  for r in $RUNNERS; do
    for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
               "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
               "GRBM_GUI_ACTIVE GRBM_COUNT"; do
      i=$((i+1))
      echo "pass $i ns=$ns runner $grp" >> $OUT/passes.txt
      timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
          python3 tools/bench_stereo.py --streams $ns --seconds 4 > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 1; }
    done
  done
done
echo done
