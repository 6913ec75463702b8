#!/bin/bash
# SQ counters of the PLL check kernel at 1,024 streams (issue, waits, memory instructions).
set -o pipefail
OUT=gpurun_out/${1:-check_sq}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  echo "pass $i $grp" >> $OUT/passes.txt
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
      python3 tools/bench_stereo.py --streams 1024 --seconds 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 1; }
done
echo done
