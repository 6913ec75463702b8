#!/bin/bash
# SQ counter passes for the PLL kernel: one stream (latency) and 256 streams (throughput).
set -o pipefail
OUT=gpurun_out/${1:-pllsq}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for ns in 1 256; do
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
        python3 tools/bench_stereo.py --streams $ns --seconds 4 > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 1; }
  done
done
echo done
