#!/bin/bash
# SQ / GRBM counter passes over configs[2] (1 GiB stereo): summarise the saturated runner with
#   python tools/pll_sq_report.py <tag> pll_sat_kernel
set -o pipefail
OUT=gpurun_out/${1:-sat_sq}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "pass $i $grp" >> $OUT/passes.txt
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
      python3 tools/bench_stereo.py --gib > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 1; }
done
echo done
