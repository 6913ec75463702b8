#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# where the predicted runner's cycles go: its two waves' body / barrier-wait cycles (A/B build
# with FMRX_AB_PROF) and SQ counters of the kernel over one 30 s stream.
set -o pipefail
OUT=gpurun_out/r03_predprof
mkdir -p $OUT
export TMPDIR=/tmp
AB=software-defined-radio-course-project_amd/build_ab/libfmrx.so
FMRX_LIB_PATH=$AB timeout -k 10 120 python tools/bench_stereo.py --streams 1 --seconds 30 > $OUT/prof.txt 2>&1 || { tail $OUT/prof.txt; exit 1; }
cat $OUT/prof.txt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "pass $i $grp" >> $OUT/passes.txt
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
      python3 tools/bench_stereo.py --streams 1 --seconds 30 > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/failed.txt; exit 2; }
done
python3 tools/pll_sq_report.py r03_predprof pll_pred_kernel
