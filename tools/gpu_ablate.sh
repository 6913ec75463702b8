#!/bin/bash
# Per-stage ablation of the fused mono kernel (FMRX_ABLATE bitmask, results wrong by design
# except 0): kernel time from bench.py's HIP events, then one PMC pass per variant with the SQ
# issue / wait counters and GRBM_GUI_ACTIVE (effective clock).  Then the clock stamps of the
# default kernel (tools/mono_stamps.py).  Report: tools/ablate_report.py <tag>.
# Usage (on the GPU box via gpurun): bash tools/gpu_ablate.sh <tag> [bitmasks...]
set -o pipefail
TAG=${1:-abl}
shift
LIST=${@:-0 1 2 4 8 16 32 6 14 62 63}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/mono_stamps.py > $OUT/mono_stamps.json 2> $OUT/mono_stamps.err || exit 1
for a in $LIST; do
  FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so FMRX_ABLATE=$a timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs \
      > $OUT/bench_$a.json 2> $OUT/bench_$a.err || exit 2
  FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so FMRX_ABLATE=$a timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $OUT/pmc_$a -o run \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs \
      > $OUT/pmc_$a.log 2>&1 || exit 3
done
echo done
