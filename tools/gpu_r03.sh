#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# A/B of the modes 2/3 resampler stage: every load hoisted ahead of the sum (libfmrx.so) vs the
# previous commit's source (build_ab/), alternating bench_modes runs of mode 2 and 3 on one box;
# the mode and bench-config parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r03_rs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mono or bench_config or modes or mode" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_modes.py --modes 2 3 > $OUT/new_$i.json 2> $OUT/new_$i.err || exit 2
  FMRX_LIB_PATH=$PWD/software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 120 python tools/bench_modes.py --modes 2 3 > $OUT/old_$i.json 2> $OUT/old_$i.err || exit 3
done
grep -h '^{' $OUT/new_*.json $OUT/old_*.json | cut -c1-200
