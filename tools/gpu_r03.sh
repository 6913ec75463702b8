#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# A/B of the stereo audio tile kernel: the 51-tap FIR unrolled (libfmrx.so) vs the runtime tap
# loop (build_ab/, -DFMRX_AB_AUDIOLOOP): kernel-trace stats of configs[4] (256 stereo streams x
# 60 s) per build; the stereo parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r03_al}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "stereo or bench_config or rds" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/new_$i -o run -- python3 tools/bench_stereo.py --streams 256 --seconds 60 > $OUT/new_$i.json 2>&1 || exit 2
  FMRX_LIB_PATH=$PWD/software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/old_$i -o run -- python3 tools/bench_stereo.py --streams 256 --seconds 60 > $OUT/old_$i.json 2>&1 || exit 3
done
grep -h '^{' $OUT/new_*.json $OUT/old_*.json
