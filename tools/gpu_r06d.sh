#!/bin/bash
# Round-6 iteration: short-call PLL forms + the pinned band-pass read.  The new seam test first,
# then the -m gpu suite, the locked-stream A/B (pre-round library; count forms below 2^19 with 8
# evaluator waves), one 10 s stream and 256 x 10 s per build, the seam.  arg: output dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "seam_calls_in_every or thread_split or two_context" > "$out/seam_tests.log" 2>&1 || { echo "seam tests failed"; tail -30 "$out/seam_tests.log"; exit 1; }
tail -1 "$out/seam_tests.log"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
A=software-defined-radio-course-project_amd
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so newcnt=,FMRX_PLL_CNT=15 \
    c8=$A/build_ab_c8/libfmrx.so,FMRX_PLL_CNT=15 c32=$A/build_ab_c32/libfmrx.so,FMRX_PLL_CNT=15 || { echo "ab failed"; exit 1; }
for spec in "new=" "c8=$A/build_ab_c8/libfmrx.so" "c32=$A/build_ab_c32/libfmrx.so"; do
  name=${spec%%=*}; path=${spec#*=}; cntv=""; [ "$name" != new ] && cntv="FMRX_PLL_CNT=15"
  env FMRX_LIB_PATH=$path $cntv timeout -k 10 200 python -u tools/bench_stereo.py --seconds 10 --streams 1 256 \
      > "$out/st10_$name.json" 2> "$out/st10_$name.err" || { echo "st10 $name failed"; exit 1; }
done
timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 > "$out/seam_py_early.json" 2>&1 || { echo "seam failed"; exit 1; }
timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 --start-block 1500 > "$out/seam_py_late.json" 2>&1 || { echo "seam late failed"; exit 1; }
timeout -k 10 120 python -u tools/seam_profile.py --blocks 1500 --start-block 8000 > "$out/seam_py_2p22.json" 2>&1 || { echo "seam 2^22 failed"; exit 1; }
cat "$out"/seam_py_*.json
timeout -k 10 300 python -u tools/bench_seam.py --blocks 3000 > "$out/seam.json" 2> "$out/seam.err" || { echo "bench_seam failed"; exit 1; }
cat "$out/seam.json"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$out/seam_prof" -o seam -- \
    python3 tools/seam_profile.py --blocks 600 --start-block 8000 > "$out/seam_prof.log" 2>&1 || { echo "seam prof failed"; exit 1; }
echo done
