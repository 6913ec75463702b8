#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests with the replayed check (the chain hands over one state a batch),
# configs[2] with it, and the cycles per interval (A/B build with FMRX_AB_PROF).
set -o pipefail
OUT=gpurun_out/r03_rep2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "predicted or saturated or speculation or pipe or long_hash or bench_config or trig_hint or many_streams" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/gib.json 2>&1 || { tail $OUT/gib.json; exit 2; }
grep -v amdgpu.ids $OUT/gib.json
AB=software-defined-radio-course-project_amd/build_ab/libfmrx.so
FMRX_LIB_PATH=$AB timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/prof.txt 2>&1 || { tail $OUT/prof.txt; exit 3; }
grep prof: $OUT/prof.txt
