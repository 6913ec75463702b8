#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests, configs[2] with the saturated runner on and off, a kernel trace.
set -o pipefail
OUT=gpurun_out/r03_pred2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "predicted or saturated or speculation or long_hash or bench_config or trig_hint or many_streams" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/gib.json 2>&1 || { tail $OUT/gib.json; exit 2; }
cat $OUT/gib.json
FMRX_PLL_SAT=0 timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/gib_nosat.json 2>&1 || exit 3
cat $OUT/gib_nosat.json
FMRX_PLL_SAT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_gib_nosat -o run --output-format csv -- \
    python3 tools/bench_stereo.py --gib > $OUT/kt_gib.log 2>&1 || { tail $OUT/kt_gib.log; exit 4; }
head -6 $OUT/kt_gib_nosat/run_kernel_stats.csv
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 --seconds 30 > $OUT/streams_30s.json 2>&1 || exit 5
cat $OUT/streams_30s.json
# A/B: the demod division through a double reciprocal (make ab AB=-DFMRX_AB_DIV)
AB=software-defined-radio-course-project_amd/build_ab/libfmrx.so
FMRX_LIB_PATH=$AB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_refdata.py -m gpu -k "mono or full_size or bench_config or thread_split or reference_demod or time_shards" -x -q --timeout 200 --timeout-method thread > $OUT/ab_tests.log 2>&1 || { tail -20 $OUT/ab_tests.log; exit 6; }
tail -1 $OUT/ab_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs > $OUT/bench_base_$i.json 2>/dev/null || exit 7
  FMRX_LIB_PATH=$AB timeout -k 10 200 python bench.py --no-cpu-baseline --no-other-configs > $OUT/bench_ab_$i.json 2>/dev/null || exit 8
done
grep -ho '"kernel_ms": [0-9.]*' $OUT/bench_base_*.json $OUT/bench_ab_*.json
