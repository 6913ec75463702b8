#!/bin/bash
# tools/gpu_dev.sh <tag> [steps...] — development GPU call: each named step under its own time
# limit, stopping at the first failure.  Steps: tests (whole GPU suite), pll (PLL / stereo tests
# only), n2 (the N=2 bench line rehearsed with gloo, both ranks on device 0), mfma (tools/ubench_mfma_add), testsall (whole GPU suite, not stopping at a failure), idx (the index-runner tests), ubench (tools/ubench_idx), stages (tools/stage_times.py), bench (bench.py, no CPU baseline), smoke.
set -o pipefail
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
           tail -2 $OUT/tests.log ;;
    testsall) timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/testsall.log 2>&1; rc=$?
           tail -30 $OUT/testsall.log; [ $rc -le 1 ] || exit 1 ;;
    pll) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pll or stereo or bench_config or trig_hint or refdata or cli" > $OUT/pll.log 2>&1 || { tail -40 $OUT/pll.log; exit 2; }
           tail -2 $OUT/pll.log ;;
    idx) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "index" > $OUT/idx.log 2>&1 || { tail -40 $OUT/idx.log; exit 6; }
           tail -2 $OUT/idx.log ;;
    ubench) timeout -k 10 60 tools/ubench_idx > $OUT/ubench_idx.txt 2>&1 || { tail $OUT/ubench_idx.txt; exit 7; }
           cat $OUT/ubench_idx.txt ;;
    mfma) timeout -k 10 60 tools/ubench_mfma_add > $OUT/ubench_mfma_add.txt 2>&1 || { tail $OUT/ubench_mfma_add.txt; exit 8; }
           cat $OUT/ubench_mfma_add.txt ;;
    stages) timeout -k 10 300 python tools/stage_times.py > $OUT/stages.json 2> $OUT/stages.err || { tail $OUT/stages.err; exit 3; }
           cat $OUT/stages.json ;;
    bench) timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
           python -c "import json; j=json.load(open('$OUT/bench.json')); print(j['value'], j['roofline']['kernel_ms'], json.dumps(j.get('baseline_configs',{}))[:1500])" ;;
    n2) FMRX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 3 --no-cpu-baseline \
          > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail $OUT/bench_n2_gloo.err; exit 9; }
          tail -c 3000 $OUT/bench_n2_gloo.json ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 5; }
           tail -1 $OUT/smoke.log ;;
  esac
done
echo all done
