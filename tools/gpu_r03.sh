#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the whole GPU suite, the bench line (N=1) and the gloo N=2 rehearsal of the driver launch line.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_a.json 2> gpurun_out/r03_bench_a.err || { tail -20 gpurun_out/r03_bench_a.err; exit 1; }
cat gpurun_out/r03_bench_a.json
FMRX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 > gpurun_out/r03_bench_n2_gloo.json 2> gpurun_out/r03_bench_n2_gloo.err || { tail -20 gpurun_out/r03_bench_n2_gloo.err; exit 1; }
cat gpurun_out/r03_bench_n2_gloo.json
