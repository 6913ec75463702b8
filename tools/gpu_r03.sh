#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the chain-step ubench variants.
set -o pipefail
OUT=gpurun_out/r03_ub2
mkdir -p $OUT
timeout -k 10 60 tools/ubench_chain > $OUT/ubench_chain.txt 2>&1 || exit 1
cat $OUT/ubench_chain.txt
