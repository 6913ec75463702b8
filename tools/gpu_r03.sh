#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests (three-wave runner on and off, its forced-miss path, many streams).
set -o pipefail
OUT=gpurun_out/r03_pipe17
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "predicted or saturated or speculation or pipe or long_hash or bench_config or trig_hint or many_streams" -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
