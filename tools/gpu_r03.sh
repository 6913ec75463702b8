#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the PLL runner tests with the 16-step form checking the chain's phases (the 64-step forms
# replay), configs[2], and 256 stereo streams x 60 s (configs[4]).
set -o pipefail
OUT=gpurun_out/r03_hyb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "predicted or saturated or speculation or pipe or long_hash or bench_config or trig_hint or many_streams" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/gib.json 2>&1 || { tail $OUT/gib.json; exit 2; }
grep -v amdgpu.ids $OUT/gib.json
timeout -k 10 300 python tools/bench_stereo.py --streams 256 --seconds 60 > $OUT/c4.json 2>&1 || { tail $OUT/c4.json; exit 3; }
grep -v amdgpu.ids $OUT/c4.json
