#!/bin/bash
# Round-6: demotion only from states inside the fast batches' range (|phase|, |integ|); the PLL,
# demotion, seam, unlocked and long-run tests.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "pll or demotion or seam or unlocked or long_hash or redo" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
