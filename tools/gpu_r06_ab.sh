#!/bin/bash
# A/B of PLL runner builds on the locked 72 s stream (tools/bench_unlocked.py --only), alternating
# libraries; args: output dir, then name=path pairs (path empty: the in-tree library)
set -o pipefail
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for pair in "$@"; do
    name=${pair%%=*}; path=${pair#*=}
    FMRX_LIB_PATH=$path timeout -k 10 120 python -u tools/bench_unlocked.py --only m0_rf51_synth_72s \
        --out "$out/${name}_$rep.json" > "$out/${name}_$rep.log" 2>&1 || exit 1
  done
done
