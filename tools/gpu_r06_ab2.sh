#!/bin/bash
# A/B of library builds and tuning environments on the locked 72 s stream (tools/bench_unlocked.py
# --only), alternating; args: output dir, then name=path[,VAR=value...] (path empty: in-tree library)
set -o pipefail
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}
    path=${rest%%,*}; envs=""
    [ "$rest" != "$path" ] && envs=$(echo "${rest#*,}" | tr ',' ' ')
    env FMRX_LIB_PATH=$path $envs timeout -k 10 120 python -u tools/bench_unlocked.py --only m0_rf51_synth_72s \
        --out "$out/${name}_$rep.json" > "$out/${name}_$rep.log" 2>&1 || exit 1
  done
done
