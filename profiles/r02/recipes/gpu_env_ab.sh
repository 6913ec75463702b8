#!/bin/bash
# A/B of an environment switch on the stereo bench: tools/gpu_env_ab.sh <tag> <VAR> "<values>" "<streams>"
set -o pipefail
OUT=gpurun_out/$1
VAR=$2
mkdir -p $OUT
for rep in 1 2; do
  for v in $3; do
    env $VAR=$v timeout -k 10 200 python tools/bench_stereo.py --streams $4 > $OUT/b_$v.$rep.json 2>> $OUT/bench.err || exit 2
  done
done
echo done
