#!/bin/bash
# Five consecutive bench.py runs on one box (report the median of >= 5 runs).
# Usage (gpurun): bash tools/bench_median.sh <tag>; then python tools/bench_median.py <tag>
set -o pipefail
OUT=gpurun_out/${1:-median}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 1
done
echo done
