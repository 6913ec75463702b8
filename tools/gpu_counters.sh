#!/bin/bash
# SQ counter passes for the fused mono kernel (one --pmc pass per group, kernel-trace off).
set -o pipefail
OUT=gpurun_out/${1:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -T -d $OUT/p$i -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $grp" >> $OUT/failed.txt; exit 1; }
done
echo done
