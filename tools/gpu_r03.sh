#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the older wave's share of a SIMD pair's span (FMRX_MONO_SPLIT, in 1/1024; default 620) swept
# again on the round's final mono kernel: bench lines cycling 620 / 645 / 660 / 675 (second sweep) on one box.
set -o pipefail
OUT=gpurun_out/${1:-r03_split2}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for sp in 620 645 660 675; do
    FMRX_MONO_SPLIT=$sp timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/s${sp}_$i.json 2> $OUT/s${sp}_$i.err || exit 2
  done
done
OUT=$OUT python - <<'PY'
import json,glob,os
out=os.environ["OUT"]
for sp in (620,645,660,675):
    r=[json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/s{sp}_*.json"))]
    ms=[x["roofline"]["kernel_ms"] for x in r]
    print(sp, [round(m,4) for m in ms], "mean %.4f" % (sum(ms)/len(ms)))
PY
