#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# A/B of the mono kernel: next chunk staged right after the FIR (libfmrx.so) vs staged at the top of its iteration
# (build_ab/: the previous commit's source), alternating bench lines on one box; mono/stereo parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r03_stage}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "mono or bench_config or stereo or modes or seek or state" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/new_$i.json 2> $OUT/new_$i.err || exit 2
  FMRX_LIB_PATH=$PWD/software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/old_$i.json 2> $OUT/old_$i.err || exit 3
done
OUT=$OUT python - <<'PY'
import json,glob,os
out=os.environ["OUT"]
for v in ("new","old"):
    r=[json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/{v}_*.json"))]
    ms=[x["roofline"]["kernel_ms"] for x in r]
    print(v, [round(m,4) for m in ms], "mean %.4f" % (sum(ms)/len(ms)))
PY
