#!/bin/bash
# tools/gpu_r03.sh — the current round-3 GPU check (edited per run; one recipe, not one per run):
# the whole GPU suite, smoke(), then tools/gpu_bench_prof.sh (bench line, kernel trace, PMC passes)
# for the mono kernel's final sources of the round.
set -o pipefail
TAG=${1:-r03_prof6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
bash tools/gpu_bench_prof.sh $TAG || exit 3
cat $OUT/bench.json
