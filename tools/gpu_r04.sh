#!/bin/bash
# tools/gpu_r04.sh — round-4 GPU record (one recipe, edited per run): the whole GPU suite, smoke(),
# the bench line + kernel trace + PMC passes (tools/gpu_bench_prof.sh), and the extra steps named
# on the command line: sq (mono SQ passes), cli (drop-in CLI vs project), overlap (tools/overlap_probe.py).
set -o pipefail
TAG=${1:-r04_a}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
bash tools/gpu_bench_prof.sh $TAG || exit 3
head -c 600 $OUT/bench.json; echo
for step in "$@"; do
  case $step in
    sq) bash tools/gpu_sq.sh ${TAG}_sq 6 || exit 4 ;;
    cli) timeout -k 10 400 python tools/bench_cli.py --mib 1024 --mode 0 > $OUT/bench_cli.json 2> $OUT/bench_cli.err || exit 5
         cat $OUT/bench_cli.json ;;
    overlap) timeout -k 10 300 python tools/overlap_probe.py > $OUT/overlap.json 2> $OUT/overlap.err || exit 6
         cat $OUT/overlap.json ;;
  esac
done
echo all done
