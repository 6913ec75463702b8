#!/bin/bash
# tools/gpu_r04.sh — round-4 GPU record: the whole GPU suite, smoke(), the bench line + kernel trace
# + PMC passes (tools/gpu_bench_prof.sh), and the extra steps named on the command line:
#   sq (mono SQ passes), cli (drop-in CLI vs project, tools/bench_cli.py), c3 (kernel trace of
#   configs[3], the mode-2 mono product, full kernel names), c4 (kernel trace of configs[4] calls +
#   tools/trace_overlap.py), overlap (tools/overlap_probe.py).
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
    c3) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c3 -o run --output-format csv -- \
          python3 tools/bench_modes.py --modes 2 --steps 10 > $OUT/kt_c3.log 2>&1 || exit 7
        tail -2 $OUT/kt_c3.log ;;
    c4) timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_c4 -o run --output-format csv -- \
          python3 tools/stage_times.py --no-gib --single 0 > $OUT/kt_c4.log 2>&1 || exit 8
        f=$(ls $OUT/kt_c4/*/run_kernel_trace.csv $OUT/kt_c4/run_kernel_trace.csv 2>/dev/null | head -1)
        python tools/trace_overlap.py $f > $OUT/overlap_c4.json && cat $OUT/overlap_c4.json ;;
    overlap) timeout -k 10 300 python tools/overlap_probe.py > $OUT/overlap.json 2> $OUT/overlap.err || exit 6
         cat $OUT/overlap.json ;;
  esac
done
echo all done
