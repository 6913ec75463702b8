#!/bin/bash
# Round-6: configs[4] per-regime ns a step (stage timer) for the in-tree build, without the demoted
# launches, and the pre-round library; the locked 72 s stream A/B.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked or pll" > "$out/dem_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/dem_tests.log"; exit 1; }
tail -1 "$out/dem_tests.log"
for rep in 1 2; do
  for spec in new= nodl=$A/build_ab_NO_DEMOTED_LAUNCH/libfmrx.so head=$A/build_ab_head/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}; pf=""; [ $rep = 1 ] && pf="--profile"
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 $pf > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json")"
  done
done
tools/gpu_r06_ab2.sh "$out/ab" new= head=$A/build_ab_head/libfmrx.so || { echo "ab failed"; exit 1; }
