#!/bin/bash
# Round-6: where configs[4]'s round-6 time goes -- the in-tree build (index demotion at 28 / 32),
# without the demoted-kernel launches, without the long forms' tail split, the pre-round library,
# alternating (tools/demote_probe.py).  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
for rep in 1 2; do
  for spec in new= nodl=$A/build_ab_NO_DEMOTED_LAUNCH/libfmrx.so nots=$A/build_ab_NO_TAIL_SPLIT/libfmrx.so head=$A/build_ab_head/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json")"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "demotion or redo_slots or seam_calls or unlocked or stereo" > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
