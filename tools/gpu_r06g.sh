#!/bin/bash
# Round-6: configs[4]'s demotions of locked streams -- the index runner's threshold (24 / 28 / 32 of
# the last 32 intervals), the no-demotion build and the pre-round library, alternating.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
for rep in 1 2; do
  for spec in new= d28=$A/build_ab_d28/libfmrx.so d32=$A/build_ab_d32/libfmrx.so nodem=$A/build_ab_nodem/libfmrx.so head=$A/build_ab_head/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json")"
  done
done
