#!/bin/bash
# Round-6: the demoted kernel in two waves (chain + one checker: dispatchable beside the pipelined
# front end's two waves a CU) on configs[4] and on the unlocked streams.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
for rep in 1 2; do
  for spec in new= d2=$A/build_ab_D2/libfmrx.so d2w2=$A/build_ab_D2W2/libfmrx.so nodl=$A/build_ab_NO_DEMOTED_LAUNCH/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cat "$out/${name}_$rep.json")"
  done
done
for spec in d2=$A/build_ab_D2/libfmrx.so d2w2=$A/build_ab_D2W2/libfmrx.so; do
  name=${spec%%=*}; path=${spec#*=}
  FMRX_LIB_PATH=$path timeout -k 10 400 python -u tools/bench_unlocked.py --out "$out/unlocked_$name.json" > "$out/unlocked_$name.log" 2>&1 || { echo "unlocked $name failed"; tail -5 "$out/unlocked_$name.log"; exit 1; }
done
python - "$out" <<'PY'
import json, sys
for n in ("d2", "d2w2"):
    d = json.load(open(f"{sys.argv[1]}/unlocked_{n}.json"))
    print(n, {k: (v["seconds"]["median"], v["ns_per_pll_step"], v["bit_exact_pcm"], v["bit_exact_pll_state"]) for k, v in d.items() if isinstance(v, dict)})
PY
