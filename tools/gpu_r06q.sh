#!/bin/bash
# Round-6: does the demoted kernel's LDS (39 / 20 / 10 KB: sub-segments of 16 / 8 / 4 batches) set
# what its launches cost configs[4]?  Probe + the unlocked streams per build.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
A=software-defined-radio-course-project_amd
for rep in 1 2; do
  for spec in new= s8=$A/build_ab_S8/libfmrx.so s4=$A/build_ab_S4/libfmrx.so; do
    name=${spec%%=*}; path=${spec#*=}
    FMRX_LIB_PATH=$path timeout -k 10 200 python -u tools/demote_probe.py --repeats 3 > "$out/${name}_$rep.json" 2> "$out/${name}_$rep.err" || { echo "$name failed"; tail -5 "$out/${name}_$rep.err"; exit 1; }
    echo "$name $(cut -c1-160 "$out/${name}_$rep.json")"
  done
done
for spec in s8=$A/build_ab_S8/libfmrx.so s4=$A/build_ab_S4/libfmrx.so; do
  name=${spec%%=*}; path=${spec#*=}
  FMRX_LIB_PATH=$path timeout -k 10 400 python -u tools/bench_unlocked.py --only unlocked_m0_rand_80s unlocked_m2_synth_170b \
      --out "$out/unlocked_$name.json" > "$out/unlocked_$name.log" 2>&1 || { echo "unlocked $name failed"; exit 1; }
  python - "$out/unlocked_$name.json" $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (v["seconds"]["median"], v["ns_per_pll_step"], v["bit_exact_pcm"]) for k, v in d.items() if isinstance(v, dict)})
PY
done
