#!/bin/bash
# Round-6: the Python two-thread seam leg's queue depth (project.cpp QUEUE_CAPACITY 3 / 16 / 64),
# three runs each, alternating.  arg: out dir.
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
for rep in 1 2 3; do
  for qd in 3 16 64; do
    timeout -k 10 120 python -u tools/bench_seam.py --blocks 3000 --queue $qd --legs serial,two_threads \
        > "$out/q${qd}_$rep.json" 2> "$out/q${qd}_$rep.err" || { echo "q$qd failed"; exit 1; }
    python - "$out/q${qd}_$rep.json" $qd <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("queue", sys.argv[2], "serial", d["serial"]["x_realtime"], "two_threads", d["two_threads"]["x_realtime"])
PY
  done
done
