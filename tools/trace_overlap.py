#!/usr/bin/env python3
"""Stage overlap inside one stereo call, from a rocprofv3 kernel trace (run_kernel_trace.csv).

The pipelined engine (api.cpp run_stereo_pipelined) puts the front end + band-pass pair, the PLL
and the audio stage on three HIP streams (three hardware queues).  A call ends with one
stereo_state_kernel; this takes the LAST call in the trace (from the first kernel after the
previous stereo_state_kernel to its own), and prints one JSON line: the call's device span, each
queue's busy time (union of its kernels' intervals) and kernel classes, the union over queues,
and the time two or more queues were busy at once (the overlap).

    python tools/trace_overlap.py <dir>/run_kernel_trace.csv
"""
import csv
import json
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def klass(name: str) -> str:
    for key in ("mono_fused", "bpf_pair", "pll_nco", "stereo_audio", "stereo_state", "copy_streams", "pll_prep",
                "pll_check", "pll_spec_lane", "pll_kernel", "pll_pipe", "pll_idx", "pll_sat", "pll_pred"):
        if key in name:
            return key
    return name.split("(")[0][-40:]


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    cols = rows[0].keys()
    qcol = next((c for c in ("Queue_Id", "Stream_Id", "Queue_ID") if c in cols), None)
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qcol, "0") if qcol else "0")
          for r in rows if not r["Kernel_Name"].startswith("__amd_rocclr")]  # (reset()'s fills, copies)
    ev.sort()
    ends = [i for i, e in enumerate(ev) if "stereo_state" in e[2]]
    if not ends:
        print(json.dumps({"error": "no stereo_state_kernel in the trace"}))
        return
    last = ends[-1]
    first = ends[-2] + 1 if len(ends) > 1 else 0
    call = ev[first:last + 1]
    t0 = min(e[0] for e in call)
    t1 = max(e[1] for e in call)
    by_q = defaultdict(list)
    classes = defaultdict(lambda: defaultdict(float))
    for s, e, n, q in call:
        by_q[q].append((s, e))
        classes[q][klass(n)] += (e - s) / 1e6
    busy = {q: union(v) / 1e6 for q, v in by_q.items()}
    all_busy = union([iv for v in by_q.values() for iv in v]) / 1e6
    out = {"kernels": len(call), "span_ms": round((t1 - t0) / 1e6, 3), "queues": len(by_q),
           "queue_busy_ms": {q: round(b, 3) for q, b in busy.items()},
           "queue_kernels_ms": {q: {k: round(v, 3) for k, v in c.items()} for q, c in classes.items()},
           "union_busy_ms": round(all_busy, 3), "overlap_ms": round(sum(busy.values()) - all_busy, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
