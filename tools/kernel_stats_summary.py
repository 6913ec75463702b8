#!/usr/bin/env python3
"""Per-kernel-class launches and time from a rocprofv3 --stats summary (run_kernel_stats.csv).

The PLL runner forms are told apart by their template arguments (pll_pipe_kernel<NB, BPI, RD, NC>:
16-step five-candidate from 2^20, 64-step five from 2^21, three-candidate from 2^22;
pll_idx_kernel<NC, NW>: 32 candidates [2^18, 2^19), 16 [2^19, 2^20)), so a trace of the CLI shows
which runners each range of the stream ran on across its --batch calls.

    python tools/kernel_stats_summary.py <dir>/run_kernel_stats.csv
"""
import csv
import json
import re
import sys
from collections import defaultdict


def klass(name: str) -> str:
    m = re.search(r"pll_pipe_kernel<(\d+), (\d+), (\d+), (\d+)>", name)
    if m:
        nb, bpi, _, nc = (int(v) for v in m.groups())
        return f"pll_pipe {nb * bpi}-step NC={nc}"
    m = re.search(r"pll_idx_kernel<(\d+), (\d+)>", name)
    if m:
        return f"pll_idx NC={m.group(1)}"
    for key in ("mono_fused", "bpf_pair", "pll_nco", "stereo_audio", "stereo_state", "copy_streams", "pll_prep",
                "pll_check", "pll_spec_lane", "pll_kernel", "pll_sat", "pll_pred"):
        if key in name:
            return key
    return name.split("(")[0][-48:]


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    calls, ms = defaultdict(int), defaultdict(float)
    for r in rows:
        k = klass(r["Name"])
        calls[k] += int(r["Calls"])
        ms[k] += float(r["TotalDurationNs"]) / 1e6
    out = {k: {"calls": calls[k], "ms": round(ms[k], 3)} for k in sorted(ms, key=ms.get, reverse=True)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
