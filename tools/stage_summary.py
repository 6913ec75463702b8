#!/usr/bin/env python3
"""One line from a tools/stage_times.py JSON: each config's best wall time and, per PLL runner
regime, ns a step.

    python tools/stage_summary.py <stage_times.json>
"""
import json
import sys

j = json.load(open(sys.argv[1]))
parts = []
for k, v in j.items():
    rs = {s.replace("runner_", ""): x["ns_per_step"] for s, x in v["stages"].items() if "ns_per_step" in x}
    parts.append(f"{k} {min(v['wall_s']):.4f}s " + " ".join(f"{s}={n}" for s, n in rs.items()))
print(" | ".join(parts))
