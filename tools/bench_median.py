#!/usr/bin/env python3
"""Median of tools/bench_median.sh's five bench lines -> one JSON object (value, kernel_ms,
roofline fractions, the five values)."""
import json
import statistics
import sys

tag = sys.argv[1]
runs = [json.loads(open(f"gpurun_out/{tag}/bench_{i}.json").read().strip().splitlines()[-1]) for i in range(1, 6)]
vals = [r["value"] for r in runs]
med = sorted(runs, key=lambda r: r["value"])[2]
print(json.dumps({"runs": 5, "values_MS_s": vals, "median_MS_s": statistics.median(vals),
                  "kernel_ms": [r["roofline"]["kernel_ms"] for r in runs],
                  "median_run": {"value": med["value"], "kernel_ms": med["roofline"]["kernel_ms"],
                                 "hbm_frac": med["roofline"]["frac"],
                                 "valu_frac": med["roofline"]["binding"]["frac"],
                                 "hbm_attainable_GBs": med["roofline"].get("hbm_attainable_GBs"),
                                 "traffic": med["roofline"].get("traffic")}}, indent=1))
