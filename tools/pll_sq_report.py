#!/usr/bin/env python3
"""Summarise tools/gpu_pll_sq.sh: SQ counters of one PLL kernel per pass (summed over launches).

    python tools/pll_sq_report.py <tag> [kernel name substring, default pll_kernel]
"""
import collections, csv, glob, sys
tag = sys.argv[1] if len(sys.argv) > 1 else "pllsq"
for f in sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")):
    agg = collections.Counter()
    for r in csv.DictReader(open(f)):
        if (sys.argv[2] if len(sys.argv) > 2 else "pll_kernel") in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f)
    for k, v in agg.items():
        print(f"  {k:24s} {v:16.0f}")
