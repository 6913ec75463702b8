#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/<tag>/p*/run_counter_collection.csv) for the fused kernel."""
import collections, csv, glob, sys
for tag in sys.argv[1:]:
    agg = {}
    for f in sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if "mono_fused" in r["Kernel_Name"]]
        last = collections.OrderedDict()
        for r in rows:
            last[r["Counter_Name"]] = float(r["Counter_Value"])
        agg.update(last)
    print(f"== {tag}")
    for k, v in agg.items():
        print(f"  {k:24s} {v:16.0f}")
    if "SQ_WAVE_CYCLES" in agg:
        wc = agg["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT"):
            if k in agg:
                print(f"  {k:24s} / WAVE_CYCLES = {agg[k]/wc:.3f}")
