#!/usr/bin/env python3
"""Mean over launches of the fused mono kernel's SQ counters (gpurun_out/<tag>/p*/ from
tools/gpu_sq.sh), with the VALU issue floor; writes the summary and the per-pass CSVs.

    python tools/sq_mean.py <tag> <dest dir> <kernel ms> <clock GHz>
"""
import collections
import csv
import glob
import os
import shutil
import sys

tag, dest, kms, ghz = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4])
os.makedirs(dest, exist_ok=True)
agg, n = collections.OrderedDict(), 0
for i, f in enumerate(sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")), 1):
    rows = [r for r in csv.DictReader(open(f)) if "mono_fused" in r["Kernel_Name"]]
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in by.items():
        agg[k] = sum(v) / len(v)
        n = len(v)
    shutil.copy(f, os.path.join(dest, f"pass{i}_mono_fused.csv"))
wc = agg["SQ_WAVE_CYCLES"]
lines = [f"== {tag}: SQ passes of mono_fused_kernel<101,10,5,64,3,4,TR=1> (the default), mean over {n} launches"]
lines += [f"  {k:24s} {v:16.0f}" for k, v in agg.items()]
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
          "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
    if k in agg:
        lines.append(f"  {k:24s} / WAVE_CYCLES = {agg[k] / wc:.3f}")
v = agg["SQ_INSTS_VALU"]
floor_cyc = v * 4 / 1024
floor_ms = floor_cyc / ghz / 1e6
lines.append(f"  VALU floor: {v:.0f} VALU wave-instructions x 4 cycles / 1024 SIMDs = {floor_cyc:.0f} cycles = "
             f"{floor_ms:.3f} ms at {ghz} GHz; kernel {kms} ms -> VALU busy {floor_ms / kms:.3f} of the SIMD cycles")
open(os.path.join(dest, "sq_default_kernel.txt"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
