#!/usr/bin/env python3
"""Table of tools/gpu_ablate.sh: per FMRX_ABLATE bitmask the kernel time (HIP events), the SQ
counters per launch (VALU instructions, VALU-active / wait fractions of wave cycles), the
effective clock (GRBM_GUI_ACTIVE / 8 / duration) and the in-kernel clock stamps.

    python tools/ablate_report.py <tag> [--md]   (reads gpurun_out/<tag>)
"""
import csv
import json
import sys
from collections import defaultdict

NAMES = {0: "full kernel", 1: "no RF FIR", 2: "no audio FIR", 4: "no demod", 8: "no byte conversion",
         16: "no global loads", 32: "no staging writes", 6: "no audio, no demod", 14: "no audio/demod/conversion",
         62: "RF FIR only (no loads/staging/conv/demod/audio)", 63: "skeleton (nothing)"}


def pmc(tag, a):
    per = defaultdict(list)
    rows = list(csv.DictReader(open(f"gpurun_out/{tag}/pmc_{a}/run_counter_collection.csv")))
    for r in rows:
        if "mono_fused" in r["Kernel_Name"]:
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key].append(float(r["Counter_Value"]))
    by = defaultdict(dict)
    dur = {}
    for r in rows:
        if "mono_fused" in r["Kernel_Name"]:
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (d, c), v in per.items():
        by[d][c] = sum(v)
    ds = sorted(by, key=int)[1:]  # drop the first (warm-up) dispatch
    avg = {c: sum(by[d][c] for d in ds) / len(ds) for c in by[ds[0]]}
    avg["dur_ns"] = sum(dur[d] for d in ds) / len(ds)
    return avg


def main():
    tag = sys.argv[1]
    rows = []
    for a in [0, 1, 2, 4, 8, 16, 32, 6, 14, 62, 63]:
        try:
            b = json.loads(open(f"gpurun_out/{tag}/bench_{a}.json").read().strip().splitlines()[-1])
            p = pmc(tag, a)
        except (OSError, IndexError, KeyError, ValueError):
            continue
        wc = p["SQ_WAVE_CYCLES"]
        rows.append({"ablate": a, "what": NAMES.get(a, str(a)), "kernel_ms": b["roofline"]["kernel_ms"],
                     "valu_insts_M": round(p["SQ_INSTS_VALU"] / 1e6, 1),
                     "valu_active_frac": round(p["SQ_ACTIVE_INST_VALU"] / wc, 3),
                     "wait_any_frac": round(p["SQ_WAIT_ANY"] / wc, 3),
                     "wait_inst_frac": round(p["SQ_WAIT_INST_ANY"] / wc, 3),
                     "lds_insts_M": round(p["SQ_INSTS_LDS"] / 1e6, 1),
                     "clock_ghz_grbm": round(p["GRBM_GUI_ACTIVE"] / 8 / p["dur_ns"], 3),
                     "pmc_kernel_ms": round(p["dur_ns"] / 1e6, 4)})
    out = {"rows": rows}
    try:
        out["stamps"] = json.loads(open(f"gpurun_out/{tag}/mono_stamps.json").read())
    except (OSError, ValueError):
        pass
    if "--md" in sys.argv:
        print("| FMRX_ABLATE | removed | kernel ms | VALU insts (M) | VALU active / wave cycles | s_waitcnt / wave cycles | issue-stall / wave cycles | LDS insts (M) | clock (GRBM, GHz) |")
        print("|---|---|---|---|---|---|---|---|---|")
        for r in rows:
            print(f"| {r['ablate']} | {r['what']} | {r['kernel_ms']} | {r['valu_insts_M']} | {r['valu_active_frac']} | "
                  f"{r['wait_any_frac']} | {r['wait_inst_frac']} | {r['lds_insts_M']} | {r['clock_ghz_grbm']} |")
    else:
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
