#!/usr/bin/env python3
"""Copy a gpu_bench_prof.sh run (gpurun_out/<tag>) into profiles/<dest>/ and recompute
profiles/traffic_mono101.json (HBM bytes per fused-kernel launch from the PMC passes).

    python tools/update_profiles.py <tag> <dest>
"""
import csv
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_hash: the stamp bench.py checks)

BENCH_HASH = bench.kernel_source_hash()

tag, dest = sys.argv[1], sys.argv[2]
src = f"gpurun_out/{tag}"
out = f"profiles/{dest}"
os.makedirs(out, exist_ok=True)
shutil.copy(f"{src}/kt/run_kernel_stats.csv", f"{out}/kernel_stats.csv")
# the traced bench's timed launches are its last `steps` fused launches (the untimed warm-up
# runs >= 1 s first): their mean duration is what bench.py's kernel_ms measures
trace = [r for r in csv.DictReader(open(f"{src}/kt/run_kernel_trace.csv")) if "mono_fused" in r["Kernel_Name"]]
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
kt_steps = 10  # tools/gpu_bench_prof.sh traces bench.py --steps 10
last = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace[-kt_steps:]]
with open(f"{out}/kernel_trace_timed_launches.json", "w") as g:
    json.dump({"kernel": "mono_fused_kernel", "launches_traced": len(trace), "timed_launches": len(last),
               "timed_mean_ns": sum(last) / len(last), "timed_ns": last,
               "note": "rocprofv3 --kernel-trace of bench.py --steps 10: the last 10 fused launches are the timed "
                       "ones (kernel_stats.csv averages every launch, warm-up included)"}, g, indent=1)
shutil.copy(f"{src}/bench.json", f"{out}/bench.json")
res = {}
for f, key in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    rows = [r for r in csv.DictReader(open(f"{src}/{f}/run_counter_collection.csv")) if "mono_fused" in r["Kernel_Name"]]
    vals = [float(r["Counter_Value"]) for r in rows]
    res[key + "_kb_per_launch"] = sum(vals) / len(vals)
    res[key + "_launches"] = len(vals)
    with open(f"{out}/{f}_mono_fused.csv", "w") as g:
        w = csv.writer(g)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "DurationNs", "Grid_Size", "Workgroup_Size",
                    "LDS_Block_Size", "VGPR_Count", "SGPR_Count"])
        for r in rows:
            w.writerow([r["Kernel_Name"][:60], r["Counter_Name"], r["Counter_Value"],
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Grid_Size"], r["Workgroup_Size"],
                        r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"]])
# effective clock (MI355X_MICROARCH.md, DVFS give-back): GRBM_GUI_ACTIVE summed over the 8 XCDs
# / 8 / the dispatch's own duration, per fused launch of the GRBM pass
clk = None
if os.path.exists(f"{src}/pmc_grbm/run_counter_collection.csv"):
    rows = [r for r in csv.DictReader(open(f"{src}/pmc_grbm/run_counter_collection.csv"))
            if "mono_fused" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
    ghz = [float(r["Counter_Value"]) / 8 / (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows]
    if ghz:
        clk = round(sorted(ghz)[len(ghz) // 2], 3)
        with open(f"{out}/pmc_grbm_mono_fused.csv", "w") as g:
            w = csv.writer(g)
            w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "DurationNs", "effective_clock_GHz"])
            for r, c in zip(rows, ghz):
                w.writerow([r["Kernel_Name"][:60], r["Counter_Name"], r["Counter_Value"],
                            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), round(c, 4)])
bline = json.load(open(f"{src}/bench.json"))
alg = bline["roofline"]["alg_bytes_per_launch"]
fetch = res["FETCH_SIZE_kb_per_launch"] * 1024 * 2  # gfx950: FETCH_SIZE counts half of a coalesced stream
write = res["WRITE_SIZE_kb_per_launch"] * 1024
res.update({
    "kernel": bline["roofline"]["kernel"], "kernel_source_sha256": BENCH_HASH,
    "effective_clock_ghz": clk,
    "clock_note": "median over the GRBM pass's fused launches of GRBM_GUI_ACTIVE / 8 / duration" if clk else None,
    "workload": "1 GiB mode-0 mono, 101-tap RF (bench.py)",
    "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE "
                  "counts half the bytes of a coalesced stream; units KiB)",
    "hbm_read_bytes_per_launch": int(fetch), "hbm_write_bytes_per_launch": int(write),
    "hbm_bytes_per_launch": int(fetch + write), "alg_bytes_per_launch": alg,
    "traffic_over_alg": round((fetch + write) / alg, 4),
    "source": f"profiles/{dest}/pmc_*_mono_fused.csv (rocprofv3 --pmc, separate passes)"})
json.dump(res, open("profiles/traffic_mono101.json", "w"), indent=1)
print(json.dumps(res, indent=1))
