#!/usr/bin/env python3
"""BASELINE configs[3] (mode-2 mono, 147/800 resampler, 1 GiB) profile of record: copy a
`tools/gpu_r05.sh <tag> mode2` run (gpurun_out/<tag>) into profiles/<dest>/ and write
profiles/traffic_mode2.json -- the warm kernel-trace duration of the timed launches, HBM bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md §HBM: gfx950's
FETCH_SIZE counts half the bytes of a coalesced stream; KiB) and the GRBM effective clock, stamped
with the hash of the fused kernel's sources.  bench.py reports configs[3]'s `traffic` only while
that hash matches the tree.

    python tools/update_profiles_mode2.py <tag> <dest>      (e.g. r05a r05/prof_mode2)
"""
import csv
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_hash: the stamp bench.py checks)

tag, dest = sys.argv[1], sys.argv[2]
src = f"gpurun_out/{tag}"
out = f"profiles/{dest}"
os.makedirs(out, exist_ok=True)
KSUB = "mono_fused_kernel<51, 10, 800"
STEPS = 20  # tools/gpu_r05.sh mode2: bench_modes.py --modes 2 --steps 20 --warmup-seconds 1.5


def rows_of(path):
    return [r for r in csv.DictReader(open(path)) if KSUB in r["Kernel_Name"]]


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


shutil.copy(f"{src}/m2_kt/run_kernel_stats.csv", f"{out}/kernel_stats.csv")
trace = sorted(rows_of(f"{src}/m2_kt/run_kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
timed = [dur(r) for r in trace[-STEPS:]]
line = [json.loads(x) for x in open(f"{src}/m2_kt.log") if x.startswith("{")][-1]
with open(f"{out}/kernel_trace_timed_launches.json", "w") as g:
    json.dump({"kernel": trace[0]["Kernel_Name"][:110], "launches_traced": len(trace), "timed_launches": len(timed),
               "timed_mean_ns": sum(timed) / len(timed), "timed_ns": timed,
               "warm_mean_ns_all": sum(dur(r) for r in trace) / len(trace),
               "bench_modes_line": line,
               "note": "rocprofv3 --kernel-trace of tools/bench_modes.py --modes 2 --steps 20 --warmup-seconds 1.5: "
                       "the last 20 fused launches are the timed ones, after >= 1.5 s of back-to-back launches"},
              g, indent=1)
res = {}
for f, key in (("m2_fetch", "FETCH_SIZE"), ("m2_write", "WRITE_SIZE")):
    rows = rows_of(f"{src}/{f}/run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in rows]
    res[key + "_kb_per_launch"] = sum(vals) / len(vals)
    res[key + "_launches"] = len(vals)
    with open(f"{out}/pmc_{key.lower()}_mode2.csv", "w") as g:
        w = csv.writer(g)
        w.writerow(["Counter_Name", "Counter_Value", "DurationNs", "VGPR_Count", "LDS_Block_Size"])
        for r in rows:
            w.writerow([r["Counter_Name"], r["Counter_Value"], dur(r), r["VGPR_Count"], r["LDS_Block_Size"]])
rows = [r for r in rows_of(f"{src}/m2_grbm/run_counter_collection.csv") if r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
ghz = sorted(float(r["Counter_Value"]) / 8 / dur(r) for r in rows)
clk = round(ghz[len(ghz) // 2], 3)
# algorithmic bytes of one launch (bench.py other_configs): u8 I+Q in, S16 mono out
blocks = int(re.search(r"(\d+) blocks", line["workload"]).group(1))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import iqgen  # noqa: E402

fm = iqgen.load_fmrx()
geo = fm.geometry(fm.default_config(2, fm.MONO))
bb, na = geo.block_bytes, geo.audio_frames
alg = blocks * bb + 2 * blocks * na
fetch = res["FETCH_SIZE_kb_per_launch"] * 1024 * 2
write = res["WRITE_SIZE_kb_per_launch"] * 1024
kt = sum(timed) / len(timed) * 1e-9
res.update({
    "kernel": "mono_fused_kernel<51,10,800,64,3,4,0,1,147,1>", "kernel_source_sha256": bench.kernel_source_hash(),
    "workload": "BASELINE configs[3]: 1 GiB mode-2 mono (147/800 resampler), 51-tap RF (tools/bench_modes.py)",
    "blocks": blocks, "alg_bytes_per_launch": alg,
    "timed_kernel_ms_trace": round(kt * 1e3, 4),
    "achieved_GBs_trace": round(alg / kt / 1e9, 1), "frac_of_8TBs_trace": round(alg / kt / 1e9 / 8000.0, 4),
    "effective_clock_ghz": clk,
    "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM; units KiB)",
    "hbm_read_bytes_per_launch": int(fetch), "hbm_write_bytes_per_launch": int(write),
    "hbm_bytes_per_launch": int(fetch + write), "traffic_over_alg": round((fetch + write) / alg, 4),
    "source": f"profiles/{dest}/ (rocprofv3 --kernel-trace and separate --pmc passes)"})
json.dump(res, open("profiles/traffic_mode2.json", "w"), indent=1)
print(json.dumps(res, indent=1))
