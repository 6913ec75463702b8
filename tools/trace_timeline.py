#!/usr/bin/env python3
"""Timeline of the last kernels / copies / HIP API calls in a rocprofv3 trace database:
    python tools/trace_timeline.py <db> [--last 60] [--api]"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--last", type=int, default=60)
ap.add_argument("--api", action="store_true", help="also HIP runtime API calls (--hip-runtime-trace)")
a = ap.parse_args()
cur = sqlite3.connect(a.db).cursor()
ev = [(s, e, "K " + (n or "")[:34]) for s, e, n in cur.execute(
    "select d.start, d.end, s.display_name from rocpd_kernel_dispatch d "
    "join rocpd_info_kernel_symbol s on s.id = d.kernel_id")]
ev += [(s, e, f"C copy {n}B") for s, e, n in cur.execute("select start, end, size from rocpd_memory_copy")]
if a.api:
    tabs = {r[0] for r in cur.execute("select name from sqlite_master")}
    if "rocpd_region" in tabs:
        ev += [(s, e, "  api " + (n or "")) for s, e, n in cur.execute(
            "select r.start, r.end, st.string from rocpd_region r join rocpd_string st on st.id = r.name_id")]
ev.sort()
last_k = max(e for s_, e, n in ev if n.startswith("K "))
ev = [x for x in ev if x[0] <= last_k][-a.last:]  # (the teardown after the last kernel dropped)
t0 = ev[0][0]
for s, e, n in ev:
    print(f"{(s - t0) / 1e3:9.1f} -> {(e - t0) / 1e3:9.1f}  {(e - s) / 1e3:6.1f}  {n}")
