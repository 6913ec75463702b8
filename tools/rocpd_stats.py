#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 SQLite result (run_results.db): name, calls, total ms, mean us."""
import glob, sqlite3, sys
for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    sym = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    dis = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    cols = [r[1] for r in c.execute(f"pragma table_info({dis})")]
    scols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name_col = 'kernel_name' if 'kernel_name' in scols else ('display_name' if 'display_name' in scols else 'name')
    rows = c.execute(f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start) from {dis} d "
                     f"join {sym} s on d.kernel_id = s.id group by s.{name_col} order by 3 desc").fetchall()
    print(f)
    for n, k, tot, avg in rows:
        short = n.split('(')[0].replace('fmrx::(anonymous namespace)::', '')[:60]
        print(f"  {short:60s} {k:6d} {tot/1e6:10.3f} ms {avg/1e3:10.1f} us")
