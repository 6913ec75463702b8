#!/usr/bin/env python3
"""Sweep the compiled fused-kernel variants (FMRX_MONO_VARIANT) on the bench workload.
Each variant runs in its own process (the variant is latched per process)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for rnd in range(2):
    for v in range(n):
        env = dict(os.environ, FMRX_MONO_VARIANT=str(v))
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10", "--warmup", "2",
                            "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(f"variant {v}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            continue
        j = json.loads(r.stdout.strip().splitlines()[-1])
        print(f"round {rnd} variant {v}: kernel {j['roofline']['kernel_ms']:.4f} ms  value {j['value']:.0f} MS/s  "
              f"valu frac {j['compute']['frac']:.3f}", flush=True)
