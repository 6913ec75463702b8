#!/usr/bin/env python3
"""Time a list of fused-kernel variants (FMRX_MONO_VARIANT), interleaved rounds, one process each."""
import json, os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vs = [int(v) for v in sys.argv[1].split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
res = {v: [] for v in vs}
for rnd in range(rounds):
    for v in vs:
        env = dict(os.environ, FMRX_MONO_VARIANT=str(v))
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10", "--warmup", "2",
                            "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print("variant", v, "FAILED", r.stderr[-800:], flush=True); continue
        res[v].append(json.loads(r.stdout.strip().splitlines()[-1])["roofline"]["kernel_ms"])
for v in vs:
    x = sorted(res[v])
    print(f"variant {v:2d}: kernel ms median {x[len(x)//2]:.4f} min {x[0]:.4f} all {x}", flush=True)
