#!/usr/bin/env python3
"""Time-parallel PLL feasibility: does a speculative restart of the stereo pilot
PLL (src/filter.cpp:136-174, project.cpp:166) bit-merge with the true trajectory?

Builds tools/pll_merge.cpp, makes the 19 kHz carrier (the reference's carrier band-pass
output, through the C oracle) of 12 s of mode-0 input for three signals -- the synthetic FM
broadcast with pilot (synth), uniform random u8 I/Q (rand) and a constant 0x80 stream (const)
-- and runs the merge measurement before and after the float trigOffset saturates (2^24).
Writes one JSON object (host-only; the oracle is the checker here, not the product).

    python tools/pll_merge.py [--seconds 12] [--restarts 24] [--max-steps 1000000] > profiles/r02/pll_merge.json
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--restarts", type=int, default=24)
    ap.add_argument("--max-steps", type=int, default=1000000)
    args = ap.parse_args()
    import iqgen
    import oracle

    tmp = tempfile.mkdtemp()
    exe = os.path.join(tmp, "pll_merge")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(REPO, "tools", "pll_merge.cpp")],
                   check=True)
    orc = oracle.Oracle()
    bb = oracle.MODES[0][0]
    nb = int(args.seconds * 2.4e6 * 2 // bb)
    out = {"what": "bit-merge of speculative PLL restarts with the true trajectory (reference arithmetic, glibc)",
           "seconds": args.seconds, "steps_per_second": 240000}
    for name, recipe in (("synth", "synth:7"), ("rand", "rand:7"), ("const", "const128")):
        iq = iqgen.make(recipe, nb * bb)
        car = orc.run(0, 51, iq, ["carrier"])["carrier"].astype(np.float32)
        f = os.path.join(tmp, f"{name}.f32")
        car.tofile(f)
        for sat in (0, 1):
            r = subprocess.run([exe, f, "19000", "240000", str(args.restarts), str(args.max_steps), str(sat)],
                               capture_output=True, text=True, check=True)
            out[f"{name}_{'after' if sat else 'before'}_2^24"] = json.loads(r.stdout)
            print(f"{name} sat={sat}: {r.stdout.strip()}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
