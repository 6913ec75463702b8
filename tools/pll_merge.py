#!/usr/bin/env python3
"""Time-parallel PLL feasibility: does a speculative restart of the stereo pilot
PLL (src/filter.cpp:136-174, project.cpp:166) bit-merge with the true trajectory?

Builds tools/pll_merge.cpp and runs the merge measurement, before and after the float
trigOffset saturates (2^24), on 19 kHz carrier files (the PLL's input, project.cpp:165, raw
float32) made by the product on a GPU with tools/make_carrier.py.  Host-only; nothing under
oracle/ is used.  Writes one JSON object.

    python tools/make_carrier.py /tmp/synth.f32 12 7          # on a GPU box
    python tools/pll_merge.py synth=/tmp/synth.f32 [--restarts 24] [--max-steps 1000000]

(profiles/r02/pll_merge.json was made in round 2 from carriers of three signals: the synthetic
broadcast, uniform random u8 I/Q and a constant 0x80 stream.)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("carriers", nargs="+", help="name=path of a raw float32 carrier file")
    ap.add_argument("--restarts", type=int, default=24)
    ap.add_argument("--max-steps", type=int, default=1000000)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp()
    exe = os.path.join(tmp, "pll_merge")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(REPO, "tools", "pll_merge.cpp")],
                   check=True)
    out = {"what": "bit-merge of speculative PLL restarts with the true trajectory (reference arithmetic, glibc)",
           "steps_per_second": 240000}
    for spec in args.carriers:
        name, f = spec.split("=", 1)
        out[f"{name}_seconds"] = os.path.getsize(f) / 4 / 240000
        for sat in (0, 1):
            r = subprocess.run([exe, f, "19000", "240000", str(args.restarts), str(args.max_steps), str(sat)],
                               capture_output=True, text=True, check=True)
            out[f"{name}_{'after' if sat else 'before'}_2^24"] = json.loads(r.stdout)
            print(f"{name} sat={sat}: {r.stdout.strip()}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
