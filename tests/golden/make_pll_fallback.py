#!/usr/bin/env python3
"""Make tests/golden/pll_fallback.npz: arguments where the PLL's certified fast paths may refuse
(csrc/pll_math.h) with glibc 2.35's float results -- the values the reference's PLL uses
(src/filter.cpp:161,168-170: float(atan2/sin/cos) of double libm calls).

    python tests/golden/make_pll_fallback.py [--atan2-pairs 4000000000]

Builds and runs tools/check_pll_cr.cpp, which walks EVERY float |x| in [2^-19, 2^30) for sin/cos
and random float pairs for atan2, keeps the superset of refusable arguments and checks the
device's fallback (csrc/pll_cr.h, compiled for the host) against glibc on all of them (it exits
non-zero on any mismatch).  The fixture keeps: every hard sin/cos argument with |x| < 1e9 (the
PLL's trigArg domain), one in 256 of those in [1e9, 2^30), and the hard atan2 pairs.  The GPU
test (test_pll_fallback_matches_glibc) runs the device fallbacks on them and requires equality.
"""
import argparse
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--atan2-pairs", type=int, default=4_000_000_000)
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="pllfb_", dir="/tmp")
    exe = os.path.join(tmp, "check_pll_cr")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o", exe,
                    os.path.join(REPO, "tools", "check_pll_cr.cpp")], check=True)
    sc, at = os.path.join(tmp, "sc.bin"), os.path.join(tmp, "at.bin")
    r1 = subprocess.run([exe, "sincos", sc], check=True, capture_output=True, text=True).stdout.strip()
    r2 = subprocess.run([exe, "atan2", str(args.atan2_pairs), str(args.seed), at], check=True,
                        capture_output=True, text=True).stdout.strip()
    s = np.fromfile(sc, np.uint32).reshape(-1, 3)
    a = np.fromfile(at, np.uint32).reshape(-1, 3)
    x = s[:, 0].view(np.float32)
    keep = (np.abs(x) < 1e9) | (np.arange(len(x)) % 256 == 0)
    s = s[keep]
    order = np.argsort(s[:, 0].view(np.float32), kind="stable")
    s = s[order]
    glibc = os.confstr("CS_GNU_LIBC_VERSION")
    np.savez_compressed(os.path.join(HERE, "pll_fallback.npz"),
                        sincos_x=s[:, 0].view(np.float32), sincos_s=s[:, 1].view(np.float32),
                        sincos_c=s[:, 2].view(np.float32),
                        atan2_y=a[:, 0].view(np.float32), atan2_x=a[:, 1].view(np.float32),
                        atan2_e=a[:, 2].view(np.float32), glibc=np.array(glibc),
                        sweep_sincos=np.array(r1), sweep_atan2=np.array(r2))
    print(glibc, r1, r2, "kept", len(s), "sincos,", len(a), "atan2")
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
