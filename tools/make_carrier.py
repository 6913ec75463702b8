"""tools/make_carrier.py -- the 19 kHz carrier band-pass output (the PLL's input,
project.cpp:165) of the bench stream, from the reference build (oracle/_ref), as raw float32:
the input of tools/pll_predict.cpp.

    python tools/make_carrier.py /tmp/carrier.f32 [seconds] [seed]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "software-defined-radio-course-project_amd"))
import fmrx  # noqa: E402
from oracle import oracle  # noqa: E402


def main() -> None:
    out = sys.argv[1]
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 18.4
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    rf_fs = 2_400_000
    n_pairs = int(seconds * rf_fs) // 25_600 * 25_600  # whole mode-0 blocks (12,800 pairs... 2 blocks)
    iq = fmrx.synth_host(seed, rf_fs, 0, n_pairs)
    r = oracle.Reference().run(0, 101, iq, fields=["carrier"])
    r["carrier"].astype(np.float32).tofile(out)
    print(f"{out}: {r['carrier'].size} carrier samples ({r['n_blocks']} blocks, seed {seed})")


if __name__ == "__main__":
    main()
