"""tools/make_carrier.py -- the 19 kHz carrier band-pass output (the PLL's input,
project.cpp:165) of the bench stream, made on the GPU by the product's own primitives
(fmrx_rf_block, then fmrx_resample with the carrier taps; tools/runner_prof.py carrier()), as
raw float32: the input of tools/pll_predict.cpp.  Needs a GPU.

    python tools/make_carrier.py /tmp/carrier.f32 [seconds] [seed]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    import numpy as np
    import torch

    import iqgen
    from runner_prof import carrier

    out = sys.argv[1]
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 18.4
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    car = carrier(fm, seconds, seed).cpu().numpy().astype(np.float32)
    car.tofile(out)
    print(f"{out}: {car.size} carrier samples (seed {seed})")


if __name__ == "__main__":
    main()
