#!/usr/bin/env python3
"""Per-form PLL runner timing on the bench stream's own carrier, from the real (locked) state.

The carrier is made on the GPU by the product's own primitives: fmrx_rf_block (front end ->
demod) of the synthetic bench stream, then the 19 kHz carrier band-pass (project.cpp:165,
fmrx_resample with up = down = 1).  `--save S`: fmrx_pll runs the carrier from the reset state
(project.cpp:106-111) and the PLL state at each trigOffset T of --trig is written to S (npz).
`--load S`: from the saved state at T, fmrx_pll runs the next --n steps (so exactly one runner
form runs, as inside a real call at T), timed, and prints ns a step per form.  With FMRX_LIB_PATH
pointing at an `make ab AB=-DFMRX_AB_PROF` build, the runners' chain / evaluator body and
barrier-wait cycles per interval are printed at exit (stderr): run one T per process.

    python tools/runner_prof.py --save /tmp/st.npz --trig 262144 --trig 1048576 ...
    python tools/runner_prof.py --load /tmp/st.npz --trig 262144 [--n 262144] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def carrier(fm, seconds: float, seed: int):
    import numpy as np
    import torch

    with fm.Receiver(0, fm.STEREO) as rx:
        bb = rx.geo.block_bytes
        nb = int(seconds * 2.4e6 * 2 // bb)
        iq = fm.synth_host(seed, 2_400_000, 0, nb * bb // 2)
        demod = rx.rf_block(iq).astype(np.float32).ravel()
        taps = fm.bpf(240000.0, 18500.0, 19500.0, rx.geo.bp_taps).astype(np.float32)
        d_in = torch.from_numpy(demod).cuda()
        d_out = torch.empty_like(d_in)
        d_state = torch.zeros(taps.size - 1, dtype=torch.float32, device="cuda")
        d_taps = torch.from_numpy(taps).cuda()
        rx.resample(d_out.data_ptr(), d_state.data_ptr(), d_in.data_ptr(), demod.size, d_taps.data_ptr(),
                    taps.size, 1, 1)
        rx.synchronize()
        return d_out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trig", type=int, action="append", required=True)
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--save")
    ap.add_argument("--load")
    args = ap.parse_args()
    import numpy as np
    import torch

    import iqgen

    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    need = max(args.trig) + (0 if args.save else args.n)
    car = carrier(fm, need / 240000.0 + 0.1, 3000)
    with fm.Receiver(0, fm.STEREO) as rx:
        if args.save:
            st = torch.tensor([0.0, 0.0, 1.0, 0.0, 1.0, 0.0], dtype=torch.float32, device="cuda")
            states, pos = {}, 0
            for t in sorted(args.trig):
                buf = car[pos:t].clone()
                rx.pll(buf.data_ptr(), t - pos, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
                rx.synchronize()
                pos = t
                states[str(t)] = st.cpu().numpy().copy()
            np.savez(args.save, **states)
            print(json.dumps({"saved": {k: v.tolist() for k, v in states.items()}}), flush=True)
            return
        saved = np.load(args.load)
        out = {"n": args.n, "lib": os.environ.get("FMRX_LIB_PATH", "libfmrx.so"), "forms": {}}
        for t in args.trig:
            st0 = saved[str(t)]
            times = []
            for _ in range(args.reps + 1):
                buf = car[t:t + args.n].clone()
                st = torch.from_numpy(st0).cuda()
                rx.synchronize()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rx.pll(buf.data_ptr(), args.n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
                rx.synchronize()
                times.append(time.perf_counter() - t0)
            best = min(times[1:])
            out["forms"][str(t)] = {"best_s": round(best, 5), "ns_per_step": round(best * 1e9 / args.n, 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
