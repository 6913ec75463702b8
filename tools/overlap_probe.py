#!/usr/bin/env python3
"""Measurement (round 4): how much parallel VALU work can run beside the serial PLL runners.

Context A runs the stereo engine on N streams (runner-dominated: one serial chain per stream,
the pipe runner's three waves on three SIMDs of a CU); context B, on its own HIP stream, runs
K launches of the fused mono kernel over 1 GiB (VALU-bound, every CU).  Times A alone, B alone,
and both enqueued together (B's end and A's end read by syncing each context).  If the runners
were unaffected and B used only idle issue slots, together ~= max(A, B); if they contend fully,
together ~= A + B.  Prints one JSON line.

    python tools/overlap_probe.py [--streams 256] [--seconds 20] [--k 300]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--k", type=int, default=300)
    args = ap.parse_args()
    import torch

    import iqgen

    fm = iqgen.load_fmrx()
    torch.cuda.set_device(0)
    a = fm.Receiver(0, fm.STEREO, n_streams=args.streams)
    bb = a.geo.block_bytes
    nb = int(args.seconds * 2.4e6 * 2 // bb)
    iq_a = torch.empty((args.streams, nb * bb), dtype=torch.uint8, device="cuda")
    pcm_a = torch.empty((args.streams, nb * a.geo.pcm_samples), dtype=torch.int16, device="cuda")
    a.synth_device_streams(list(range(args.streams)), 0, nb * bb // 2, iq_a.data_ptr(), nb * bb)
    b = fm.Receiver(0, fm.MONO, rf_taps=101)
    nbb = (1 << 30) // bb
    iq_b = torch.empty(nbb * bb, dtype=torch.uint8, device="cuda")
    pcm_b = torch.empty(nbb * b.geo.audio_frames, dtype=torch.int16, device="cuda")
    b.synth_device(7, 0, nbb * bb // 2, iq_b.data_ptr())
    a.synchronize()
    b.synchronize()

    def run_a():
        a.reset()
        a.process_device(iq_a.data_ptr(), nb, pcm_a.data_ptr())

    def run_b():
        for _ in range(args.k):
            b.process_device(iq_b.data_ptr(), nbb, pcm_b.data_ptr())

    # warm-up: A once at full size, B for > 1 s (clock ramp)
    run_a()
    a.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        run_b()
        b.synchronize()
    res = {"streams": args.streams, "seconds": args.seconds, "k_mono": args.k}
    for rep in range(2):
        t0 = time.perf_counter()
        run_a()
        a.synchronize()
        ta = time.perf_counter() - t0
        t0 = time.perf_counter()
        run_b()
        b.synchronize()
        tb = time.perf_counter() - t0
        a.reset()
        a.synchronize()
        t0 = time.perf_counter()
        a.process_device(iq_a.data_ptr(), nb, pcm_a.data_ptr())
        run_b()
        b.synchronize()
        tb_end = time.perf_counter() - t0
        a.synchronize()
        ta_end = time.perf_counter() - t0
        res[f"rep{rep}"] = {"a_alone": round(ta, 4), "b_alone": round(tb, 4), "together_b_end": round(tb_end, 4),
                            "together_a_end": round(ta_end, 4), "sum": round(ta + tb, 4),
                            "max": round(max(ta, tb), 4)}
    print(json.dumps(res), flush=True)
    a.close()
    b.close()


if __name__ == "__main__":
    main()
