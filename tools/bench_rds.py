#!/usr/bin/env python3
"""RDS front half throughput (rds_thread body, project.cpp:200-271) on device-resident demod.

    python tools/bench_rds.py [--streams 1,32,256] [--seconds 10] [--mode 0]

Per stream count: demod test signals (tests/iqgen.py make_rds_demod) uploaded once, then
fmrx_rds_device over the whole run timed with a device sync on both sides.  The PLL (one
lane per stream, strictly serial) bounds every configuration; the FIR front end and the
mixer are parallel kernels.  Prints one JSON line per stream count.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,32,256")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()
    import torch

    import iqgen

    fm = iqgen.load_fmrx()
    geo = fm.geometry(fm.default_config(args.mode, fm.STEREO))
    nif, bp_fs = geo.if_samples, geo.bp_fs
    nb = int(args.seconds * bp_fs) // nif
    base = iqgen.make_rds_demod(3, nb * nif, bp_fs)
    for ns in (int(v) for v in args.streams.split(",")):
        d_in = torch.from_numpy(np.tile(base, (ns, 1))).cuda()
        d_out = torch.empty_like(d_in)
        with fm.Receiver(args.mode, fm.STEREO, n_streams=ns) as rx:
            rx.rds_device(d_in.data_ptr(), nb, d_out.data_ptr())  # warm-up: code objects, buffers sized
            rx.synchronize()
            rx.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rx.rds_device(d_in.data_ptr(), nb, d_out.data_ptr())
            rx.synchronize()
            dt = time.perf_counter() - t0
        sig = nb * nif / bp_fs
        print(json.dumps({"workload": f"RDS front half, mode {args.mode}, {ns} stream(s) x {sig:.1f} s",
                          "seconds": round(dt, 4), "x_realtime_per_stream": round(sig / dt, 2),
                          "stream_seconds_per_s": round(ns * sig / dt, 1),
                          "ns_per_sample_step": round(dt / (nb * nif) * 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
