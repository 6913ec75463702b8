#!/usr/bin/env python3
"""Stereo (REF_EXACT, project.cpp output) throughput on one GPU: BASELINE configs[2] (one
stream) and configs[4]'s per-GPU share (many independent streams), device-resident input.
Prints one JSON line per configuration with the per-stage kernel split from HIP events."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 32, 256])
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--gib", action="store_true",
                    help="BASELINE configs[2]: one stream of 1 GiB (83,886 mode-0 blocks) in ONE call (the reference's "
                         "CPU time on these bytes is bench.py's configs[2] cpu_baseline)")
    args = ap.parse_args()
    if args.gib:
        return gib(args)
    import torch
    import iqgen

    fm = iqgen.load_fmrx()
    for ns in args.streams:
        rx = fm.Receiver(args.mode, fm.STEREO, n_streams=ns)
        bb = rx.geo.block_bytes
        nb = int(args.seconds * rx.geo.rf_fs * 2 // bb)
        iq = torch.empty((ns, nb * bb), dtype=torch.uint8, device="cuda")
        pcm = torch.empty((ns, nb * rx.geo.pcm_samples), dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        for s in range(ns):
            rx.synth_device(s, 0, nb * bb // 2, iq[s].data_ptr())
        rx.synchronize()
        rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())  # warm-up: code objects, buffers sized
        rx.synchronize()
        rx.reset()
        t0 = time.perf_counter()
        rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        dt = time.perf_counter() - t0
        iq_pairs = ns * nb * bb // 2
        print(json.dumps({"config": f"mode-{args.mode} stereo, {ns} stream(s) x {nb * bb / 2 / rx.geo.rf_fs:.1f} s",
                          "seconds": round(dt, 4), "MS_per_s": round(iq_pairs / dt / 1e6, 1),
                          "x_realtime_per_stream": round(nb * bb / 2 / rx.geo.rf_fs / dt, 1),
                          "stream_seconds_per_s": round(ns * nb * bb / 2 / rx.geo.rf_fs / dt, 1)}), flush=True)
        rx.close()
        del iq, pcm
        torch.cuda.empty_cache()


def gib(args):
    import torch

    import iqgen

    fm = iqgen.load_fmrx()
    rx = fm.Receiver(args.mode, fm.STEREO)
    bb = rx.geo.block_bytes
    nb = (1 << 30) // bb
    iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
    pcm = torch.empty(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
    rx.synth_device(0, 0, nb * bb // 2, iq.data_ptr())
    rx.synchronize()
    t0 = time.perf_counter()
    rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
    rx.synchronize()
    dt = time.perf_counter() - t0
    sig = nb * bb / 2 / rx.geo.rf_fs
    out = {"config": f"BASELINE configs[2]: mode-{args.mode} stereo, one stream, 1 GiB ({nb} blocks, {sig:.1f} s) "
                     "in one call, device-resident", "seconds": round(dt, 3),
           "MS_per_s": round(nb * bb / 2 / dt / 1e6, 1), "x_realtime": round(sig / dt, 1)}
    print(json.dumps(out), flush=True)
    rx.close()


if __name__ == "__main__":
    main()
