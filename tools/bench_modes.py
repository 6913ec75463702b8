#!/usr/bin/env python3
"""Mono product throughput per mode (BASELINE configs[3] is mode 2: the 147/800 polyphase
resampler over a 7,497-tap prototype, 51 taps per output) on 1 GiB of device-resident
synthetic I/Q per mode.  One step = fmrx_process_device over the whole GiB (RF front end +
demod + audio resampler + S16).  Prints one JSON line per mode.

    python tools/bench_modes.py [--modes 0 1 2 3] [--steps 5] [--rf-taps 51] [--warmup-seconds 1]
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
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rf-taps", type=int, default=51)
    ap.add_argument("--warmup-seconds", type=float, default=1.0,
                    help="untimed back-to-back steps first (the clock ramp, DESIGN §5.1), as bench.py")
    args = ap.parse_args()
    import torch

    import iqgen

    fm = iqgen.load_fmrx()
    for mode in args.modes:
        with fm.Receiver(mode, fm.MONO, rf_taps=args.rf_taps) as rx:
            bb, na, rf_fs = rx.geo.block_bytes, rx.geo.audio_frames, rx.geo.rf_fs
            nb = (1 << 30) // bb
            d_iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
            d_pcm = torch.empty(nb * na, dtype=torch.int16, device="cuda")
            torch.cuda.synchronize()
            rx.synth_device(100 + mode, 0, nb * bb // 2, d_iq.data_ptr())
            rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())  # warm-up
            rx.synchronize()
            t_w = time.perf_counter()
            while time.perf_counter() - t_w < args.warmup_seconds:
                for _ in range(64):
                    rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
                rx.synchronize()
            rx.kernel_timing(reset=1)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
            rx.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            kern_ms, _ = rx.kernel_timing(reset=-1)
        n_iq = nb * bb // 2
        print(json.dumps({"workload": f"mode-{mode} mono, {args.rf_taps}-tap RF, {nb} blocks ({nb * bb} B) per step",
                          "ms_per_step": round(dt * 1e3, 4), "MS_per_s": round(n_iq / dt / 1e6, 1),
                          "x_realtime": round(n_iq / rf_fs / dt, 1), "rf_kernel_ms": round(kern_ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
