#!/usr/bin/env python3
"""Per-call breakdown of the per-block seam (fmrx_rf_block + fmrx_audio_block, one 12,800-byte
mode-0 block a call, one context, host buffers): wall time of each call on the host, for a
rocprofv3 --kernel-trace / --memory-copy-trace run to split into kernels, copies and the rest.

    python tools/seam_profile.py [--blocks 1000] [--start-block 0]
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
    ap.add_argument("--blocks", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--start-block", type=int, default=0,
                    help="skip this many blocks first in one fused call (a later trigOffset regime)")
    args = ap.parse_args()
    import iqgen

    fm = iqgen.load_fmrx()
    L = fm.lib()
    geo = fm.geometry(fm.default_config(0, fm.STEREO))
    bb, nif, npcm = geo.block_bytes, geo.if_samples, geo.pcm_samples
    nb = args.start_block + args.warmup + args.blocks
    iq = fm.synth_host(5, geo.rf_fs, 0, nb * bb // 2)
    demod = np.zeros((nb, nif), np.float32)
    pcm = np.zeros((nb, npcm), np.int16)
    # raw addresses (argtypes c_void_p take ints): no slice or ctypes object per call
    iq_p, dm_p, pcm_p = iq.ctypes.data, demod.ctypes.data, pcm.ctypes.data
    dm_b, pcm_b = demod.strides[0], pcm.strides[0]
    t_rf, t_au = [], []
    with fm.Receiver(0, fm.STEREO) as rx:
        if args.start_block:
            rx.process(iq[: args.start_block * bb])
        for b in range(args.start_block, nb):
            t0 = time.perf_counter()
            rc = L.fmrx_rf_block(rx.h, iq_p + b * bb, 1, dm_p + b * dm_b)
            t1 = time.perf_counter()
            rc |= L.fmrx_audio_block(rx.h, dm_p + b * dm_b, 1, pcm_p + b * pcm_b)
            t2 = time.perf_counter()
            assert rc == 0, L.fmrx_last_error()
            if b >= args.start_block + args.warmup:
                t_rf.append(t1 - t0)
                t_au.append(t2 - t1)
    med = lambda x: round(float(np.median(x)) * 1e3, 4)  # noqa: E731
    budget = bb / 2 / geo.rf_fs
    print(json.dumps({"blocks": args.blocks, "start_block": args.start_block, "rf_ms_median": med(t_rf),
                      "audio_ms_median": med(t_au), "block_ms_median": med(np.add(t_rf, t_au)),
                      "x_realtime_serial": round(budget * len(t_rf) / float(np.sum(np.add(t_rf, t_au))), 2)}))


if __name__ == "__main__":
    main()
