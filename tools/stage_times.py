#!/usr/bin/env python3
"""Where a stereo call's device time goes, per stage (fmrx_debug_stage_timing): BASELINE
configs[4] (256 streams x 60 s) and configs[2] (one 1 GiB stream), each call timed plain first
(wall), then once more with the stage events armed.  ns per PLL step per runner regime from the
runner launches that ran their segment alone.  One JSON line.

    python tools/stage_times.py [--streams 256] [--seconds 60] [--no-gib] [--single 10]

--single S adds one stream of S seconds (the single-stream real-time factor, x_realtime).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def run(fm, ns, nb, seeds, reps=1):
    import torch

    rx = fm.Receiver(0, fm.STEREO, n_streams=ns)
    bb = rx.geo.block_bytes
    iq = torch.empty((ns, nb * bb), dtype=torch.uint8, device="cuda")
    pcm = torch.empty((ns, nb * rx.geo.pcm_samples), dtype=torch.int16, device="cuda")
    if ns == 1:
        rx.synth_device(seeds[0], 0, nb * bb // 2, iq.data_ptr())
    else:
        rx.synth_device_streams(seeds, 0, nb * bb // 2, iq.data_ptr(), nb * bb)
    rx.synchronize()
    walls = []
    for _ in range(1 + reps):  # the first call sizes the buffers
        rx.reset()
        t0 = time.perf_counter()
        rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        walls.append(time.perf_counter() - t0)
    rx.reset()
    rx.stage_timing(1)
    t0 = time.perf_counter()
    rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
    rx.synchronize()
    wall_timed = time.perf_counter() - t0
    st = rx.stage_timing(-1)
    rx.close()
    stages = {k: {"ms": round(v[0], 3), "launches": v[1]} for k, v in st.items()}
    for k, v in st.items():
        if v[2] > 0:
            stages[k]["steps"] = int(v[2])
            stages[k]["ns_per_step"] = round(v[0] * 1e6 / v[2], 2)
    return {"streams": ns, "blocks": nb, "wall_s": [round(w, 4) for w in walls[1:]],
            "wall_s_with_events": round(wall_timed, 4), "sum_stage_ms": round(sum(v[0] for v in st.values()), 2),
            "stages": stages}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--no-gib", action="store_true")
    ap.add_argument("--single", type=float, default=10.0)
    args = ap.parse_args()
    import torch

    import iqgen

    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    out = {}
    nb = int(args.seconds * 2.4e6 * 2 // 12800)
    out["configs[4]"] = run(fm, args.streams, nb, list(range(args.streams)))
    if args.single > 0:
        nb1 = int(args.single * 2.4e6 * 2 // 12800)
        r = run(fm, 1, nb1, [3000], reps=3)
        r["x_realtime"] = round(nb1 * 12800 / 2 / 2.4e6 / min(r["wall_s"]), 1)
        out["single_%gs" % args.single] = r
    if not args.no_gib:
        out["configs[2]"] = run(fm, 1, (1 << 30) // 12800, [3000])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
