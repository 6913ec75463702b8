#!/usr/bin/env python3
"""The stereo PLL (filter.cpp:157-171) outside the locked regime: bit-exactness and speed.

For every `unlocked_*` entry of tests/golden/hashes.json (random bytes, a pilot-less broadcast,
heavy noise, a mode-2 stream whose PLL runs at the upsampled if_fs) and the locked 72 s synth run
beside them, one stereo call over the whole stream (device-resident input), checked against the
reference build's PCM SHA-256 and final PLL state, then timed again from a reset with the
per-stage HIP-event timer armed: seconds, ns a PLL step, per-regime ns a step and the
self-certifying runners' redone intervals (fmrx_debug_pll_redos).  Writes one JSON object.

    python tools/bench_unlocked.py [--out profiles/r06/unlocked.json] [--only NAME ...] [--cpu]
"""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)



def load_input(fm, rx, h, torch):
    import iqgen

    bb = rx.geo.block_bytes
    n = h["n_blocks"] * bb
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    kind, _, arg = h["recipe"].partition(":")
    if kind in iqgen.SYNTH_FLAGS:  # the same generator on the device (identical bytes)
        rx.synth_device(int(arg) | iqgen.SYNTH_FLAGS[kind], 0, n // 2, d.data_ptr())
        rx.synchronize()
    else:
        d.copy_(torch.from_numpy(iqgen.make(h["recipe"], n, rx.geo.rf_fs)))
    return d


def pll_state(rx):
    """The context's final PLL floats {integrator, phaseEst, fbI, fbQ, ncoOut_state, trigOffset}
    (state blob: header, halo, audio history, demod history, PLL 8 floats; tests _stream_blob)."""
    import numpy as np

    blob = rx.get_state()
    hdr = np.frombuffer(blob[:40], np.uint32)
    off = 40 + int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64
    return np.frombuffer(blob[off: off + 24], np.float32)


def run_one(fm, name, h, torch, bench_mod, cpu=False):
    import numpy as np

    rx = fm.Receiver(h["mode"], fm.STEREO, rf_taps=h["rf_taps"])
    d_iq = load_input(fm, rx, h, torch)
    assert hashlib.sha256(d_iq.cpu().numpy().tobytes()).hexdigest() == h["input_sha256"], name
    nb = h["n_blocks"]
    d_pcm = torch.empty(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
    redos = torch.zeros(fm.REDO_SLOTS, dtype=torch.int32, device="cuda")
    rx.debug_pll_redos(redos.data_ptr())
    t0 = time.perf_counter()
    rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
    rx.synchronize()
    first = time.perf_counter() - t0
    rx.debug_pll_redos(None)
    pcm_ok = hashlib.sha256(d_pcm.cpu().numpy().tobytes()).hexdigest() == h["pcm_sha256"]
    st = pll_state(rx)
    st_ok = bool(np.array_equal(st.view(np.uint32), np.asarray(h["pll_state_last"], np.float32).view(np.uint32)))
    times = []
    for _ in range(3):
        rx.reset()
        t0 = time.perf_counter()
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
        rx.synchronize()
        times.append(time.perf_counter() - t0)
    lat = bench_mod.stage_latency(rx, lambda: rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr()))
    steps = nb * rx.geo.if_samples
    sig = nb * rx.geo.block_bytes / 2 / rx.geo.rf_fs
    times.sort()
    med = times[len(times) // 2]
    out = {"recipe": h["recipe"], "mode": h["mode"], "n_blocks": nb, "signal_seconds": round(sig, 2),
           "pll_steps": steps, "bit_exact_pcm": pcm_ok, "bit_exact_pll_state": st_ok,
           "final_phaseEst": float(st[1]), "seconds_first_call": round(first, 4),
           "seconds": {"median": round(med, 4), "min": round(times[0], 4), "max": round(times[-1], 4), "runs": 3},
           "ns_per_pll_step": round(med * 1e9 / steps, 2), "x_realtime": round(sig / med, 1),
           "redone_intervals": dict(zip(fm.REDO_RANGES, redos.cpu().tolist()[:4])),
           "demoted_steps": dict(zip(fm.REDO_RANGES, redos.cpu().tolist()[4:])),
           "runner_ms": lat["runner_ms"], "regimes": lat["regimes"], "stage_ms": lat["stage_ms"]}
    if cpu:  # the reference's own stereo path on the same bytes (bench.py's CPU-baseline leg)
        out["cpu_reference"] = bench_mod.cpu_baseline_stereo_stream(d_iq.cpu().numpy(), h, steps, sig)
    rx.close()
    del d_iq, d_pcm
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--cpu", action="store_true", help="time the reference's CPU path on each input too")
    args = ap.parse_args()
    import torch

    import iqgen

    torch.cuda.init()
    fm = iqgen.load_fmrx()
    import bench as bench_mod

    with open(os.path.join(REPO, "tests", "golden", "hashes.json")) as f:
        hashes = json.load(f)
    names = [k for k in hashes if k.startswith("unlocked_")] + ["m0_rf51_synth_72s"]
    if args.only:
        names = [n for n in names if n in args.only]
    res = {}
    for name in names:
        res[name] = run_one(fm, name, hashes[name], torch, bench_mod, args.cpu)
        print(json.dumps({name: res[name]}), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
