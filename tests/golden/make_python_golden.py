#!/usr/bin/env python3
"""Golden vectors from the reference's PYTHON models (test infrastructure, this container only).

The arctan demodulator (model/fmSupportLib.py:34-63 fmDemodArctan) and the PSD estimate
(model/fmSupportLib.py:83-157 estimatePSD, numpy FFT, float64) exist only in the Python
models; the C++ PSD (src/fourier.cpp:35-117, float DFT) is added from oracle/_ref for the same
inputs.  The model module is imported read-only from /root/reference/model (numpy, math and
cmath only; no side effects); nothing of it is copied.  Writes:

  py_arctan.npz  float32 I/Q blocks, the model's float64 demod per block with the phase
                 carried across blocks, and the phase after each block
  py_psd.npz     float32 test signals; per (signal, freq_bins, Fs) the model's freq/psd
                 (float64) and the C++ estimatePSD's freq/psd (float32)

Usage: python tests/golden/make_python_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, "/root/reference/model")

import fmSupportLib as model  # noqa: E402
import iqgen  # noqa: E402
import oracle  # noqa: E402

# (signal name, freq_bins, Fs)
PSD_CASES = [("tones", 512, 240000.0), ("tones", 256, 240000.0), ("demod", 1024, 240000.0),
             ("demod", 4096, 240000.0), ("noise", 512, 48000.0)]


def arctan_inputs() -> tuple[np.ndarray, np.ndarray]:
    """An FM-modulated unit phasor with noise (I/Q after the RF filter, float32), including
    exact zeros and large phase jumps so that the unwrap branch is taken."""
    n = 4 * 2048
    t = np.arange(n) / 240000.0
    msg = 0.6 * np.sin(2 * np.pi * 1000.0 * t) + 0.3 * np.sin(2 * np.pi * 7300.0 * t)
    phase = 2 * np.pi * 75000.0 * np.cumsum(msg) / 240000.0
    noise = (iqgen.rand_bytes(5, 2 * n).astype(np.float64) - 127.5) / 1275.0
    i = np.cos(phase) + noise[:n]
    q = np.sin(phase) + noise[n:]
    i[100:104] = 0.0
    q[102:106] = 0.0
    i[3000:3010] *= -1.0  # phase jumps of ~pi
    return i.astype(np.float32), q.astype(np.float32)


def psd_signal(name: str) -> np.ndarray:
    n = 16384
    if name == "tones":
        t = np.arange(n) / 240000.0
        x = np.sin(2 * np.pi * 19000.0 * t) + 0.1 * np.sin(2 * np.pi * 57000.0 * t)
        x += (iqgen.rand_bytes(11, n).astype(np.float64) - 127.5) / 12750.0
    elif name == "demod":
        iq = iqgen.make("synth:7", 26 * 12800, 2400000)
        x = oracle.Oracle().run(0, 51, iq, ["demod"])["demod"][:n].astype(np.float64)
    else:
        x = (iqgen.rand_bytes(12, n).astype(np.float64) - 127.5) / 127.5
    return x.astype(np.float32)


def main() -> None:
    oracle.build(ref=True)
    ref = oracle.Reference()
    i, q = arctan_inputs()
    blocks = np.split(np.arange(i.size), 4)
    demod, phases, prev = [], [], 0.0
    for b in blocks:
        d, prev = model.fmDemodArctan(i[b].astype(np.float64), q[b].astype(np.float64), prev)
        demod.append(d)
        phases.append(prev)
    np.savez_compressed(os.path.join(HERE, "py_arctan.npz"), i=i, q=q, demod=np.concatenate(demod),
                        phases=np.array(phases), block=blocks[0].size)

    out = {}
    for name in sorted({c[0] for c in PSD_CASES}):
        out[f"x_{name}"] = psd_signal(name)
    for name, nb, fs in PSD_CASES:
        x = out[f"x_{name}"]
        f, p = model.estimatePSD(x.astype(np.float64), nb, fs)
        cf, cp = ref.estimate_psd(x, nb, fs)
        key = f"{name}_{nb}_{int(fs)}"
        out[f"py_freq_{key}"], out[f"py_psd_{key}"] = np.asarray(f), np.asarray(p)
        out[f"cpp_freq_{key}"], out[f"cpp_psd_{key}"] = cf, cp
        print(key, "python vs C++ max |dB|", float(np.abs(np.asarray(p) - cp).max()))
    np.savez_compressed(os.path.join(HERE, "py_psd.npz"), cases=np.array([f"{n}_{b}_{int(f)}" for n, b, f in PSD_CASES]),
                        **out)


if __name__ == "__main__":
    main()
