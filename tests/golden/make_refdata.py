#!/usr/bin/env python3
"""Fixtures from the reference's OWN data files (test infrastructure; needs /root/reference).

/root/reference/data holds two inputs on this path:

  fm_demod_10.bin, fm_demod_11.bin   5,120 float32 each: FM demod of blocks 10 and 11 of a real
                                     broadcast recording, dumped by model/fmMonoBlock.py:277-280
                                     (5,120 = one Python block; 8 mode-0 C++ blocks of 640)
  q_block_time.dat -> q_filt_time.dat  10,240 Q samples (u8 values) and their 151-tap LPF
                                     (2.4 MHz, 100 kHz) at 6 significant digits, written by
                                     logVector (src/logfunc.cpp:23-43) in the lab era

This script copies those inputs into tests/golden/refdata.npz (a fixture is data) and adds the
reference build's outputs on them (oracle/_ref/libfmref.so: src/filter.cpp driven in
audio_thread order, project.cpp:132-196):

  pcm_<k>, pcm_mono_<k>, pll_<k>   stereo R,L PCM, mono-product PCM and the PLL state after
                                   every block, for k = 10, 11 and 10_11 (the two dumps back to
                                   back: 16 contiguous blocks of the same recording)

The .dat pair is stored as parsed (q as float64 u8 values, the filtered text values as float64).
Usage: python tests/golden/make_refdata.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402

DATA = "/root/reference/data"


def main() -> None:
    oracle.build(ref=True)
    ref = oracle.Reference()
    d10 = np.fromfile(os.path.join(DATA, "fm_demod_10.bin"), np.float32)
    d11 = np.fromfile(os.path.join(DATA, "fm_demod_11.bin"), np.float32)
    out = {"demod_10": d10, "demod_11": d11}
    for k, d in (("10", d10), ("11", d11), ("10_11", np.concatenate([d10, d11]))):
        r = ref.run_audio(0, d, ["pcm", "pcm_mono", "pll_state"])
        out[f"pcm_{k}"], out[f"pcm_mono_{k}"], out[f"pll_{k}"] = r["pcm"], r["pcm_mono"], r["pll_state"]
    q = np.loadtxt(os.path.join(DATA, "q_block_time.dat"))
    y = np.loadtxt(os.path.join(DATA, "q_filt_time.dat"))
    assert np.array_equal(q[:, 0], np.arange(q.shape[0])) and np.array_equal(y[:, 0], q[:, 0])
    out["q_block"], out["q_filt"] = q[:, 1], y[:, 1]
    np.savez_compressed(os.path.join(HERE, "refdata.npz"), **out)
    print("refdata.npz:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
