#!/usr/bin/env python3
"""Generate the golden fixtures from the REFERENCE ITSELF (test infrastructure).

Runs the reference's own src/filter.cpp + src/iofunc.cpp (compiled in place from
/root/reference by oracle/Makefile into oracle/_ref/libfmref.so, driven in project.cpp's
sequential block order by oracle/ref_driver.cpp) on deterministic inputs and writes:

  taps.npz              every tap table the receive chain designs (filter.cpp:14-64)
  case_<name>.npz       per-stage outputs of short runs (inputs are regenerated from a recipe
                        and checked against the stored SHA-256)
  hashes.json           SHA-256 of the S16 output of longer runs (10 s of signal)

Inputs (no reference data file holds I/Q — data/samples*.raw are missing blobs):
  synth:<seed>  the repo's deterministic FM-stereo generator (libfmrx fmrx_synth_host,
                integer-only, identical bytes on host and GPU)
  rand:<seed>   uniform random bytes from tests/iqgen.py (splitmix64, numpy-only)
  const128      all bytes 128 (x = 0.0): the reference outputs all-zero PCM

Usage: python tests/golden/make_golden.py   (needs /root/reference; not run on the GPU box)
"""
from __future__ import annotations

import hashlib
import json
import os
import platform
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle  # noqa: E402
import iqgen  # noqa: E402

# Small per-stage cases: (name, mode, rf_taps, input recipe, n_blocks, fields stored in full)
ALL = ["demod", "mono_exact", "mono_indep", "pcm", "pcm_mono", "channel", "carrier", "nco",
       "mixer", "stereo", "left", "right", "pll_state"]
CASES = [
    ("m0_rf51_synth", 0, 51, "synth:1", 16, ALL),
    ("m0_rf101_synth", 0, 101, "synth:2", 16, ALL),
    ("m0_rf51_rand", 0, 51, "rand:7", 24, ALL),
    ("m0_rf101_rand", 0, 101, "rand:8", 8, ["demod", "mono_indep", "pcm", "pcm_mono"]),
    ("m0_rf51_const", 0, 51, "const128", 4, ["pcm", "pcm_mono", "demod"]),
    ("m0_rf51_one", 0, 51, "synth:3", 1, ALL),
    ("m1_rf51_synth", 1, 51, "synth:4", 12, ALL),
    ("m1_rf101_rand", 1, 101, "rand:9", 6, ["demod", "mono_indep", "pcm", "pcm_mono"]),
    ("m2_rf51_synth", 2, 51, "synth:5", 2, ["pcm", "pcm_mono", "pll_state"]),
    ("m3_rf51_synth", 3, 51, "synth:6", 1, ["pcm", "pcm_mono", "pll_state"]),
]
# Long runs, hash only: (name, mode, rf_taps, recipe, seconds of signal)
LONG = [
    ("m0_rf51_synth_10s", 0, 51, "synth:11", 10.0),
    ("m0_rf101_synth_10s", 0, 101, "synth:12", 10.0),
    ("m1_rf51_synth_10s", 1, 51, "synth:13", 10.0),
    ("m2_rf51_synth_4s", 2, 51, "synth:14", 4.0),
    ("m3_rf51_synth_8s", 3, 51, "synth:15", 8.0),
    ("m0_rf51_rand_2s", 0, 51, "rand:16", 2.0),
    ("m0_rf51_synth_72s", 0, 51, "synth:17", 72.0),  # PLL trigOffset saturates at 69.9 s
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main() -> None:
    oracle.build(ref=True)
    ref = oracle.Reference()
    meta = {"glibc": platform.libc_ver(), "generator": "oracle/_ref/libfmref.so (reference "
            "src/filter.cpp + src/iofunc.cpp, g++ -O3, no -march) via oracle/ref_driver.cpp"}

    taps = {}
    for mode, (bb, nif, na, rf_fs, if_fs, bp_fs, up, down) in oracle.MODES.items():
        for t in (51, 101):
            taps[f"rf_m{mode}_{t}"] = ref.lpf(rf_fs, 100000, t, 1)
        taps[f"audio_m{mode}"] = ref.lpf(if_fs, 16000, 51 * up, up)
        taps[f"ch_m{mode}"] = ref.bpf(bp_fs, 22000.0, 54000.0, 51)
        taps[f"ca_m{mode}"] = ref.bpf(bp_fs, 18500, 19500, 51)
    # primitive-level KATs on tiny random vectors (reference functions called directly)
    rng = iqgen.bytes_("rand:21", 4096)
    x = (rng.astype(np.float32) - 128.0) / 128.0
    prim = {}
    prim["norm_in"] = rng[:512]
    prim["norm_out"] = ref.normalize(rng[:512])
    c = taps["rf_m0_51"]
    st = np.linspace(-0.5, 0.5, 50).astype(np.float32)
    for up, down in ((1, 10), (1, 1), (3, 7)):
        o, s2 = ref.resample(x[:1000], st, c, up, down)
        prim[f"resample_{up}_{down}_out"], prim[f"resample_{up}_{down}_state"] = o, s2
    prim["resample_in"], prim["resample_state"] = x[:1000], st
    d, pv = ref.fmdemod(x[:600], x[600:1200], [0.25, -0.5])
    prim["demod_i"], prim["demod_q"], prim["demod_out"], prim["demod_prev"] = x[:600], x[600:1200], d, pv
    pin = np.sin(2 * np.pi * 19000 / 240000 * np.arange(3000)).astype(np.float32) * 0.1
    po, ps = ref.pll(pin, 19000, 240000, 2, 0, 0.01, [0, 0, 1, 0, 1, 0])
    prim["pll_in"], prim["pll_out"], prim["pll_state"] = pin, po, ps
    np.savez_compressed(os.path.join(HERE, "taps.npz"), **taps, **prim)

    for name, mode, rf_taps, recipe, nb, fields in CASES:
        bb = oracle.MODES[mode][0]
        iq = iqgen.make(recipe, nb * bb, oracle.MODES[mode][3])
        out = ref.run(mode, rf_taps, iq, fields)
        arrs = {k: v for k, v in out.items() if k in fields}
        np.savez_compressed(os.path.join(HERE, f"case_{name}.npz"), mode=mode, rf_taps=rf_taps,
                            recipe=recipe, n_blocks=nb, input_sha256=sha(iq), **arrs)
        print(f"case {name}: {nb} blocks, fields {sorted(arrs)}")

    hashes = {"meta": meta}
    for name, mode, rf_taps, recipe, secs in LONG:
        bb, _, _, rf_fs = oracle.MODES[mode][:4]
        nb = int(secs * rf_fs * 2 // bb)
        iq = iqgen.make(recipe, nb * bb, rf_fs)
        out = ref.run(mode, rf_taps, iq, ["pcm", "pcm_mono", "pll_state"])
        hashes[name] = {"mode": mode, "rf_taps": rf_taps, "recipe": recipe, "n_blocks": nb,
                        "input_sha256": sha(iq), "pcm_sha256": sha(out["pcm"]),
                        "pcm_mono_sha256": sha(out["pcm_mono"]),
                        "pll_state_last": [float(v) for v in out["pll_state"][-6:]]}
        print(f"long {name}: {nb} blocks")
    with open(os.path.join(HERE, "hashes.json"), "w") as f:
        json.dump(hashes, f, indent=1)


if __name__ == "__main__":
    main()
