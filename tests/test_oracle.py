"""Pin the C restatement (oracle/fmrx_oracle.c) against the reference's own outputs.

The golden fixtures under tests/golden were produced by the reference's src/filter.cpp and
src/iofunc.cpp (compiled from /root/reference, driven in project.cpp order); every
comparison here is bit-exact.  Tests marked with the `ref` fixture additionally run the
reference build live (this container only) on fresh inputs.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import iqgen
import oracle
from conftest import case_input, golden_cases, load_case, long_runs, unlocked_runs


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_taps_match_reference(orc, taps_golden, mode):
    bb, nif, na, rf_fs, if_fs, bp_fs, up, down = oracle.MODES[mode]
    for t in (51, 101):
        assert np.array_equal(bits(orc.lpf(rf_fs, 100000, t, 1)), bits(taps_golden[f"rf_m{mode}_{t}"]))
    assert np.array_equal(bits(orc.lpf(if_fs, 16000, 51 * up, up)), bits(taps_golden[f"audio_m{mode}"]))
    assert np.array_equal(bits(orc.bpf(bp_fs, 22000, 54000, 51)), bits(taps_golden[f"ch_m{mode}"]))
    assert np.array_equal(bits(orc.bpf(bp_fs, 18500, 19500, 51)), bits(taps_golden[f"ca_m{mode}"]))


def test_primitives_match_reference(orc, taps_golden):
    g = taps_golden
    assert np.array_equal(bits(orc.normalize(g["norm_in"])), bits(g["norm_out"]))
    c = g["rf_m0_51"]
    for up, down in ((1, 10), (1, 1), (3, 7)):
        o, s = orc.resample(g["resample_in"], g["resample_state"], c, up, down)
        assert np.array_equal(bits(o), bits(g[f"resample_{up}_{down}_out"]))
        assert np.array_equal(bits(s), bits(g[f"resample_{up}_{down}_state"]))
    d, pv = orc.fmdemod(g["demod_i"], g["demod_q"], [0.25, -0.5])
    assert np.array_equal(bits(d), bits(g["demod_out"]))
    assert np.array_equal(bits(pv), bits(g["demod_prev"]))
    po, ps = orc.pll(g["pll_in"], 19000, 240000, 2, 0, 0.01, [0, 0, 1, 0, 1, 0])
    assert np.array_equal(bits(po), bits(g["pll_out"]))
    assert np.array_equal(bits(ps), bits(g["pll_state"]))


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_matches_golden_case(orc, name):
    z = load_case(name)
    iq = case_input(z)
    assert sha(iq) == z["input_sha256"], "input generator drifted"
    fields = [k for k in oracle.FIELDS if k in z]
    out = orc.run(z["mode"], z["rf_taps"], iq, fields)
    assert out["n_blocks"] == z["n_blocks"]
    for f in fields:
        assert np.array_equal(bits(out[f]), bits(z[f])), f"{name}:{f} differs"


@pytest.mark.parametrize("name", sorted(long_runs()))
def test_oracle_matches_long_hashes(orc, name):
    h = long_runs()[name]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    assert sha(iq) == h["input_sha256"]
    out = orc.run(h["mode"], h["rf_taps"], iq, ["pcm", "pcm_mono", "pll_state"])
    assert sha(out["pcm"]) == h["pcm_sha256"]
    assert sha(out["pcm_mono"]) == h["pcm_mono_sha256"]


@pytest.mark.parametrize("name", ["unlocked_m0_nopilot_80s", "unlocked_m2_synth_170b"])
def test_oracle_matches_unlocked_hashes(orc, name):
    """The C restatement on a PLL that never locks, past the trigOffset stick (~20 s each; the
    other two unlocked fixtures, random bytes and heavy noise, matched too when they were made)."""
    h = unlocked_runs()[name]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    assert sha(iq) == h["input_sha256"]
    out = orc.run(h["mode"], h["rf_taps"], iq, ["pcm", "pll_state"])
    assert sha(out["pcm"]) == h["pcm_sha256"]
    assert np.array_equal(bits(out["pll_state"][-6:]), bits(np.asarray(h["pll_state_last"], np.float32)))


def test_const128_is_silence(orc):
    out = orc.run(0, 51, np.full(12800 * 3, 128, np.uint8), ["pcm", "pcm_mono", "demod"])
    assert not out["pcm"].any() and not out["pcm_mono"].any() and not out["demod"].any()


def test_quantizer_x86_semantics(orc):
    # static_cast<short>(x*16384) on x86-64: cvttss2si then 16-bit store (project.cpp:187)
    x = np.array([0.0, 1.0, -1.0, 1.99993896484375, 2.0, -2.0, 2.5, 1e6, -1e6, 1.4e5, 2e5,
                  np.inf, -np.inf, np.nan, 131071.99, -131072.0, 3.0517578125e-05, -3.0e-05],
                 np.float32)
    got = orc.quant(x)
    want = []
    for v in x:
        if np.isnan(v):
            want.append(0)
            continue
        p = np.float32(v) * np.float32(16384)
        t = -(2**31) if (not (p < 2.0**31) or p < -(2.0**31)) else int(p)
        want.append(np.int16(np.uint16(t & 0xFFFF).view(np.int16)))
    assert np.array_equal(got, np.array(want, np.int16))


def test_random_input_exercises_wrap(orc):
    z = load_case("m0_rf51_rand")
    mono = z["mono_indep"]
    assert (np.abs(mono * 16384.0) >= 32768).any(), "stress input must overflow int16"


# ---- live comparisons with the reference build (this container only) -------------------

@pytest.mark.parametrize("mode,rf_taps,recipe,nb", [(0, 51, "synth:31", 9), (0, 101, "rand:32", 5),
                                                   (1, 51, "rand:33", 7), (1, 101, "synth:34", 4)])
def test_oracle_vs_reference_live(orc, ref, mode, rf_taps, recipe, nb):
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    iq = iqgen.make(recipe, nb * bb + 777, rf_fs)  # ragged tail is dropped by both
    a = orc.run(mode, rf_taps, iq)
    b = ref.run(mode, rf_taps, iq)
    for f in oracle.FIELDS:
        assert np.array_equal(bits(a[f]), bits(b[f])), f


# ---- RDS front half (project.cpp:200-271) ------------------------------------------------

from conftest import load_rds, rds_cases, rds_input  # noqa: E402

RDS_FIELDS = ("channel", "carrier", "nco", "rds")


@pytest.mark.parametrize("name", rds_cases())
def test_oracle_rds_matches_golden(orc, name):
    z = load_rds(name)
    if z["n_blocks"] > 100:
        pytest.skip("long case: GPU tests compare it; the oracle pass is covered by the short ones")
    out = orc.rds(z["mode"], rds_input(orc, z))
    for f in RDS_FIELDS:
        if f in z:
            assert np.array_equal(bits(out[f]), bits(z[f])), f
        assert sha(out[f]) == z[f + "_sha256"], f


@pytest.mark.parametrize("mode,nb", [(0, 11), (1, 9)])
def test_oracle_rds_vs_reference_live(orc, ref, mode, nb):
    nif = oracle.MODES[mode][1]
    demod = iqgen.make_rds_demod(50 + mode, nb * nif, oracle.MODES[mode][5])
    demod[::97] *= -3.0  # impulsive samples
    a, b = orc.rds(mode, demod), ref.rds(mode, demod)
    for f in RDS_FIELDS:
        assert np.array_equal(bits(a[f]), bits(b[f])), f


# ---- arctan demodulator and PSD estimate (floating-point, tolerances) ---

import os  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# Tolerances (dB) of the PSD estimate: the reference's Python model is float64 (numpy FFT);
# the oracle/GPU run an accurate double transform and round the per-segment dB to float, then
# average in float like fourier.cpp:109-116 -> within 2e-3 dB of the model on every bin.  The
# C++ estimatePSD is an O(N^2) float DFT whose own error reaches ~1 dB on weak bins at N=4096,
# so it is compared on the bins within 40 dB of its maximum, to 0.01 dB.
PSD_TOL_MODEL_DB = 2e-3
PSD_TOL_CPP_DB = 1e-2
PSD_CPP_RANGE_DB = 40.0


def psd_cases():
    z = np.load(os.path.join(GOLD, "py_psd.npz"))
    return [str(c) for c in z["cases"]]


def check_psd(z, key, freq, psd):
    py, cp = z[f"py_psd_{key}"], z[f"cpp_psd_{key}"]
    assert np.array_equal(freq, z[f"cpp_freq_{key}"])
    assert np.allclose(freq, z[f"py_freq_{key}"], rtol=0, atol=0)
    assert np.abs(psd - py).max() <= PSD_TOL_MODEL_DB
    strong = cp > cp.max() - PSD_CPP_RANGE_DB
    assert np.abs(psd - cp)[strong].max() <= PSD_TOL_CPP_DB


def test_oracle_arctan_matches_python_model(orc):
    z = np.load(os.path.join(GOLD, "py_arctan.npz"))
    b = int(z["block"])
    prev, outs = 0.0, []
    for k in range(z["i"].size // b):
        d, prev = orc.fm_demod_arctan(z["i"][k * b:(k + 1) * b], z["q"][k * b:(k + 1) * b], prev)
        outs.append(d)
        assert prev == z["phases"][k]
    assert np.array_equal(np.concatenate(outs), z["demod"])  # float64, bit for bit


@pytest.mark.parametrize("key", psd_cases())
def test_oracle_psd_matches_python_model_and_cpp(orc, key):
    z = np.load(os.path.join(GOLD, "py_psd.npz"))
    name, nb, fs = key.rsplit("_", 2)
    freq, psd = orc.estimate_psd(z[f"x_{name}"], int(nb), float(fs))
    check_psd(z, key, freq, psd)


def test_oracle_psd_vs_reference_live(orc, ref):
    x = (iqgen.rand_bytes(77, 8192).astype(np.float32) - 127.5) / 127.5
    x += np.sin(np.arange(8192) * 0.3).astype(np.float32)
    f1, p1 = orc.estimate_psd(x, 512, 96000.0)
    f2, p2 = ref.estimate_psd(x, 512, 96000.0)
    assert np.array_equal(f1, f2)
    strong = p2 > p2.max() - PSD_CPP_RANGE_DB
    assert np.abs(p1 - p2)[strong].max() <= PSD_TOL_CPP_DB


def test_oracle_mixer_and_lr(orc):
    """The oracle's mixer (filter.cpp:176-184) and LRExtraction (filter.cpp:186-199), the checkers
    of the GPU elementwise test: float product then doubling; the float sum/difference times the
    double 0.5, rounded back to float."""
    rng = np.random.default_rng(5)
    a = rng.standard_normal(1000).astype(np.float32)
    b = rng.standard_normal(1000).astype(np.float32)
    assert np.array_equal(orc.mixer(a, b), np.float32(2) * (a * b))
    left, right = orc.lr(a, b)
    assert np.array_equal(left, ((a + b).astype(np.float64) * 0.5).astype(np.float32))
    assert np.array_equal(right, ((a - b).astype(np.float64) * 0.5).astype(np.float32))
