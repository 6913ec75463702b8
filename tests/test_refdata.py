"""The reference's OWN data files as inputs (tests/golden/refdata.npz, made by
tests/golden/make_refdata.py from /root/reference/data):

* data/fm_demod_10.bin, fm_demod_11.bin -- 5,120 float32 each of real broadcast FM demod
  (blocks 10 and 11 of a recording, model/fmMonoBlock.py:277-280) = 8 mode-0 blocks each --
  through the audio stage (project.cpp:132-196): stereo R,L PCM, the mono product and the PLL
  state after every block, bit-exact against the reference build (oracle/_ref) on the same
  floats;
* data/q_block_time.dat -> data/q_filt_time.dat -- a 151-tap LPF (2.4 MHz, 100 kHz) known-answer
  test from the reference's lab era (logVector, src/logfunc.cpp:23-43): the Q bytes normalised
  as (q - 127) / 128 (that lab's convention, not readStdinBlockData's -128: it is the one the
  text file matches), filtered by impulseResponseLPF + resample (filter.cpp:14-37, 67-103) and
  compared with the file at its 6-significant-digit text precision past the 150-sample start
  transient (the file's first 150 rows are not the zero-state filter's).

CPU tests pin the oracle to the fixture; GPU tests run the HIP path through the C ABI.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = ["10", "11", "10_11"]
KAT_TOL = 1e-5  # q_filt_time.dat prints 6 significant digits of values |y| <= ~1.1 (5e-6 half-ulp)
KAT_SKIP = 150  # start transient: rows 0..149 of the file are not the zero-state filter's


@pytest.fixture(scope="module")
def rd():
    return dict(np.load(os.path.join(HERE, "golden", "refdata.npz")))


def demod_of(rd, k):
    return np.concatenate([rd["demod_10"], rd["demod_11"]]) if k == "10_11" else rd[f"demod_{k}"]


def q_input(rd):
    return ((rd["q_block"] - 127.0) / 128.0).astype(np.float32)


# ---- CPU: the oracle against the reference build's outputs on the reference's data ------------

@pytest.mark.parametrize("k", KEYS)
def test_oracle_audio_on_reference_demod(orc, rd, k):
    out = orc.run_audio(0, demod_of(rd, k), ["pcm", "pcm_mono", "pll_state"])
    assert np.array_equal(out["pcm"], rd[f"pcm_{k}"])
    assert np.array_equal(out["pcm_mono"], rd[f"pcm_mono_{k}"])
    assert np.array_equal(out["pll_state"].view(np.uint32), rd[f"pll_{k}"].view(np.uint32))


def test_oracle_q_filt_kat(orc, rd):
    h = orc.lpf(2.4e6, 100e3, 151, 1)
    y, _ = orc.resample(q_input(rd), np.zeros(150, np.float32), h, 1, 1)
    err = np.abs(y.astype(np.float64) - rd["q_filt"])
    assert err[KAT_SKIP:].max() < KAT_TOL, err[KAT_SKIP:].max()
    assert err[:KAT_SKIP].max() > 0.1  # the transient really is different data


def test_reference_data_is_real_signal(rd):
    """Guard against a degenerate fixture: real broadcast audio, not silence or clipping."""
    for k in KEYS:
        pcm = rd[f"pcm_{k}"]
        assert np.abs(pcm).max() > 1000 and np.count_nonzero(pcm) > 0.9 * pcm.size
    assert rd["q_block"].size == 10240 and rd["q_filt"].size == 10240


# ---- GPU: the HIP path through the C ABI ----------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("k", KEYS)
def test_audio_block_on_reference_demod(fmrx, rd, k):
    pytest.importorskip("torch").cuda.init()
    d = demod_of(rd, k)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        assert np.array_equal(rx.audio_block(d), rd[f"pcm_{k}"])
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        assert np.array_equal(rx.audio_block(d), rd[f"pcm_mono_{k}"])


@pytest.mark.gpu
def test_audio_block_on_reference_demod_split_calls(fmrx, rd):
    """The 16 contiguous blocks in uneven calls (3, 8, 5 blocks: the split crosses the seam
    between the two dumps at block 8) give the one-call PCM."""
    pytest.importorskip("torch").cuda.init()
    d = demod_of(rd, "10_11")
    nif = 640
    for ch, key in ((fmrx.STEREO, "pcm_10_11"), (fmrx.MONO, "pcm_mono_10_11")):
        with fmrx.Receiver(0, ch) as rx:
            parts, pos = [], 0
            for n in (3, 8, 5):
                parts.append(rx.audio_block(d[pos * nif:(pos + n) * nif]))
                pos += n
        assert np.array_equal(np.concatenate(parts), rd[key]), ch


@pytest.mark.gpu
def test_resample_q_filt_kat(fmrx, rd):
    """fmrx_impulse_response_lpf(151 taps) + fmrx_resample on the device against the reference's
    q_filt_time.dat, and bit-exact against the oracle's resample of the same floats."""
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    h = fmrx.lpf(2.4e6, 100e3, 151, 1)
    x = q_input(rd)
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        d_x = torch.from_numpy(x).cuda()
        d_h = torch.from_numpy(h).cuda()
        d_st = torch.zeros(150, dtype=torch.float32, device="cuda")
        d_y = torch.zeros(x.size, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        n = rx.resample(d_y.data_ptr(), d_st.data_ptr(), d_x.data_ptr(), x.size, d_h.data_ptr(), 151, 1, 1)
        rx.synchronize()
        y = d_y.cpu().numpy()
        st = d_st.cpu().numpy()
    assert n == x.size
    err = np.abs(y.astype(np.float64) - rd["q_filt"])
    assert err[KAT_SKIP:].max() < KAT_TOL, err[KAT_SKIP:].max()
    import oracle

    want, want_st = oracle.Oracle().resample(x, np.zeros(150, np.float32), h, 1, 1)
    assert np.array_equal(y.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(st.view(np.uint32), want_st.view(np.uint32))
