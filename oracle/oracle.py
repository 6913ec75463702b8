"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes loaders for the two CPU checkers:
  * ``Oracle``    -> oracle/liboracle.so, the plain-C restatement (fmrx_oracle.c);
  * ``Reference`` -> oracle/_ref/libfmref.so, the reference's OWN src/filter.cpp +
                     src/iofunc.cpp compiled from /root/reference with a sequential
                     project.cpp driver (ref_driver.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libfmref.so")
REF_SRC = "/root/reference"

_fp = C.POINTER(C.c_float)
_i16p = C.POINTER(C.c_int16)
_u8p = C.POINTER(C.c_uint8)


class Outputs(C.Structure):
    """Mirror of orc_outputs / ref_outputs (same field order)."""

    _fields_ = [
        ("demod", _fp), ("mono_exact", _fp), ("mono_indep", _fp), ("pcm", _i16p),
        ("pcm_mono", _i16p), ("channel", _fp), ("carrier", _fp), ("nco", _fp), ("mixer", _fp),
        ("stereo", _fp), ("left", _fp), ("right", _fp), ("pll_state", _fp),
    ]


FIELDS = [f for f, _ in Outputs._fields_]
PER_IF = {"demod", "channel", "carrier", "nco", "mixer"}
PER_AUDIO = {"mono_exact", "mono_indep", "pcm_mono", "stereo", "left", "right"}

# project.cpp:304-364 -> (block_bytes, if_samples, audio_frames, rf_fs, if_fs, bp_fs, up, down)
MODES = {
    0: (12800, 640, 128, 2400000, 240000, 240000, 1, 5),
    1: (6144, 768, 128, 1152000, 288000, 288000, 1, 6),
    2: (2048000, 102400, 18816, 2400000, 240000 * 147, 240000, 147, 800),
    3: (5898240, 327680, 56448, 2304000, 256000 * 441, 256000, 441, 2560),
}


def build(ref: bool | None = None) -> None:
    """Build liboracle.so, and _ref/libfmref.so when the reference sources are present."""
    targets = ["oracle"]
    if ref is None:
        ref = os.path.isdir(REF_SRC)
    if ref:
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _as_u8(iq) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(iq, dtype=np.uint8))


class _Lib:
    prefix = ""
    path = ""

    def __init__(self):
        if not os.path.exists(self.path):
            raise FileNotFoundError(f"{self.path} not built (run oracle.build())")
        self.lib = C.CDLL(self.path)

    def _run(self, fn, mode: int, rf_taps: int, iq, fields=None, demod=None) -> dict:
        bb, nif, na = MODES[mode][:3]
        if demod is not None:  # audio stage only: demod blocks in
            demod = np.ascontiguousarray(demod, np.float32)
            nb = demod.size // nif
        else:
            iq = _as_u8(iq)
            nb = iq.size // bb
        fields = fields or FIELDS
        arrays = {}
        o = Outputs()
        for f in FIELDS:
            if f not in fields:
                continue
            if f in PER_IF:
                a = np.zeros(nb * nif, np.float32)
            elif f == "pcm":
                a = np.zeros(nb * 2 * na, np.int16)
            elif f == "pcm_mono":
                a = np.zeros(nb * na, np.int16)
            elif f == "pll_state":
                a = np.zeros(nb * 6, np.float32)
            else:
                a = np.zeros(nb * na, np.float32)
            arrays[f] = a
            setattr(o, f, _ptr(a, _i16p if a.dtype == np.int16 else _fp))
        fn.restype = C.c_long
        if demod is not None:
            fn.argtypes = [C.c_int, _fp, C.c_size_t, C.POINTER(Outputs)]
            n = fn(mode, _ptr(demod, _fp), nb, C.byref(o))
        else:
            fn.argtypes = [C.c_int, C.c_int, _u8p, C.c_size_t, C.POINTER(Outputs)]
            n = fn(mode, rf_taps, _ptr(iq, _u8p), iq.size, C.byref(o))
        if n < 0:
            raise ValueError("bad mode")
        arrays["n_blocks"] = n
        return arrays

    def run_audio(self, mode: int, demod, fields=None) -> dict:
        """audio_thread alone (project.cpp:132-196) over whole demod blocks (if_samples each),
        plus the private-history mono product; the same output fields as run()."""
        return self._run(getattr(self.lib, self.prefix + "run_audio"), mode, 51, None, fields, demod)

    def lpf(self, fs, fc, taps, gain=1):
        h = np.zeros(taps, np.float32)
        f = getattr(self.lib, self.prefix + "lpf")
        f.argtypes = [_fp, C.c_float, C.c_float, C.c_int, C.c_int]
        f(_ptr(h, _fp), fs, fc, taps, gain)
        return h

    def bpf(self, fs, fb, fe, taps):
        h = np.zeros(taps, np.float32)
        f = getattr(self.lib, self.prefix + "bpf")
        f.argtypes = [_fp, C.c_float, C.c_float, C.c_float, C.c_int]
        f(_ptr(h, _fp), fs, fb, fe, taps)
        return h

    def resample(self, x, state, coeff, up, down):
        x = np.ascontiguousarray(x, np.float32)
        state = np.array(state, np.float32)
        coeff = np.ascontiguousarray(coeff, np.float32)
        out = np.zeros(x.size * up // down, np.float32)
        f = getattr(self.lib, self.prefix + "resample")
        f.argtypes = [_fp, _fp, _fp, C.c_int, _fp, C.c_int, C.c_int, C.c_int]
        f(_ptr(out, _fp), _ptr(state, _fp), _ptr(x, _fp), x.size, _ptr(coeff, _fp), coeff.size, up, down)
        return out, state

    def fmdemod(self, i, q, prev):
        i = np.ascontiguousarray(i, np.float32)
        q = np.ascontiguousarray(q, np.float32)
        prev = np.array(prev, np.float32)
        out = np.zeros(i.size, np.float32)
        f = getattr(self.lib, self.prefix + "fmdemod")
        f.argtypes = [_fp, _fp, _fp, _fp, C.c_int]
        f(_ptr(out, _fp), _ptr(prev, _fp), _ptr(i, _fp), _ptr(q, _fp), i.size)
        return out, prev

    def pll(self, x, freq, fs, nco_scale, phase_adjust, norm_bw, state):
        io = np.array(x, np.float32)
        st = np.array(state, np.float32)
        f = getattr(self.lib, self.prefix + "pll")
        f.argtypes = [_fp, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _fp]
        f(_ptr(io, _fp), io.size, freq, fs, nco_scale, phase_adjust, norm_bw, _ptr(st, _fp))
        return io, st

    def rds(self, mode: int, demod) -> dict:
        """RDS front half (project.cpp:200-271) over whole demod blocks: channel, carrier (PLL
        input), nco (PLL output) and rds (mixer output), if_samples per block each."""
        demod = np.ascontiguousarray(demod, np.float32)
        nif = MODES[mode][1]
        nb = demod.size // nif
        out = {k: np.zeros(nb * nif, np.float32) for k in ("channel", "carrier", "nco", "rds")}
        f = getattr(self.lib, self.prefix + "rds")
        f.restype = C.c_long
        f.argtypes = [C.c_int, _fp, C.c_size_t, _fp, _fp, _fp, _fp]
        n = f(mode, _ptr(demod, _fp), nb, *(_ptr(out[k], _fp) for k in ("channel", "carrier", "nco", "rds")))
        if n < 0:
            raise ValueError("bad mode")
        return out

    def estimate_psd(self, samples, freq_bins: int, fs: float):
        """estimatePSD (fourier.cpp:35-117): (freq, psd_db), freq_bins/2 floats each."""
        x = np.ascontiguousarray(samples, np.float32)
        freq = np.zeros(freq_bins // 2, np.float32)
        psd = np.zeros(freq_bins // 2, np.float32)
        f = getattr(self.lib, self.prefix + "estimate_psd")
        f.restype = C.c_int
        f.argtypes = [_fp, C.c_size_t, C.c_int, C.c_float, _fp, _fp]
        if f(_ptr(x, _fp), x.size, freq_bins, fs, _ptr(freq, _fp), _ptr(psd, _fp)) < 0:
            raise ValueError("need at least one segment")
        return freq, psd

    def normalize(self, b):
        b = _as_u8(b)
        out = np.zeros(b.size, np.float32)
        f = getattr(self.lib, self.prefix + "normalize")
        f.argtypes = [_u8p, C.c_int, _fp]
        f(_ptr(b, _u8p), b.size, _ptr(out, _fp))
        return out


class Oracle(_Lib):
    """The C restatement (fmrx_oracle.c)."""

    prefix = "orc_"
    path = ORACLE_SO

    def run(self, mode, rf_taps, iq, fields=None):
        return self._run(self.lib.orc_run, mode, rf_taps, iq, fields)

    def fm_demod_arctan(self, i, q, prev_phase=0.0):
        """fmDemodArctan (model/fmSupportLib.py:34-63) in float64: (demod, last phase)."""
        i = np.ascontiguousarray(i, np.float64)
        q = np.ascontiguousarray(q, np.float64)
        out = np.zeros(i.size, np.float64)
        pv = C.c_double(prev_phase)
        _dp = C.POINTER(C.c_double)
        f = self.lib.orc_fm_demod_arctan
        f.argtypes = [_dp, _dp, _dp, _dp, C.c_int]
        f(out.ctypes.data_as(_dp), C.byref(pv), i.ctypes.data_as(_dp), q.ctypes.data_as(_dp), i.size)
        return out, pv.value

    def mixer(self, a, b):
        """mixer (filter.cpp:176-184): 2 (a b) in float."""
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        out = np.zeros(a.size, np.float32)
        f = self.lib.orc_mixer
        f.argtypes = [_fp, _fp, _fp, C.c_int]
        f(_ptr(out, _fp), _ptr(a, _fp), _ptr(b, _fp), a.size)
        return out

    def lr(self, mono, stereo):
        """LRExtraction (filter.cpp:186-199): (left, right) = ((m + s) 0.5, (m - s) 0.5)."""
        m = np.ascontiguousarray(mono, np.float32)
        st = np.ascontiguousarray(stereo, np.float32)
        left, right = np.zeros(m.size, np.float32), np.zeros(m.size, np.float32)
        f = self.lib.orc_lr
        f.argtypes = [_fp, _fp, _fp, _fp, C.c_int]
        f(_ptr(left, _fp), _ptr(right, _fp), _ptr(m, _fp), _ptr(st, _fp), m.size)
        return left, right

    def quant(self, x):
        f = self.lib.orc_quant
        f.restype = C.c_int16
        f.argtypes = [C.c_float]
        return np.array([f(float(v)) for v in np.asarray(x, np.float32)], np.int16)


class Reference(_Lib):
    """The reference's own filter.cpp / iofunc.cpp behind a sequential project.cpp driver."""

    prefix = "ref_"
    path = REF_SO

    def run(self, mode, rf_taps, iq, fields=None):
        return self._run(self.lib.ref_run, mode, rf_taps, iq, fields)

    def run_mono(self, mode, rf_taps, iq):
        """Sequential mono-only receive path (the CPU baseline)."""
        iq = _as_u8(iq)
        bb, _, na = MODES[mode][:3]
        nb = iq.size // bb
        out = np.zeros(nb * na, np.int16)
        f = self.lib.ref_run_mono
        f.restype = C.c_long
        f.argtypes = [C.c_int, C.c_int, _u8p, C.c_size_t, _i16p]
        f(mode, rf_taps, _ptr(iq, _u8p), iq.size, _ptr(out, _i16p))
        return out


def reference_available() -> bool:
    return os.path.exists(REF_SO)
