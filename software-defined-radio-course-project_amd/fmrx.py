"""fmrx.py — Python host binding of libfmrx.so (the C ABI in include/fmrx.h).

Mirrors the reference's per-block interface (src/project.cpp rf_thread / audio_thread bodies
and the filter.h primitives) for tests, the bench and Python callers.  There is no CPU
compute path here: everything numeric runs in the HIP kernels of libfmrx.so, and loading
fails loudly if the library has not been built.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
# FMRX_LIB_PATH: an A/B build of the same sources (Makefile `ab` target; measurements only)
LIB_PATH = os.environ.get("FMRX_LIB_PATH") or os.path.join(PKG_DIR, "libfmrx.so")
HEADER = os.path.join(REPO, "include", "fmrx.h")

FMRX_OK, FMRX_EINVAL, FMRX_EHIP, FMRX_ENOMEM, FMRX_ESTATE = 0, -1, -2, -3, -4
MONO, STEREO = 1, 2


class FmrxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fmrx error {code}: {msg}")
        self.code = code


class Config(C.Structure):
    _fields_ = [("mode", C.c_int), ("channels", C.c_int), ("rf_taps", C.c_int),
                ("bp_taps", C.c_int), ("audio_taps", C.c_int), ("n_streams", C.c_int),
                ("device", C.c_int)]


class Geometry(C.Structure):
    _fields_ = [("rf_fs", C.c_int), ("rf_decim", C.c_int), ("if_fs", C.c_int), ("bp_fs", C.c_int),
                ("audio_up", C.c_int), ("audio_down", C.c_int), ("rf_taps", C.c_int),
                ("bp_taps", C.c_int), ("audio_taps_total", C.c_int), ("block_bytes", C.c_size_t),
                ("iq_pairs", C.c_size_t), ("if_samples", C.c_size_t), ("audio_frames", C.c_size_t),
                ("pcm_samples", C.c_size_t)]


_vp, _sz, _fp, _i16p, _u8p = C.c_void_p, C.c_size_t, C.POINTER(C.c_float), C.POINTER(C.c_int16), C.POINTER(C.c_uint8)

# name -> (restype, argtypes); every function declared in include/fmrx.h
PROTOTYPES = {
    "fmrx_config_default": (C.c_int, [C.POINTER(Config), C.c_int, C.c_int]),
    "fmrx_geometry": (C.c_int, [C.POINTER(Config), C.POINTER(Geometry)]),
    "fmrx_create": (C.c_int, [C.POINTER(Config), C.POINTER(_vp)]),
    "fmrx_destroy": (None, [_vp]),
    "fmrx_reset": (C.c_int, [_vp]),
    "fmrx_last_error": (C.c_char_p, []),
    "fmrx_version": (C.c_char_p, []),
    "fmrx_state_size": (C.c_int, [_vp, C.POINTER(_sz)]),
    "fmrx_get_state": (C.c_int, [_vp, _vp, _sz]),
    "fmrx_set_state": (C.c_int, [_vp, _vp, _sz]),
    "fmrx_history_bytes": (C.c_int, [_vp, C.POINTER(_sz)]),
    "fmrx_seek": (C.c_int, [_vp, _vp, _sz, C.c_int]),
    "fmrx_process": (C.c_int, [_vp, _vp, _sz, _vp]),
    "fmrx_rf_block": (C.c_int, [_vp, _vp, _sz, _vp]),
    "fmrx_audio_block": (C.c_int, [_vp, _vp, _sz, _vp]),
    "fmrx_rds_block": (C.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "fmrx_rds_device": (C.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "fmrx_fm_demod_arctan": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int]),
    "fmrx_estimate_psd": (C.c_int, [_vp, _vp, _sz, C.c_int, C.c_float, _vp, _vp]),
    "fmrx_psd_device": (C.c_int, [_vp, _vp, _sz, C.c_int, C.c_float, _vp]),
    "fmrx_process_device": (C.c_int, [_vp, _vp, _sz, _vp]),
    "fmrx_process_device_ex": (C.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "fmrx_synchronize": (C.c_int, [_vp]),
    "fmrx_stream": (_vp, [_vp]),
    "fmrx_kernel_timing": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_long)]),
    "fmrx_impulse_response_lpf": (C.c_int, [_fp, C.c_float, C.c_float, C.c_int, C.c_int]),
    "fmrx_impulse_response_bpf": (C.c_int, [_fp, C.c_float, C.c_float, C.c_float, C.c_int]),
    "fmrx_resample": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int, _vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "fmrx_fm_demod": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int]),
    "fmrx_pll": (C.c_int, [_vp, _vp, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _vp]),
    "fmrx_mixer": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int]),
    "fmrx_lr_extraction": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int]),
    "fmrx_normalize_iq": (C.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "fmrx_quantize": (C.c_int, [_vp, _vp, _sz, _vp]),
    "fmrx_synth_host": (C.c_int, [C.c_uint64, C.c_int, C.c_uint64, _sz, _vp]),
    "fmrx_synth_device": (C.c_int, [_vp, C.c_uint64, C.c_int, C.c_uint64, _sz, _vp]),
    "fmrx_synth_device_streams": (C.c_int, [_vp, _vp, _sz, C.c_int, C.c_uint64, _sz, _vp, _sz]),
    "fmrx_test_pll_fallback": (C.c_int, [_vp, C.c_int, _vp, _vp, _sz, _vp]),
    "fmrx_debug_mono_stamps": (C.c_int, [_vp, _vp, _sz, C.POINTER(_sz)]),
    "fmrx_debug_pll_stats": (C.c_int, [_vp, _vp]),
    "fmrx_debug_set_knob": (C.c_int, [_vp, C.c_int, C.c_double]),
    "fmrx_debug_pll_redos": (C.c_int, [_vp, _vp]),
    "fmrx_debug_stage_timing": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                          C.POINTER(C.c_long), C.c_int]),
}

# fmrx_debug_stage_timing's stage kinds (csrc/fmrx_internal.h StageKind)
STAGES = ["front_end", "bandpass_pair", "pll_prep", "runner_lane", "runner_pred", "runner_sat", "runner_pipe20",
          "runner_pipe21", "runner_pipe22", "pll_check", "pll_tail", "pll_nco", "audio", "runner_idx17", "runner_idx18",
          "runner_idx19", "runner_cnt17", "runner_cnt18", "runner_cnt19", "runner_cnt20", "runner_cnt21", "runner_stick"]

# fmrx_debug_set_knob's knobs (include/fmrx.h FMRX_KNOB_*): none changes the output; the
# pll_inject / pll_pipe_miss / pll_hint_skew test hooks make the PLL runners redo work
KNOBS = {"pll_spec": 0, "pll_sat": 1, "pll_pred": 2, "pll_pipe": 3, "pll_idx": 4, "stereo_chunks": 5,
         "mono_split": 6, "bpf_tile": 7, "halo_kernel": 8, "pll_inject": 9, "pll_pipe_miss": 10,
         "pll_hint_skew": 11, "pll_cnt": 12, "pll_stick": 13, "stereo_head": 14,
         "stereo_lead": 15, "audio_defer": 16, "stereo_tail": 17}
# fmrx_debug_pll_redos's trigOffset ranges (slots r and 4 + r of each stream's 8)
REDO_RANGES = ["[2^17,2^20)", "[2^20,2^21)", "[2^21,2^22)", "[2^22,2^24]"]
REDO_SLOTS = 8
# knobs every new Receiver applies after fmrx_create (tests set it per test, e.g. with
# monkeypatch.setattr; the library itself reads only the tuning knobs' environment variables)
DEFAULT_KNOBS: dict = {}

_lib = None


def header_symbols() -> list[str]:
    """Function names declared in include/fmrx.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fmrx_[a-z0-9_]+)\s*\(", txt)))


def lib() -> C.CDLL:
    """Load libfmrx.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built; run `make -C {PKG_DIR}` "
                              "(the HIP extension is required, there is no CPU path)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != FMRX_OK:
        raise FmrxError(rc, lib().fmrx_last_error().decode())


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def default_config(mode: int = 0, channels: int = MONO, **kw) -> Config:
    cfg = Config()
    _check(lib().fmrx_config_default(C.byref(cfg), mode, channels))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def geometry(cfg: Config) -> Geometry:
    g = Geometry()
    _check(lib().fmrx_geometry(C.byref(cfg), C.byref(g)))
    return g


def lpf(fs: float, fc: float, taps: int, gain: int = 1) -> np.ndarray:
    """impulseResponseLPF (src/filter.cpp:14-37)."""
    h = np.zeros(taps, np.float32)
    _check(lib().fmrx_impulse_response_lpf(h.ctypes.data_as(_fp), fs, fc, taps, gain))
    return h


def bpf(fs: float, fb: float, fe: float, taps: int) -> np.ndarray:
    """impulseResponseBPF (src/filter.cpp:39-64)."""
    h = np.zeros(taps, np.float32)
    _check(lib().fmrx_impulse_response_bpf(h.ctypes.data_as(_fp), fs, fb, fe, taps))
    return h


def synth_host(seed: int, rf_fs: int, first_pair: int, n_pairs: int) -> np.ndarray:
    out = np.zeros(2 * n_pairs, np.uint8)
    _check(lib().fmrx_synth_host(seed, rf_fs, first_pair, n_pairs, _np_ptr(out)))
    return out


class Receiver:
    """One libfmrx context: ``n_streams`` independent IQ streams on one GPU.

    Host-buffer methods mirror the reference's block loop; ``*_device`` methods take
    device pointers (e.g. ``torch.Tensor.data_ptr()``) and enqueue on the context stream.
    """

    def __init__(self, mode: int = 0, channels: int = MONO, rf_taps: int = 51, n_streams: int = 1,
                 device: int = 0, bp_taps: int = 51, audio_taps: int = 51, knobs: dict | None = None):
        self.cfg = default_config(mode, channels, rf_taps=rf_taps, n_streams=n_streams,
                                  device=device, bp_taps=bp_taps, audio_taps=audio_taps)
        self.geo = geometry(self.cfg)
        h = C.c_void_p()
        _check(lib().fmrx_create(C.byref(self.cfg), C.byref(h)))
        self.h = h
        self.n_streams = n_streams
        self.channels = channels
        for k, v in {**DEFAULT_KNOBS, **(knobs or {})}.items():
            self.set_knob(k, v)

    def set_knob(self, name: str, value: float) -> None:
        """fmrx_debug_set_knob (include/fmrx.h FMRX_KNOB_*; KNOBS names them)."""
        _check(lib().fmrx_debug_set_knob(self.h, KNOBS[name], float(value)))

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().fmrx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- sizes
    @property
    def block_bytes(self) -> int:
        return self.geo.block_bytes

    def n_blocks(self, n_bytes_per_stream: int) -> int:
        return n_bytes_per_stream // self.geo.block_bytes

    # ---- host entry points
    def _streams(self, iq: np.ndarray) -> tuple[np.ndarray, int]:
        iq = np.ascontiguousarray(iq, np.uint8).reshape(self.n_streams, -1)
        nb = iq.shape[1] // self.geo.block_bytes
        return np.ascontiguousarray(iq[:, : nb * self.geo.block_bytes]), nb

    def process(self, iq: np.ndarray) -> np.ndarray:
        """Full blocks of u8 I/Q (per stream) -> S16 PCM (R,L interleaved for stereo)."""
        iq, nb = self._streams(iq)
        out = np.zeros((self.n_streams, nb * self.geo.pcm_samples), np.int16)
        if nb:
            _check(lib().fmrx_process(self.h, _np_ptr(iq), nb, _np_ptr(out)))
        return out if self.n_streams > 1 else out[0]

    def rf_block(self, iq: np.ndarray) -> np.ndarray:
        """rf_thread body (project.cpp:48-70): u8 I/Q -> demod floats."""
        iq, nb = self._streams(iq)
        out = np.zeros((self.n_streams, nb * self.geo.if_samples), np.float32)
        if nb:
            _check(lib().fmrx_rf_block(self.h, _np_ptr(iq), nb, _np_ptr(out)))
        return out if self.n_streams > 1 else out[0]

    def audio_block(self, demod: np.ndarray) -> np.ndarray:
        """audio_thread body (project.cpp:132-195): demod floats -> S16."""
        d = np.ascontiguousarray(demod, np.float32).reshape(self.n_streams, -1)
        nb = d.shape[1] // self.geo.if_samples
        out = np.zeros((self.n_streams, nb * self.geo.pcm_samples), np.int16)
        if nb:
            _check(lib().fmrx_audio_block(self.h, _np_ptr(d), nb, _np_ptr(out)))
        return out if self.n_streams > 1 else out[0]

    def rds_block(self, demod: np.ndarray, want_nco: bool = False, want_channel: bool = False):
        """rds_thread body (project.cpp:200-271): demod floats -> RDS mixer output (and
        optionally the PLL output and the 54-60 kHz channel).  Returns a dict of arrays."""
        d = np.ascontiguousarray(demod, np.float32).reshape(self.n_streams, -1)
        nb = d.shape[1] // self.geo.if_samples
        n = nb * self.geo.if_samples
        d = np.ascontiguousarray(d[:, :n])
        out = {"rds": np.zeros((self.n_streams, n), np.float32)}
        if want_nco:
            out["nco"] = np.zeros((self.n_streams, n), np.float32)
        if want_channel:
            out["channel"] = np.zeros((self.n_streams, n), np.float32)
        if nb:
            _check(lib().fmrx_rds_block(self.h, _np_ptr(d), nb, _np_ptr(out["rds"]),
                                        _np_ptr(out["nco"]) if want_nco else None,
                                        _np_ptr(out["channel"]) if want_channel else None))
        return {k: (v if self.n_streams > 1 else v[0]) for k, v in out.items()}

    def rds_device(self, d_demod: int, n_blocks: int, d_rds: int, d_nco: int | None = None,
                   d_channel: int | None = None) -> None:
        _check(lib().fmrx_rds_device(self.h, d_demod, n_blocks, d_rds, d_nco, d_channel))

    def estimate_psd(self, samples: np.ndarray, freq_bins: int, fs: float):
        """estimatePSD (fourier.cpp:35-117) on the GPU: (freq, psd_db)."""
        x = np.ascontiguousarray(samples, np.float32)
        freq = np.zeros(freq_bins // 2, np.float32)
        psd = np.zeros(freq_bins // 2, np.float32)
        _check(lib().fmrx_estimate_psd(self.h, _np_ptr(x), x.size, freq_bins, fs, _np_ptr(freq), _np_ptr(psd)))
        return freq, psd

    def psd_device(self, d_samples: int, n: int, freq_bins: int, fs: float, d_psd: int) -> None:
        _check(lib().fmrx_psd_device(self.h, d_samples, n, freq_bins, fs, d_psd))

    def fm_demod_arctan(self, d_out: int, d_prev_phase: int, d_i: int, d_q: int, n: int) -> None:
        """fmDemodArctan (fmSupportLib.py:34-63) on device buffers (float in/out, double phase)."""
        _check(lib().fmrx_fm_demod_arctan(self.h, d_out, d_prev_phase, d_i, d_q, n))

    # ---- device entry points (pointers are device addresses)
    def process_device(self, d_iq: int, n_blocks: int, d_pcm: int, d_mono: int | None = None) -> None:
        _check(lib().fmrx_process_device_ex(self.h, d_iq, n_blocks, d_pcm, d_mono))

    def synchronize(self) -> None:
        _check(lib().fmrx_synchronize(self.h))

    def stream(self) -> int:
        return lib().fmrx_stream(self.h)

    def synth_device(self, seed: int, first_pair: int, n_pairs: int, d_out: int) -> None:
        _check(lib().fmrx_synth_device(self.h, seed, self.geo.rf_fs, first_pair, n_pairs, d_out))

    def synth_device_streams(self, seeds, first_pair: int, n_pairs: int, d_out: int, stride: int) -> None:
        """One launch for several streams: stream k (seed seeds[k]) at d_out + k * stride bytes."""
        sd = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))
        _check(lib().fmrx_synth_device_streams(self.h, sd.ctypes.data, sd.size, self.geo.rf_fs, first_pair,
                                               n_pairs, d_out, stride))

    def kernel_timing(self, reset: int = 0) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_long()
        _check(lib().fmrx_kernel_timing(self.h, reset, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # ---- state
    def get_state(self) -> bytes:
        n = C.c_size_t()
        _check(lib().fmrx_state_size(self.h, C.byref(n)))
        buf = (C.c_uint8 * n.value)()
        _check(lib().fmrx_get_state(self.h, C.addressof(buf), n.value))
        return bytes(buf)

    def set_state(self, blob: bytes) -> None:
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        _check(lib().fmrx_set_state(self.h, C.addressof(buf), len(blob)))

    def reset(self) -> None:
        _check(lib().fmrx_reset(self.h))

    # ---- time shards of one recording (mono product)
    def history_bytes(self) -> int:
        """Raw bytes before a shard that fully determine the mono product's state there."""
        n = C.c_size_t()
        _check(lib().fmrx_history_bytes(self.h, C.byref(n)))
        return n.value

    def seek(self, prev, n: int | None = None) -> None:
        """Continue, on the next call, a stream whose preceding bytes are `prev`: a host
        array (n_streams x n u8, or 1-D for one stream) or, with `n` given, a device address
        of n_streams x n bytes."""
        if n is not None:
            _check(lib().fmrx_seek(self.h, prev, n, 1))
            return
        a = np.ascontiguousarray(np.asarray(prev, np.uint8).reshape(self.cfg.n_streams, -1))
        _check(lib().fmrx_seek(self.h, a.ctypes.data, a.shape[1], 0))

    # ---- filter.h primitives on device pointers
    def resample(self, d_out, d_state, d_in, n_in, d_coeff, taps, up, down) -> int:
        n = C.c_int()
        _check(lib().fmrx_resample(self.h, d_out, d_state, d_in, n_in, d_coeff, taps, up, down, C.byref(n)))
        return n.value

    def fm_demod(self, d_out, d_prev, d_i, d_q, n) -> None:
        _check(lib().fmrx_fm_demod(self.h, d_out, d_prev, d_i, d_q, n))

    def pll(self, d_io, n, freq, fs, nco_scale, phase_adjust, norm_bw, d_state) -> None:
        _check(lib().fmrx_pll(self.h, d_io, n, freq, fs, nco_scale, phase_adjust, norm_bw, d_state))

    def mixer(self, d_out, d_a, d_b, n) -> None:
        _check(lib().fmrx_mixer(self.h, d_out, d_a, d_b, n))

    def lr_extraction(self, d_l, d_r, d_m, d_s, n) -> None:
        _check(lib().fmrx_lr_extraction(self.h, d_l, d_r, d_m, d_s, n))

    def normalize_iq(self, d_iq, n_pairs, d_i, d_q) -> None:
        _check(lib().fmrx_normalize_iq(self.h, d_iq, n_pairs, d_i, d_q))

    def quantize(self, d_x, n, d_out) -> None:
        _check(lib().fmrx_quantize(self.h, d_x, n, d_out))

    def test_pll_fallback(self, kind: int, d_a, d_b, n: int, d_out) -> None:
        """Test hook: the PLL's fallback libm on device (0 sincos, 1 atan2, 2 NCO cos)."""
        _check(lib().fmrx_test_pll_fallback(self.h, kind, d_a, d_b, n, d_out))

    def debug_mono_stamps(self, d_stamps: int | None, n_workgroups: int = 0) -> int:
        """Diagnostic clock stamps of the fused mono kernel (fmrx.h); returns the stamp slots a
        call may need (6 u64 each)."""
        need = _sz()
        _check(lib().fmrx_debug_mono_stamps(self.h, d_stamps, n_workgroups, C.byref(need)))
        return need.value

    def stage_timing(self, op: int) -> dict | None:
        """Per-stage device time of the stereo engine (fmrx_debug_stage_timing): op 1 arms,
        0 reads, -1 reads and disarms; a read returns {stage: (ms, launches, steps)}."""
        n = len(STAGES)
        ms, steps, la = (C.c_double * n)(), (C.c_double * n)(), (C.c_long * n)()
        _check(lib().fmrx_debug_stage_timing(self.h, op, ms, steps, la, n))
        if op == 1:
            return None
        return {STAGES[k]: (ms[k], la[k], steps[k]) for k in range(n) if la[k]}

    def debug_pll_stats(self, d_counts: int | None) -> None:
        """Diagnostic speculative-PLL counters (fmrx.h): d_counts[0] += runner batches that did
        not verify, d_counts[1] += batches checked (2 u64 on the device); None turns it off."""
        _check(lib().fmrx_debug_pll_stats(self.h, d_counts))

    def debug_pll_redos(self, d_counts) -> None:
        """fmrx_debug_pll_redos: per stream and trigOffset range of the self-certifying runners
        (REDO_RANGES), redone intervals and demoted steps (n_streams x 8 u32 on the device, zeroed
        by the caller: [r] redone intervals, [4 + r] demoted steps; None turns it off)."""
        _check(lib().fmrx_debug_pll_redos(self.h, d_counts))


def build() -> None:
    """Compile libfmrx.so and the fmrx CLI for gfx950 (hipcc cross-compiles without a GPU)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", PKG_DIR, "-j8"], check=True)
