"""GPU parity: libfmrx's HIP kernels (through the C ABI) against the reference's outputs.

Every comparison is bit-exact (integer PCM and the float bit patterns of intermediates):
  * golden fixtures produced by the reference itself (tests/golden, make_golden.py);
  * the C restatement oracle (pinned to those fixtures) on fresh seeded inputs;
  * size-independent properties at BASELINE sizes: call-split invariance, state
    checkpoint/resume, and windowed oracle checks anywhere inside a 1 GiB stream (the mono
    product has finite memory, so an oracle run started one block early is exact).
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import iqgen
import oracle
from conftest import bench_runs, case_input, golden_cases, load_case, long_runs, unlocked_runs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")



def knobs(monkeypatch, fm, **kw):
    """Knobs (fmrx_debug_set_knob) of the Receivers this test creates; the test hooks among them
    (pll_inject, pll_pipe_miss, pll_hint_skew) are not readable from the environment."""
    monkeypatch.setattr(fm, "DEFAULT_KNOBS", {**fm.DEFAULT_KNOBS, **kw})

def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def same(a, b):
    return np.array_equal(bits(a), bits(b))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()


MONO_CASES = [n for n in golden_cases() if "pcm_mono" in load_case(n)]
STEREO_CASES = [n for n in golden_cases() if "pcm" in load_case(n)]


# ---- fused mono product ---------------------------------------------------------------------

@pytest.mark.parametrize("name", MONO_CASES)
def test_mono_pcm_matches_reference(fmrx, name):
    z = load_case(name)
    iq = case_input(z)
    with fmrx.Receiver(z["mode"], fmrx.MONO, rf_taps=z["rf_taps"]) as rx:
        pcm = rx.process(iq)
    assert np.array_equal(pcm, z["pcm_mono"]), name


@pytest.mark.parametrize("name", [n for n in MONO_CASES if "mono_indep" in load_case(n)])
def test_mono_float_matches_reference(fmrx, name):
    z = load_case(name)
    iq = case_input(z)
    with fmrx.Receiver(z["mode"], fmrx.MONO, rf_taps=z["rf_taps"]) as rx:
        nb = z["n_blocks"]
        d_iq = torch.from_numpy(iq).cuda()
        d_pcm = torch.zeros(nb * rx.geo.audio_frames, dtype=torch.int16, device="cuda")
        d_mono = torch.zeros(nb * rx.geo.audio_frames, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr(), d_mono.data_ptr())
        rx.synchronize()
        assert same(d_mono.cpu().numpy(), z["mono_indep"])
        assert np.array_equal(d_pcm.cpu().numpy(), z["pcm_mono"])


@pytest.mark.parametrize("name", [n for n in golden_cases() if "demod" in load_case(n)])
def test_rf_block_demod_matches_reference(fmrx, name):
    z = load_case(name)
    with fmrx.Receiver(z["mode"], fmrx.MONO, rf_taps=z["rf_taps"]) as rx:
        demod = rx.rf_block(case_input(z))
    assert same(demod, z["demod"])


@pytest.mark.parametrize("name", [n for n in MONO_CASES if "demod" in load_case(n)])
def test_mono_audio_block_from_reference_demod(fmrx, name):
    z = load_case(name)
    with fmrx.Receiver(z["mode"], fmrx.MONO, rf_taps=z["rf_taps"]) as rx:
        pcm = rx.audio_block(z["demod"])
    assert np.array_equal(pcm, z["pcm_mono"])


@pytest.mark.parametrize("mode,rf_taps", [(0, 51), (0, 101), (1, 51), (1, 101)])
def test_mono_call_split_and_resume(fmrx, orc, mode, rf_taps):
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    nb = 37
    iq = iqgen.make("synth:41", nb * bb, rf_fs)
    want = orc.run(mode, rf_taps, iq, ["pcm_mono"])["pcm_mono"]
    with fmrx.Receiver(mode, fmrx.MONO, rf_taps=rf_taps) as rx:
        got = rx.process(iq)
        assert np.array_equal(got, want)
        rx.reset()
        parts, pos = [], 0
        na = rx.geo.audio_frames
        for n in (1, 2, 5, 1, 11, 3, 14):  # ragged call sizes, 37 blocks in total
            parts.append(rx.process(iq[pos * bb:(pos + n) * bb]))
            pos += n
            if pos == 9:  # checkpoint / resume through a second context
                blob = rx.get_state()
                with fmrx.Receiver(mode, fmrx.MONO, rf_taps=rf_taps) as rx2:
                    rx2.set_state(blob)
                    tail = rx2.process(iq[pos * bb:])
                assert np.array_equal(tail, want[pos * na:])
        assert np.array_equal(np.concatenate(parts), want)


@pytest.mark.parametrize("mode,nb", [(0, 23), (1, 19), (2, 5)])
def test_stereo_call_split_and_resume(fmrx, orc, mode, nb):
    """REF_EXACT stereo across ragged call sizes and a checkpoint / resume into a second
    context: the blob carries the demod history, PLL state, mixer tail and mono delay line of
    every stream (3 streams, each its own input)."""
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    ns = 3
    iqs = [iqgen.make(f"synth:{71 + k}", nb * bb, rf_fs) for k in range(ns)]
    want = np.stack([orc.run(mode, 51, x, ["pcm"])["pcm"] for x in iqs])
    iq = np.stack(iqs)
    with fmrx.Receiver(mode, fmrx.STEREO, n_streams=ns) as rx:
        ps = rx.geo.pcm_samples
        parts, pos = [], 0
        for n in (1, 3, 2, nb - 6):
            parts.append(rx.process(iq[:, pos * bb:(pos + n) * bb]))
            pos += n
            if pos in (1, 4):  # checkpoint / resume through a second context
                blob = rx.get_state()
                with fmrx.Receiver(mode, fmrx.STEREO, n_streams=ns) as rx2:
                    rx2.set_state(blob)
                    tail = rx2.process(iq[:, pos * bb:])
                assert np.array_equal(tail, want[:, pos * ps:]), (mode, pos)
        assert np.array_equal(np.concatenate(parts, axis=1), want)


def test_create_refuses_streams_beyond_grid_limit(fmrx):
    """n_streams lands on grid.y of every per-stream launch: fmrx_create refuses a count no
    device can launch (EINVAL at create time, before any allocation)."""
    with pytest.raises(fmrx.FmrxError) as e:
        fmrx.Receiver(0, fmrx.STEREO, n_streams=2**31 - 1)
    assert e.value.code == fmrx.FMRX_EINVAL


def test_state_blob_keeps_seek_staleness(fmrx):
    """A blob taken between fmrx_seek and the next fused call restores a stale audio history:
    the split API's audio stage must refuse it in the second context too (ESTATE)."""
    bb = oracle.MODES[0][0]
    iq = iqgen.make("synth:5", 3 * bb)
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        rx.process(iq[:bb])
        rx.seek(iq[:2 * bb])
        blob = rx.get_state()
        demod = np.zeros(rx.geo.if_samples, np.float32)
        with pytest.raises(fmrx.FmrxError):
            rx.audio_block(demod)
        with fmrx.Receiver(0, fmrx.MONO) as rx2:
            rx2.set_state(blob)
            with pytest.raises(fmrx.FmrxError):
                rx2.audio_block(demod)
            rx2.process(iq[2 * bb:])  # a fused call refreshes the history
            rx2.audio_block(demod)


def test_state_blob_header_errors(fmrx):
    """fmrx_set_state names what is wrong with a foreign blob: another format version, another
    context shape, a non-zero reserved word (FMRX_ESTATE each, the context unchanged)."""
    with fmrx.Receiver(0, fmrx.STEREO) as rx, fmrx.Receiver(0, fmrx.MONO) as other:
        good = rx.get_state()
        for word, val, msg in ((1, 1, "version 1, expected 2"), (0, 7, "not an fmrx state blob"),
                               (9, 5, "reserved word 9")):
            bad = bytearray(good)
            bad[4 * word: 4 * word + 4] = np.uint32(val).tobytes()
            with pytest.raises(fmrx.FmrxError) as e:
                rx.set_state(bytes(bad))
            assert e.value.code == fmrx.FMRX_ESTATE and msg in str(e.value), str(e.value)
        with pytest.raises(fmrx.FmrxError) as e:
            rx.set_state(other.get_state() + bytes(len(good)))
        assert "another context shape" in str(e.value)
        rx.set_state(good)


def test_trig_hint_after_set_state(fmrx, monkeypatch):
    """The host-side trigOffset bounds that pick which PLL runners launch (api.cpp TrigTrack)
    follow a restored blob: a stream restored at 2^20 - 2,000 crosses into the predicted
    runner's range within the call and one at 2^24 - 3,000 into the saturated runner's; the PCM
    equals the lane runner's alone (knob pll_pred=0, knob pll_sat=0: every segment on it), and
    every batch verified -- a runner left out by a wrong bound would leave its waves unrun."""
    bb = oracle.MODES[0][0]
    iq = iqgen.make("synth:91", 30 * bb)

    def run(trig):
        with fmrx.Receiver(0, fmrx.STEREO) as rx:
            blob = bytearray(rx.get_state())
            hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
            pll_off = 40 + int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64
            pll = np.frombuffer(bytes(blob[pll_off: pll_off + 32]), np.float32).copy()
            pll[5] = trig
            blob[pll_off: pll_off + 32] = pll.tobytes()
            rx.set_state(bytes(blob))
            counts = torch.zeros(2, dtype=torch.int64, device="cuda")
            rx.debug_pll_stats(counts.data_ptr())
            got = rx.process(iq)
            rx.debug_pll_stats(None)
        return got, counts.cpu().tolist()

    for trig in (1048576.0 - 2000, 16777216.0 - 3000):
        got, (resumed, checked) = run(trig)
        assert checked > 0 and resumed == 0, (trig, resumed, checked)
        knobs(monkeypatch, fmrx, pll_pred=0)
        knobs(monkeypatch, fmrx, pll_sat=0)
        want, _ = run(trig)
        knobs(monkeypatch, fmrx, pll_pred=1, pll_sat=1)
        assert np.array_equal(got, want), trig


@pytest.mark.parametrize("mode,nb", [(2, 6), (3, 4)])
def test_polyphase_mono_split_resume_and_mixed_api(fmrx, orc, mode, nb):
    """Modes 2/3 run the rational resampler inside the fused kernel; its history must survive
    call splits, a checkpoint into a second context, and hand-over to the split API."""
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    iq = iqgen.make("synth:61", nb * bb, rf_fs)
    want = orc.run(mode, 51, iq, ["pcm_mono"])["pcm_mono"]
    na = oracle.MODES[mode][2]
    with fmrx.Receiver(mode, fmrx.MONO) as rx:
        parts, pos = [], 0
        for n in (1, 2, nb - 3):
            parts.append(rx.process(iq[pos * bb:(pos + n) * bb]))
            pos += n
            if pos == 1:
                with fmrx.Receiver(mode, fmrx.MONO) as rx2:
                    rx2.set_state(rx.get_state())
                    assert np.array_equal(rx2.process(iq[bb:]), want[na:])
        assert np.array_equal(np.concatenate(parts), want)
        rx.reset()
        first = rx.process(iq[:2 * bb])  # fused ...
        rest = rx.audio_block(rx.rf_block(iq[2 * bb:]))  # ... then the reference's thread split
        assert np.array_equal(np.concatenate([first, rest]), want)


@pytest.mark.parametrize("mode,nb", [(0, 7), (1, 5), (2, 3)])
def test_thread_split_block_by_block(fmrx, orc, mode, nb):
    """project.cpp's thread split on one context, block by block: rf_block(b) then
    audio_block(b) (the audio stage owns the audio history, the RF stage must not touch it)."""
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    iq = iqgen.make("synth:62", nb * bb, rf_fs)
    with fmrx.Receiver(mode, fmrx.MONO) as rx:
        got = [rx.audio_block(rx.rf_block(iq[b * bb:(b + 1) * bb])) for b in range(nb)]
    assert np.array_equal(np.concatenate(got), orc.run(mode, 51, iq, ["pcm_mono"])["pcm_mono"])
    with fmrx.Receiver(mode, fmrx.STEREO) as rx:
        got = [rx.audio_block(rx.rf_block(iq[b * bb:(b + 1) * bb])) for b in range(nb)]
    assert np.array_equal(np.concatenate(got), orc.run(mode, 51, iq, ["pcm"])["pcm"])


@pytest.mark.parametrize("channels", [2, 1])
def test_two_context_thread_split_overlaps(fmrx, orc, channels):
    """INTEGRATION.md Option 1 in its overlapping form: project.cpp's two threads, each with
    its OWN context -- context A only runs fmrx_rf_block (it owns the RF histories and the
    demodulator's previous sample), context B only fmrx_audio_block (the band-pass histories,
    PLL, shared audio_state and mono delay) -- joined by a bounded queue of depth 3
    (QUEUE_CAPACITY, project.cpp:17,71-80,133-141).  48 blocks one per call: B's PCM equals
    the oracle's, and the stages really ran concurrently (ctypes drops the GIL; each context
    has its own lock)."""
    import queue
    import threading
    import time

    nb, bb = 48, 12800
    iq = iqgen.make("synth:63", nb * bb)
    q = queue.Queue(maxsize=3)
    spans = {"rf": [], "audio": []}
    out, errors = [], []
    with fmrx.Receiver(0, channels) as ra, fmrx.Receiver(0, channels) as rb:
        def rf_thread():
            try:
                for b in range(nb):
                    t0 = time.perf_counter()
                    d = ra.rf_block(iq[b * bb:(b + 1) * bb])
                    spans["rf"].append((t0, time.perf_counter()))
                    q.put(d)
            except Exception as e:  # pragma: no cover - surfaced below
                errors.append(e)
            q.put(None)

        def audio_thread():
            try:
                while (d := q.get()) is not None:
                    t0 = time.perf_counter()
                    out.append(rb.audio_block(d))
                    spans["audio"].append((t0, time.perf_counter()))
            except Exception as e:  # pragma: no cover
                errors.append(e)

        ts = [threading.Thread(target=rf_thread), threading.Thread(target=audio_thread)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
    assert not errors, errors
    field = "pcm" if channels == 2 else "pcm_mono"
    assert len(out) == nb
    assert np.array_equal(np.concatenate(out), orc.run(0, 51, iq, [field])[field])
    overlapped = sum(1 for a0, a1 in spans["audio"] for r0, r1 in spans["rf"] if r0 < a1 and a0 < r1)
    assert overlapped >= nb // 4, overlapped


def test_mono_multistream_independent(fmrx, orc):
    nb, bb = 23, 12800
    ins = [iqgen.make(r, nb * bb) for r in ("synth:51", "rand:52", "synth:53", "const128")]
    with fmrx.Receiver(0, fmrx.MONO, rf_taps=101, n_streams=len(ins)) as rx:
        out = rx.process(np.stack(ins))
    for s, iq in enumerate(ins):
        assert np.array_equal(out[s], orc.run(0, 101, iq, ["pcm_mono"])["pcm_mono"]), s


@pytest.mark.parametrize("channels,n_streams,share", [(1, 3, None), (1, 4, "900"), (2, 2, None)])
def test_unequal_wave_shares_multistream(fmrx, orc, monkeypatch, channels, n_streams, share):
    """The fused kernel's two-waves-per-SIMD split (mono_fused.hip mono_share: workgroups w and
    w + grid/2 share a span, the first taking kOlderShare/1024 of it) with several streams:
    ~2,048 workgroups (3 streams: 682 even segments each, 2,046 workgroups), an extreme share
    (knob mono_split=900), and the stereo engine's front end.  Every stream equals the oracle."""
    if share is not None:
        knobs(monkeypatch, fmrx, mono_split=float(share))
    nb, bb = 420, 12800  # 2,800 chunks per stream: enough for the full-chip grid
    recipes = [("synth:%d" if s % 2 == 0 else "rand:%d") % (300 + s) for s in range(n_streams)]
    ins = np.stack([iqgen.make(r, nb * bb) for r in recipes])
    taps = 101 if channels == 1 else 51
    with fmrx.Receiver(0, channels, rf_taps=taps, n_streams=n_streams) as rx:
        out = rx.process(ins)
    field = "pcm" if channels == 2 else "pcm_mono"
    for s_ in range(n_streams):
        assert np.array_equal(out[s_], orc.run(0, taps, ins[s_], [field])[field]), s_


@pytest.mark.parametrize("mode,rf_taps,nb,cuts", [(0, 101, 40, (1, 7, 23)), (0, 51, 12, (3,)),
                                                   (1, 51, 30, (2, 17)), (2, 51, 4, (1, 3)), (3, 101, 3, (1, 2))])
def test_time_shards_with_seek_equal_whole_stream(fmrx, mode, rf_taps, nb, cuts):
    """fmrx_seek: a recording cut at block boundaries, each shard processed by a
    fresh context that first seeks to the bytes in front of it (the whole prefix, or only the
    last history_bytes of it), gives the whole recording's mono PCM bit for bit -- including
    the first cut, whose prefix is shorter than the history (the stream began inside it)."""
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    iq = iqgen.make("synth:31", nb * bb, rf_fs)
    with fmrx.Receiver(mode, fmrx.MONO, rf_taps=rf_taps) as rx:
        whole = rx.process(iq)
        hb = rx.history_bytes()
    edges = [0, *cuts, nb]
    for trim in (False, True):
        pieces = []
        for a, b in zip(edges, edges[1:]):
            with fmrx.Receiver(mode, fmrx.MONO, rf_taps=rf_taps) as rx:
                if a:
                    prev = iq[: a * bb]
                    rx.seek(prev[-hb:] if trim else prev)
                pieces.append(rx.process(iq[a * bb: b * bb]))
        assert np.array_equal(np.concatenate(pieces), whole), trim


def test_time_shard_worker_and_seek_errors(fmrx):
    """dist.fmrx_time_shard_fn (device-side history + seek) over 3 shards equals one context on
    the whole stream; seek is refused for stereo and leaves the split API's audio stage
    without history until a fused call."""
    d = iqgen.load_module("dist")
    nb, seed = 25, 4242
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        bb, na = rx.geo.block_bytes, rx.geo.pcm_samples
        iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
        want = torch.empty(nb * na, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        rx.synth_device(seed, 0, nb * bb // 2, iq.data_ptr())
        rx.process_device(iq.data_ptr(), nb, want.data_ptr())
        rx.synchronize()
    proc = d.fmrx_time_shard_fn(fmrx, 0, seed, 0)
    got = torch.cat([proc(d.shard(nb, 3, r)) for r in range(3)])
    assert torch.equal(got.cpu(), want.cpu())
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        with pytest.raises(RuntimeError):
            rx.seek(np.zeros(100, np.uint8))
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        rx.seek(np.full(64, 128, np.uint8))
        with pytest.raises(RuntimeError):
            rx.audio_block(np.zeros(640, np.float32))
        rx.process(np.full(12800, 128, np.uint8))
        rx.audio_block(np.zeros(640, np.float32))


def test_partial_block_dropped_and_empty(fmrx, orc):
    iq = iqgen.make("synth:55", 3 * 12800 + 5000)
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        assert rx.process(iq[:1000]).size == 0
        rx.reset()
        got = rx.process(iq)
    assert np.array_equal(got, orc.run(0, 51, iq, ["pcm_mono"])["pcm_mono"])


@pytest.mark.parametrize("name", [n for n in long_runs() if long_runs()[n]["mode"] in (0, 1)])
def test_mono_long_hash(fmrx, name):
    h = long_runs()[name]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    with fmrx.Receiver(h["mode"], fmrx.MONO, rf_taps=h["rf_taps"]) as rx:
        assert sha(rx.process(iq)) == h["pcm_mono_sha256"]


def test_full_size_1gib_windowed(fmrx, orc):
    """BASELINE config 2 at full size: 1 GiB of synthetic I/Q, 101-tap RF, mono.  The GPU
    generates the bytes; windows anywhere in the output are checked bit-exactly against the
    oracle run on that window's bytes (started one block early: finite filter memory)."""
    nbytes = 1 << 30
    bb, na = 12800, 128
    nb = nbytes // bb
    with fmrx.Receiver(0, fmrx.MONO, rf_taps=101) as rx:
        d_iq = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        d_pcm = torch.empty(nb * na, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        rx.synth_device(77, 0, nbytes // 2, d_iq.data_ptr())
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
        rx.synchronize()
        pcm = d_pcm.cpu().numpy()
        rng = np.random.default_rng(0)
        for b in [0, 1, 2, nb // 2, nb - 2, nb - 1] + list(rng.integers(1, nb - 1, 10)):
            b0 = max(0, int(b) - 1)
            win = d_iq[b0 * bb:(int(b) + 1) * bb].cpu().numpy()
            assert np.array_equal(win, iqgen.load_fmrx().synth_host(77, 2400000, b0 * bb // 2, win.size // 2))
            want = orc.run(0, 101, win, ["pcm_mono"])["pcm_mono"][(int(b) - b0) * na:]
            assert np.array_equal(pcm[int(b) * na:(int(b) + 1) * na], want), b


# ---- stereo engine (project.cpp output) -----------------------------------------------------

@pytest.mark.parametrize("name", STEREO_CASES)
def test_stereo_pcm_matches_reference(fmrx, name):
    z = load_case(name)
    iq = case_input(z)
    with fmrx.Receiver(z["mode"], fmrx.STEREO, rf_taps=z["rf_taps"]) as rx:
        nb = z["n_blocks"]
        d_iq = torch.from_numpy(iq).cuda()
        d_pcm = torch.zeros(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
        d_mono = torch.zeros(nb * rx.geo.audio_frames, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr(), d_mono.data_ptr())
        rx.synchronize()
        pcm = d_pcm.cpu().numpy()
        if "mono_exact" in z:
            assert same(d_mono.cpu().numpy(), z["mono_exact"]), "REF_EXACT mono differs"
    assert np.array_equal(pcm, z["pcm"]), name


@pytest.mark.parametrize("name", [n for n in STEREO_CASES if "demod" in load_case(n)])
def test_stereo_audio_block_from_reference_demod(fmrx, name):
    z = load_case(name)
    with fmrx.Receiver(z["mode"], fmrx.STEREO, rf_taps=z["rf_taps"]) as rx:
        pcm = rx.audio_block(z["demod"])
    assert np.array_equal(pcm, z["pcm"])


def test_stereo_call_split(fmrx, orc):
    nb, bb = 19, 12800
    iq = iqgen.make("synth:61", nb * bb)
    want = orc.run(0, 51, iq, ["pcm"])["pcm"]
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        parts, pos = [], 0
        for n in (1, 4, 2, 9, 3):
            parts.append(rx.process(iq[pos * bb:(pos + n) * bb]))
            pos += n
    assert np.array_equal(np.concatenate(parts), want)


def test_stereo_multistream(fmrx, orc):
    nb, bb = 9, 12800
    ins = [iqgen.make(f"synth:{70 + s}", nb * bb) for s in range(5)]
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=5) as rx:
        out = rx.process(np.stack(ins))
    for s, iq in enumerate(ins):
        assert np.array_equal(out[s], orc.run(0, 51, iq, ["pcm"])["pcm"]), s


@pytest.mark.parametrize("mode,n_streams,nb,chunks,lead", [(0, 5, 48, "3", 0), (0, 1, 64, "4", 0), (1, 3, 40, "2", 0),
                                                           (2, 2, 3, "2", 0), (0, 70, 120, None, 0),
                                                           (0, 5, 48, "4", 1), (0, 70, 120, None, 2),
                                                           (0, 70, 120, None, -1), (1, 3, 40, "2", -1),
                                                           (0, 70, 120, None, -2), (0, 5, 48, "4", -2),
                                                           (0, 70, 120, None, -3), (0, 70, 120, None, -4),
                                                           (0, 5, 48, "3", -4), (0, 5, 48, "2", -3)])
def test_stereo_pipelined_chunks(fmrx, orc, monkeypatch, mode, n_streams, nb, chunks, lead):
    """The pipelined stereo engine (api.cpp run_stereo_pipelined): a call's blocks in chunks,
    front end + band-pass of chunk k + 1 and audio of chunk k - 1 on their own HIP streams beside
    the PLL of chunk k, every chunk reading the call's buffers at its offset (a chunk's RF halo
    is the call's own bytes in front of it).  knob stereo_chunks forces the chunk count (None: the
    default, 8 from 16 streams, fewer when a chunk would hold < 2^14 samples); two calls in a row
    check the carried state.  Modes 0/1 take the tiled audio kernel, mode 2 the per-frame one.
    lead > 0: the paced schedule (chunk k's front end after chunk k - lead's PLL); lead <= 0: knob
    audio_defer = -lead (0 each chunk's audio beside the next PLL, 1 every chunk's after the last
    PLL, 2 all but the last chunk's beside the last PLL, 2 + e the first e of those beside the PLL
    before the last; e is clamped to K - 2, so 2 chunks with e = 1 is the plain 2 form)."""
    kw = {"stereo_lead": float(max(lead, 0)), "audio_defer": float(max(-lead, 0))}
    if chunks is not None:
        kw["stereo_chunks"] = float(chunks)
    knobs(monkeypatch, fmrx, **kw)
    bb = oracle.MODES[mode][0]
    rf_fs = oracle.MODES[mode][3]
    recipes = [("synth:%d" if s % 3 else "rand:%d") % (500 + s) for s in range(n_streams)]
    ins = np.stack([iqgen.make(r, 2 * nb * bb, rf_fs) for r in recipes])
    with fmrx.Receiver(mode, fmrx.STEREO, n_streams=n_streams) as rx:
        a = np.atleast_2d(rx.process(np.ascontiguousarray(ins[:, :nb * bb])))
        b = np.atleast_2d(rx.process(np.ascontiguousarray(ins[:, nb * bb:])))
    for s in sorted({0, n_streams // 2, n_streams - 1}):
        want = orc.run(mode, 51, ins[s], ["pcm"])["pcm"]
        assert np.array_equal(np.concatenate([a[s], b[s]]), want), s


@pytest.mark.parametrize("head,tail", [(8, 2), (2, 16), (16, 1)])
def test_stereo_pipelined_head_tail(fmrx, orc, monkeypatch, head, tail):
    """The pipelined engine's first and last chunk sizes (knobs stereo_head / stereo_tail, in 16ths
    of a middle chunk): 70 streams, the default 8 chunks, bit-exact against the oracle."""
    knobs(monkeypatch, fmrx, stereo_head=float(head), stereo_tail=float(tail))
    n_streams, nb, bb = 70, 120, 12800
    recipes = [("synth:%d" if s % 3 else "rand:%d") % (600 + s) for s in range(n_streams)]
    ins = np.stack([iqgen.make(r, nb * bb) for r in recipes])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=n_streams) as rx:
        out = np.atleast_2d(rx.process(ins))
    for s in (0, 35, 69):
        assert np.array_equal(out[s], orc.run(0, 51, ins[s], ["pcm"])["pcm"]), s


def test_stereo_pipelined_checkpoint_resume(fmrx, orc, monkeypatch):
    """The pipelined engine's carried state (demod history, PLL with its trigOffset hint, mixer
    tail, mono delay; api.cpp run_stereo_pipelined) through a checkpoint: 16 streams (the
    engine's default threshold) in pipelined calls, the blob into a second context, which goes
    on pipelined, bit-exact against the oracle on three streams."""
    knobs(monkeypatch, fmrx, stereo_chunks=3)
    ns, nb, bb = 16, 30, 12800
    iq = np.stack([iqgen.make(f"synth:{620 + k}", 2 * nb * bb) for k in range(ns)])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
        a = rx.process(np.ascontiguousarray(iq[:, :nb * bb]))
        blob = rx.get_state()
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx2:
        rx2.set_state(blob)
        b = rx2.process(np.ascontiguousarray(iq[:, nb * bb:]))
    for s in (0, 7, 15):
        want = orc.run(0, 51, iq[s], ["pcm"])["pcm"]
        assert np.array_equal(np.concatenate([a[s], b[s]]), want), s


@pytest.mark.parametrize("channels,n_streams", [(2, 70), (1, 130), (2, 1100), (2, 4200)])
def test_many_streams_cross_wave_boundaries(fmrx, orc, channels, n_streams):
    """Many streams of different content: the PLL runs one stream per wave until the streams
    outnumber the SIMDs (1,024 on MI355X), then two or four per wave with streams by 16-lane
    row (the split sin/cos form; 1,100 streams), and beyond 4 per wave lanes split by stream
    without it (4,200 streams: 8 per wave); the fused kernel's segments per stream shrink as
    streams grow."""
    nb, bb = 3, 12800
    recipes = [("synth:%d" if s % 3 else "rand:%d") % (200 + s) for s in range(n_streams)]
    ins = np.stack([iqgen.make(r, nb * bb) for r in recipes])
    with fmrx.Receiver(0, channels, n_streams=n_streams) as rx:
        out = rx.process(ins)
    field = "pcm" if channels == 2 else "pcm_mono"
    for s in sorted({0, 1, 63, 64, 65, n_streams // 2, n_streams // 2 + 1, n_streams - 2, n_streams - 1}):
        assert np.array_equal(out[s], orc.run(0, 51, ins[s], [field])[field]), s


@pytest.mark.parametrize("env", [{"pll_spec": "0"}, {"pll_inject": "0"},
                                 {"pll_inject": "7"}])
@pytest.mark.parametrize("n_streams,nb", [(1, 450), (6, 40), (1100, 2)])
def test_pll_speculation_fallbacks(fmrx, orc, monkeypatch, env, n_streams, nb):
    """The speculative PLL (stereo.hip pll_spec_kernel -> pll_check_kernel -> pll_kernel from
    the first batch that differs) equals the reference whatever the runner got wrong: with the
    test hook knob pll_inject=k the runner corrupts batch 1 + (k + s) % (nb - 1) of every
    stream s, so every stream resumes at its own batch (and a wave of several streams, at 1,100
    streams, at the earliest of them); knob pll_spec=0 is the plain certified launch.  450
    blocks cross the 2^18-sample segment boundary."""
    knobs(monkeypatch, fmrx, **{k: float(v) for k, v in env.items()})
    bb = 12800
    recipes = [("synth:%d" if s % 3 else "rand:%d") % (900 + s) for s in range(n_streams)]
    ins = np.stack([iqgen.make(r, nb * bb) for r in recipes])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=n_streams) as rx:
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        out = np.atleast_2d(rx.process(ins))
        rx.debug_pll_stats(None)
        if n_streams == 1:
            out2 = np.atleast_2d(rx.process(ins))  # a second call from the carried state
    resumed, checked = counts.cpu().tolist()
    if "pll_inject" in env:  # every stream's corrupted batch was caught and resumed
        assert checked > 0 and resumed >= n_streams, (resumed, checked)
    else:  # the plain launch: nothing speculative ran
        assert (resumed, checked) == (0, 0)
    for s in sorted({0, min(1, n_streams - 1), n_streams // 2, n_streams - 1}):
        assert np.array_equal(out[s], orc.run(0, 51, ins[s], ["pcm"])["pcm"]), s
    if n_streams == 1:
        want2 = orc.run(0, 51, np.concatenate([ins[0], ins[0]]), ["pcm"])["pcm"][nb * 512 // 2:]
        assert np.array_equal(out2[0], want2)


@pytest.mark.parametrize("skew", [4194304.0, 1048576.0, 16777216.0])
def test_pll_wrong_hint_fails_safe(fmrx, orc, monkeypatch, skew):
    """The host picks a segment's runners from its trigOffset bounds (api.cpp TrigTrack).  With
    the bounds deliberately wrong (test hook knob pll_hint_skew: the host believes the streams
    are `skew` samples further on), the runners launched leave the streams alone; the pre-pass's
    fail[] sentinel (0) then makes pll_kernel resume each such stream's whole segment on the
    certified path: slower, bit-identical (stats: every checked batch resumed)."""
    knobs(monkeypatch, fmrx, pll_hint_skew=skew)
    nb, bb, n_streams = 30, 12800, 3
    ins = np.stack([iqgen.make(f"synth:{950 + s}", nb * bb) for s in range(n_streams)])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=n_streams) as rx:
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        out = rx.process(ins)
        rx.debug_pll_stats(None)
    resumed, checked = counts.cpu().tolist()
    assert checked > 0 and resumed == checked, (resumed, checked)
    for s in range(n_streams):
        assert np.array_equal(out[s], orc.run(0, 51, ins[s], ["pcm"])["pcm"]), s


@pytest.mark.parametrize("name", sorted(long_runs()))
def test_stereo_long_hash(fmrx, name):
    h = long_runs()[name]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    with fmrx.Receiver(h["mode"], fmrx.STEREO, rf_taps=h["rf_taps"]) as rx:
        assert sha(rx.process(iq)) == h["pcm_sha256"]


def test_seam_calls_in_every_pll_regime(fmrx):
    """The per-block seam deep into a stream: the 72 s long run (past the 2^24 trigOffset stick)
    cut into long fused calls with runs of short calls between them, in every PLL regime --
    single blocks through fmrx_rf_block + fmrx_audio_block (project.cpp's thread split: 640
    steps a call, launch_pll's 16-step forms only) and 2-9-block fused calls (either side of
    kPllShortCall = 4,096 steps, the long forms' tails on the 16-step forms).  The whole PCM
    against the reference build's hash; the PLL state too."""
    h = long_runs()["m0_rf51_synth_72s"]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    nb = h["n_blocks"]
    iq = iqgen.make(h["recipe"], nb * bb, rf_fs)
    # block boundaries: runs of short calls at trigOffsets 2^17.., 2^19.., 2^20.., 2^21.., 2^22.., the stick
    runs = [(150, 12), (900, 12), (1700, 12), (3400, 12), (7000, 12), (26300, 12)]
    sizes = [1, 2, 3, 5, 6, 7, 9]
    parts, b = [], 0
    with fmrx.Receiver(h["mode"], fmrx.STEREO, rf_taps=h["rf_taps"]) as rx:
        for start, count in runs:
            parts.append(rx.process(iq[b * bb:start * bb]))
            b = start
            for k in range(count):
                m = sizes[k % len(sizes)]
                chunk = iq[b * bb:(b + m) * bb]
                parts.append(rx.audio_block(rx.rf_block(chunk)) if m == 1 else rx.process(chunk))
                b += m
        parts.append(rx.process(iq[b * bb:]))
        assert same(_pll_floats(rx), np.asarray(h["pll_state_last"], np.float32))
    assert sha(np.concatenate(parts)) == h["pcm_sha256"]


def test_seam_driver_native(fmrx):
    """bin/fmrx_seam (csrc/seam_bench.cpp): the per-block seam from C++ in project.cpp's call
    pattern, serially on one context and on two threads / two contexts with a depth-3 queue, from
    block 0 and from past the 2^22 trigOffset: the two legs' PCM are equal (exit 0) and the JSON
    line is well formed."""
    import json
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(fmrx.LIB_PATH), "bin", "fmrx_seam")
    for start in (0, 6600):
        r = subprocess.run([exe, "--blocks", "300", "--warmup", "10", "--start", str(start)], capture_output=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr.decode()[-400:]
        d = json.loads(r.stdout.decode())
        assert d["two_threads"]["pcm_equals_serial"] and d["start_block"] == start
        assert d["serial"]["x_realtime"] > 0 and d["two_threads"]["x_realtime"] > 0


def test_stereo_long_hash_three_streams(fmrx):
    """The saturated-segment runner (pll_sat.hip) with several waves: three copies of the 72 s
    long run in one 3-stream call, each stream's PCM against the reference build's hash."""
    h = long_runs()["m0_rf51_synth_72s"]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    with fmrx.Receiver(h["mode"], fmrx.STEREO, rf_taps=h["rf_taps"], n_streams=3) as rx:
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        out = rx.process(np.stack([iq, iq, iq]))
        rx.debug_pll_stats(None)
    for s in range(3):
        assert sha(out[s]) == h["pcm_sha256"], s
    resumed, checked = counts.cpu().tolist()
    assert checked > 0 and resumed <= checked // 10000, (resumed, checked)


def _stream_blob(multi: bytes, single_hdr: bytes, ns: int, s: int) -> bytes:
    """Stream s's slice of an n_streams state blob, as a 1-stream blob (api.cpp state_io order:
    halo, audio history, demod history, PLL, mixer tail, mono state)."""
    hdr = np.frombuffer(multi[:40], np.uint32)
    sizes = [int(hdr[6]), 4 * int(hdr[7]), 4 * 64, 4 * 8, 4 * 64, 4 * 8]
    out, off = [single_hdr[:40]], 40
    for z in sizes:
        out.append(multi[off + s * z: off + (s + 1) * z])
        off += ns * z
    assert off == len(multi)
    return b"".join(out)


def test_saturated_runner_wide_grid(fmrx):
    """pll_sat.hip on a grid of 4-wave workgroups (300 streams, one a wave): every stream's PLL
    is put at trigOffset 2^24 through the state blob, 40 blocks run in one call, and streams
    across the workgroups are compared with the same stream alone in a 1-stream context (whose
    saturated runner the long-run hashes pin to the reference build)."""
    ns, nb, bb = 300, 40, 12800
    ins = np.stack([iqgen.make("synth:%d" % (600 + s % 7), (nb + 2) * bb) for s in range(ns)])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
        rx.process(ins[:, : 2 * bb])  # a state to start from
        blob = bytearray(rx.get_state())
        hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
        pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
        pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
        pll[:, 5] = 16777216.0
        blob[pll_off: pll_off + ns * 32] = pll.tobytes()
        rx.set_state(bytes(blob))
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        out = rx.process(ins[:, 2 * bb:])
        rx.debug_pll_stats(None)
    resumed, checked = counts.cpu().tolist()
    assert checked > 0 and resumed == 0, (resumed, checked)
    for s in (0, 1, 63, 64, 255, 256, 299):
        with fmrx.Receiver(0, fmrx.STEREO) as r1:
            r1.process(ins[s, : 2 * bb])
            r1.set_state(_stream_blob(bytes(blob), r1.get_state(), ns, s))
            assert np.array_equal(r1.process(ins[s, 2 * bb:]), out[s]), s


def _unlocked_input(rx, h):
    """A fixture's input on the device: the synth recipes generated there (identical bytes),
    random bytes uploaded."""
    n = h["n_blocks"] * rx.geo.block_bytes
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    kind, _, arg = h["recipe"].partition(":")
    if kind in iqgen.SYNTH_FLAGS:
        rx.synth_device(int(arg) | iqgen.SYNTH_FLAGS[kind], 0, n // 2, d.data_ptr())
        rx.synchronize()
    else:
        d.copy_(torch.from_numpy(iqgen.make(h["recipe"], n, rx.geo.rf_fs)))
    assert sha(d.cpu().numpy()) == h["input_sha256"]
    return d


def _pll_floats(rx):
    """A 1-stream context's PLL state {integrator, phaseEst, fbI, fbQ, ncoOut_state, trigOffset}
    from its state blob (api.cpp state_io order: halo, audio history, demod history, PLL)."""
    blob = rx.get_state()
    hdr = np.frombuffer(blob[:40], np.uint32)
    off = 40 + int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64
    return np.frombuffer(blob[off: off + 24], np.float32)


@pytest.mark.parametrize("name", sorted(unlocked_runs()))
def test_unlocked_pll_long_hash(fmrx, name):
    """The PLL where it never locks or slips cycles (filter.cpp:157-171; random bytes, no pilot,
    heavy noise, mode 2's PLL handed the upsampled if_fs, project.cpp:166,348), 17-19 M steps
    each, through every runner form and the trigOffset stick: one device-resident call, the PCM
    and the final PLL state against the reference build's."""
    h = unlocked_runs()[name]
    with fmrx.Receiver(h["mode"], fmrx.STEREO, rf_taps=h["rf_taps"]) as rx:
        d_iq = _unlocked_input(rx, h)
        d_pcm = torch.empty(h["n_blocks"] * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
        redos = torch.zeros(fmrx.REDO_SLOTS, dtype=torch.int32, device="cuda")
        rx.debug_pll_redos(redos.data_ptr())
        rx.process_device(d_iq.data_ptr(), h["n_blocks"], d_pcm.data_ptr())
        rx.synchronize()
        rx.debug_pll_redos(None)
        assert sha(d_pcm.cpu().numpy()) == h["pcm_sha256"], name
        assert same(_pll_floats(rx), np.asarray(h["pll_state_last"], np.float32))
    # every one of these streams misses most intervals somewhere: demoted there
    assert redos.cpu().numpy()[4:].sum() > 0, redos.cpu().numpy()


@pytest.mark.parametrize("name", [n for n in long_runs() if long_runs()[n]["mode"] in (2, 3)])
def test_polyphase_mono_long_hash(fmrx, name):
    h = long_runs()[name]
    bb, rf_fs = oracle.MODES[h["mode"]][0], oracle.MODES[h["mode"]][3]
    iq = iqgen.make(h["recipe"], h["n_blocks"] * bb, rf_fs)
    with fmrx.Receiver(h["mode"], fmrx.MONO, rf_taps=h["rf_taps"]) as rx:
        assert sha(rx.process(iq)) == h["pcm_mono_sha256"]


@pytest.mark.parametrize("name", sorted(bench_runs()))
def test_bench_config_full_size_hash(fmrx, name):
    """BASELINE configs[2] (mode-0 stereo, ONE 1 GiB stream: 223.7 s of signal, two thirds of
    it past the PLL's trigOffset saturation, project.cpp:132-196 / filter.cpp:136-174) and
    configs[3] (mode-2 mono, 1 GiB) at full size on exactly bench.py's device-generated input,
    against the reference build's PCM hash of the same bytes."""
    h = bench_runs()[name]
    bb = oracle.MODES[h["mode"]][0]
    nb = h["n_blocks"]
    with fmrx.Receiver(h["mode"], h["channels"], rf_taps=h["rf_taps"]) as rx:
        d_iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
        d_pcm = torch.empty(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        rx.synth_device(int(h["recipe"][6:]), 0, nb * bb // 2, d_iq.data_ptr())
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
        rx.synchronize()
        assert sha(d_iq.cpu().numpy()) == h["input_sha256"]
        assert sha(d_pcm.cpu().numpy()) == h["pcm_sha256"], name


# ---- filter.h primitives --------------------------------------------------------------------

def _d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_primitives(fmrx, taps_golden):
    g = taps_golden
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        c = _d(g["rf_m0_51"])
        for up, down in ((1, 10), (1, 1), (3, 7)):
            x, st = _d(g["resample_in"]), _d(g["resample_state"])
            out = torch.zeros(1000 * up // down, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            n = rx.resample(out.data_ptr(), st.data_ptr(), x.data_ptr(), 1000, c.data_ptr(), 51, up, down)
            rx.synchronize()
            assert n == out.numel()
            assert same(out.cpu().numpy(), g[f"resample_{up}_{down}_out"])
            assert same(st.cpu().numpy(), g[f"resample_{up}_{down}_state"])
        i, q, prev = _d(g["demod_i"]), _d(g["demod_q"]), _d(np.array([0.25, -0.5], np.float32))
        out = torch.zeros(600, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.fm_demod(out.data_ptr(), prev.data_ptr(), i.data_ptr(), q.data_ptr(), 600)
        rx.synchronize()
        assert same(out.cpu().numpy(), g["demod_out"]) and same(prev.cpu().numpy(), g["demod_prev"])
        io, st = _d(g["pll_in"]), _d(np.array([0, 0, 1, 0, 1, 0], np.float32))
        torch.cuda.synchronize()
        rx.pll(io.data_ptr(), io.numel(), 19000, 240000, 2, 0, 0.01, st.data_ptr())
        rx.synchronize()
        assert same(io.cpu().numpy(), g["pll_out"]) and same(st.cpu().numpy(), g["pll_state"])
        b = _d(g["norm_in"])
        fi = torch.zeros(256, dtype=torch.float32, device="cuda")
        fq = torch.zeros(256, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.normalize_iq(b.data_ptr(), 256, fi.data_ptr(), fq.data_ptr())
        rx.synchronize()
        assert same(fi.cpu().numpy(), g["norm_out"][0::2]) and same(fq.cpu().numpy(), g["norm_out"][1::2])


@pytest.mark.parametrize("trig,phase,freq,fs,n,offset", [
    (0.0, 0.0, 19000, 240000, 4103, 0),              # n % 16 != 0: exact tail
    (16777200.0, 0.25, 19000, 240000, 700, 0),       # trigOffset sticks at 2^24 inside a batch
    (16777216.0, 0.3, 19000, 240000, 6000, 0),       # stuck from the start: the runner's sin/cos skipping
    (0.5, 0.0, 19000, 240000, 300, 0),               # non-integer trigOffset: exact path only
    (3.0e7, 0.0, 19000, 240000, 300, 0),             # past 2^24: exact path only
    (0.0, 6.0e8, 19000, 240000, 300, 0),             # |phaseEst| beyond the batch's range check
    (131072.0, 6.0e8, 19000, 240000, 20000, 0),      # the same in the index runner's range: every
                                                     # interval redone, then the stream demoted
    (0.0, 0.0, 114000, 240000, 2000, 0),             # RDS's 114 kHz loop
    (0.0, 0.0, 19000, 35280000, 2000, 0),            # mode 2's upsampled fs (project.cpp:166)
    (0.0, 0.0, 19000, 240000, 1000, 1),              # unaligned samples: exact path only
])
def test_pll_primitive_states(fmrx, orc, trig, phase, freq, fs, n, offset):
    """fmrx_pll (filter.cpp:136-174) from states the optimistic batches must refuse or handle
    at their edges (trigOffset saturation, non-integer or huge trigOffset, huge phase, tails,
    unaligned input), against the oracle's PLL on the same state."""
    rng = np.random.default_rng(int(trig) + n)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * freq / fs * t + 0.3) + 0.01 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([1e-4, phase, 0.6, 0.8, 1.0, trig], np.float32)
    want_x, want_st = orc.pll(x, freq, fs, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(np.concatenate([np.zeros(offset, np.float32), x]))
        st = _d(st0)
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr() + 4 * offset, n, freq, fs, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        assert same(buf.cpu().numpy()[offset:], want_x)
        assert same(st.cpu().numpy(), want_st)


@pytest.mark.parametrize("freq,nco_scale", [(19000, 2.0), (114000, 0.5)])  # pilot (project.cpp:166), RDS (:226)
@pytest.mark.parametrize("inject", [None, "3"])
@pytest.mark.parametrize("sat,pipe", [("1", "1"), ("1", "0"), ("0", "0")])
def test_pll_saturated_runner(fmrx, orc, monkeypatch, inject, sat, pipe, freq, nco_scale):
    """A segment that starts with trigOffset stuck at 2^24 (filter.cpp:165-166 in float, 69.9 s
    into a stream): the three-wave runner (pll_pred.hip pll_pipe_kernel, which takes one stream
    a workgroup), with it off the saturated-segment runner (pll_sat.hip), with both off the
    two-wave predicted runner; and a corrupted runner batch (check + certified resume).  The
    speculation counters must show every batch verified without the corruption -- a runner
    that disagrees with the exact path would otherwise pass here, fixed up by the resume."""
    knobs(monkeypatch, fmrx, pll_sat=float(sat))
    knobs(monkeypatch, fmrx, pll_pipe=float(pipe))
    if inject is not None:
        knobs(monkeypatch, fmrx, pll_inject=float(inject))
    n = 20000
    rng = np.random.default_rng(24)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * freq / 240000 * t + 0.3) + 0.01 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([2e-4, 1.7, 0.6, 0.8, 1.0, 16777216.0], np.float32)
    want_x, want_st = orc.pll(x, freq, 240000, nco_scale, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, freq, 240000, nco_scale, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        assert checked == n // 16
        assert (resumed > 0) if inject is not None else (resumed == 0), (resumed, checked)


@pytest.mark.parametrize("trig0", [1048576.0, 2097185.0, 4194204.0, 4194321.0, 16772216.0, 1048575.0])
@pytest.mark.parametrize("inject", [None, "5"])
@pytest.mark.parametrize("pred,pipe", [("1", "1"), ("1", "0"), ("0", "0")])
def test_pll_predicted_runner(fmrx, orc, monkeypatch, trig0, inject, pred, pipe):
    """Segments from trigOffset 2^20 up to the 2^24 stick: the predicted-trigArg runners
    (pll_pred.hip: three waves one stream a workgroup -- five candidates in 16-step intervals from
    2^20, in 64-step ones from 2^21, three candidates from 2^22; knob pll_pipe=0: the two-wave
    runner throughout; knob pll_pred=0: the lane runner), starting at 2^20, at 2^21 + 33, 100 steps
    below 2^22 (its form runs on past it), at 2^22 + 17, and 5,000 steps below the stick (its pr
    stops rising inside the segment); 2^20 - 1 runs its first step on the index runner's
    [2^19, 2^20) form (pll_idx_kernel; the lane runner with knob pll_pipe=0).  A corrupted batch
    must be caught and resumed; without it every batch verifies."""
    knobs(monkeypatch, fmrx, pll_pred=float(pred))
    knobs(monkeypatch, fmrx, pll_pipe=float(pipe))
    if inject is not None:
        knobs(monkeypatch, fmrx, pll_inject=float(inject))
    n = 20000
    rng = np.random.default_rng(int(trig0) % 1000)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.7) + 0.02 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([-3e-4, -0.9, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        # each launch counts its whole batches: a range split at a form's edge loses one
        assert n // 16 - 1 <= checked <= n // 16, checked
        assert (resumed > 0) if inject is not None else (resumed == 0), (resumed, checked)


@pytest.mark.parametrize("trig0", [1048600.0, 2097185.0, 4194321.0, 16772216.0, 16777216.0])
@pytest.mark.parametrize("miss", ["1", "2", "77", "155", "156", "311", "312", "1248", "5000"])
@pytest.mark.parametrize("stick", [1, 0])
def test_pll_pipe_redo(fmrx, orc, monkeypatch, trig0, miss, stick):
    """The three-wave runner's miss path (pll_pipe_kernel): knob pll_pipe_miss=k makes its check
    report interval k as missed (past the last interval: the last), so the chain redoes that
    interval and the two after it exactly and the evaluators restart from the corrected phase.
    20,000 steps = batch 0 + 156 intervals of 128 steps + 1 batch from 2^21 (k = 1, 77, 155 and
    156: the first, a middle one and the verdicts read after the loop; larger k: the last), and in
    [2^20, 2^21) the count runner's 128-step intervals or, with pll_cnt = 0, the 16-step form's
    1,249 (1,248 and 1,249 the last two).  From the stuck trigOffset 2^24
    (and 5,000 steps before it: the handover inside the call) the stick form (knob pll_stick = 1:
    the interval's two thresholds once, three e a step) or the plain three-candidate form (0).
    Bit-exact, every batch verifies."""
    knobs(monkeypatch, fmrx, pll_pipe_miss=float(miss), pll_stick=stick)
    n = 20000
    rng = np.random.default_rng(int(trig0) % 977)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.2) + 0.005 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([1e-4, 0.4, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        # each launch counts its whole batches: a range split at a form's edge (the stick) loses one
        assert n // 16 - 1 <= checked <= n // 16 and resumed == 0, (resumed, checked)


@pytest.mark.parametrize("trig0", [131072.0, 262177.0, 524188.0, 600000.0, 1043576.0, 125000.0])
@pytest.mark.parametrize("inject", [None, "5"])
@pytest.mark.parametrize("idx", ["1", "0", "2", None])
def test_pll_index_runner(fmrx, orc, monkeypatch, trig0, inject, idx):
    """trigOffset in [2^17, 2^20): the index runner (pll_pred.hip pll_idx_kernel: the chain forms
    trigArg itself and reads its e from a lane of a candidate row -- 32 candidates from 2^17 and
    from 2^18, 16 from 2^19; knob pll_idx=1: from 2^18 only, the lane runner below), starting at
    2^17 (the default, knob pll_idx=2 or unset, starts there; with 1 the lane runner hands over at
    2^18), at 2^18 + 33, 100 steps below 2^19 (the 2^18 form hands over to the 2^19 one
    inside the call), at 600,000, and 5,000 steps below 2^20 (the three-wave runner takes over);
    125,000 starts on the lane runner and crosses into it.  knob pll_idx=0: the lane runner below
    2^20.  Bit-exact against the oracle; a forced miss
    (knob pll_inject) is redone exactly, and without it no batch is."""
    if idx is None:
        knobs(monkeypatch, fmrx, pll_idx=2)
    else:
        knobs(monkeypatch, fmrx, pll_idx=float(idx))
    if inject is not None:
        knobs(monkeypatch, fmrx, pll_inject=float(inject))
    n = 20000
    rng = np.random.default_rng(int(trig0) % 1009)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.4) + 0.02 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([2e-4, 0.8, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        assert n // 16 - 2 <= checked <= n // 16, checked
        assert (resumed > 0) if inject is not None else (resumed == 0), (resumed, checked)


@pytest.mark.parametrize("trig0", [131072.0, 262177.0, 524188.0, 700000.0, 1048500.0, 1048576.0, 1500000.0,
                                   2097100.0, 3000000.0])
@pytest.mark.parametrize("hook", [None, ("pll_inject", 5), ("pll_pipe_miss", 1), ("pll_pipe_miss", 300)])
@pytest.mark.parametrize("cnt", [31, 0])
def test_pll_count_runner(fmrx, orc, monkeypatch, trig0, hook, cnt):
    """trigOffset in [2^17, 2^22) on the count runner (pll_pred.hip pll_cnt_kernel: one compare
    of the phase against a row of exact thresholds and a bit count pick each step's e; knob
    pll_cnt = 31: every form from 2^17 to 2^22 on it, 0: none -- the index and three-wave runners),
    starting at each form's edge, just below the next edge (the call crosses into the next form)
    and inside; with a forced miss (pll_inject: counted as resumed; pll_pipe_miss k: interval k
    redone, k past the last: the last) the interval is redone exactly.  Bit-exact against the
    oracle, state included."""
    knobs(monkeypatch, fmrx, pll_cnt=cnt)
    if hook is not None:
        knobs(monkeypatch, fmrx, **{hook[0]: hook[1]})
    n = 20000
    rng = np.random.default_rng(int(trig0) % 991)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.9) + 0.02 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([1.5e-4, -0.3, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        assert n // 16 - 2 <= checked <= n // 16, checked
        if hook is not None and hook[0] == "pll_inject":
            assert resumed > 0, (resumed, checked)


@pytest.mark.parametrize("trig0", [131100.0, 300000.0, 700000.0])
@pytest.mark.parametrize("miss", ["1", "2", "600", "1248", "1249", "5000"])
def test_pll_index_redo(fmrx, orc, monkeypatch, trig0, miss):
    """The index runner's miss path: knob pll_pipe_miss=k makes its check report interval k as
    missed (past the last: the last), so the chain redoes it and the two after it exactly and the
    evaluators restart from the corrected phase.  20,000 steps = interval 0 + 1,249 intervals of
    16 steps + a tail (1,248 and 1,249: the verdicts read after the loop).  Bit-exact."""
    knobs(monkeypatch, fmrx, pll_pipe_miss=float(miss))
    n = 20000
    rng = np.random.default_rng(int(trig0) % 983)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.2) + 0.005 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([1e-4, 0.4, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
        resumed, checked = counts.cpu().tolist()
        assert checked == n // 16 and resumed == 0, (resumed, checked)


def test_index_runner_streams(fmrx, monkeypatch):
    """pll_idx_kernel over many streams (200: four waves each still fit the SIMDs), every stream
    put at trigOffset 2^18 - 4,000 through the state blob (the runners need the streams at one
    known trigOffset: the 2^17 form hands over to the 2^18 one inside the call; knob pll_idx=1:
    the lane runner to 2^18), 24 blocks in one call: the PCM equals the same call with the index
    runner off (knob pll_idx=0: the lane runner, checked by pll_check_kernel), and no batch is
    redone."""
    ns, nb, bb = 200, 24, 12800
    ins = np.stack([iqgen.make("synth:%d" % (700 + s % 5), (nb + 2) * bb) for s in range(ns)])
    outs = []
    for idx in ("2", "1", "0"):
        knobs(monkeypatch, fmrx, pll_idx=float(idx))
        with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
            rx.process(ins[:, : 2 * bb])
            blob = bytearray(rx.get_state())
            hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
            pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
            pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
            pll[:, 5] = 262144.0 - 4000.0
            blob[pll_off: pll_off + ns * 32] = pll.tobytes()
            rx.set_state(bytes(blob))
            counts = torch.zeros(2, dtype=torch.int64, device="cuda")
            rx.debug_pll_stats(counts.data_ptr())
            outs.append(rx.process(ins[:, 2 * bb:]))
            rx.debug_pll_stats(None)
        resumed, checked = counts.cpu().tolist()
        assert checked > 0 and resumed == 0, (idx, resumed, checked)
    assert np.array_equal(outs[0], outs[2]) and np.array_equal(outs[1], outs[2])


def test_count_runner_streams(fmrx, monkeypatch):
    """pll_cnt_kernel over many streams (200: a CU each still fits), every stream put at trigOffset
    2^20 - 10,000 through the state blob (the [2^19, 2^20) form hands over to the [2^20, 2^21) one
    inside the call), 24 blocks in one call: the PCM equals the same call with the count runner off
    (knob pll_cnt = 0: the index runner and the three-wave runner's 16-step form), and no batch is
    redone on the inject hook's account."""
    ns, nb, bb = 200, 24, 12800
    ins = np.stack([iqgen.make("synth:%d" % (740 + s % 5), (nb + 2) * bb) for s in range(ns)])
    outs = []
    for cnt in (12, 0):
        knobs(monkeypatch, fmrx, pll_cnt=cnt)
        with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
            rx.process(ins[:, : 2 * bb])
            blob = bytearray(rx.get_state())
            hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
            pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
            pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
            pll[:, 5] = 1048576.0 - 10000.0
            blob[pll_off: pll_off + ns * 32] = pll.tobytes()
            rx.set_state(bytes(blob))
            counts = torch.zeros(2, dtype=torch.int64, device="cuda")
            redos = torch.zeros((ns, fmrx.REDO_SLOTS), dtype=torch.int32, device="cuda")
            rx.debug_pll_stats(counts.data_ptr())
            rx.debug_pll_redos(redos.data_ptr())
            outs.append(rx.process(ins[:, 2 * bb:]))
            rx.debug_pll_stats(None)
            rx.debug_pll_redos(None)
        resumed, checked = counts.cpu().tolist()
        assert checked > 0 and resumed == 0, (cnt, resumed, checked)
        r = redos.cpu().numpy()
        # locked streams: no demotion, and nothing below 2^19 or past 2^21 in this range
        assert not r[:, 4:].any() and not r[:, 2:4].any(), r.sum(axis=0)
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("trig0,slots", [(4194304.0 - 6000.0, (2, 3)), (1048576.0 - 3000.0, (0, 1)),
                                         (300000.0, (0,))])
def test_pll_redo_slots(fmrx, monkeypatch, trig0, slots):
    """fmrx_debug_pll_redos files each runner launch's redone intervals by its trigOffset range
    (fmrx.REDO_RANGES): 4 streams put at trig0 through the state blob run 24 blocks (15,360 steps)
    with knob pll_pipe_miss = 3 (interval 3 of every launch reported missed) and without.  Hooked:
    every stream has at least one redo in each range the call crosses (`slots`); every slot of a
    range it does not cross is zero, hooked or not (redos and demoted steps); the PCM is
    identical."""
    ns, nb, bb = 4, 24, 12800
    ins = np.stack([iqgen.make("synth:%d" % (760 + s), (nb + 2) * bb) for s in range(ns)])
    res = {}
    for hook in (None, 3):
        knobs(monkeypatch, fmrx, pll_pipe_miss=-1 if hook is None else hook)
        with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
            rx.process(ins[:, : 2 * bb])
            blob = bytearray(rx.get_state())
            hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
            pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
            pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
            pll[:, 5] = trig0
            blob[pll_off: pll_off + ns * 32] = pll.tobytes()
            rx.set_state(bytes(blob))
            redos = torch.zeros((ns, fmrx.REDO_SLOTS), dtype=torch.int32, device="cuda")
            rx.debug_pll_redos(redos.data_ptr())
            out = rx.process(ins[:, 2 * bb:])
            rx.debug_pll_redos(None)
        res[hook] = (out, redos.cpu().numpy())
    (o0, r0), (o1, r1) = res[None], res[3]
    assert np.array_equal(o0, o1)
    # (the PLL state put out of its loop's lock makes some streams miss most intervals for a while:
    # those demote, with their demoted steps in the same range's slot)
    for sl in range(4):
        if sl in slots:
            assert (r1[:, sl] >= 1).all(), (sl, r0[:, sl], r1[:, sl])
        else:
            for r in (r0, r1):
                assert not r[:, sl].any() and not r[:, 4 + sl].any(), (sl, r0, r1)


@pytest.mark.parametrize("trig0", [131100.0, 300000.0, 700000.0, 1500000.0, 3000000.0, 6000000.0, 16770000.0,
                                   16777216.0])
@pytest.mark.parametrize("miss", [-2, -40])
@pytest.mark.parametrize("cnt", [12, 0])
@pytest.mark.parametrize("inject", [None, 3])
def test_pll_demotion(fmrx, orc, monkeypatch, trig0, miss, cnt, inject):
    """A stream whose intervals keep missing (an unlocked loop; forced here by knob pll_pipe_miss
    = -k: every interval from k - 1 on) is demoted by each self-certifying runner once 24 of its
    last 32 intervals missed: the rest of the launch's range runs on the exact path
    (pll_run_fast).  20,000 steps from each form's range (index 2^17 / 2^18, count or index 2^19,
    count or 16-step three-wave 2^20, five-candidate 2^21, three-candidate 2^22, the stick's
    handover and the stick): bit-exact against the oracle, state included, and the demoted steps
    filed in the range's slot.  pll_inject: the runners and the demoted stream's chain (pll_demote.hip)
    each corrupt one batch -- the checkers catch it, the chain recomputes from there (resumed)."""
    knobs(monkeypatch, fmrx, pll_pipe_miss=miss, pll_cnt=cnt)
    if inject is not None:
        knobs(monkeypatch, fmrx, pll_inject=inject)
    n = 20000
    rng = np.random.default_rng(int(trig0) % 997)
    t = np.arange(n)
    x = (0.1 * np.cos(2 * np.pi * 19000 / 240000 * t + 0.3) + 0.02 * rng.standard_normal(n)).astype(np.float32)
    st0 = np.array([1e-4, 0.4, 0.6, 0.8, 1.0, trig0], np.float32)
    want_x, want_st = orc.pll(x, 19000, 240000, 2.0, 0.0, 0.01, st0)
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        buf = _d(x)
        st = _d(st0)
        redos = torch.zeros(fmrx.REDO_SLOTS, dtype=torch.int32, device="cuda")
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_redos(redos.data_ptr())
        rx.debug_pll_stats(counts.data_ptr())
        torch.cuda.synchronize()
        rx.pll(buf.data_ptr(), n, 19000, 240000, 2.0, 0.0, 0.01, st.data_ptr())
        rx.synchronize()
        rx.debug_pll_redos(None)
        rx.debug_pll_stats(None)
        assert same(buf.cpu().numpy(), want_x)
        assert same(st.cpu().numpy(), want_st)
    r = redos.cpu().numpy()
    # (from interval 39 on, a short launch may end before 24 misses; a launch under 64 intervals
    # never demotes -- the stick handover's 7,216- and 12,784-step ranges of 256-step intervals)
    if miss == -2 and trig0 != 16770000.0:
        assert r[4:].sum() > 0, r
        if inject is not None:
            assert counts.cpu().tolist()[0] > 0


@pytest.mark.parametrize("mixed", [False, True])
def test_pipe_runner_streams(fmrx, monkeypatch, mixed):
    """pll_pipe_kernel over many streams (300: three waves each still fit the SIMDs), every
    stream put at trigOffset 2^22 - 6,000 through the state blob (the runners need the streams at
    one known trigOffset: the 2^21 form hands over to the 2^22 one inside the call), 24 blocks in
    one call: every batch verifies, and the PCM equals the same call with the three-wave runner
    off (knob pll_pipe=0: the two-wave runner, checked by pll_check_kernel).  mixed: the streams
    at three trigOffsets (2^22 / 2^21 / 2^20 + k, as a set_state or seek can leave them), so the
    host's bounds differ and the segment runners (two-wave, saturated, lane) take them, checked."""
    ns, nb, bb = 300, 24, 12800
    ins = np.stack([iqgen.make("synth:%d" % (900 + s % 7), (nb + 2) * bb) for s in range(ns)])
    outs = []
    for pipe in ("1", "0"):
        knobs(monkeypatch, fmrx, pll_pipe=float(pipe))
        with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
            rx.process(ins[:, : 2 * bb])
            blob = bytearray(rx.get_state())
            hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
            pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
            pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
            if mixed:
                pll[:, 5] = np.array([(4194304.0, 2097152.0, 1048576.0)[k % 3] + k for k in range(ns)], np.float32)
            else:
                pll[:, 5] = 4194304.0 - 6000.0
            blob[pll_off: pll_off + ns * 32] = pll.tobytes()
            rx.set_state(bytes(blob))
            counts = torch.zeros(2, dtype=torch.int64, device="cuda")
            rx.debug_pll_stats(counts.data_ptr())
            outs.append(rx.process(ins[:, 2 * bb:]))
            rx.debug_pll_stats(None)
        resumed, checked = counts.cpu().tolist()
        assert checked > 0 and resumed == 0, (pipe, resumed, checked)
    assert np.array_equal(outs[0], outs[1])


def test_predicted_runner_rows(fmrx, monkeypatch):
    """pll_pred.hip with two streams a wave (1,100 streams: 16-lane rows; knob pll_pred=2 launches
    it although its 550 two-wave groups would share SIMDs, where the host leaves such counts to
    the lane runner), every stream put at its own trigOffset in [2^21, 2^21 + 1100) through the
    state blob -- except stream 5, at 1,000, which sends its wave (streams 4 and 5) to the lane
    runner -- 40 blocks in one call, every batch verified, and streams on both sides compared
    with the same stream alone."""
    knobs(monkeypatch, fmrx, pll_pred=2)
    ns, nb, bb = 1100, 40, 12800
    ins = np.stack([iqgen.make("synth:%d" % (700 + s % 5), (nb + 2) * bb) for s in range(ns)])
    with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns) as rx:
        rx.process(ins[:, : 2 * bb])
        blob = bytearray(rx.get_state())
        hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
        pll_off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
        pll = np.frombuffer(bytes(blob[pll_off: pll_off + ns * 32]), np.float32).reshape(ns, 8).copy()
        pll[:, 5] = 2097152.0 + np.arange(ns, dtype=np.float32)
        pll[5, 5] = 1000.0
        blob[pll_off: pll_off + ns * 32] = pll.tobytes()
        rx.set_state(bytes(blob))
        counts = torch.zeros(2, dtype=torch.int64, device="cuda")
        rx.debug_pll_stats(counts.data_ptr())
        out = rx.process(ins[:, 2 * bb:])
        rx.debug_pll_stats(None)
    resumed, checked = counts.cpu().tolist()
    assert checked > 0 and resumed == 0, (resumed, checked)
    for s in (0, 4, 5, 6, 1023, 1099):
        with fmrx.Receiver(0, fmrx.STEREO) as r1:
            r1.process(ins[s, : 2 * bb])
            r1.set_state(_stream_blob(bytes(blob), r1.get_state(), ns, s))
            assert np.array_equal(r1.process(ins[s, 2 * bb:]), out[s]), s


def test_quantize_and_elementwise(fmrx, orc):
    x = np.array([0, 1, -1, 1.99993896484375, 2, -2, 2.5, 1e6, -1e6, 1.4e5, np.inf, -np.inf, np.nan,
                  131071.99, -131072, 3.05e-5] * 4, np.float32)
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        dx = _d(x)
        dq = torch.zeros(x.size, dtype=torch.int16, device="cuda")
        a, b = _d(x[::-1].copy()), _d(np.nan_to_num(x))
        mix = torch.zeros(x.size, dtype=torch.float32, device="cuda")
        l = torch.zeros_like(mix)
        r = torch.zeros_like(mix)
        torch.cuda.synchronize()
        rx.quantize(dx.data_ptr(), x.size, dq.data_ptr())
        rx.mixer(mix.data_ptr(), a.data_ptr(), b.data_ptr(), x.size)
        rx.lr_extraction(l.data_ptr(), r.data_ptr(), a.data_ptr(), b.data_ptr(), x.size)
        rx.synchronize()
    assert np.array_equal(dq.cpu().numpy(), orc.quant(x))
    xa, xb = x[::-1].copy(), np.nan_to_num(x)
    assert same(mix.cpu().numpy(), orc.mixer(xa, xb))
    want_l, want_r = orc.lr(xa, xb)
    assert same(l.cpu().numpy(), want_l)
    assert same(r.cpu().numpy(), want_r)


def test_device_synth_equals_host(fmrx):
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        d = torch.empty(2 * 300001, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        rx.synth_device(9, 123456, 300001, d.data_ptr())
        rx.synchronize()
        assert np.array_equal(d.cpu().numpy(), fmrx.synth_host(9, 2400000, 123456, 300001))
        # several streams in one launch (configs[4]'s per-rank input), rows with a gap between
        seeds, n, stride = [5, 300, 7, 2**40 + 3, 62 | 1 << 56, 63 | 6 << 57], 70001, 2 * 70001 + 6
        m = torch.full((len(seeds) * stride,), 0xAB, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        rx.synth_device_streams(seeds, 999, n, m.data_ptr(), stride)
        rows = m.cpu().numpy()
        for k, sd in enumerate(seeds):
            assert np.array_equal(rows[k * stride:k * stride + 2 * n], fmrx.synth_host(sd, 2400000, 999, n)), sd
            assert (rows[k * stride + 2 * n:(k + 1) * stride] == 0xAB).all()  # nothing past the row


# ---- the PLL's fallback libm (refused arguments) against glibc ---------------------------------

def test_pll_fallback_matches_glibc(fmrx):
    """Where the PLL's certified fast paths refuse, the device falls back to csrc/pll_cr.h; its
    floats must equal glibc's (filter.cpp:161,168-170) on every refusable argument of the fixture
    (all hard sin/cos arguments |x| < 1e9 and a sample beyond, hard atan2 pairs)."""
    import os

    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "pll_fallback.npz"))
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        x = torch.from_numpy(z["sincos_x"]).cuda()
        out = torch.empty(2 * x.numel(), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.test_pll_fallback(0, x.data_ptr(), None, x.numel(), out.data_ptr())
        rx.synchronize()
        got = out.cpu().numpy().reshape(-1, 2)
        assert same(got[:, 0], z["sincos_s"]) and same(got[:, 1], z["sincos_c"])
        nco = torch.empty(x.numel(), dtype=torch.float32, device="cuda")
        rx.test_pll_fallback(2, x.data_ptr(), None, x.numel(), nco.data_ptr())
        rx.synchronize()
        assert same(nco.cpu().numpy(), z["sincos_c"])
        y, xx = torch.from_numpy(z["atan2_y"]).cuda(), torch.from_numpy(z["atan2_x"]).cuda()
        e = torch.empty(y.numel(), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rx.test_pll_fallback(1, y.data_ptr(), xx.data_ptr(), y.numel(), e.data_ptr())
        rx.synchronize()
        assert same(e.cpu().numpy(), z["atan2_e"])


# ---- the `project` drop-in CLI (stdin u8 -> stdout S16) --------------------------------------

def _cli(fmrx, args, data, timeout=300):
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(fmrx.LIB_PATH), "bin", "fmrx")
    r = subprocess.run([exe] + [str(a) for a in args], input=data, capture_output=True, timeout=timeout)
    return r


# project.cpp:179-195 writes the 2-channel R,L stream whatever `channels` is (it is only logged,
# :301-302), and fewer than two arguments select the default mode 0 (:278-279).
_CLI_ARGS = [((), 0), (("3",), 0), ((0, 1), 0), ((0, 2), 0), ((1, 2), 1), ((1, 1), 1), ((2, 1), 2), ((3, 2), 3)]


# batch 5 only where a call holds several batches (modes 2/3 run one or two blocks)
@pytest.mark.parametrize("args,mode,batch", [a + (1,) for a in _CLI_ARGS] + [a + (5,) for a in _CLI_ARGS if a[1] < 2])
def test_cli_project_contract(fmrx, orc, args, mode, batch):
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    nb = {0: 23, 1: 17, 2: 2, 3: 1}[mode]
    iq = iqgen.make("synth:91", nb * bb + 4321, rf_fs)  # ragged tail is dropped
    r = _cli(fmrx, list(args) + ["--batch", batch], iq.tobytes())
    assert r.returncode == 0, r.stderr.decode()
    got = np.frombuffer(r.stdout, np.int16)
    want = orc.run(mode, 51, iq, ["pcm"])["pcm"]
    assert got.size == nb * 2 * oracle.MODES[mode][2]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode,rf_taps", [(0, 51), (0, 101), (2, 51)])
def test_cli_mono_product_flag(fmrx, orc, mode, rf_taps):
    bb, rf_fs = oracle.MODES[mode][0], oracle.MODES[mode][3]
    nb = {0: 19, 2: 2}[mode]
    iq = iqgen.make("synth:92", nb * bb, rf_fs)
    r = _cli(fmrx, [mode, 1, "--mono-product", "--rf-taps", rf_taps, "--batch", 4], iq.tobytes())
    assert r.returncode == 0, r.stderr.decode()
    want = orc.run(mode, rf_taps, iq, ["pcm_mono"])["pcm_mono"]
    assert np.array_equal(np.frombuffer(r.stdout, np.int16), want)


def test_cli_bytes_equal_reference_project(fmrx, orc):
    """Byte-compare `fmrx` and `fmrx 0 1` with the reference's own `project` executable
    (oracle/_ref/project, built from src/project.cpp in place).  project exit(1)s at EOF while
    blocks may still be queued (project.cpp:51-54), so its stdout is a prefix of the full
    stream: compare on its length and require the full stream to equal the oracle's."""
    import os
    import subprocess

    ref = os.path.join(os.path.dirname(os.path.dirname(fmrx.LIB_PATH)), "oracle", "_ref", "project")
    if not os.path.exists(ref):
        pytest.skip("oracle/_ref/project not built")
    iq = iqgen.make("synth:93", 40 * 12800, 2400000).tobytes()
    pr = subprocess.run([ref, "0", "1"], input=iq, capture_output=True, timeout=120)
    want_prefix = pr.stdout
    full = orc.run(0, 51, np.frombuffer(iq, np.uint8), ["pcm"])["pcm"].tobytes()
    assert len(want_prefix) > 0 and full[: len(want_prefix)] == want_prefix
    for args in ([], [0, 1]):
        r = _cli(fmrx, args, iq)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout == full
        assert r.stdout[: len(want_prefix)] == want_prefix


@pytest.mark.parametrize("nbytes", [0, 12799, 12800])
def test_cli_empty_and_short_input(fmrx, orc, nbytes):
    import os
    import subprocess

    iq = iqgen.make("rand:3", nbytes, 2400000)
    exe = os.path.join(os.path.dirname(fmrx.LIB_PATH), "bin", "fmrx")
    r = subprocess.run([exe, "0", "2", "--batch", "4"], input=iq.tobytes(), capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got = np.frombuffer(r.stdout, np.int16)
    if nbytes < 12800:
        assert got.size == 0
    else:
        assert np.array_equal(got, orc.run(0, 51, iq, ["pcm"])["pcm"])


# ---- RDS front half (rds_thread body, project.cpp:200-271) -----------------------------------

from conftest import load_rds, rds_cases, rds_input  # noqa: E402


@pytest.mark.parametrize("name", rds_cases())
def test_rds_matches_reference(fmrx, orc, name):
    z = load_rds(name)
    demod = rds_input(orc, z)
    with fmrx.Receiver(z["mode"], fmrx.STEREO) as rx:
        out = rx.rds_block(demod, want_nco=True, want_channel=True)
    for f in ("channel", "nco", "rds"):
        if f in z:
            assert same(out[f], z[f]), f
        assert sha(out[f]) == z[f + "_sha256"], f


def test_rds_call_split_and_reset(fmrx, orc):
    z = load_rds("m0_rds57")
    demod, nif = z["demod"], oracle.MODES[0][1]
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        parts, b = [], 0
        for nb in (1, 5, 2, 16):
            parts.append(rx.rds_block(demod[b * nif:(b + nb) * nif])["rds"])
            b += nb
        assert same(np.concatenate(parts), z["rds"])
        rx.reset()
        assert same(rx.rds_block(demod)["rds"], z["rds"])


@pytest.mark.parametrize("env", [{"pll_spec": "0"}, {"pll_inject": "3"}])
def test_rds_pll_speculation_fallbacks(fmrx, monkeypatch, env):
    """The RDS loop (114 kHz, ncoScale 0.5) through the same speculative launch: the plain
    certified launch and a runner with one corrupted batch both give the fixture's bits."""
    knobs(monkeypatch, fmrx, **{k: float(v) for k, v in env.items()})
    z = load_rds("m0_rds57")
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        assert same(rx.rds_block(z["demod"])["rds"], z["rds"])


def test_rds_multistream_and_device_api(fmrx, orc):
    nif, nb = oracle.MODES[1][1], 10
    ins = [iqgen.make_rds_demod(60 + s, nb * nif, oracle.MODES[1][5]) for s in range(3)]
    ins[2] = ins[2] * np.float32(-2.5)
    want = [orc.rds(1, x) for x in ins]
    with fmrx.Receiver(1, fmrx.STEREO, n_streams=3) as rx:
        got = rx.rds_block(np.stack(ins), want_nco=True, want_channel=True)
    for s in range(3):
        for f in ("rds", "nco", "channel"):
            assert same(got[f][s], want[s][f]), (s, f)
    # device entry point: n_streams x (n_blocks * if_samples) contiguous, two calls of halves
    with fmrx.Receiver(1, fmrx.STEREO, n_streams=3) as rx:
        half = nb // 2 * nif
        outs = []
        for h in range(2):
            d_in = torch.from_numpy(np.stack([x[h * half:(h + 1) * half] for x in ins])).cuda()
            d_out = torch.empty_like(d_in)
            d_nco = torch.empty_like(d_in)
            rx.rds_device(d_in.data_ptr(), nb // 2, d_out.data_ptr(), d_nco.data_ptr())
            rx.synchronize()
            outs.append((d_out.cpu().numpy(), d_nco.cpu().numpy()))
    for s in range(3):
        assert same(np.concatenate([o[0][s] for o in outs]), want[s]["rds"]), s
        assert same(np.concatenate([o[1][s] for o in outs]), want[s]["nco"]), s


# ---- arctan demodulator and PSD estimate (floating point: tolerances stated) -----------------

import os  # noqa: E402

from test_oracle import GOLD, check_psd, psd_cases  # noqa: E402

# fmDemodArctan on the GPU: double atan2 of float I/Q, wrapped, rounded to float.  Against the
# model's float64 output the error is the final float rounding (<= 2^-24 relative) plus the
# model's own cancellation error on its growing unwrapped phase (~1e-12 here).
ARCTAN_RTOL = 2.0 ** -23
ARCTAN_ATOL = 1e-9


def test_arctan_demod_matches_python_model(fmrx):
    z = np.load(os.path.join(GOLD, "py_arctan.npz"))
    b = int(z["block"])
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        prev = torch.zeros(1, dtype=torch.float64, device="cuda")
        outs = []
        for k in range(z["i"].size // b):
            di = torch.from_numpy(z["i"][k * b:(k + 1) * b].copy()).cuda()
            dq = torch.from_numpy(z["q"][k * b:(k + 1) * b].copy()).cuda()
            do = torch.empty_like(di)
            rx.fm_demod_arctan(do.data_ptr(), prev.data_ptr(), di.data_ptr(), dq.data_ptr(), b)
            rx.synchronize()
            outs.append(do.cpu().numpy())
            # the carried phase is the principal value: equal to the model's mod 2 pi
            dphi = float(prev.cpu()[0]) - float(z["phases"][k])
            assert abs(dphi - 2 * np.pi * round(dphi / (2 * np.pi))) < 1e-9
    got = np.concatenate(outs).astype(np.float64)
    np.testing.assert_allclose(got, z["demod"], rtol=ARCTAN_RTOL, atol=ARCTAN_ATOL)


@pytest.mark.parametrize("key", psd_cases())
def test_psd_matches_python_model_and_cpp(fmrx, key):
    z = np.load(os.path.join(GOLD, "py_psd.npz"))
    name, nb, fs = key.rsplit("_", 2)
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        freq, psd = rx.estimate_psd(z[f"x_{name}"], int(nb), float(fs))
    check_psd(z, key, freq, psd)


def test_psd_device_api_and_errors(fmrx, orc):
    x = (iqgen.rand_bytes(78, 5000).astype(np.float32) - 127.5) / 127.5
    with fmrx.Receiver(0, fmrx.MONO) as rx:
        d_x = torch.from_numpy(x).cuda()
        d_p = torch.empty(256, dtype=torch.float32, device="cuda")
        rx.psd_device(d_x.data_ptr(), x.size, 512, 48000.0, d_p.data_ptr())  # 9 segments, ragged tail
        rx.synchronize()
        _, want = orc.estimate_psd(x, 512, 48000.0)
        assert np.abs(d_p.cpu().numpy() - want).max() <= 1e-3
        for bad in ((x, 500, 48000.0), (x[:100], 512, 48000.0), (x, 16384, 48000.0)):
            with pytest.raises(fmrx.FmrxError):
                rx.estimate_psd(*bad)


# ---- tuning knobs: no value of any accepted range changes the output; the rest is refused --------

KNOB_SWEEP = {  # include/fmrx.h FMRX_KNOB_* accepted ranges, every value or a spread of them
    "pll_spec": [0, 1], "pll_sat": [0, 1], "pll_pred": [0, 1, 2], "pll_pipe": [0, 1], "pll_idx": [0, 1, 2],
    "pll_cnt": list(range(32)), "pll_stick": [0, 1], "stereo_chunks": [0, 1, 2, 3, 4, 5, 7, 8, 9, 16, 33, 64],
    "stereo_head": [1, 2, 7, 8, 9, 16, 17, 63, 64], "stereo_tail": [1, 2, 8, 15, 16, 64],
    "stereo_lead": [0, 1, 2, 3, 7, 64], "audio_defer": [0, 1, 2, 3, 4, 5, 9, 10, 64], "bpf_tile": [0, 1],
}
KNOB_RANGES = {"pll_spec": (0, 1), "pll_sat": (0, 1), "pll_pred": (0, 2), "pll_pipe": (0, 1), "pll_idx": (0, 2),
               "stereo_chunks": (0, 64), "mono_split": (-1, 1023), "bpf_tile": (0, 1), "halo_kernel": (0, 1),
               "pll_cnt": (0, 31), "pll_stick": (0, 1), "stereo_head": (1, 64), "stereo_lead": (0, 64),
               "audio_defer": (0, 64), "stereo_tail": (1, 64), "pll_inject": (-1, 1 << 30),
               "pll_pipe_miss": (-(1 << 30), 1 << 30), "pll_hint_skew": (-16777216.0, 16777216.0)}


def _at_trig(rx, ns, trig):
    """Put every stream's PLL at trigOffset `trig` through the state blob (the runner regimes)."""
    blob = bytearray(rx.get_state())
    hdr = np.frombuffer(bytes(blob[:40]), np.uint32)
    off = 40 + ns * (int(hdr[6]) + 4 * int(hdr[7]) + 4 * 64)
    pll = np.frombuffer(bytes(blob[off: off + ns * 32]), np.float32).reshape(ns, 8).copy()
    pll[:, 5] = trig
    blob[off: off + ns * 32] = pll.tobytes()
    rx.set_state(bytes(blob))


def test_knob_sweep_bit_exact(fmrx, orc):
    """Every tuning knob (api.cpp kKnobs) over its accepted range, one at a time, through
    fmrx_debug_set_knob: a 20-stream 40-block stereo call from power-on (the pipelined engine:
    chunking, deferral, band-pass form) against the oracle, the same call with every stream's PLL put
    at trigOffset 2^19 - 6,000 and at 2^22 - 6,000 (the count / index / three-wave runners, their
    handovers) against the default knobs' output there, and a 20-stream mono call (mono_split,
    halo_kernel) against the oracle: bit-exact for every value."""
    ns, nb, bb = 20, 40, 12800
    ins = np.stack([iqgen.make("synth:%d" % (880 + s), nb * bb) for s in range(ns)])
    want = np.stack([orc.run(0, 51, ins[s], ["pcm"])["pcm"] for s in range(ns)])
    want_m = np.stack([orc.run(0, 51, ins[s], ["pcm_mono"])["pcm_mono"] for s in range(ns)])

    def stereo(knobs, trig=None):
        with fmrx.Receiver(0, fmrx.STEREO, n_streams=ns, knobs=knobs) as rx:
            if trig is not None:
                rx.process(ins[:, : 2 * bb])
                _at_trig(rx, ns, trig)
            return rx.process(ins if trig is None else ins[:, 2 * bb:])

    base = {t: stereo({}, t) for t in (524288.0 - 6000.0, 4194304.0 - 6000.0)}
    for name, values in KNOB_SWEEP.items():
        for v in values:
            assert np.array_equal(stereo({name: v}), want), (name, v)
            for t, b in base.items():
                assert np.array_equal(stereo({name: v}, t), b), (name, v, t)
    for name, values in (("mono_split", [-1, 0, 1, 330, 512, 660, 1023]), ("halo_kernel", [0, 1])):
        for v in values:
            with fmrx.Receiver(0, fmrx.MONO, n_streams=ns, knobs={name: v}) as rx:
                assert np.array_equal(rx.process(ins), want_m), (name, v)


def test_knob_out_of_range_refused(fmrx, monkeypatch):
    """A value outside a knob's range (include/fmrx.h), a fraction for an integer knob, NaN or an
    unknown knob: fmrx_debug_set_knob returns FMRX_EINVAL and the context keeps running; a bad
    environment variable makes fmrx_create refuse the context."""
    with fmrx.Receiver(0, fmrx.STEREO) as rx:
        for name, (lo, hi) in KNOB_RANGES.items():
            rx.set_knob(name, lo)
            rx.set_knob(name, hi)
            for bad in (lo - 1, hi + 1, float("nan")) + ((lo + 0.5,) if name != "pll_hint_skew" else ()):
                with pytest.raises(fmrx.FmrxError) as e:
                    rx.set_knob(name, bad)
                assert e.value.code == fmrx.FMRX_EINVAL, (name, bad)
        with pytest.raises(fmrx.FmrxError):
            fmrx._check(fmrx.lib().fmrx_debug_set_knob(rx.h, 99, 0.0))
    for var, val in (("FMRX_PLL_CNT", "32"), ("FMRX_AUDIO_DEFER", "-1"), ("FMRX_STEREO_HEAD", "0"),
                     ("FMRX_PLL_SPEC", "yes"), ("FMRX_MONO_SPLIT", "1024")):
        monkeypatch.setenv(var, val)
        with pytest.raises(fmrx.FmrxError) as e:
            fmrx.Receiver(0, fmrx.STEREO)
        assert e.value.code == fmrx.FMRX_EINVAL and var in str(e.value), (var, val)
        monkeypatch.delenv(var)
