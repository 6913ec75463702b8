"""dist.py — many independent IQ streams sharded over GPUs (BASELINE configs[4]).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Streams have fully
private state, so the only communication is the final GATHER of the int16 PCM to
rank 0.  Shards are contiguous stream ranges; ranks with fewer streams pad their send buffer
so that the collective moves equal-sized messages, and rank 0 drops the padding.

The per-rank work is a callable ``process(stream_ids) -> tensor[len(ids), pcm_len]`` so the
same sharding/gather code runs over libfmrx on GPUs (``fmrx_process_fn``) and, in the CPU
tests, over the oracle with the gloo backend.

ONE long recording can be cut in time instead (mono product only): rank r takes a
contiguous range of blocks and seeks to the raw bytes in front of it (``fmrx_seek``: the mono
product's state is a function of a bounded run of preceding bytes), so the gathered PCM is the
whole recording's, bit for bit (``run_time_sharded``, ``fmrx_time_shard_fn``).  The stereo
PLL is a serial recurrence: stereo streams are replicas only.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch
import torch.distributed as dist


def shard(n_streams: int, world: int, rank: int) -> range:
    """Contiguous, balanced stream range of `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_streams, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_pcm(local: torch.Tensor, n_streams: int, pcm_len: int, world: int, rank: int,
               dst: int = 0) -> torch.Tensor | None:
    """Gather every rank's [n_local, pcm_len] int16 PCM to `dst` as [n_streams, pcm_len].

    Messages are padded to the largest shard so one equal-size collective suffices.
    """
    max_local = len(shard(n_streams, world, 0))
    send = torch.zeros((max_local, pcm_len), dtype=local.dtype, device=local.device)
    send[: local.shape[0]] = local
    # RCCL/NCCL and gloo have no int16 type: move the PCM as raw bytes (gloo: host memory).
    send8 = send.view(torch.uint8)
    if dist.get_backend() == "gloo" and send8.is_cuda:
        send8 = send8.cpu()
    bufs = [torch.empty_like(send8) for _ in range(world)] if rank == dst else None
    dist.gather(send8, bufs, dst=dst)
    if rank != dst:
        return None
    parts = [bufs[r].view(local.dtype)[: len(shard(n_streams, world, r))] for r in range(world)]
    return torch.cat(parts, 0)


def run_sharded(process: Callable[[Sequence[int]], torch.Tensor], n_streams: int, pcm_len: int,
                world: int, rank: int) -> torch.Tensor | None:
    """Process this rank's shard and gather the PCM of all streams on rank 0."""
    ids = shard(n_streams, world, rank)
    local = process(list(ids))
    assert local.shape == (len(ids), pcm_len), (local.shape, len(ids), pcm_len)
    return gather_pcm(local, n_streams, pcm_len, world, rank)


def fmrx_process_fn(fmrx, mode: int, channels: int, n_blocks: int, device: int, rf_taps: int = 51):
    """GPU per-rank worker: synthesize each stream on the device (seed = global stream id),
    run them as one multi-stream libfmrx context, return the device PCM tensor."""

    def process(ids: Sequence[int]) -> torch.Tensor:
        n = len(ids)
        rx = fmrx.Receiver(mode, channels, rf_taps=rf_taps, n_streams=max(n, 1), device=device)
        try:
            bb = rx.geo.block_bytes
            pcm_len = n_blocks * rx.geo.pcm_samples
            out = torch.empty((n, pcm_len), dtype=torch.int16, device=f"cuda:{device}")
            if n == 0:
                return out
            iq = torch.empty((n, n_blocks * bb), dtype=torch.uint8, device=f"cuda:{device}")
            torch.cuda.synchronize(device)
            rx.synth_device_streams(list(ids), 0, n_blocks * bb // 2, iq.data_ptr(), n_blocks * bb)
            rx.process_device(iq.data_ptr(), n_blocks, out.data_ptr())
            rx.synchronize()
            return out
        finally:
            rx.close()

    return process


def _flag_device(pg: bool, device):
    """Where a collective's small tensors live: the GPU for RCCL, host memory for gloo."""
    return device if pg and dist.get_backend() == "nccl" else "cpu"


def all_ok(ok: bool, pg: bool, device=None) -> bool:
    """Every rank learns whether EVERY rank succeeded so far (MAX over ranks of an error flag).
    A rank that failed before a collective must not leave the others blocked in it: each rank
    calls this at the same points, and all of them skip the collectives together when any failed."""
    if not pg:
        return ok
    t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=_flag_device(pg, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) == 0


def per_rank(values: Sequence[float], pg: bool, device=None) -> list[list[float]]:
    """Every rank's `values` (same length on every rank), in rank order, on every rank."""
    t = torch.tensor(list(values), dtype=torch.float64, device=_flag_device(pg, device))
    if not pg:
        return [t.tolist()]
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.tolist() for p in parts]


def gather_chunked(chunks, n_streams: int, pcm_len: int, world: int, rank: int, pg: bool):
    """Gather a rank's PCM time chunk by time chunk as each one finishes: `chunks` is a list of
    (col0, tensor[n_local, cols], done) with `done` a torch.cuda.Event recorded after the chunk's
    work on the stream that computes it (None: already complete).  RCCL: the collective's stream
    waits for the event, so chunk c's gather runs beside chunk c + 1's processing; gloo: the host
    waits for chunk c alone, then moves it.  Returns (rank 0: [n_streams, pcm_len], else None;
    the time the last chunk's processing was seen complete)."""
    import time

    nccl = pg and dist.get_backend() == "nccl"
    full = None
    t_proc = None
    for k, (c0, part, done) in enumerate(chunks):
        last = k == len(chunks) - 1
        if done is not None:
            if nccl and not last:
                torch.cuda.current_stream(part.device).wait_event(done)
            else:
                done.synchronize()
        if last:
            t_proc = time.perf_counter()
        got = gather_pcm(part, n_streams, part.shape[1], world, rank) if pg else part
        if got is not None:
            if full is None:
                full = torch.empty((n_streams, pcm_len), dtype=got.dtype, device=got.device)
            full[:, c0:c0 + got.shape[1]] = got
    return full, t_proc


def run_leg(setup: Callable[[], object], process: Callable[[object], torch.Tensor], n_streams: int, pcm_len: int,
            world: int, rank: int, pg: bool, device=None, cleanup: Callable[[object], None] | None = None,
            post: Callable[[object], dict] | None = None, repeats: int = 1,
            reset: Callable[[object], None] | None = None) -> dict:
    """One timed multi-stream step with failure agreement (the collective skeleton of
    streams_leg, also run on the CPU with gloo by the tests).

    setup() prepares this rank's shard (untimed; may raise); process(state) -> [n_local, pcm_len]
    PCM is the timed step (may raise).  Timing = barrier -> process -> gather to rank 0.  Before
    the barrier and again before the gather every rank agrees on success (all_ok), so a rank
    that raised does not leave the others in a collective.  Returns a dict on every rank:
    `error` when any rank failed, else per-rank seconds (total, process, gather) and, on rank 0,
    `gathered` ([n_streams, pcm_len]).  repeats > 1: the timed step that many times, reset(state)
    (untimed) before each after the first; the result is the repeat of median total time, with
    `runs` (every repeat's max-over-ranks total) beside it, and the last repeat's PCM."""
    import time

    err, state = None, None
    try:
        state = setup()
    except Exception as e:  # noqa: BLE001 -- reported, and every rank skips the collectives
        err = f"rank {rank} setup: {e!r}"
    try:
        if not all_ok(err is None, pg, device):
            return {"error": err or "another rank failed in setup; collectives skipped"}
        reps = []
        for rep in range(max(1, repeats)):
            if rep > 0 and reset is not None:
                try:
                    reset(state)
                except Exception as e:  # noqa: BLE001
                    err = f"rank {rank} reset: {e!r}"
                if not all_ok(err is None, pg, device):
                    return {"error": err or "another rank failed in a reset; collectives skipped"}
            if pg:
                dist.barrier()
            if device is not None and torch.cuda.is_available():
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            local = None
            try:
                local = process(state)
                if isinstance(local, torch.Tensor):
                    assert local.shape[1:] == (pcm_len,), (tuple(local.shape), pcm_len)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank} process: {e!r}"
            t1 = time.perf_counter()
            if not all_ok(err is None, pg, device):
                return {"error": err or "another rank failed in the timed step; gather skipped"}
            if isinstance(local, torch.Tensor):
                gathered = gather_pcm(local, n_streams, pcm_len, world, rank) if pg else local
                t_proc = t1
            else:  # time chunks enqueued: each gathered as soon as it is done, beside the later ones
                gathered, t_proc = gather_chunked(local, n_streams, pcm_len, world, rank, pg)
            if device is not None and torch.cuda.is_available():
                torch.cuda.synchronize(device)
            t2 = time.perf_counter()
            ranks = per_rank([t2 - t0, t_proc - t0, t2 - t_proc], pg, device)
            reps.append({"per_rank": ranks, "total": max(r[0] for r in ranks), "process": max(r[1] for r in ranks),
                         "gather": max(r[2] for r in ranks)})
        order = sorted(range(len(reps)), key=lambda k: reps[k]["total"])
        res = dict(reps[order[len(order) // 2]])
        res["runs"] = [r["total"] for r in reps]
        if rank == 0:
            res["gathered"] = gathered
            if post is not None:  # after the timed step, untimed (rank 0's shard only)
                try:
                    res["post"] = post(state)
                except Exception as e:  # noqa: BLE001 -- diagnostic only
                    res["post"] = {"error": repr(e)}
        return res
    finally:
        if cleanup is not None and state is not None:
            cleanup(state)


def streams_leg(fmrx, n_streams: int, seconds: float, world: int, rank: int, device: int,
                mode: int = 0, expect: dict | None = None, warmup: bool = True,
                collective: bool | None = None, profile: Callable | None = None,
                gather_chunks: int = 1, repeats: int = 1) -> dict | None:
    """BASELINE configs[4] as one timed step: `n_streams` independent stereo streams (stream id
    = synth seed) of `seconds` each, this rank's contiguous shard processed as ONE multi-stream
    device-resident call, then the S16 PCM gathered to rank 0 (RCCL over xGMI; gloo rehearses
    it).  Timing = barrier -> process -> gather, max over ranks, with every rank's own split
    (`per_rank`: seconds, seconds_process, seconds_gather) so a multi-GPU run shows which rank
    or which phase is slow.  The input is synthesized on the device in one launch before the
    timed region; `warmup` runs one untimed full-size call first (code objects, scratch sized)
    and restarts from the power-on state.  `expect` maps stream id -> the reference build's PCM
    SHA-256 (tests/golden/hashes.json streams_*); rank 0 checks those streams of the gathered
    PCM (`parity` says "unpinned" when none are recorded for this length).  `collective`
    (default: world > 1) routes the barrier, gather and timing reduction through the process
    group; without it (one rank, no process group) the rank's PCM is the result.  A failure on
    any rank is agreed on before each collective (run_leg), so no rank hangs in one.
    `gather_chunks` K > 1 (with a process group): the shard runs as K calls over consecutive time
    chunks (the context carries every state across them: the same PCM as one call), each chunk's
    PCM gathered as soon as it is done while the next is processed (gather_chunked), so only the
    last chunk's gather follows the processing.  `repeats`: the timed step that many times from
    the power-on state (fmrx_reset between them, untimed): the line's times are the median
    repeat's, `runs` / `median` / `min` / `max` the totals.  Returns rank 0's result dict (None
    elsewhere)."""
    import hashlib
    import time

    ids = list(shard(n_streams, world, rank))
    pg = world > 1 if collective is None else collective
    dev = torch.device("cuda", device)
    geo = fmrx.geometry(fmrx.default_config(mode, fmrx.STEREO))
    bb = geo.block_bytes
    nb = int(seconds * geo.rf_fs * 2 // bb)
    pcm_len = nb * geo.pcm_samples
    K = max(1, min(gather_chunks, nb)) if pg else 1
    cuts = [nb * k // K for k in range(K + 1)]  # block boundaries of the time chunks
    t_synth = [0.0]
    redos = [None]  # this rank's streams x 8 redo slots (fmrx_debug_pll_redos), warm-up call

    def setup():
        rx = fmrx.Receiver(mode, fmrx.STEREO, n_streams=max(1, len(ids)), device=device)
        try:
            # one input and one output buffer a time chunk (stream-major within the chunk)
            iqs = [torch.empty((max(1, len(ids)), (cuts[k + 1] - cuts[k]) * bb), dtype=torch.uint8, device=dev)
                   for k in range(K)]
            outs = [torch.empty((len(ids), (cuts[k + 1] - cuts[k]) * geo.pcm_samples), dtype=torch.int16,
                                device=dev) for k in range(K)]
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            if ids:
                for k in range(K):
                    rx.synth_device_streams(ids, cuts[k] * bb // 2, (cuts[k + 1] - cuts[k]) * bb // 2,
                                            iqs[k].data_ptr(), (cuts[k + 1] - cuts[k]) * bb)
                rx.synchronize()
            t_synth[0] = time.perf_counter() - t
            if ids and warmup:
                # the untimed warm-up does the timed step's work exactly (same input, same
                # power-on state): the runners' per-stream redo counts are taken here
                redo = torch.zeros((len(ids), fmrx.REDO_SLOTS), dtype=torch.int32, device=dev)
                rx.debug_pll_redos(redo.data_ptr())
                for k in range(K):
                    rx.process_device(iqs[k].data_ptr(), cuts[k + 1] - cuts[k], outs[k].data_ptr())
                rx.synchronize()
                rx.debug_pll_redos(None)
                redos[0] = redo.cpu().numpy()
                rx.reset()
        except Exception:
            rx.close()
            raise
        return rx, iqs, outs

    def process(state):
        rx, iqs, outs = state
        if K == 1:
            if ids:
                rx.process_device(iqs[0].data_ptr(), nb, outs[0].data_ptr())
                rx.synchronize()
            return outs[0]
        ext = torch.cuda.ExternalStream(rx.stream(), device=dev)
        chunks = []
        for k in range(K):
            done = None
            if ids:
                rx.process_device(iqs[k].data_ptr(), cuts[k + 1] - cuts[k], outs[k].data_ptr())
                done = torch.cuda.Event()
                done.record(ext)
            chunks.append((cuts[k] * geo.pcm_samples, outs[k], done))
        return chunks

    # profile(rx, run) (optional, rank 0): one more call of rank 0's shard, e.g. with the stage
    # timing armed (bench.stage_latency); its result is the line's `latency`
    post = None
    if profile is not None and ids:
        def post(st):
            def run():
                for k in range(K):
                    st[0].process_device(st[1][k].data_ptr(), cuts[k + 1] - cuts[k], st[2][k].data_ptr())
            return profile(st[0], run)
    def reset(st):
        st[0].reset()
        st[0].synchronize()

    res = run_leg(setup, process, n_streams, pcm_len, world, rank, pg, dev, cleanup=lambda st: st[0].close(),
                  post=post, repeats=repeats, reset=reset)
    if rank != 0:
        return None
    if "error" in res:
        return {"error": res["error"], "n_gpus": world}
    gathered = res.pop("gathered")
    assert gathered.shape == (n_streams, pcm_len), gathered.shape
    sig_s = nb * bb / 2 / geo.rf_fs
    total = res["total"]
    max_local = len(shard(n_streams, world, 0))
    out = {"workload": f"BASELINE configs[4]: {n_streams} independent mode-{mode} stereo streams x {sig_s:g} s, "
                       f"{world} rank(s), streams sharded contiguously"
                       + (", S16 PCM gathered to rank 0" if pg else ", PCM left on the one rank (no gather)")
                       + (f" in {K} time chunks, each gathered beside the next one's processing" if K > 1 else ""),
           "n_gpus": world, "seconds": round(total, 4), "seconds_process": round(res["process"], 4),
           "seconds_gather": round(res["gather"], 4), "gather_bytes": int(gathered.numel() * 2),
           "seconds_note": ("seconds_process ends when the last time chunk's processing is seen complete and "
                            "includes the gathers of the chunks before it (overlapped with processing on RCCL, "
                            "host-blocking on gloo); seconds_gather is the last chunk's gather only")
           if K > 1 else "seconds_process: the call; seconds_gather: the gather after it",
           "runs": [round(x, 4) for x in res["runs"]], "median": round(total, 4),
           "min": round(min(res["runs"]), 4), "max": round(max(res["runs"]), 4),
           "gather_chunks": K,
           # every rank sends an equal (padded) message per chunk; rank 0 receives world of them
           "gather_bytes_sent_per_rank": int(max_local * pcm_len * 2) if pg else 0,
           "gather_GBs_after_processing": (round(max_local * pcm_len * 2 * world / K / res["gather"] / 1e9, 2)
                                           if pg and res["gather"] > 0 else None),
           "MS_per_s": round(n_streams * nb * bb / 2 / total / 1e6, 1),
           "stream_seconds_per_s": round(n_streams * sig_s / total, 1),
           "x_realtime_per_stream": round(sig_s / total, 2), "synth_seconds_untimed": round(t_synth[0], 3),
           "dist": {"world_size": dist.get_world_size() if pg else 1,
                    "backend": ({"nccl": "RCCL"}.get(dist.get_backend(), dist.get_backend()) if pg else None)},
           "per_rank": [{"rank": r, "streams": len(shard(n_streams, world, r)), "seconds": round(v[0], 4),
                         "seconds_process": round(v[1], 4), "seconds_gather": round(v[2], 4)}
                        for r, v in enumerate(res["per_rank"])]}
    if "post" in res:
        out["latency"] = res["post"]
    if redos[0] is not None and len(ids):
        # rank 0's shard: the streams whose redone intervals (a trigArg outside the runner's
        # candidates) cost the most serial time -- the slowest of them sets the call's wall time
        r, dm = redos[0][:, :4], redos[0][:, 4:]
        tot = r.sum(axis=1)
        worst = [int(i) for i in tot.argsort()[::-1][:8]]
        out["redos"] = {"streams": len(ids), "ranges": fmrx.REDO_RANGES,
                        "total_per_range": [int(x) for x in r.sum(axis=0)],
                        "max_per_range": [int(x) for x in r.max(axis=0)],
                        "worst_streams": [{"stream": ids[i], "redos": [int(x) for x in r[i]]} for i in worst],
                        "demoted_streams": int((dm.sum(axis=1) > 0).sum()),
                        "demoted_steps_per_range": [int(x) for x in dm.sum(axis=0)],
                        "source": "fmrx_debug_pll_redos over the untimed warm-up call (same input, same state): "
                                  "redone intervals by the runner launch's trigOffset range; demoted: steps run on "
                                  "the exact path after most intervals missed (pll_demote)"}
    if expect:
        host = gathered.cpu().numpy()
        got = {sid: hashlib.sha256(host[sid].tobytes()).hexdigest() for sid in expect}
        out["checked_streams"] = sorted(expect)
        bad = sorted(sid for sid in expect if got[sid] != expect[sid])
        out["bit_exact_vs_reference"] = not bad
        if bad:
            out["mismatched_streams"] = bad
    else:
        out["parity"] = f"unpinned: no reference hashes recorded for {n_streams} streams x {nb} blocks"
    return out


def run_time_sharded(process: Callable[[range], torch.Tensor], n_blocks: int, pcm_per_block: int,
                     world: int, rank: int) -> torch.Tensor | None:
    """One stream cut in time: rank r processes blocks shard(n_blocks, world, r) (its
    `process(blocks) -> tensor[len(blocks) * pcm_per_block]` seeks to the bytes in front of the
    range first); rank 0 receives the whole stream's PCM, in order."""
    blocks = shard(n_blocks, world, rank)
    local = process(blocks)
    assert local.shape == (len(blocks) * pcm_per_block,), (local.shape, len(blocks), pcm_per_block)
    got = gather_pcm(local.view(len(blocks), pcm_per_block), n_blocks, pcm_per_block, world, rank)
    return None if got is None else got.reshape(-1)


def fmrx_time_shard_fn(fmrx, mode: int, seed: int, device: int, rf_taps: int = 51):
    """GPU per-rank worker for run_time_sharded: the shard and the history bytes in front of it
    are synthesized on the device (the generator is position-addressable), the context seeks to
    the history, then processes the shard as one device-resident mono call."""

    def process(blocks: range) -> torch.Tensor:
        rx = fmrx.Receiver(mode, fmrx.MONO, rf_taps=rf_taps, device=device)
        try:
            bb, pcm = rx.geo.block_bytes, rx.geo.pcm_samples
            out = torch.empty(len(blocks) * pcm, dtype=torch.int16, device=f"cuda:{device}")
            if len(blocks) == 0:
                return out
            start = blocks.start * bb
            pre = min(rx.history_bytes(), start)
            buf = torch.empty(pre + len(blocks) * bb, dtype=torch.uint8, device=f"cuda:{device}")
            torch.cuda.synchronize(device)
            rx.synth_device(seed, (start - pre) // 2, buf.numel() // 2, buf.data_ptr())
            rx.seek(buf.data_ptr(), pre)
            rx.process_device(buf.data_ptr() + pre, len(blocks), out.data_ptr())
            rx.synchronize()
            return out
        finally:
            rx.close()

    return process
