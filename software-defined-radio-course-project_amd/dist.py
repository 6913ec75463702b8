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


def streams_leg(fmrx, n_streams: int, seconds: float, world: int, rank: int, device: int,
                mode: int = 0, expect: dict | None = None, warmup: bool = True,
                collective: bool | None = None) -> dict | None:
    """BASELINE configs[4] as one timed step: `n_streams` independent stereo streams (stream id
    = synth seed) of `seconds` each, this rank's contiguous shard processed as ONE multi-stream
    device-resident call, then the S16 PCM gathered to rank 0 (RCCL over xGMI; gloo rehearses
    it).  Timing = barrier -> process -> gather, max over ranks.  The input is synthesized on the
    device in one launch before the timed region; `warmup` runs one untimed full-size call first
    (code objects, scratch sized) and restarts from the power-on state.  `expect` maps stream id
    -> the reference build's PCM SHA-256 (tests/golden/hashes.json streams_*); rank 0 checks
    those streams of the gathered PCM.  `collective` (default: world > 1) routes the barrier,
    gather and timing reduction through the initialised process group; without it (one rank, no
    process group) the rank's PCM is the result.  Returns rank 0's result dict (None elsewhere)."""
    import hashlib
    import time

    ids = list(shard(n_streams, world, rank))
    rx = fmrx.Receiver(mode, fmrx.STEREO, n_streams=max(1, len(ids)), device=device)
    try:
        bb = rx.geo.block_bytes
        nb = int(seconds * rx.geo.rf_fs * 2 // bb)
        pcm_len = nb * rx.geo.pcm_samples
        dev = torch.device("cuda", device)
        iq = torch.empty((max(1, len(ids)), nb * bb), dtype=torch.uint8, device=dev)
        out = torch.empty((len(ids), pcm_len), dtype=torch.int16, device=dev)
        torch.cuda.synchronize(dev)
        t_synth = time.perf_counter()
        if ids:
            rx.synth_device_streams(ids, 0, nb * bb // 2, iq.data_ptr(), nb * bb)
        t_synth = time.perf_counter() - t_synth
        if ids and warmup:
            rx.process_device(iq.data_ptr(), nb, out.data_ptr())
            rx.synchronize()
            rx.reset()
        pg = world > 1 if collective is None else collective
        if pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if ids:
            rx.process_device(iq.data_ptr(), nb, out.data_ptr())
            rx.synchronize()
        t1 = time.perf_counter()
        gathered = gather_pcm(out, n_streams, pcm_len, world, rank) if pg else out
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        t = torch.tensor([t2 - t0, t1 - t0, t2 - t1],
                         device=dev if pg and dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        if pg:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        total, proc, gat = (float(v) for v in t)
        if rank != 0:
            return None
        assert gathered.shape == (n_streams, pcm_len), gathered.shape
        sig_s = nb * bb / 2 / rx.geo.rf_fs
        res = {"workload": f"BASELINE configs[4]: {n_streams} independent mode-{mode} stereo streams x {sig_s:g} s, "
                           f"{world} rank(s), streams sharded contiguously"
                           + (", S16 PCM gathered to rank 0" if pg else ", PCM left on the one rank (no gather)"),
               "n_gpus": world, "seconds": round(total, 4), "seconds_process": round(proc, 4),
               "seconds_gather": round(gat, 4), "gather_bytes": int(gathered.numel() * 2),
               "MS_per_s": round(n_streams * nb * bb / 2 / total / 1e6, 1),
               "stream_seconds_per_s": round(n_streams * sig_s / total, 1),
               "x_realtime_per_stream": round(sig_s / total, 2), "synth_seconds_untimed": round(t_synth, 3)}
        if expect:
            got = {sid: hashlib.sha256(gathered[sid].cpu().numpy().tobytes()).hexdigest() for sid in expect}
            res["checked_streams"] = sorted(expect)
            res["bit_exact_vs_reference"] = all(got[sid] == expect[sid] for sid in expect)
        return res
    finally:
        rx.close()


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
