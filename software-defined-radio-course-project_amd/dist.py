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
            for k, sid in enumerate(ids):
                rx.synth_device(sid, 0, n_blocks * bb // 2, iq[k].data_ptr())
            rx.process_device(iq.data_ptr(), n_blocks, out.data_ptr())
            rx.synchronize()
            return out
        finally:
            rx.close()

    return process


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
