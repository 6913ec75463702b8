#!/usr/bin/env python3
"""ONE long mono recording cut in time over the GPUs (MONO only).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/bench_time_shards.py --gib-per-rank 1 [--check]

Rank r owns blocks shard(n_blocks, N, r) of one stream (seed fixed: the same recording on every
rank), synthesizes them and the history bytes in front of them on its device (untimed), seeks
to the history (`fmrx_seek`) and processes its shard as one device-resident mono call (timed:
max over ranks, barrier + sync on both sides).  The PCM is gathered to rank 0 over RCCL.
--check: rank 0 also runs the whole recording in one context and compares bit for bit (the
recording must fit one GPU).  FMRX_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs.
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib-per-rank", type=float, default=1.0)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--rf-taps", type=int, default=101)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import iqgen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("FMRX_BENCH_BACKEND", "nccl")
    dev = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    fm = iqgen.load_fmrx()
    d = iqgen.load_module("dist")
    rx = fm.Receiver(args.mode, fm.MONO, rf_taps=args.rf_taps, device=dev)
    bb, na = rx.geo.block_bytes, rx.geo.pcm_samples
    n_blocks = int(args.gib_per_rank * (1 << 30)) // bb * world
    blocks = d.shard(n_blocks, world, rank)
    start = blocks.start * bb
    pre = min(rx.history_bytes(), start)
    buf = torch.empty(pre + len(blocks) * bb, dtype=torch.uint8, device="cuda")
    out = torch.empty(len(blocks) * na, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rx.synth_device(args.seed, (start - pre) // 2, buf.numel() // 2, buf.data_ptr())
    rx.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):  # untimed: the same shard (code objects, caches)
        rx.seek(buf.data_ptr(), pre)
        rx.process_device(buf.data_ptr() + pre, len(blocks), out.data_ptr())
    rx.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rx.seek(buf.data_ptr(), pre)
    rx.process_device(buf.data_ptr() + pre, len(blocks), out.data_ptr())
    rx.synchronize()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    t_gather = 0.0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
        g0 = time.perf_counter()
        got = d.gather_pcm(out.view(len(blocks), na), n_blocks, na, world, rank)
        t_gather = time.perf_counter() - g0
        got = None if got is None else got.reshape(-1)
    else:
        got = out
    if rank == 0:
        line = {"config": f"one mode-{args.mode} mono recording of {n_blocks * bb / 2**30:.2f} GiB "
                          f"({n_blocks} blocks, {n_blocks * bb / 2 / rx.geo.rf_fs:.0f} s, rf_taps "
                          f"{args.rf_taps}) cut in time over {world} rank(s), fmrx_seek per shard, "
                          f"PCM gathered to rank 0",
                "n_gpus": world, "seconds_process": round(dt, 5), "seconds_gather": round(t_gather, 4),
                "MS_per_s": round(n_blocks * bb / 2 / dt / 1e6, 1), "scaling": "weak"}
        if args.check:
            whole = torch.empty(n_blocks * bb, dtype=torch.uint8, device="cuda")
            ref = torch.empty(n_blocks * na, dtype=torch.int16, device="cuda")
            one = fm.Receiver(args.mode, fm.MONO, rf_taps=args.rf_taps, device=dev)
            one.synth_device(args.seed, 0, n_blocks * bb // 2, whole.data_ptr())
            one.process_device(whole.data_ptr(), n_blocks, ref.data_ptr())
            one.synchronize()
            line["bit_exact_vs_one_context"] = bool(torch.equal(got.to(ref.device), ref))
            one.close()
        print(json.dumps(line), flush=True)
    rx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
