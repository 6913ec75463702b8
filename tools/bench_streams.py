#!/usr/bin/env python3
"""BASELINE configs[4]: many independent 2.4 MS/s stereo streams sharded across GPUs, one
process per GPU, RCCL gather of the S16 audio to rank 0.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/bench_streams.py --streams 256 --seconds 10

Rank 0 prints one JSON line: aggregate IQ MS/s and stream-seconds per second (max-over-ranks
timing of synth-free processing + the gather), and the gather's own time.
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
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--check", action="store_true", help="rank 0 re-runs the first and last stream alone")
    ap.add_argument("--no-warmup", action="store_true", help="time the first (buffer-sizing) call")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import iqgen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FMRX_BENCH_BACKEND=gloo rehearses several ranks on fewer GPUs (devices shared, the
    # gather through host memory); the default is RCCL with one GPU per rank.
    backend = os.environ.get("FMRX_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    fm = iqgen.load_fmrx()
    dmod = iqgen.load_module("dist")
    ids = list(dmod.shard(args.streams, world, rank))
    rx = fm.Receiver(args.mode, fm.STEREO, n_streams=max(1, len(ids)), device=local)
    bb = rx.geo.block_bytes
    nb = int(args.seconds * rx.geo.rf_fs * 2 // bb)
    pcm_len = nb * rx.geo.pcm_samples
    iq = torch.empty((max(1, len(ids)), nb * bb), dtype=torch.uint8, device="cuda")
    out = torch.empty((len(ids), pcm_len), dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    for k, sid in enumerate(ids):
        rx.synth_device(sid, 0, nb * bb // 2, iq[k].data_ptr())
    rx.synchronize()
    if ids and not args.no_warmup:  # full-size call first (code objects, scratch sized), then a fresh state
        rx.process_device(iq.data_ptr(), nb, out.data_ptr())
        rx.synchronize()
        rx.reset()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if ids:
        rx.process_device(iq.data_ptr(), nb, out.data_ptr())
        rx.synchronize()
    t1 = time.perf_counter()
    gathered = dmod.gather_pcm(out, args.streams, pcm_len, world, rank)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t = torch.tensor([t2 - t0, t1 - t0, t2 - t1], device="cuda" if backend == "nccl" else "cpu",
                     dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    total, proc, gat = (float(v) for v in t)
    if rank == 0:
        assert gathered.shape == (args.streams, pcm_len)
        if args.check:  # the gathered PCM of two streams equals a single-stream run
            for sid in (0, args.streams - 1):
                with fm.Receiver(args.mode, fm.STEREO, device=local) as one:
                    d = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
                    o = torch.empty(pcm_len, dtype=torch.int16, device="cuda")
                    one.synth_device(sid, 0, nb * bb // 2, d.data_ptr())
                    one.process_device(d.data_ptr(), nb, o.data_ptr())
                    one.synchronize()
                assert torch.equal(o.cpu(), gathered[sid].cpu()), sid
        sig_s = nb * bb / 2 / rx.geo.rf_fs
        print(json.dumps({
            "config": f"BASELINE configs[4]: {args.streams} independent mode-{args.mode} stereo streams "
                      f"x {sig_s:.1f} s, {world} rank(s), {'RCCL' if backend == 'nccl' else backend} gather of S16 PCM to rank 0",
            "n_gpus": world, "seconds_total": round(total, 4), "seconds_process": round(proc, 4),
            "seconds_gather": round(gat, 4), "gather_bytes": int(gathered.numel() * 2),
            "MS_per_s": round(args.streams * nb * bb / 2 / total / 1e6, 1),
            "stream_seconds_per_s": round(args.streams * sig_s / total, 1),
            "x_realtime_per_stream": round(sig_s / total, 2)}), flush=True)
    rx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
