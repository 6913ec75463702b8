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
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import iqgen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
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
    t = torch.tensor([t2 - t0, t1 - t0, t2 - t1], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    total, proc, gat = (float(v) for v in t)
    if rank == 0:
        assert gathered.shape == (args.streams, pcm_len)
        sig_s = nb * bb / 2 / rx.geo.rf_fs
        print(json.dumps({
            "config": f"BASELINE configs[4]: {args.streams} independent mode-{args.mode} stereo streams "
                      f"x {sig_s:.1f} s, {world} GPU(s), RCCL gather of S16 PCM to rank 0",
            "n_gpus": world, "seconds_total": round(total, 4), "seconds_process": round(proc, 4),
            "seconds_gather": round(gat, 4), "gather_bytes": int(gathered.numel() * 2),
            "MS_per_s": round(args.streams * nb * bb / 2 / total / 1e6, 1),
            "stream_seconds_per_s": round(args.streams * sig_s / total, 1),
            "x_realtime_per_stream": round(sig_s / total, 2)}), flush=True)
    rx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
