#!/usr/bin/env python3
"""BASELINE configs[4]: many independent 2.4 MS/s stereo streams sharded across GPUs, one
process per GPU, RCCL gather of the S16 audio to rank 0 (dist.streams_leg, the same leg
bench.py runs).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/bench_streams.py --streams 256 --seconds 60 --check

Rank 0 prints one JSON line: aggregate IQ MS/s and stream-seconds per second (max-over-ranks
timing of processing + the gather), and the gather's own time.  --check compares the gathered
PCM of the streams tests/golden/hashes.json holds for this stream length (streams_*: the
reference build's PCM hashes) and fails if they differ or none are recorded.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--check", action="store_true",
                    help="rank 0 checks the streams hashes.json records against the reference build")
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
    nb = int(args.seconds * 2400000 * 2 // 12800) if args.mode == 0 else None
    expect = None
    if args.check:
        expect = iqgen.stream_hashes(args.streams, nb) if args.mode == 0 else {}
        if not expect:
            raise SystemExit(f"--check: no reference hashes for {args.streams} streams x {args.seconds} s")
    # collective=True: the gather goes through the process group even for one rank (RCCL)
    res = dmod.streams_leg(fm, args.streams, args.seconds, world, rank, local, mode=args.mode, expect=expect,
                           warmup=not args.no_warmup, collective=True)
    if rank == 0:
        res["backend"] = "RCCL" if backend == "nccl" else backend
        print(json.dumps(res), flush=True)
        if expect and not res["bit_exact_vs_reference"]:
            raise SystemExit("gathered PCM differs from the reference build's hashes")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
