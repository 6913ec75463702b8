"""Worker for tests/test_distributed.py: one rank of the sharded multi-stream runner (or, with
argv[3] == "time", of one stream cut in time) on CPU (gloo), with the oracle as the per-rank
receiver.  Rank 0 saves the gathered PCM to argv[2]."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import iqgen  # noqa: E402
import oracle  # noqa: E402

MODE, NB, BB, NA = 0, 2, 12800, 128


def process(ids):
    orc = oracle.Oracle()
    rows = [orc.run(MODE, 51, iqgen.make(f"rand:{100 + i}", NB * BB), ["pcm"])["pcm"] for i in ids]
    if not rows:
        return torch.empty((0, NB * NA * 2), dtype=torch.int16)
    return torch.from_numpy(np.stack(rows))


TIME_RECIPE = "synth:77"


def process_time(n_blocks):
    """One stream cut in time, the oracle as the receiver: it starts from the zero state, so
    it is run from one whole block before the shard (more than the mono product's memory:
    100 RF pairs + 50 demod samples) and that block's output is dropped -- the CPU analogue
    of fmrx_seek."""
    whole = iqgen.make(TIME_RECIPE, n_blocks * BB)

    def process(blocks):
        if len(blocks) == 0:
            return torch.empty(0, dtype=torch.int16)
        pre = min(1, blocks.start)
        seg = whole[(blocks.start - pre) * BB: blocks.stop * BB]
        pcm = oracle.Oracle().run(MODE, 51, seg, ["pcm_mono"])["pcm_mono"]
        return torch.from_numpy(np.ascontiguousarray(pcm[pre * NA:]))

    return process


def leg_with_failure(d, n_streams, world, rank, where):
    """dist.run_leg with rank 1 raising in `where` ("setup" or "process"): every rank must
    return (no rank left in a collective) with the error reported; rank 0 records it."""
    def setup():
        if where == "setup" and rank == 1:
            raise RuntimeError("injected setup failure")
        return list(d.shard(n_streams, world, rank))

    def run(ids):
        if where == "process" and rank == 1:
            raise RuntimeError("injected process failure")
        return process(ids)

    return d.run_leg(setup, run, n_streams, NB * NA * 2, world, rank, True)


def leg_chunked(d, n_streams, world, rank, n_chunks=3):
    """dist.run_leg with the PCM handed over as time chunks (dist.gather_chunked: each chunk
    gathered on its own, rank 0 stitching the columns back)."""
    def run(ids):
        full = process(ids)
        cols = full.shape[1]
        cuts = [cols * k // n_chunks for k in range(n_chunks + 1)]
        return [(cuts[k], full[:, cuts[k]:cuts[k + 1]].contiguous(), None) for k in range(n_chunks)]

    return d.run_leg(lambda: list(d.shard(n_streams, world, rank)), run, n_streams, NB * NA * 2, world, rank, True)


def leg_repeats(d, n_streams, world, rank, repeats=3):
    """dist.run_leg timing the step `repeats` times with a reset between (bench.py's configs[4]
    median of repeats): every repeat gathers; the result carries every repeat's total."""
    resets = []

    def reset(ids):
        resets.append(len(ids))

    res = d.run_leg(lambda: list(d.shard(n_streams, world, rank)), process, n_streams, NB * NA * 2, world, rank,
                    True, repeats=repeats, reset=reset)
    assert len(resets) == repeats - 1, resets
    if rank == 0:
        assert len(res["runs"]) == repeats and res["total"] == sorted(res["runs"])[repeats // 2], res
    return res


def main():
    n_streams, out_path = int(sys.argv[1]), sys.argv[2]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    d = iqgen.load_module("dist")
    if len(sys.argv) > 3 and sys.argv[3] in ("setup", "process", "ok", "chunks", "repeats"):  # dist.run_leg
        res = (leg_chunked(d, n_streams, world, rank) if sys.argv[3] == "chunks"
               else leg_repeats(d, n_streams, world, rank) if sys.argv[3] == "repeats"
               else leg_with_failure(d, n_streams, world, rank, sys.argv[3]))
        if rank == 0:
            if "error" in res:
                np.save(out_path, np.frombuffer(res["error"].encode(), np.uint8))
            else:
                np.save(out_path, res["gathered"].numpy())
        dist.destroy_process_group()
        return
    if len(sys.argv) > 3 and sys.argv[3] == "time":  # argv[1] = blocks of the one stream
        got = d.run_time_sharded(process_time(n_streams), n_streams, NA, world, rank)
    else:
        got = d.run_sharded(process, n_streams, NB * NA * 2, world, rank)
    if rank == 0:
        np.save(out_path, got.numpy())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
