"""Worker for tests/test_distributed.py: one rank of the sharded multi-stream runner on CPU
(gloo), with the oracle as the per-rank receiver.  Rank 0 saves the gathered PCM to argv[2]."""
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


def main():
    n_streams, out_path = int(sys.argv[1]), sys.argv[2]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    d = iqgen.load_module("dist")
    got = d.run_sharded(process, n_streams, NB * NA * 2, world, rank)
    if rank == 0:
        np.save(out_path, got.numpy())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
