"""Worker for tests/test_gpu_distributed.py: one rank of BASELINE configs[4]'s sharded
multi-stream runner with libfmrx on the GPU (dist.fmrx_process_fn + dist.run_sharded).

    dist_gpu_worker.py <n_streams> <n_blocks> <mode> <channels> <out.npy>

Rendezvous from the env (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT).  Backend gloo: several
ranks share device 0 and the PCM gather goes through host memory (the same sharding, padding
and byte-view gather code as RCCL).  Rank 0 saves the gathered [n_streams, pcm_len] int16 PCM.
Must be started as a fresh process (subprocess.Popen) before anything touches the GPU."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import iqgen  # noqa: E402


def leg(n_streams, seconds, chunks, out_path):
    """dist.streams_leg (bench.py's configs[4] step) over gloo with `chunks` time chunks of
    overlapped gather; rank 0 writes the result line as JSON."""
    import json

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    d = iqgen.load_module("dist")
    geo = fm.geometry(fm.default_config(0, fm.STEREO))
    expect = iqgen.stream_hashes(n_streams, int(seconds * geo.rf_fs * 2 // geo.block_bytes))
    res = d.streams_leg(fm, n_streams, seconds, world, rank, 0, expect=expect, gather_chunks=chunks)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    if sys.argv[1] == "leg":
        leg(int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
        return
    n_streams, n_blocks, mode, channels = (int(a) for a in sys.argv[1:5])
    out_path = sys.argv[5]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    d = iqgen.load_module("dist")
    geo = fm.geometry(fm.default_config(mode, channels))
    pcm_len = n_blocks * geo.pcm_samples
    got = d.run_sharded(d.fmrx_process_fn(fm, mode, channels, n_blocks, device=0), n_streams, pcm_len,
                        world, rank)
    if rank == 0:
        np.save(out_path, got.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
