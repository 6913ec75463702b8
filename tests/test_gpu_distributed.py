"""BASELINE configs[4] on the GPU: independent stereo streams sharded over ranks, PCM gathered
to rank 0 (dist.run_sharded over libfmrx, the path bench/SCALE runs on 8 GPUs).

* gloo, world size 2, both ranks on device 0 (one GPU per box here): the GPU per-rank worker
  (dist.fmrx_process_fn: device synthesis, one multi-stream context per rank), the shard
  padding and the int16-as-bytes gather, against the oracle per stream;
* RCCL, world size 1: tools/bench_streams.py under torch.distributed.run (RCCL init, the
  device-side gather, its --check against single-stream contexts).
Ranks are fresh processes (subprocess.Popen), started from a parent that only spawns them.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import iqgen
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_world(tmp_path, world, *args, out_name="pcm.npy"):
    port = _free_port()
    out = tmp_path / out_name
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_worker.py")]
                                      + [str(a) for a in args] + [str(out)], env=env))
    try:
        for p in procs:
            assert p.wait(timeout=240) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return out


@pytest.mark.parametrize("n_streams,n_blocks,check", [(256, 4, (0, 127, 128, 255)), (5, 3, (0, 2, 3, 4))])
def test_configs4_sharded_stereo_world2_gloo(fmrx, orc, tmp_path, n_streams, n_blocks, check):
    got = np.load(_gpu_world(tmp_path, 2, n_streams, n_blocks, 0, fmrx.STEREO))
    bb, na = 12800, 128
    assert got.shape == (n_streams, n_blocks * na * 2)
    for sid in check:
        iq = fmrx.synth_host(sid, 2400000, 0, n_blocks * bb // 2)
        want = orc.run(0, 51, iq, ["pcm"])["pcm"]
        assert np.array_equal(got[sid], want), sid
    # streams are distinct (the gather did not replicate a shard)
    assert not np.array_equal(got[0], got[-1])


def test_configs4_rccl_one_rank_bench_streams(fmrx):
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(REPO, "tools", "bench_streams.py"), "--streams", "16", "--seconds", "0.5", "--check"]
    r = subprocess.run(cmd, capture_output=True, timeout=240, env=dict(os.environ))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    line = [l for l in r.stdout.decode().splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["backend"] == "RCCL"
    assert res["gather_bytes"] == 16 * int(0.5 * 2400000 * 2 // 12800) * 256 * 2
    # the gathered PCM against the reference build's hashes (tests/golden/hashes.json
    # streams_c4_short), not against another GPU run
    assert res["checked_streams"] == [0, 7, 8, 15] and res["bit_exact_vs_reference"] is True


@pytest.mark.parametrize("chunks", [1, 3])
def test_configs4_leg_world2_gloo_time_chunks(tmp_path, chunks):
    """dist.streams_leg as bench.py runs configs[4] at N > 1, rehearsed with gloo on one device:
    16 streams x 0.5 s in `chunks` time chunks, each chunk's PCM gathered as soon as its CUDA
    event completes (dist.gather_chunked) while the next chunk is processed; the stitched PCM
    equals the reference build's hashes (tests/golden/hashes.json streams_c4_short)."""
    path = _gpu_world(tmp_path, 2, "leg", 16, 0.5, chunks, out_name="leg.json")
    res = json.loads(path.read_text())
    assert res["gather_chunks"] == chunks and res["n_gpus"] == 2, res
    assert res["checked_streams"] == [0, 7, 8, 15] and res["bit_exact_vs_reference"] is True, res
    assert res["gather_bytes_sent_per_rank"] == 8 * int(0.5 * 2400000 * 2 // 12800) * 256 * 2
