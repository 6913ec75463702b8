"""Multi-process sharding + gather (BASELINE configs[4]) on CPU: world_size 2, gloo.

The per-rank work is the oracle (CPU) instead of libfmrx (GPU); the sharding, padding and
gather code is the same code path the GPU runner uses over RCCL."""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import iqgen
import oracle

MODE, NB, BB, NA = 0, 2, 12800, 128
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_balanced_and_covering():
    d = iqgen.load_module("dist")
    for n in (1, 5, 8, 31, 256):
        for w in (1, 2, 3, 8):
            rs = [d.shard(n, w, r) for r in range(w)]
            assert [i for r in rs for i in r] == list(range(n))
            assert max(map(len, rs)) - min(map(len, rs)) <= 1


def _run_world2(tmp_path, *args):
    port = _free_port()
    out = tmp_path / "pcm.npy"
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(args[0]),
                                       str(out)] + [str(a) for a in args[1:]], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    return np.load(out)


@pytest.mark.parametrize("n_streams", [5, 2, 1])
def test_gather_world2_matches_serial(n_streams, orc, tmp_path):
    got = _run_world2(tmp_path, n_streams)
    want = np.stack([orc.run(MODE, 51, iqgen.make(f"rand:{100 + i}", NB * BB), ["pcm"])["pcm"]
                     for i in range(n_streams)])
    assert got.shape == want.shape and np.array_equal(got, want)


@pytest.mark.parametrize("n_blocks", [7, 2, 1])
def test_time_shards_world2_match_whole_stream(n_blocks, orc, tmp_path):
    """One recording cut in time over 2 ranks (dist.run_time_sharded): every rank restarts from
    the bytes in front of its shard, and the gathered mono PCM equals the whole stream's."""
    got = _run_world2(tmp_path, n_blocks, "time")
    whole = iqgen.make("synth:77", n_blocks * BB)
    want = orc.run(MODE, 51, whole, ["pcm_mono"])["pcm_mono"]
    assert got.shape == want.shape and np.array_equal(got, want)


@pytest.mark.parametrize("where", ["setup", "process"])
def test_run_leg_failure_on_one_rank_does_not_hang(where, tmp_path):
    """A rank that raises before the barrier or before the gather (bench.py's configs[4] step at
    N > 1) must not leave the other rank blocked in the collective: dist.run_leg agrees on
    success first, both ranks return, and rank 0 reports the failing rank's error."""
    got = _run_world2(tmp_path, 3, where)
    msg = got.tobytes().decode()
    assert "injected" in msg or "another rank failed" in msg, msg


def test_run_leg_world2_gathers(orc, tmp_path):
    got = _run_world2(tmp_path, 3, "ok")
    want = np.stack([orc.run(MODE, 51, iqgen.make(f"rand:{100 + i}", NB * BB), ["pcm"])["pcm"] for i in range(3)])
    assert np.array_equal(got, want)


def test_run_leg_world2_gathers_time_chunks(orc, tmp_path):
    """The chunked gather (dist.gather_chunked, bench.py's configs[4] at N > 1): each rank hands
    over its PCM as three time chunks, gathered one by one; rank 0 stitches the same PCM."""
    got = _run_world2(tmp_path, 3, "chunks")
    want = np.stack([orc.run(MODE, 51, iqgen.make(f"rand:{100 + i}", NB * BB), ["pcm"])["pcm"] for i in range(3)])
    assert np.array_equal(got, want)


def test_run_leg_world2_repeats(orc, tmp_path):
    """The timed step repeated (bench.py's configs[4] median of five): reset between repeats, every
    repeat gathers, the median repeat's times reported beside all of them; the same PCM."""
    got = _run_world2(tmp_path, 3, "repeats")
    want = np.stack([orc.run(MODE, 51, iqgen.make(f"rand:{100 + i}", NB * BB), ["pcm"])["pcm"] for i in range(3)])
    assert np.array_equal(got, want)
