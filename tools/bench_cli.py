#!/usr/bin/env python3
"""End-to-end drop-in timing: stdin u8 I/Q -> stdout S16, the `fmrx` CLI
(pipelined: pinned ring of 3 batch slots, H2D / receive / D2H overlapped).

    python tools/bench_cli.py [--mib 1024] [--mode 0] [--batch 2048]

Writes the synthetic stream to a file first (untimed), then times each CLI form reading it on
stdin and writing a file.  Prints one JSON line.  The reference's own `project` on the same
1 GiB stream is timed by bench.py's cpu_baseline leg (configs[2] "threaded_project"), the only
place a measurement runs anything under oracle/; its stereo bytes are compared with the CLI's
in tests/test_gpu_parity.py (test_cli_*).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()

    import iqgen

    fm = iqgen.load_fmrx()
    geo = fm.geometry(fm.default_config(args.mode, fm.STEREO))
    bb, rf_fs = geo.block_bytes, geo.rf_fs
    nbytes = args.mib << 20
    tmp = tempfile.mkdtemp(prefix="fmrx_cli_", dir="/tmp")
    src = os.path.join(tmp, "iq.u8")
    chunk = 32 << 20  # pairs per piece
    with open(src, "wb") as f:
        for p0 in range(0, nbytes // 2, chunk):
            f.write(fm.synth_host(5, rf_fs, p0, min(chunk, nbytes // 2 - p0)).tobytes())
    exe = os.path.join(os.path.dirname(fm.LIB_PATH), "bin", "fmrx")
    res = {"config": f"mode {args.mode}, {args.mib} MiB synthetic u8 I/Q on stdin -> S16 on stdout",
           "blocks": nbytes // bb, "batch_blocks": args.batch}
    outs = {}
    # `fmrx <mode> 1` writes project's R,L stream like `<mode> 2` (project.cpp:179-195); the
    # 1-channel mono product is the --mono-product extension
    runs = [("fmrx_stereo", [exe, str(args.mode), "2", "--batch", str(args.batch)]),
            ("fmrx_channels1", [exe, str(args.mode), "1", "--batch", str(args.batch)]),
            ("fmrx_mono_product", [exe, str(args.mode), "1", "--mono-product", "--batch", str(args.batch)])]
    for name, cmd in runs:
        dst = os.path.join(tmp, name + ".s16")
        with open(src, "rb") as fi, open(dst, "wb") as fo:
            t0 = time.perf_counter()
            r = subprocess.run(cmd, stdin=fi, stdout=fo, stderr=subprocess.PIPE, timeout=900)
            dt = time.perf_counter() - t0
        if r.returncode != 0:
            raise SystemExit(f"{name} failed: {r.stderr.decode()[-500:]}")
        outs[name] = np.fromfile(dst, np.int16)
        res[name] = {"seconds": round(dt, 3), "MS_per_s": round(nbytes / 2 / dt / 1e6, 2),
                     "x_realtime": round(nbytes / 2 / rf_fs / dt, 1), "pcm_bytes": int(outs[name].nbytes)}
    res["channels1_equals_stereo"] = bool(np.array_equal(outs["fmrx_channels1"], outs["fmrx_stereo"]))
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
