#!/usr/bin/env python3
"""End-to-end drop-in timing: stdin u8 I/Q -> stdout S16, the `fmrx` CLI
(pipelined: pinned ring of 3 batch slots, H2D / receive / D2H overlapped) beside the
reference's own `project` executable (oracle/_ref/project, built from src/*.cpp in place).

    python tools/bench_cli.py [--mib 1024] [--mode 0] [--batch 2048]

Writes the synthetic stream to a file first (untimed), then times each program reading it on
stdin and writing a file.  The reference exits at EOF with blocks still queued
(project.cpp:51-54), so its stereo PCM is checked as a bit-exact PREFIX of fmrx's.  Prints
one JSON line.
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
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--no-reference", action="store_true")
    args = ap.parse_args()

    import iqgen
    import oracle

    fm = iqgen.load_fmrx()
    bb, rf_fs = oracle.MODES[args.mode][0], oracle.MODES[args.mode][3]
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
    ref = os.path.join(REPO, "oracle", "_ref", "project")
    if not args.no_reference and os.path.exists(ref):
        runs.append(("reference_project", [ref, str(args.mode), "2"]))
    for name, cmd in runs:
        dst = os.path.join(tmp, name + ".s16")
        with open(src, "rb") as fi, open(dst, "wb") as fo:
            t0 = time.perf_counter()
            r = subprocess.run(cmd, stdin=fi, stdout=fo, stderr=subprocess.PIPE, timeout=900)
            dt = time.perf_counter() - t0
        # the reference ends with exit(1) at EOF by design (project.cpp:51-54)
        if r.returncode != 0 and name != "reference_project":
            raise SystemExit(f"{name} failed: {r.stderr.decode()[-500:]}")
        outs[name] = np.fromfile(dst, np.int16)
        res[name] = {"seconds": round(dt, 3), "MS_per_s": round(nbytes / 2 / dt / 1e6, 2),
                     "x_realtime": round(nbytes / 2 / rf_fs / dt, 1), "pcm_bytes": int(outs[name].nbytes)}
    if "reference_project" in outs:
        a, b = outs["reference_project"], outs["fmrx_stereo"]
        res["reference_prefix_bit_exact"] = bool(len(a) <= len(b) and np.array_equal(a, b[: len(a)]))
        res["reference_blocks_written"] = int(len(a) // (2 * oracle.MODES[args.mode][2]))
    res["channels1_equals_stereo"] = bool(np.array_equal(outs["fmrx_channels1"], outs["fmrx_stereo"]))
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
