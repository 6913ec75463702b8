#!/usr/bin/env python3
"""configs[4] (256 stereo streams x 60 s, one GPU) with its demotion record: how many locked streams
the runners demote (pll_demote) and what the call costs -- for A/B builds of the demotion rule
(FMRX_LIB_PATH).  One JSON line.

    python tools/demote_probe.py [--seconds 60] [--repeats 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--profile", action="store_true", help="one more call with the stage timer: ns a step per regime")
    args = ap.parse_args()
    import torch

    import iqgen

    torch.cuda.set_device(0)
    fm = iqgen.load_fmrx()
    dmod = iqgen.load_module("dist")
    nb = int(args.seconds * 2400000 * 2 // 12800)
    prof = None
    if args.profile:
        sys.path.insert(0, REPO)
        import bench
        prof = bench.stage_latency
    res = dmod.streams_leg(fm, 256, args.seconds, 1, 0, 0, expect=iqgen.stream_hashes(256, nb) or None,
                           repeats=args.repeats, profile=prof)
    r = res.get("redos", {})
    lat = res.get("latency") or {}
    print(json.dumps({"lib": fm.LIB_PATH, "median": res.get("median"), "runs": res.get("runs"),
                      "bit_exact": res.get("bit_exact_vs_reference"), "demoted_streams": r.get("demoted_streams"),
                      "demoted_steps_per_range": r.get("demoted_steps_per_range"),
                      "redos_total_per_range": r.get("total_per_range"),
                      "regimes_ns": {k: v["ns_per_step"] for k, v in (lat.get("regimes") or {}).items()},
                      "stage_ms": lat.get("stage_ms")}), flush=True)


if __name__ == "__main__":
    main()
