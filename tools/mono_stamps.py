#!/usr/bin/env python3
"""Clock and occupancy stamps of the fused mono kernel (bench workload: mode 0, 101-tap RF,
1 GiB device-resident).  After ~2 s of back-to-back launches (steady clock), one launch with
per-workgroup stamps (fmrx_debug_mono_stamps: shader clock and 100 MHz counters at the start
and end of each workgroup's work, HW_ID, XCC_ID; MI355X_MICROARCH.md DVFS item 6):

  * in-kernel clock = d(s_memtime) / d(s_memrealtime) x 100 MHz, median over workgroups;
  * workgroup lifetimes against the launch's span (start / end spread, idle tail);
  * the same per XCD.

    python tools/mono_stamps.py [--warm-seconds 2] > profiles/r02/mono_stamps.json
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
    ap.add_argument("--warm-seconds", type=float, default=2.0)
    ap.add_argument("--idle", action="store_true", help="stamp a launch that follows a sync (boost clock)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import iqgen

    fm = iqgen.load_fmrx()
    rx = fm.Receiver(0, fm.MONO, rf_taps=101)
    bb, na = rx.geo.block_bytes, rx.geo.audio_frames
    nb = (1 << 30) // bb
    iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
    pcm = torch.empty(nb * na, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rx.synth_device(1000, 0, nb * bb // 2, iq.data_ptr())
    rx.synchronize()
    need = rx.debug_mono_stamps(None)
    st = torch.zeros(6 * need, dtype=torch.int64, device="cuda")
    t0 = time.perf_counter()
    launches = 0
    while time.perf_counter() - t0 < args.warm_seconds:
        for _ in range(50):
            rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        launches += 50
    # steady state: the stamped launch is the last of 40 back-to-back launches (no idle gap
    # in front of it, as in bench.py's timed loop); --idle stamps a launch after a sync instead
    if not args.idle:
        for _ in range(40):
            rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        launches += 40
    rx.debug_mono_stamps(st.data_ptr(), need)
    rx.kernel_timing(reset=1)  # HIP events around the stamped launch on the context stream
    rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
    rx.synchronize()
    ev_ms, _ = rx.kernel_timing(reset=-1)
    rx.debug_mono_stamps(None)
    a = st.cpu().numpy().reshape(-1, 6).astype(np.int64)
    a = a[a[:, 3] > 0]  # workgroups that ran
    t0c, t1c, r0, r1, hw, xcc = (a[:, i] for i in range(6))
    clk = (t1c - t0c) / np.maximum(r1 - r0, 1) * 0.1  # GHz (100 MHz realtime counter)
    span = (r1.max() - r0.min()) * 10.0  # ns
    life = (r1 - r0) * 10.0
    out = {
        "workload": "bench.py configs[1]: mode-0 mono, 101-tap RF, 1 GiB, one stamped launch after "
                    f"{launches} warm launches ({args.warm_seconds} s), "
                    + ("after a sync (idle in front)" if args.idle else "the last of 41 back-to-back launches"),
        "workgroups": int(len(a)),
        "clock_ghz_median": round(float(np.median(clk)), 3),
        "clock_ghz_p05_p95": [round(float(np.percentile(clk, 5)), 3), round(float(np.percentile(clk, 95)), 3)],
        "launch_span_us": round(span / 1e3, 2),
        "hip_event_kernel_us": round(ev_ms * 1e3, 2),
        "wg_lifetime_us_median": round(float(np.median(life)) / 1e3, 2),
        "wg_lifetime_over_span_mean": round(float(life.mean() / span), 4),
        "start_spread_us": round(float((r0.max() - r0.min()) * 10.0) / 1e3, 2),
        "end_spread_us": round(float((r1.max() - r1.min()) * 10.0) / 1e3, 2),
        "end_p05_p50_p95_us_from_first_start": [round(float(np.percentile((r1 - r0.min()) * 10.0, q)) / 1e3, 2)
                                                for q in (5, 50, 95)],
        "per_xcc": {},
    }
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        out["per_xcc"][int(x)] = {"workgroups": int(m.sum()), "clock_ghz_median": round(float(np.median(clk[m])), 3),
                                  "end_us_max": round(float((r1[m].max() - r0.min()) * 10.0) / 1e3, 2),
                                  "lifetime_us_median": round(float(np.median(life[m])) / 1e3, 2)}
    cu = (hw >> 8) & 0xF  # gfx9 HW_ID: CU_ID bits 11:8, SH_ID 12, SE_ID 15:13, SIMD 5:4
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    slots = {}
    for x, s_, c_, sm in zip(xcc.tolist(), se.tolist(), cu.tolist(), simd.tolist()):
        slots[(x, s_, c_, sm)] = slots.get((x, s_, c_, sm), 0) + 1
    v = np.array(list(slots.values()))
    out["waves_per_simd_hist"] = {int(k): int((v == k).sum()) for k in sorted(set(v.tolist()))}
    # the two waves of each SIMD: does the first-dispatched one finish first, and by how much?
    wave_id = hw & 0xF
    groups = {}
    for i, key in enumerate(zip(xcc.tolist(), se.tolist(), cu.tolist(), simd.tolist())):
        groups.setdefault(key, []).append(i)
    first_ends_first, slot0_ends_first, lowid_ends_first, n2 = 0, 0, 0, 0
    e_old, e_young, gap = [], [], []
    wg = np.nonzero(st.cpu().numpy().reshape(-1, 6)[:, 3] > 0)[0]
    for idx in groups.values():
        if len(idx) != 2:
            continue
        n2 += 1
        a_, b_ = idx
        old, young = (a_, b_) if t0c[a_] <= t0c[b_] else (b_, a_)
        e_old.append((r1[old] - r0.min()) * 10.0 / 1e3)
        e_young.append((r1[young] - r0.min()) * 10.0 / 1e3)
        gap.append(abs(int(r1[a_]) - int(r1[b_])) * 10.0 / 1e3)
        first_ends_first += r1[old] <= r1[young]
        s0 = a_ if wave_id[a_] < wave_id[b_] else b_
        slot0_ends_first += r1[s0] <= r1[a_ + b_ - s0]
        lo = a_ if wg[a_] < wg[b_] else b_
        lowid_ends_first += r1[lo] <= r1[a_ + b_ - lo]
    out["simd_pairs"] = {
        "pairs": n2,
        "first_started_ends_first": int(first_ends_first),
        "lower_wave_slot_ends_first": int(slot0_ends_first),
        "lower_workgroup_id_ends_first": int(lowid_ends_first),
        "end_us_first_started_mean": round(float(np.mean(e_old)), 2) if e_old else None,
        "end_us_second_started_mean": round(float(np.mean(e_young)), 2) if e_young else None,
        "end_gap_us_mean": round(float(np.mean(gap)), 2) if gap else None,
    }
    ids = wg
    out["end_us_mean_by_wg_id_quarter"] = [round(float(np.mean((r1[(ids >= q * len(ids) // 4) & (ids < (q + 1) * len(ids) // 4)] - r0.min()) * 10.0)) / 1e3, 2) for q in range(4)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
