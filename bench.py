#!/usr/bin/env python3
"""bench.py — BASELINE.json headline: IQ Msamples/s (and x real-time) per GPU on the mode-0
mono path, configs[1]: 101-tap RF LPF + 10x decimate + FM demod + 51-tap audio LPF / 5x
decimate -> S16, on 1 GiB of synthetic 2.4 MS/s u8 I/Q resident in HBM.

One "step" = one pass of the fused receive kernel over the whole 1 GiB stream (83,886 full
reference blocks; the 1,024-byte tail is dropped like the reference drops partial blocks).
Multi-GPU: one process per GPU (torch.distributed.run); every rank receives its own
independent stream (weak scaling, no data-path collective); timing is the max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

Prints ONE JSON line on rank 0.  `roofline` prices the fused kernel against HBM (SURVEY
§8d algorithmic bytes: 2 B/IQ in + 2 B per mono audio frame out) from HIP-event kernel
times on the context stream; `compute` gives the same kernel against the FP32 VALU roof.
`cpu_baseline` times the reference's own src/filter.cpp mono path (oracle/_ref, 1 core) on
the same bytes and reports whether its PCM equals the GPU's bit for bit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
VALU_F32_PEAK_TOPS = 78.6      # 157.3 TF FP32 vector / 2: separate mul + add, no FMA
RT_RATE = 2.4e6                # mode 0 real time: 2.4 MS/s complex
STREAM_BYTES = 1 << 30         # BASELINE config 2: 1 GiB synthetic IQ
RF_TAPS = 101


# compiled variants of the fused kernel (csrc/mono_fused.hip kVariants), default index 6
_VARIANTS = ["mono_fused_kernel<101,10,5,256,3,3>", "mono_fused_kernel<101,10,5,128,3,3>",
             "mono_fused_kernel<101,10,5,64,3,3>", "mono_fused_kernel<101,10,5,128,5,3>",
             "mono_fused_kernel<101,10,5,256,3,5>", "mono_fused_kernel<101,10,5,64,3,3,TR=1>",
             "mono_fused_kernel<101,10,5,64,3,4,TR=1>"]


def kernel_name() -> str:
    return _VARIANTS[int(os.environ.get("FMRX_MONO_VARIANT", "6"))]  # csrc kDefaultVariant


KERNEL_SOURCES = ("mono_fused.hip", "dsp_device.h", "mono_launch.h")


def kernel_source_hash() -> str:
    """sha256 over the fused kernel's sources: profiles/traffic_mono101.json carries the hash of
    the sources its PMC passes ran, and bench.py reports `traffic` only while they still match."""
    import hashlib

    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, "software-defined-radio-course-project_amd", "csrc", f), "rb") as g:
            h.update(g.read())
    return h.hexdigest()[:16]


def host_info() -> dict:
    """The host the CPU baselines run on (SURVEY §8d ii): CPU model, nproc, the affinity mask,
    a cgroup CPU quota if any, and the cores the baseline may use.  On the gpurun box nproc and
    the affinity mask show the whole machine; the box's CPU share is exported as
    OMP_NUM_THREADS (16 per GPU), which the all-cores baseline honours."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as g:
                    quota = int(parts[0]) / int(g.read())
            break
        except (OSError, ValueError, IndexError):
            continue
    usable = affinity
    if quota is not None:
        usable = min(usable, max(1, int(quota)))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "cpu_share_env": share, "usable_cores": usable}


def hbm_copy_bandwidth(src, reps: int = 20) -> float:
    """GB/s of a device-to-device copy of `src` (bytes read + bytes written), median of reps."""
    import torch

    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dst.copy_(src)
        b.record()
        b.synchronize()
        times.append(a.elapsed_time(b) * 1e-3)
    del dst
    times.sort()
    return round(2 * src.numel() * src.element_size() / times[len(times) // 2] / 1e9, 1)


def warm_up(step, sync, n_steps: int, min_seconds: float) -> int:
    """Untimed steps: n_steps, continuing until min_seconds of back-to-back work have passed.
    Returns the number of steps run."""
    t0 = time.perf_counter()
    done = 0
    while done < n_steps or time.perf_counter() - t0 < min_seconds:
        for _ in range(min(64, n_steps - done) if done < n_steps else 64):
            step()
            done += 1
        sync()
    return done


def flops_per_iq(rf_taps: int) -> float:
    # per IQ pair: RF 2 ch x taps x (mul+add) / 10, demod ~9/10, audio 51x2/50
    return 2 * rf_taps * 2 / 10 + 0.9 + 51 * 2 / 50


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--min-warmup-seconds", type=float, default=1.0,
                    help="untimed warm-up runs at least this long (clock ramp), besides the W steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-bytes", type=int, default=STREAM_BYTES)
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the extra BASELINE configs (stereo 1 GiB, mode-2 mono at N=1; the 256-stream "
                         "stereo configs[4] at every N)")
    ap.add_argument("--streams-seconds", type=float, default=60.0,
                    help="configs[4] stream length (256 stereo streams sharded over the ranks)")
    ap.add_argument("--gather-chunks", type=int, default=4,
                    help="configs[4] at N > 1: time chunks whose PCM is gathered beside the next one's processing")
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed repeats of configs[2] and configs[4] (median, min, max reported)")
    ap.add_argument("--dry-run", action="store_true",
                    help="the launch only: every rank joins the process group and rank 0 prints n_gpus (no GPU)")
    args = ap.parse_args()

    # --gpus N means N GPUs: without a launcher's WORLD_SIZE, start N ranks under
    # torch.distributed.run as a child process (nothing has touched the GPU yet) and exit with
    # its status; under a launcher, its world size must be N
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {env_world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        sys.exit(dry_run())

    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FMRX_BENCH_BACKEND=gloo rehearses the N>1 path where there are fewer GPUs than ranks
    # (ranks share devices; barriers and the timing reduction go through gloo on the CPU).
    # The data path has no collective either way: every rank owns an independent stream.
    backend = os.environ.get("FMRX_BENCH_BACKEND", "nccl")
    dev = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    import iqgen

    fmrx = iqgen.load_fmrx()
    rx = fmrx.Receiver(0, fmrx.MONO, rf_taps=RF_TAPS, device=dev if world > 1 else 0)
    bb, na = rx.geo.block_bytes, rx.geo.audio_frames
    nb = STREAM_BYTES // bb
    n_iq = nb * bb // 2
    d_iq = torch.empty(STREAM_BYTES, dtype=torch.uint8, device="cuda")
    d_pcm = torch.empty(nb * na, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    rx.synth_device(1000 + rank, 0, STREAM_BYTES // 2, d_iq.data_ptr())  # untimed input gen
    rx.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    # Untimed warm-up: W steps, and at least --min-warmup-seconds of back-to-back steps.  The
    # MI355X raises its clock over ~0.5 s of sustained load (profiles/r02/warmup/: the same
    # kernel takes 0.66 ms per GiB after 3 warm-up steps and 0.57 ms once the clock has ramped,
    # the same 0.57 ms over 1,500 timed steps), so the timed K steps measure the sustained rate.
    warmup_steps_run = warm_up(lambda: rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr()), rx.synchronize,
                               args.warmup, args.min_warmup_seconds)
    rx.kernel_timing(reset=1)  # arm per-launch HIP events on the context stream
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rx.process_device(d_iq.data_ptr(), nb, d_pcm.data_ptr())
    rx.synchronize()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, launches = rx.kernel_timing(reset=-1)
    ranks = None
    if dist is not None:  # every rank's own (seconds, kernel ms): a slow rank shows by name
        dmod = iqgen.load_module("dist")
        ranks = dmod.per_rank([elapsed, kern_ms], True, torch.device("cuda", dev))
        elapsed, kern_ms = max(r[0] for r in ranks), max(r[1] for r in ranks)

    total_iq = n_iq * args.steps * world
    value = total_iq / elapsed / 1e6  # IQ Msamples/s, whole job
    alg_bytes = 2 * n_iq + 2 * nb * na  # per launch: u8 I+Q in, S16 mono out
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    flops = flops_per_iq(RF_TAPS) * n_iq
    line = {
        # value = whole-job aggregate over all ranks (per_gpu_MS_s = value / n_gpus)
        "metric": "IQ Msamples/s (and x real-time) per GPU, mode-0 mono 2.4MS/s->48kS/s",
        "value": round(value, 1),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warmup_steps_run,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "x_realtime_per_gpu": round(value / world * 1e6 / RT_RATE, 1),
        "config": {
            "workload": "BASELINE configs[1]: mode-0 mono, 101-tap RF LPF + 10x decimate + FM demod "
                        "+ 51-tap audio LPF/5x decimate -> S16, 1 GiB synthetic u8 IQ per GPU "
                        "(83,886 reference blocks), device-resident",
            "mode": 0, "channels": 1, "rf_taps": RF_TAPS, "stream_bytes_per_gpu": nb * bb,
            "blocks_per_gpu": nb, "parallelism": f"streams x{world} (one independent stream per GPU)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": kernel_name(),
            "kernel_ms": round(kern_ms, 4),
            "launches_timed": launches,
            "alg_bytes_per_launch": alg_bytes,
        },
        "compute": {
            "bound": "valu_f32_no_fma",
            "achieved": round(flops / (kern_ms * 1e-3) / 1e12, 2),
            "peak": VALU_F32_PEAK_TOPS,
            "unit": "Tflop/s",
            "frac": round(flops / (kern_ms * 1e-3) / 1e12 / VALU_F32_PEAK_TOPS, 4),
            "flop_per_iq": round(flops_per_iq(RF_TAPS), 2),
        },
    }
    # the attainable HBM bandwidth next to the datasheet peak -- a device-to-device
    # copy of the 1 GiB input (read + write counted), after the timed region
    line["roofline"]["hbm_attainable_GBs"] = hbm_copy_bandwidth(d_iq)
    line["roofline"]["frac_of_attainable"] = round(achieved / line["roofline"]["hbm_attainable_GBs"], 4)
    # binding roof: the kernel is bound by the FP32 VALU without FMA (bit parity), not by HBM
    line["roofline"]["binding"] = dict(line["compute"])
    # PMC traffic of record, only while it was measured on this kernel's sources
    traffic_file = os.path.join(REPO, "profiles", "traffic_mono101.json")
    if os.path.exists(traffic_file):
        with open(traffic_file) as f:
            rec = json.load(f)
        if rec.get("kernel") == kernel_name() and rec.get("kernel_source_sha256") == kernel_source_hash():
            line["roofline"]["traffic"] = rec.get("hbm_bytes_per_launch")
            line["roofline"]["traffic_source"] = rec.get("source")
            if rec.get("effective_clock_ghz"):
                line["roofline"]["binding"]["effective_clock_ghz_pmc"] = rec["effective_clock_ghz"]
                line["roofline"]["binding"]["frac_at_effective_clock"] = round(
                    line["compute"]["frac"] * 2.4 / rec["effective_clock_ghz"], 4)
        else:
            line["roofline"]["traffic_note"] = "profiles/traffic_mono101.json is for other kernel sources: not reported"
    line["per_gpu_MS_s"] = round(value / world, 1)
    line["aggregate_MS_s"] = round(value, 1)
    if ranks is not None:
        line["dist"] = {"world_size": dist.get_world_size(),
                        "backend": {"nccl": "RCCL"}.get(dist.get_backend(), dist.get_backend()),
                        "per_rank": [{"rank": r, "seconds": round(v[0], 4), "kernel_ms": round(v[1], 4)}
                                     for r, v in enumerate(ranks)]}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N=1 only
        host = host_info()
        line["cpu_baseline"] = cpu_baseline(d_iq, d_pcm, args.cpu_sample_bytes, bb, na)
        line["cpu_baseline"]["host"] = host
        line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(d_iq, args.cpu_sample_bytes, bb, host["usable_cores"])
        if line["cpu_baseline_all_cores"] is not None:
            line["cpu_baseline_all_cores"]["host"] = host
    if not args.no_other_configs:
        del d_iq, d_pcm
        rx.close()
        torch.cuda.empty_cache()
        line["baseline_configs"] = other_configs(fmrx, args.repeats) if world == 1 else {}
        c4 = streams_config(fmrx, world, rank, dev if world > 1 else 0, args.streams_seconds, args.gather_chunks,
                            args.repeats)
        if rank == 0:
            line["baseline_configs"]["configs[4]"] = c4
            if world == 1 and not args.no_cpu_baseline and isinstance(c4, dict) and "error" not in c4:
                c4["cpu_baseline"] = guarded(cpu_streams_baseline, fmrx, args.streams_seconds, c4)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def relaunch(n: int) -> int:
    """bench.py --gpus n without a launcher: the same command as n ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1), run as a child."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def dry_run() -> int:
    """The launch alone (tests/test_bench_contract.py): every rank joins a gloo process group and
    rank 0 prints the world size it would report as n_gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world}), flush=True)
    return 0


# Serial-chain floors of the PLL runners (the stereo configs are latency-bound), two
# per regime: (1) issue: VALU instructions a step on the runner's critical wave (csrc/pll_pred.hip
# chain4_3 / chain4_5, pll_cnt_kernel, pll_idx_kernel, stereo.hip pll_spec_lane_kernel,
# pll_sat.hip) x ~4.2 cycles a wave64 VALU issue on gfx950 (tools/ubench_dep.hip); (2) latency:
# the step's dependent cycles measured with its data in registers (tools/ubench_cnt.hip, one wave,
# profiles/r05/ubench/ubench_cnt.txt: the index step mode 0, the count step mode 3, the five- and
# three-candidate asm blocks modes 15 / 16; the lane runner is issue-bound, its latency floor
# is its issue floor).  Both at the 2.4 GHz peak engine clock.
CHAIN_VALU_PER_STEP = {"runner_lane": 35.5, "runner_pred": 16.0, "runner_sat": 8.0, "runner_pipe20": 12.0,
                       "runner_pipe21": 12.0, "runner_pipe22": 9.0, "runner_idx17": 11.0, "runner_idx18": 11.0,
                       "runner_idx19": 11.0, "runner_cnt17": 7.0, "runner_cnt18": 7.0, "runner_cnt19": 7.0,
                       "runner_cnt20": 7.0, "runner_cnt21": 7.0, "runner_stick": 9.0}
CHAIN_LATENCY_CYCLES = {"runner_pipe20": 57.5, "runner_pipe21": 57.5, "runner_pipe22": 43.0, "runner_idx17": 91.3,
                        "runner_idx18": 91.3, "runner_idx19": 91.3, "runner_cnt17": 59.8, "runner_cnt18": 59.8,
                        "runner_cnt19": 59.8, "runner_cnt20": 59.8, "runner_cnt21": 59.8, "runner_stick": 43.0}
VALU_ISSUE_CYCLES = 4.2
PEAK_CLOCK_GHZ = 2.4


def stage_latency(rx, run) -> dict:
    """One more call of `run` with fmrx_debug_stage_timing armed: device ms per stage of the
    stereo engine and, per PLL runner regime, ns per serial step against the chain's
    instruction floor (CHAIN_VALU_PER_STEP)."""
    rx.reset()
    rx.stage_timing(1)
    run()
    rx.synchronize()
    st = rx.stage_timing(-1)
    stages = {k: round(v[0], 3) for k, v in st.items()}
    regimes = {}
    for k, (ms, _, steps) in st.items():
        if steps > 0 and k in CHAIN_VALU_PER_STEP:
            ns = ms * 1e6 / steps
            floor = CHAIN_VALU_PER_STEP[k] * VALU_ISSUE_CYCLES / PEAK_CLOCK_GHZ
            lat = max(floor, CHAIN_LATENCY_CYCLES.get(k, 0.0) / PEAK_CLOCK_GHZ)
            regimes[k] = {"steps_per_stream": int(steps), "ns_per_step": round(ns, 2),
                          "floor_ns_per_step": round(floor, 2), "frac": round(floor / ns, 3),
                          "latency_floor_ns_per_step": round(lat, 2), "frac_of_latency_floor": round(lat / ns, 3)}
    runner_ms = sum(v[0] for k, v in st.items() if k.startswith("runner_"))
    return {"bound": "serial PLL chain (one recurrence a stream)", "stage_ms": stages,
            "runner_ms": round(runner_ms, 2), "non_runner_ms": round(sum(v[0] for v in st.values()) - runner_ms, 2),
            "regimes": regimes,
            "floor_note": f"floor: chain VALU a step x {VALU_ISSUE_CYCLES} cycles at {PEAK_CLOCK_GHZ} GHz "
                          "(bench.CHAIN_VALU_PER_STEP); latency_floor: the step's measured dependent cycles with "
                          "its data in registers (bench.CHAIN_LATENCY_CYCLES, tools/ubench_cnt.hip) at the same "
                          "clock; stage ms from HIP events, overlapping stages add up"}


def cpu_reference_stereo(host_iq, gpu_pcm) -> dict:
    """SURVEY §8d CPU plan for configs[2]: the reference's own stereo path (oracle/_ref: the
    sequential project.cpp driver over src/filter.cpp, 1 core) on the same 1 GiB, and the
    reference's two-thread `project 0 2` executable reading it on stdin (it exits at EOF with
    blocks still queued, project.cpp:51-54, so its PCM is compared as a prefix)."""
    import hashlib

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    if not oracle.reference_available():
        return {"error": "oracle/_ref not built"}
    nb = host_iq.size // 12800
    t0 = time.perf_counter()
    pcm = oracle.Reference().run(0, 51, host_iq, ["pcm"])["pcm"]
    dt = time.perf_counter() - t0
    out = {"value": round(host_iq.size / 2 / dt / 1e6, 2), "unit": "MS/s", "cores": 1, "kind": "reference",
           "sample": f"the same {nb} blocks, sequential project.cpp order (oracle/_ref)", "seconds": round(dt, 3),
           "x_realtime": round(host_iq.size / 2 / RT_RATE / dt, 1),
           "bit_exact_vs_gpu": hashlib.sha256(pcm.tobytes()).hexdigest() == hashlib.sha256(gpu_pcm.tobytes()).hexdigest()}
    exe = os.path.join(REPO, "oracle", "_ref", "project")
    if os.path.exists(exe):
        out["threaded_project"] = guarded(threaded_project, exe, host_iq, gpu_pcm)
    return out


def cpu_baseline_stereo_stream(host_iq, h: dict, steps: int, sig: float) -> dict:
    """The CPU baseline of one long stereo stream (tools/bench_unlocked.py: the PLL outside its
    locked regime): the reference's stereo path (oracle/_ref, src/filter.cpp in project.cpp order,
    1 core) on the same bytes, against the reference build's PCM hash of h (hashes.json)."""
    import hashlib

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    if not oracle.reference_available():
        return {"error": "oracle/_ref not built"}
    t0 = time.perf_counter()
    pcm = oracle.Reference().run(h["mode"], h["rf_taps"], host_iq, ["pcm"])["pcm"]
    dt = time.perf_counter() - t0
    return {"seconds": round(dt, 3), "cores": 1, "ns_per_pll_step": round(dt * 1e9 / steps, 1),
            "x_realtime": round(sig / dt, 1), "kind": "reference",
            "bit_exact": hashlib.sha256(pcm.tobytes()).hexdigest() == h["pcm_sha256"],
            "sample": "the whole stream, oracle/_ref (src/filter.cpp in project.cpp order, whole chain)"}


def threaded_project(exe, host_iq, gpu_pcm) -> dict:
    """The reference's two-thread `project 0 2` on the same bytes (stdin file -> stdout file)."""
    import subprocess
    import tempfile

    import numpy as np

    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        src, dst = os.path.join(d, "iq.u8"), os.path.join(d, "pcm.s16")
        host_iq.tofile(src)
        with open(src, "rb") as fi, open(dst, "wb") as fo:
            t0 = time.perf_counter()
            subprocess.run([exe, "0", "2"], stdin=fi, stdout=fo, stderr=subprocess.DEVNULL, timeout=120)
            dt = time.perf_counter() - t0
        got = np.fromfile(dst, np.int16)
    return {"seconds": round(dt, 3), "x_realtime": round(host_iq.size / 2 / RT_RATE / dt, 1), "cores": 2,
            "blocks_written": int(got.size // 256),
            "prefix_bit_exact_vs_gpu": bool(got.size > 0 and np.array_equal(got, gpu_pcm[: got.size])),
            "exit_code_note": "project exits 1 at EOF (project.cpp:51-54), not an error here",
            "sample": "src/project.cpp built as src/Makefile (oracle/_ref/project 0 2), stdin -> file"}


def guarded(fn, *args) -> dict:
    """A CPU-baseline leg that cannot take the GPU results with it: its failure (a timeout, a
    non-zero exit) is recorded under its own key."""
    try:
        return fn(*args)
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)}


def other_configs(fmrx, repeats: int = 5) -> dict:
    """The other single-GPU BASELINE configs, timed on the same box (extra keys; `value` stays
    configs[1]): configs[2] mode-0 stereo as ONE 1 GiB stream in one call (the serial PLL bounds
    it), configs[3] mode-2 mono (147/800 resampler) over 1 GiB, device-resident, synthetic."""
    import torch

    out = {}
    try:
        rx = fmrx.Receiver(0, fmrx.STEREO)
        bb = rx.geo.block_bytes
        nb = STREAM_BYTES // bb
        iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
        pcm = torch.empty(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
        rx.synth_device(3000, 0, nb * bb // 2, iq.data_ptr())
        # warm-up at full size (the first full-size call grows the demod / band-pass / PLL
        # scratch buffers; that allocation must not sit inside the timed call), then restart
        rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        runs = []
        for _ in range(max(1, repeats)):  # each timed call from the power-on state (fmrx_reset)
            rx.reset()
            rx.synchronize()
            t0 = time.perf_counter()
            rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
            rx.synchronize()
            runs.append(time.perf_counter() - t0)
        dt = sorted(runs)[len(runs) // 2]
        sig = nb * bb / 2 / RT_RATE
        out["configs[2]"] = {"workload": f"mode-0 stereo (REF_EXACT), one stream, 1 GiB ({nb} blocks) in one call",
                             "seconds": round(dt, 3), "MS_per_s": round(nb * bb / 2 / dt / 1e6, 1),
                             "x_realtime": round(sig / dt, 1), "runs": [round(x, 4) for x in runs],
                             "median": round(dt, 4), "min": round(min(runs), 4), "max": round(max(runs), 4)}
        par, host_iq, host_pcm = parity_vs_reference("bench_c2_m0_stereo_gib", iq, pcm, keep=True)
        out["configs[2]"].update(par)
        out["configs[2]"]["latency"] = stage_latency(rx, lambda: rx.process_device(iq.data_ptr(), nb, pcm.data_ptr()))
        rx.close()
        del iq, pcm
        torch.cuda.empty_cache()
        out["configs[2]"]["cpu_baseline"] = guarded(cpu_reference_stereo, host_iq, host_pcm)
        del host_iq, host_pcm
        rx = fmrx.Receiver(2, fmrx.MONO)
        bb = rx.geo.block_bytes
        nb = STREAM_BYTES // bb
        iq = torch.empty(nb * bb, dtype=torch.uint8, device="cuda")
        pcm = torch.empty(nb * rx.geo.pcm_samples, dtype=torch.int16, device="cuda")
        rx.synth_device(3001, 0, nb * bb // 2, iq.data_ptr())
        warm_up(lambda: rx.process_device(iq.data_ptr(), nb, pcm.data_ptr()), rx.synchronize, 2, 1.0)
        steps = 10
        rx.kernel_timing(reset=1)
        t0 = time.perf_counter()
        for _ in range(steps):
            rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        dt = (time.perf_counter() - t0) / steps
        kms, _ = rx.kernel_timing(reset=-1)
        na = rx.geo.audio_frames
        n_iq = nb * bb // 2
        alg = nb * bb + 2 * nb * na  # u8 I+Q in, S16 mono out (2.037 B/IQ)
        # flop per IQ (mul and add apart): RF 51 taps x 2 channels / decimation 10,
        # demod ~0.9, the resampler's 51 taps per output at 18,816 outputs per 1,024,000 IQ
        fl = 2 * 51 * 2 / 10 + 0.9 + 51 * 2 * na / (bb // 2)
        out["configs[3]"] = {"workload": f"mode-2 mono, 147/800 polyphase resampler, 1 GiB ({nb} blocks)",
                             "ms_per_step": round(dt * 1e3, 4), "MS_per_s": round(nb * bb / 2 / dt / 1e6, 1),
                             "x_realtime": round(nb * bb / 2 / rx.geo.rf_fs / dt, 1),
                             "roofline": {"bound": "hbm", "kernel": "mono_fused_kernel<51,10,AU=147>",
                                          "kernel_ms": round(kms, 4), "alg_bytes_per_launch": alg,
                                          "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                          "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                          "binding": {"bound": "valu_f32_no_fma", "flop_per_iq": round(fl, 2),
                                                      "achieved": round(fl * n_iq / (kms * 1e-3) / 1e12, 2),
                                                      "peak": VALU_F32_PEAK_TOPS, "unit": "Tflop/s",
                                                      "frac": round(fl * n_iq / (kms * 1e-3) / 1e12 / VALU_F32_PEAK_TOPS, 4)}}}
        # PMC traffic of record (profiles/traffic_mode2.json: warm trace + separate FETCH_SIZE /
        # WRITE_SIZE passes of this kernel), only while it was measured on these kernel sources
        tf = os.path.join(REPO, "profiles", "traffic_mode2.json")
        roof = out["configs[3]"]["roofline"]
        if os.path.exists(tf):
            with open(tf) as f:
                rec = json.load(f)
            if rec.get("kernel_source_sha256") == kernel_source_hash():
                roof["traffic"] = rec.get("hbm_bytes_per_launch")
                roof["traffic_over_alg"] = rec.get("traffic_over_alg")
                roof["trace_kernel_ms"] = rec.get("timed_kernel_ms_trace")
                roof["traffic_source"] = rec.get("source")
            else:
                roof["traffic"] = None
                roof["traffic_note"] = "profiles/traffic_mode2.json is for other kernel sources: not reported"
        # the timed steps carried state from step to step: the parity pass starts fresh
        rx.reset()
        rx.process_device(iq.data_ptr(), nb, pcm.data_ptr())
        rx.synchronize()
        par, host_iq, host_pcm = parity_vs_reference("bench_c3_m2_mono_gib", iq, pcm, keep=True)
        out["configs[3]"].update(par)
        rx.close()
        del iq, pcm
        torch.cuda.empty_cache()
        out["configs[3]"]["cpu_baseline"] = guarded(cpu_reference_mono2, host_iq, host_pcm)
    except Exception as e:  # the headline line must still print
        out["error"] = repr(e)
    return out


def cpu_reference_mono2(host_iq, gpu_pcm) -> dict:
    """configs[3]'s CPU baseline: the reference's mode-2 mono path (oracle/_ref, src/filter.cpp's
    resample with up 147 / down 800, 1 core, sequential) on the same 1 GiB."""
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    if not oracle.reference_available():
        return {"error": "oracle/_ref not built"}
    t0 = time.perf_counter()
    pcm = oracle.Reference().run_mono(2, 51, host_iq)
    dt = time.perf_counter() - t0
    return {"value": round(host_iq.size / 2 / dt / 1e6, 2), "unit": "MS/s", "cores": 1, "kind": "reference",
            "sample": f"the same {host_iq.size // 2048000} blocks, sequential mono path (oracle/_ref)",
            "seconds": round(dt, 3), "bit_exact_vs_gpu": bool(np.array_equal(pcm, gpu_pcm))}


def parity_vs_reference(key: str, d_iq, d_pcm, keep: bool = False):
    """Full-size parity of an extra config, after its timing: SHA-256 of the bench's input and
    of the GPU's PCM against the reference build's over the same bytes (tests/golden/hashes.json
    `bench_*`, written by tests/golden/make_golden.py --bench-only through oracle/_ref)."""
    import hashlib

    with open(os.path.join(REPO, "tests", "golden", "hashes.json")) as f:
        want = json.load(f)[key]
    h_iq, h_pcm = d_iq.cpu().numpy(), d_pcm.cpu().numpy()
    got_in = hashlib.sha256(h_iq.tobytes()).hexdigest()
    got_pcm = hashlib.sha256(h_pcm.tobytes()).hexdigest()
    res = {"input_matches_fixture": got_in == want["input_sha256"],
           "bit_exact_vs_reference": got_in == want["input_sha256"] and got_pcm == want["pcm_sha256"],
           "parity_source": f"tests/golden/hashes.json {key}: reference build (oracle/_ref) "
                            f"{want['field']} SHA-256 over the same {want['n_blocks']} blocks"}
    return (res, h_iq, h_pcm) if keep else res


def streams_config(fmrx, world: int, rank: int, dev: int, seconds: float, gather_chunks: int = 1,
                   repeats: int = 5) -> dict | None:
    """BASELINE configs[4] at this N (extra key; `value` stays configs[1]): 256 independent
    mode-0 stereo streams of `seconds` each, sharded contiguously over the ranks (one process per
    GPU), each rank's shard one device-resident multi-stream call, the S16 PCM gathered to rank 0
    over RCCL (dist.streams_leg); max-over-ranks time of processing + gather.  Rank 0 checks
    streams 0, 127, 128, 255 of the gathered PCM against the reference build's hashes
    (tests/golden/hashes.json streams_c4_60s; other lengths: the streams recorded for them)."""
    import iqgen
    import torch

    dmod = iqgen.load_module("dist")
    # the same geometry streams_leg sizes its run from (mode 0 stereo)
    geo = fmrx.geometry(fmrx.default_config(0, fmrx.STEREO))
    expect = iqgen.stream_hashes(256, int(seconds * geo.rf_fs * 2 // geo.block_bytes)) or None
    try:  # streams_leg agrees on failure across ranks before each collective (dist.run_leg)
        res = dmod.streams_leg(fmrx, 256, seconds, world, rank, dev, expect=expect, profile=stage_latency,
                               gather_chunks=gather_chunks, repeats=repeats)
    except Exception as e:  # the headline line must still print
        res = {"error": repr(e)} if rank == 0 else None
    torch.cuda.empty_cache()
    return res


def _stereo_worker(args):
    """One host core: the reference's stereo path (oracle/_ref) over one configs[4] stream held in
    shared memory (row k of n rows); returns its start / end time and PCM SHA-256."""
    import hashlib
    from multiprocessing import shared_memory

    import numpy as np

    shm_name, k, n_rows, row_bytes, barrier = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    ref = oracle.Reference()
    shm = shared_memory.SharedMemory(name=shm_name)
    try:
        row = np.ndarray((n_rows, row_bytes), np.uint8, shm.buf)[k]
        barrier.wait()
        t0 = time.perf_counter()
        pcm = ref.run(0, 51, row, ["pcm"])["pcm"]
        t1 = time.perf_counter()
        del row
    finally:
        shm.close()
    return t0, t1, hashlib.sha256(pcm.tobytes()).hexdigest()


def cpu_streams_baseline(fmrx, seconds: float, c4: dict) -> dict:
    """configs[4]'s CPU baseline (SURVEY §8d ii): the reference's own stereo path (oracle/_ref,
    src/filter.cpp in project.cpp order) with one stream per usable host core, all at once, on a
    sample of the 256 streams spread over the ids, their PCM checked against the reference build's
    hashes; the 256-stream time on those cores is extrapolated (ceil(256 / cores) rounds of the
    measured wall)."""
    import math
    import multiprocessing as mp
    from multiprocessing import shared_memory

    import numpy as np
    import torch

    import iqgen

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    if not oracle.reference_available():
        return {"error": "oracle/_ref not built"}
    host = host_info()
    cores = max(1, host["usable_cores"])
    ids = [k * 256 // cores for k in range(cores)] if cores < 256 else list(range(256))
    rx = fmrx.Receiver(0, fmrx.STEREO)
    bb = rx.geo.block_bytes
    nb = int(seconds * rx.geo.rf_fs * 2 // bb)
    row_bytes = nb * bb
    expect = iqgen.stream_hashes(256, nb)
    shm = shared_memory.SharedMemory(create=True, size=len(ids) * row_bytes)
    try:
        rows = np.ndarray((len(ids), row_bytes), np.uint8, shm.buf)
        d = torch.empty(row_bytes, dtype=torch.uint8, device="cuda")
        for k, sid in enumerate(ids):  # the inputs, untimed (the same generator as the GPU leg's)
            rx.synth_device(sid, 0, row_bytes // 2, d.data_ptr())
            rx.synchronize()
            rows[k] = d.cpu().numpy()
        del d, rows
        rx.close()
        torch.cuda.empty_cache()
        ctx = mp.get_context("spawn")
        with ctx.Manager() as mgr:
            barrier = mgr.Barrier(len(ids))
            with ctx.Pool(len(ids)) as pool:
                res = pool.map(_stereo_worker, [(shm.name, k, len(ids), row_bytes, barrier) for k in range(len(ids))])
    finally:
        shm.close()
        shm.unlink()
    wall = max(r[1] for r in res) - min(r[0] for r in res)
    per = [r[1] - r[0] for r in res]
    rounds = math.ceil(256 / len(ids))
    est = wall * rounds
    bad = [sid for sid, r in zip(ids, res) if expect.get(sid) is not None and r[2] != expect[sid]]
    return {"value": round(len(ids) * nb * bb / 2 / wall / 1e6, 2), "unit": "MS/s", "cores": len(ids),
            "kind": "reference", "streams_timed": ids,
            "sample": f"{len(ids)} of the 256 streams x {seconds:g} s, one process per usable core, concurrently "
                      "(oracle/_ref: src/filter.cpp in project.cpp order)",
            "seconds_wall": round(wall, 3), "seconds_per_stream_mean": round(sum(per) / len(per), 3),
            "seconds_256_streams_extrapolated": round(est, 2),
            "extrapolation": f"ceil(256 / {len(ids)}) = {rounds} rounds of the measured wall on {len(ids)} cores",
            "gpu_speedup_vs_extrapolated": round(est / c4["seconds"], 1) if c4.get("seconds") else None,
            "bit_exact_vs_reference": not bad and all(expect.get(sid) for sid in ids),
            "mismatched_streams": bad, "host": host}


def cpu_baseline(d_iq, d_pcm, sample_bytes, bb, na):
    """The reference's own mono path (oracle/_ref: src/filter.cpp + src/iofunc.cpp, g++ -O3,
    sequential project.cpp order, 1 core) on the first `sample_bytes` of the same stream."""
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    nbs = sample_bytes // bb
    host = d_iq[: nbs * bb].cpu().numpy()
    if oracle.reference_available():
        ref, kind = oracle.Reference(), "reference"
        t0 = time.perf_counter()
        pcm = ref.run_mono(0, RF_TAPS, host)
    else:
        ref, kind = oracle.Oracle(), "port"
        t0 = time.perf_counter()
        pcm = ref.run(0, RF_TAPS, host, ["pcm_mono"])["pcm_mono"]
    dt = time.perf_counter() - t0
    # The GPU's last step re-processed the same 1 GiB with carried state, so compare the
    # first sample from a fresh context.
    import iqgen

    fm = iqgen.load_fmrx()
    fresh = fm.Receiver(0, fm.MONO, rf_taps=RF_TAPS)
    out = d_pcm.new_empty(nbs * na)
    fresh.process_device(d_iq.data_ptr(), nbs, out.data_ptr())
    fresh.synchronize()
    parity = bool(np.array_equal(out.cpu().numpy(), pcm))
    fresh.close()
    return {"value": round(nbs * bb / 2 / dt / 1e6, 2), "unit": "MS/s", "cores": 1, "kind": kind,
            "sample": f"first {nbs} blocks ({nbs * bb} B, {nbs * bb / 2 / RT_RATE:.1f} s of signal) "
                      f"of the rank-0 stream, sequential mono path",
            "seconds": round(dt, 2), "bit_exact_vs_gpu": parity}


def _ref_worker(args):
    """One host core: the reference mono path over one contiguous slice (its own stream)."""
    chunk, barrier = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    ref = oracle.Reference()
    barrier.wait()
    t0 = time.perf_counter()
    ref.run_mono(0, RF_TAPS, chunk)
    return t0, time.perf_counter()


def cpu_baseline_all_cores(d_iq, sample_bytes, bb, cores):
    """the reference's mono path with one stream per host core, all at once.
    The GiB is cut into one contiguous slice per core (each slice an independent stream, so
    only the timing is meaningful); spawned processes, no GPU.  Rate = bytes / wall span."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    if not oracle.reference_available():
        return None
    cores = max(1, cores)  # host_info()["usable_cores"]
    nbs = sample_bytes // bb
    host = d_iq[: nbs * bb].cpu().numpy()
    per = nbs // cores
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        barrier = mgr.Barrier(cores)
        with ctx.Pool(cores) as pool:
            spans = pool.map(_ref_worker, [(host[i * per * bb:(i + 1) * per * bb], barrier) for i in range(cores)])
    dt = max(t1 for _, t1 in spans) - min(t0 for t0, _ in spans)
    return {"value": round(cores * per * bb / 2 / dt / 1e6, 2), "unit": "MS/s", "cores": cores, "kind": "reference",
            "sample": f"{cores} contiguous slices of {per} blocks, one process per core, concurrently",
            "seconds": round(dt, 3)}


if __name__ == "__main__":
    main()
