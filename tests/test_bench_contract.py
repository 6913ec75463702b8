"""bench.py's output contract (the driver parses this line every round): one JSON line with
the metric, whole-job value, timing fields, roofline and the CPU baseline keys.  A short run
(2 steps, 1 warmup) on the GPU, in a child process (it owns the device while it runs)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(*extra):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1", *extra],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_json_contract():
    j = _run("--no-cpu-baseline", "--streams-seconds", "0.5")
    for k, t in (("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int),
                 ("warmup", int), ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str),
                 ("dtype", str), ("data", str), ("config", dict), ("roofline", dict)):
        assert isinstance(j[k], t), k
    assert j["n_gpus"] == 1 and j["steps"] == 2 and j["warmup"] == 1 and j["scaling"] == "weak"
    assert j["vs_baseline"] is None and j["higher_is_better"] is True
    assert "workload" in j["config"]
    oc = j["baseline_configs"]  # the other single-GPU BASELINE configs, same box
    assert "error" not in oc, oc
    assert oc["configs[2]"]["x_realtime"] > 1 and oc["configs[3]"]["MS_per_s"] > 0
    # configs[2] and configs[4] timed five times each (bench.py --repeats): median, min, max
    for c in ("configs[2]", "configs[4]"):
        r = oc[c]
        assert len(r["runs"]) == 5 and r["min"] <= r["median"] <= r["max"], r
    assert oc["configs[2]"]["seconds"] == round(oc["configs[2]"]["median"], 3)
    # full-size parity of both extra configs against the reference build's PCM hashes of the
    # same bytes (tests/golden/hashes.json bench_*): /root/reference/src/project.cpp:132-196
    for c in ("configs[2]", "configs[3]"):
        assert oc[c]["input_matches_fixture"] is True, oc[c]
        assert oc[c]["bit_exact_vs_reference"] is True, oc[c]
        # every config carries its CPU baseline (the reference's own path, oracle/_ref, same bytes)
        cb = oc[c]["cpu_baseline"]
        assert cb["kind"] == "reference" and cb["cores"] == 1 and cb["value"] > 0 and cb["bit_exact_vs_gpu"] is True, cb
    assert oc["configs[2]"]["cpu_baseline"]["threaded_project"]["prefix_bit_exact_vs_gpu"] is True
    # configs[3] priced against HBM and the no-FMA VALU like the headline; the stereo configs
    # against the serial chain's instruction floor per PLL regime
    r3 = oc["configs[3]"]["roofline"]
    assert 0 < r3["frac"] < 1 and 0 < r3["binding"]["frac"] < 1 and r3["kernel_ms"] > 0
    # its PMC traffic only with the stamp of the kernel sources that ran (profiles/traffic_mode2.json)
    assert r3.get("traffic") is None or (r3["traffic_source"] and 1.0 <= r3["traffic_over_alg"] < 1.1), r3
    for c in ("configs[2]", "configs[4]"):
        lat = oc[c]["latency"]
        assert lat["runner_ms"] > 0 and lat["regimes"], lat
        for k, r in lat["regimes"].items():
            assert k.startswith("runner_") and 0 < r["frac"] <= 1.0 and r["ns_per_step"] > r["floor_ns_per_step"], (k, r)
            # and against the chain's measured dependent latency (tools/ubench_cnt.hip)
            assert r["latency_floor_ns_per_step"] >= r["floor_ns_per_step"] and 0 < r["frac_of_latency_floor"] <= 1.0, (k, r)
    # configs[4] (256 stereo streams; 0.5 s each here, 60 s by default) checked against the
    # reference build's per-stream hashes
    c4 = oc["configs[4]"]
    assert "error" not in c4, c4
    assert c4["n_gpus"] == 1 and c4["checked_streams"] == [0, 7, 8, 15] and c4["bit_exact_vs_reference"] is True
    # the self-certifying runners' redone intervals per stream, from the untimed warm-up call
    assert c4["redos"]["streams"] == 256 and len(c4["redos"]["worst_streams"]) == 8, c4.get("redos")
    # each rank's own split (one rank here) and the process group it ran in
    assert c4["dist"]["world_size"] == 1 and len(c4["per_rank"]) == 1 and c4["per_rank"][0]["streams"] == 256
    rf = j["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] in ("GB/s", "TFLOP/s")
    assert 0 < rf["frac"] < 1 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # value = IQ pairs of the whole job / wall time; the kernel alone is faster than a step
    assert j["value"] > 1e5 and rf["kernel_ms"] <= j["ms_per_step"] * 1.05
    # the binding roof next to HBM; per-GPU and aggregate rates spelled out
    assert rf["binding"]["bound"] == "valu_f32_no_fma" and 0 < rf["binding"]["frac"] < 1
    assert j["aggregate_MS_s"] == j["value"] and j["per_gpu_MS_s"] == round(j["value"] / j["n_gpus"], 1)
    # the attainable HBM bandwidth (device copy) sits below the datasheet peak
    assert 1000 < rf["hbm_attainable_GBs"] < 1.1 * rf["peak"]
    # traffic only with the stamp of the kernel sources that ran
    if rf["traffic"] is not None:
        assert rf["traffic_source"]


def test_bench_cpu_baseline_keys():
    j = _run("--cpu-sample-bytes", str(64 * 12800), "--no-other-configs")
    cb = j["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["cores"] == 1 and cb["value"] > 0
    assert cb["bit_exact_vs_gpu"] is True
    for key in ("cpu_baseline", "cpu_baseline_all_cores"):
        h = j[key]["host"]
        assert h["nproc"] >= 1 and h["cpu_model"] and 1 <= h["usable_cores"] <= h["affinity_cpus"]
    assert j["cpu_baseline_all_cores"]["cores"] == j["cpu_baseline_all_cores"]["host"]["usable_cores"]
