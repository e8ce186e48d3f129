"""bench.py's contract on the GPU: the N = 1 line, and the N > 1 row-partitioned path
rehearsed with two ranks on the one MI355X over gloo (RCCL refuses two ranks on one device;
the 8-GPU RCCL run is the driver's). Fresh child processes under torch.distributed.run, as
the driver launches them."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_gpu_line(cuda):
    r = subprocess.run([sys.executable, "bench.py", "--config", "geotext", "--steps", "3",
                        "--warmup", "1", "--no-train-step", "--no-cpu-baseline"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "variants", "dense_kernels"):
        assert key in rec, key
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["warmup"] == 1
    rf = rec["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rec["value_kind"] == "edge-centric"
    # the live PMC pass ran (rocprofv3 child processes): frac is measured bytes / kernel time
    assert "traffic" in rf["live_pmc"], rf["live_pmc"]
    assert rf["traffic"] == rf["live_pmc"]["traffic"] > 0 and 0 < rf["frac"] <= 1
    assert rf["edge_centric_achieved"] > 0 and rf["frac_vs_achievable"] > 0
    # the same launch under rocprofv3 --kernel-trace in the same run backs the kernel time
    assert rf["kernel_trace_ms"] > 0 and rf["kernel_trace"]["dispatches"] >= 1, rf.get("kernel_trace")
    assert "kernel_trace_le_step" in rf
    assert rec["variants"]["uniform"]["roofline"]["traffic"] > 0
    assert rec["variants"]["uniform"]["kernel_ms"] > 0 and rec["variants"]["k1500"]["kernel_ms"] > 0
    # the like-for-like point of the scaling series: the same SpMM in the mode N > 1 runs
    if not rec["config"]["mode"].endswith("fast"):
        assert rec["variants"]["fast"]["mode"] == "fast" and rec["variants"]["fast"]["kernel_ms"] > 0
    assert "mode_resolution" in rec["config"]
    dk = {k: v for k, v in rec["dense_kernels"].items() if isinstance(v, dict)}
    assert len(dk) == 8 and all(v["TFLOPs"] > 0 and v["frac"] < 1 for v in dk.values())
    assert sum(v.get("math") == "bf16x6" for v in dk.values()) == 4  # NT x 2, TN, fused


def test_bench_two_ranks_gloo(cuda):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--config", "twitter-us", "--steps", "3", "--warmup", "1",
           "--dist-backend", "gloo", "--exchange-ab"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=500, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    # the headline line is out before any extra: the exchange A/B follows as one 'ALT' line
    lines = r.stdout.splitlines()
    head = next(i for i, ln in enumerate(lines) if ln.startswith("{"))
    alt_at = [i for i, ln in enumerate(lines) if ln.startswith("ALT ")]
    assert len(alt_at) == 1 and alt_at[0] > head
    alt = json.loads(lines[alt_at[0]][4:])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "row2"
    # one mode for every rank and every N: the whole graph's
    assert rec["config"]["mode_resolution"].startswith("the whole graph")
    assert rec["config"]["mode"].split("->")[1] in ("fast", "ordered", "rowwise")
    d = rec["distributed"]
    assert d["world_size"] == 2 and d["backend"] == "gloo"
    for key in ("exchange", "exchange_ms", "local_spmm_ms", "comm_fraction"):
        assert key in d, key
    assert d["exchange_ms"] > 0 and d["local_spmm_ms"] > 0
    # the chunk-count calibration rides in the headline line (same exchange, 1/2/4 chunks)
    ab = d["chunks_ab"]
    assert set(ab["ms_per_step"]) == {"1", "2", "4"} and all(v > 0 for v in ab["ms_per_step"].values())
    assert set(ab["model_ms"]) == {"1", "2", "4"} and ab["chosen"] == d["chunks"]
    assert d["xgmi_link_GBps_fit"] > 0 and d["xgmi_links"] == 1
    assert "alternatives" not in rec
    assert "feature_parallel" in alt and "exchange_halo" in alt, alt
