#!/usr/bin/env python
"""Benchmark of the graphconvgeo hot path on MI355X: the GCN normalized-adjacency SpMM.

Metric (BASELINE.json): "GCN SpMM fwd GB/s (achieved HBM) + edges/s, Twitter-World graph,
1/2/4/8 GPU". One step = one forward SpMM Y = H . Z over the whole Twitter-World-scale
synthetic graph (N = 1.4M users, E = 20M edges, nnz(H) = 2E + N, hidden K = 300, fp32),
the S.dot(H, .) of mlpconv.py:73. Inputs are resident in HBM before the timed region.

  value     = algorithmic bytes per step / step time (GB/s), bytes per SURVEY.md §8d:
              B = 4(N+1) + 8 nnz + 4 K nnz + 4 K N
  edges/s   = nnz(H) / step time
  N > 1     : H row-partitioned (nnz-balanced) over N ranks, each step = RCCL exchange of Z
              over xGMI (all-gather, or halo all-to-all of only the referenced rows) pipelined
              with the local SpMM over column chunks; total work fixed -> "strong" scaling.

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from graphconvgeo_amd import sparse as gs  # noqa: E402
from graphconvgeo_amd.synth import CONFIGS, SEED, synthetic_graph  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_ACHIEVABLE_GBS = 6300.0  # MI355X_MICROARCH.md:296, "~6.3 TB/s achievable"
MFMA_F32_PEAK_TFLOPS = 157.3  # dense f32 MFMA (v_mfma_f32_16x16x4_f32) at 2.4 GHz
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def spmm_bytes(n_rows: int, nnz: int, K: int) -> int:
    """Edge-centric algorithmic bytes of one CSR SpMM."""
    return 4 * (n_rows + 1) + 8 * nnz + 4 * K * nnz + 4 * K * n_rows


def compulsory_bytes(n_rows: int, nnz: int, K: int, n_cols: int) -> int:
    """indptr + (idx, val) + Z read once + Y written once."""
    return 4 * (n_rows + 1) + 8 * nnz + 4 * K * n_cols + 4 * K * n_rows


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def scipy_baseline(H, K: int, budget_s: float = 30.0) -> dict:
    """The reference's own executor: S.dot(H, Z) (mlpconv.py:73) is scipy's `H @ Z`
    (csr_matvecs, single-threaded whatever the host) on the bench graph against the full N x K
    float32 operand, 1 warm-up then the median of up to 3 runs (time.perf_counter) --
    SURVEY.md §8d -- bounded by `budget_s`: the whole graph while 4 runs fit the budget
    (World: ~5.5 s per run on the GPU box's EPYC), else the leading rows that do (the same
    rows every run; GB/s from that sample's bytes)."""
    import scipy

    Z = np.random.default_rng(SEED + 5).standard_normal((H.shape[1], K), dtype=np.float32)
    # probe ~1/20 of the graph to size the sample
    n = H.shape[0]
    stop = int(np.searchsorted(H.indptr, H.nnz // 20, side="left"))
    t0 = time.perf_counter()
    H[:max(stop, 1)] @ Z
    est = (time.perf_counter() - t0) * H.nnz / max(int(H.indptr[max(stop, 1)]), 1)
    rows = n
    if 4 * est > budget_s:  # full graph does not fit: the leading rows that do
        frac = budget_s / (4 * est)
        rows = max(1, int(np.searchsorted(H.indptr, int(frac * H.nnz), side="left")))
    S = H if rows == n else H[:rows]
    t0 = time.perf_counter()
    S @ Z  # warm-up
    t_warm = time.perf_counter() - t0
    ts = []
    for _ in range(3):
        if ts and sum(ts) + t_warm + ts[-1] > budget_s:
            break
        t0 = time.perf_counter()
        S @ Z
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    what = (f"full graph: all {n} rows" if rows == n else
            f"rows [0, {rows}) of the same graph (budget {budget_s:.0f} s)")
    return {"value": round(spmm_bytes(rows, S.nnz, K) / t / 1e9, 3), "unit": "GB/s",
            "cores": 1, "kind": "reference",
            "edges_per_s": round(S.nnz / t, 1), "seconds_per_spmm": round(t * H.nnz / S.nnz, 3),
            "sample": f"{what}: scipy {scipy.__version__} H @ Z ({S.nnz} nnz x K={K}), 1 "
                      f"warm-up ({t_warm:.2f} s) + median of {len(ts)} "
                      f"({', '.join(f'{x:.2f}' for x in ts)} s), single-threaded scipy "
                      f"csr_matvecs on {cpu_model()} ({os.cpu_count()} host cpus)"}


def cpu_baseline(H, K: int, budget_s: float) -> dict:
    """Labelled extra: the oracle (C port of scipy csr_matvecs, 1 thread) on a bounded row
    sample of the same graph: consecutive row blocks of ~1M nonzeros until `budget_s` is spent."""
    from oracle import gcn_oracle as O

    rng = np.random.default_rng(SEED + 5)
    Z = rng.standard_normal((H.shape[1], K), dtype=np.float32)
    O.spmm_f32(H[:1000], Z)  # warm-up
    rows_done = nnz_done = 0
    t_total = 0.0
    r = 0
    n = H.shape[0]
    while r < n and t_total < budget_s:
        stop = int(np.searchsorted(H.indptr, H.indptr[r] + 1_000_000, side="left"))
        stop = min(max(stop, r + 1), n)
        blk = H[r:stop]
        t0 = time.perf_counter()
        O.spmm_f32(blk, Z)
        t_total += time.perf_counter() - t0
        rows_done += stop - r
        nnz_done += blk.nnz
        r = stop
    gbs = spmm_bytes(rows_done, nnz_done, K) / t_total / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "edges_per_s": round(nnz_done / t_total, 1),
            "sample": f"rows [0, {rows_done}) of the same graph: {nnz_done} nnz x K={K} "
                      f"in {t_total:.1f}s, oracle/spmm_oracle.c (scipy csr_matvecs port), "
                      f"1 thread on {cpu_model()} ({os.cpu_count()} host cpus)"}


def cpu_multicore(H, K: int, budget_s: float) -> dict:
    """Extra, labelled: torch's CPU CSR x dense on every host thread torch uses (SURVEY.md
    §8d optional multi-core reference) -- not the reference's executor, which is 1-thread."""
    import torch as _t

    n = H.shape[0]
    stop = int(np.searchsorted(H.indptr, min(H.nnz, 8_000_000), side="left"))
    blk = H[:max(stop, 1)]
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        A = _t.sparse_csr_tensor(_t.from_numpy(blk.indptr.astype(np.int64)),
                                 _t.from_numpy(blk.indices.astype(np.int64)),
                                 _t.from_numpy(blk.data), size=blk.shape)
    Z = _t.randn((n, K), dtype=_t.float32)
    _t.sparse.mm(A, Z)
    reps, t_total = 0, 0.0
    while t_total < budget_s and reps < 50:
        t0 = time.perf_counter()
        _t.sparse.mm(A, Z)
        t_total += time.perf_counter() - t0
        reps += 1
    t = t_total / reps
    return {"value": round(spmm_bytes(blk.shape[0], blk.nnz, K) / t / 1e9, 3), "unit": "GB/s",
            "cores": _t.get_num_threads(), "kind": "torch.sparse.mm (CPU, multi-thread)",
            "edges_per_s": round(blk.nnz / t, 1),
            "sample": f"rows [0, {blk.shape[0]}): {blk.nnz} nnz x K={K}, {reps} reps"}


PROFILE_ROUNDS = ("r04", "r03", "r02", "r01")  # newest first
PMC_COUNTERS = ("FETCH_SIZE", "WRITE_SIZE")  # one rocprofv3 pass each (TCC slots, guide §PMC)
PMC_KERNEL = "spmm_rows_kernel"


def library_hash() -> str:
    """Source hash of the library this run measures (graphconvgeo_amd/_build.source_hash; the
    binding refuses a library built from other sources, _native._check_fresh)."""
    from graphconvgeo_amd import _build
    return _build.source_hash()


def load_traffic(workload: str, per_launch_bytes: int):
    """Fallback when the live PMC pass cannot run: L2->fabric bytes per launch (2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md:298) from the newest committed
    rocprofv3 PMC summary of this workload -- only one stamped with the source hash of the
    library this run loads (a summary of another build describes other kernels)."""
    want = library_hash()
    for rnd in PROFILE_ROUNDS:
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_{workload}.json")
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get("gcg_source_hash") != want or rec.get("algorithmic_bytes_per_launch") != per_launch_bytes:
            continue
        return rec.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def under_profiler() -> bool:
    """True inside a rocprofv3 run (its tool library is preloaded): no nested PMC pass."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(
        k.startswith("ROCPROF") for k in os.environ)


def _read_counter(d: str, counter: str, kernel: str = PMC_KERNEL):
    import csv
    import glob
    per = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    did = int(row["Dispatch_Id"])
                    per[did] = per.get(did, 0.0) + float(row["Counter_Value"])
    return [per[k] for k in sorted(per)]


def _read_kernel_trace(d: str, kernel: str = PMC_KERNEL):
    """Per-dispatch durations (ns, dispatch order) of `kernel` from a rocprofv3 kernel trace."""
    import csv
    import glob
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"]:
                    rows.append((int(row.get("Dispatch_Id", 0) or 0),
                                 int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    return [ns for _d, ns in sorted(rows)]


def live_traffic(H, K: int, mode: str, timeout_s: int = 240, keep_dir: str = "",
                 tag: str = "headline", launches: int = 20, warmup: int = 5) -> dict:
    """Measured in this run, before this process touches the GPU, by child processes that replay
    the bench's own SpMM launch (tools/pmc_probe.py: the same graph, empty_dense layout, mode and
    gather hint), each under `timeout -s KILL`:
      1. `rocprofv3 --kernel-trace --stats`: the kernel's average duration on THIS box
         (`kernel_trace_ms`) over the bench's own loop -- `warmup` untimed launches, then
         `launches` back to back, the dispatches of that timed loop only -- and the probe's wall
         clock per step over the same loop under the profiler (`traced_ms_per_step`): the
         profile that backs the line's kernel time, and the profiler's own overhead beside it
         (VERDICT r05 item 3);
      2. `--pmc FETCH_SIZE`, 3. `--pmc WRITE_SIZE` (separate passes, guide §PMC): HBM-side bytes
         per launch, 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the gfx950 correction of
         MI355X_MICROARCH.md:298), the mean over the launches after the plan-building one.
    The bytes are L2->fabric bytes: reads the Infinity Cache serves are counted too (no gfx950
    TCC counter separates them, profiles/HISTORY.md §3), so they bound the DRAM bytes from above.
    keep_dir: copy the kernel-trace stats CSV there (`<tag>_kernel_stats.csv`)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {"error": "rocprofv3 not found"}
    tmpd = tempfile.mkdtemp(prefix="gcg_pmc_")
    t0 = time.perf_counter()
    out = {}
    try:
        graph = os.path.join(tmpd, "graph.npz")
        np.savez(graph, n=np.int64(H.shape[0]), indptr=H.indptr, indices=H.indices, data=H.data)
        probe = [sys.executable, os.path.join(ROOT, "tools", "pmc_probe.py"), graph, "--K",
                 str(K), "--mode", mode]

        def run(name, prof_args, n_launch, n_warm=0):
            cmd = (["timeout", "-s", "KILL", str(timeout_s), prof] + prof_args +
                   ["--output-format", "csv", "-d", os.path.join(tmpd, name), "-o", name, "--"] +
                   probe + ["--launches", str(n_launch), "--warmup", str(n_warm)])
            t1 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s + 30)
            print(f"bench: live {name} pass rc={r.returncode} in {time.perf_counter() - t1:.1f} s",
                  file=sys.stderr, flush=True)
            if r.returncode != 0:
                raise RuntimeError(f"{name} pass rc={r.returncode}: {(r.stderr or r.stdout)[-300:]}")
            for line in r.stdout.splitlines():
                if line.startswith("PROBE "):
                    return json.loads(line[6:])
            return {}

        # 1. kernel trace: the kernel's own duration on this box, over the bench's loop
        try:
            n_launch = max(int(launches), 1)
            probe_rec = run("kt", ["--kernel-trace", "--stats"], n_launch, max(int(warmup), 0))
            ns = _read_kernel_trace(os.path.join(tmpd, "kt"))
            if len(ns) < n_launch:
                raise RuntimeError(f"kernel trace: {len(ns)} {PMC_KERNEL} dispatches")
            ns = ns[-n_launch:]  # the timed loop's dispatches (plan + warm-up dropped)
            out["kernel_trace"] = {
                "avg_ms": round(float(np.mean(ns)) / 1e6, 4),
                "min_ms": round(min(ns) / 1e6, 4), "max_ms": round(max(ns) / 1e6, 4),
                "dispatches": len(ns), "warmup": max(int(warmup), 0),
                "traced_ms_per_step": probe_rec.get("ms_per_step"),
                "source": "rocprofv3 --kernel-trace --stats of tools/pmc_probe.py (this run): "
                          "the bench's warm-up + timed loop, its timed dispatches"}
            if keep_dir:
                import glob
                os.makedirs(keep_dir, exist_ok=True)
                for fn in glob.glob(os.path.join(tmpd, "kt", "**", "*kernel_stats.csv"),
                                    recursive=True):
                    shutil.copy(fn, os.path.join(keep_dir, f"{tag}_kernel_stats.csv"))
        except (OSError, subprocess.SubprocessError, RuntimeError, KeyError, ValueError) as exc:
            out["kernel_trace"] = {"error": repr(exc)[:300]}
        # 2, 3. the counters, one pass each
        vals = {}
        for c in PMC_COUNTERS:
            run(c, ["--pmc", c], 4)
            v = _read_counter(os.path.join(tmpd, c), c)
            if len(v) < 2:
                raise RuntimeError(f"{c}: {len(v)} {PMC_KERNEL} dispatches in the counter CSV")
            vals[c] = v[1:]  # drop the plan-building call's launch
        fetch = float(np.mean(vals["FETCH_SIZE"]))
        write = float(np.mean(vals["WRITE_SIZE"]))
        out.update({"traffic": int(2 * fetch * 1024 + write * 1024),
                    "FETCH_SIZE_KiB_per_launch": round(fetch, 1),
                    "WRITE_SIZE_KiB_per_launch": round(write, 1),
                    "dispatches": {c: len(v) for c, v in vals.items()},
                    "spread": round(max(max(v) / min(v) for v in vals.values()) - 1, 4),
                    "gcg_source_hash": library_hash(),
                    "pass_s": round(time.perf_counter() - t0, 1)})
        return out
    except (OSError, subprocess.SubprocessError, RuntimeError, KeyError, ValueError) as exc:
        out["error"] = repr(exc)[:300]
        return out
    finally:
        shutil.rmtree(tmpd, ignore_errors=True)


def roofline_record(kbytes: int, k_ms: float, traffic, traffic_src: str, kernel: str) -> dict:
    """SURVEY.md §8d roofline for the headline kernel. `achieved` / `frac` are the MEASURED
    bytes (rocprofv3 PMC traffic per launch) over the HIP-event kernel time against the 8 TB/s
    HBM spec -- a physical rate, <= 1 of peak; the edge-centric algorithmic model (one K-wide
    row read per nonzero) is kept beside it as `edge_centric_*`: it counts
    re-reads the Infinity Cache serves, so on the power-law graph it exceeds the peak."""
    edge = kbytes / (k_ms * 1e-3) / 1e9
    rec = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": kernel,
           "kernel_ms": round(k_ms, 3), "algorithmic_bytes_per_launch": kbytes,
           "edge_centric_achieved": round(edge, 1),
           "edge_centric_frac": round(edge / HBM_PEAK_GBS, 4)}
    if traffic:
        ach = traffic / (k_ms * 1e-3) / 1e9
        rec.update(achieved=round(ach, 1), frac=round(ach / HBM_PEAK_GBS, 4),
                   frac_vs_achievable=round(ach / HBM_ACHIEVABLE_GBS, 4),
                   achieved_kind=("measured bytes per launch (rocprofv3 PMC 2 x FETCH_SIZE + "
                                  "WRITE_SIZE: L2->fabric, Infinity-Cache hits included) / "
                                  "HIP-event kernel time"),
                   traffic=int(traffic), traffic_over_algorithmic=round(traffic / kbytes, 4),
                   traffic_source=traffic_src)
    else:  # no measured bytes: the model, labelled as such
        rec.update(achieved=round(edge, 1), frac=round(edge / HBM_PEAK_GBS, 4),
                   achieved_kind="edge-centric algorithmic bytes / kernel time (no PMC traffic "
                                 "measured in this run)", traffic=None)
    return rec


def time_events(fn, reps: int, dev) -> float:
    """Per-call ms of fn() with HIP events on the current stream (fn launches there): the median
    of the calls, so one host-side hiccup between an event and its launch does not move it."""
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize(dev)
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def host_mode(H, mode: str) -> str:
    """The mode 'auto' resolves to for host CSR H (sparse.auto_mode), without a device."""
    if mode != "auto":
        return mode
    lens = np.diff(H.indptr)
    return gs.auto_mode(H.shape[0], H.nnz, int(lens.max()) if lens.size else 0)


def spmm_variant(cfg, kind: str, K: int, mode: str, reps: int, dev, H=None, live=None) -> dict:
    """SURVEY.md §8d second run: the same SpMM on the uniform-degree graph of the same size,
    where no hub rows are served from the Infinity Cache -- the honest HBM-gather case. `live`:
    this graph's live PMC pass (live_traffic), run before the process touched the GPU."""
    if H is None:
        H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=kind)
    A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
    g = torch.Generator(device=dev).manual_seed(SEED)
    Z = gs.empty_dense(H.shape[0], K, dev).copy_(torch.randn((H.shape[0], K), generator=g, device=dev))
    Y = gs.empty_dense(H.shape[0], K, dev)
    eff = resolve_mode(A, mode)
    gs.spmm(A, Z, out=Y, mode=eff)
    gs.spmm(A, Z, out=Y, mode=eff)
    k_ms = time_events(lambda: gs.spmm(A, Z, out=Y, mode=eff), reps, dev)
    B = spmm_bytes(H.shape[0], H.nnz, K)
    gbs = B / (k_ms * 1e-3) / 1e9
    if live and "traffic" in live:
        traffic, src = live["traffic"], "live rocprofv3 --pmc pass of this run (bench.live_traffic)"
    else:
        traffic, src = load_traffic(f"{cfg.name}-{kind}-k{K}-{eff}", B)
    rec = {"graph": kind, "mode": eff, "nnz_H": H.nnz, "kernel_ms": round(k_ms, 3),
           "value": round(gbs, 1), "value_kind": "edge-centric", "unit": "GB/s",
           "edges_per_s": round(H.nnz / (k_ms * 1e-3), 1),
           "roofline": roofline_record(B, k_ms, traffic, src, "spmm_rows_kernel")}
    if live and "error" in live:
        rec["live_pmc_error"] = live["error"]
    kt = (live or {}).get("kernel_trace") or {}
    if "avg_ms" in kt:
        rec["roofline"]["kernel_trace_ms"] = kt["avg_ms"]
        rec["roofline"]["kernel_trace"] = kt
    del A, Z, Y
    return rec


def dense_kernels_bench(reps: int, dev) -> dict:
    """The output layer's MFMA kernels (T.dot(h, W2) + b2, softmax-CE and their gradients,
    mlpconv.py:88-95) at Twitter-World's shapes -- 840k target rows x K=300 x C=930 -- each
    timed alone with HIP events (median of `reps` launches after one warm-up), TFLOP/s against
    the dense f32 MFMA peak (steady state: 5 untimed launches first). Random data; parity is
    in tests/test_dense_gpu.py."""
    import math

    from graphconvgeo_amd import dense
    T, K, C = 840_000, 300, 930
    g = torch.Generator(device=dev).manual_seed(SEED + 21)
    P = gs.empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
    W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + C))
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
    W_kc = dense._WeightCache().get(W, False)  # [K][round4(C)]: fused layer / dgrad operand
    W_ck = dense._WeightCache().get(W, True)   # [C][round4(K)]: NT forward operand
    G = gs.empty_dense(T, C, dev)
    dP = gs.empty_dense(T, K, dev)
    loss = torch.empty(T, device=dev)
    hits = torch.empty(T, device=dev)
    kernels = {
        "gemm_nt: P.W2 + b2 (mlpconv.py:88)":
            lambda: dense.gemm_nt(P, W_ck, bias=b, out=G, math="bf16x6"),
        "gemm_nt: dP = G.W2^T": lambda: dense.gemm_nt(G, W_kc, out=dP, math="bf16x6"),
        "gemm_nt f32 MFMA: P.W2 + b2": lambda: dense.gemm_nt(P, W_ck, bias=b, out=G, math="f32"),
        "gemm_nt f32 MFMA: dP = G.W2^T": lambda: dense.gemm_nt(G, W_kc, out=dP, math="f32"),
        "gemm_tn: dW2 = P^T.G (split-K)": lambda: dense.gemm_tn(P, G, math="bf16x6"),
        "gemm_tn f32 MFMA: dW2 = P^T.G (split-K)": lambda: dense.gemm_tn(P, G, math="f32"),
        "fused: P.W2 + b2 -> softmax-CE, hits, dlogits (mlpconv.py:88-95)":
            lambda: dense._fused(P, W_kc, b, y, 1.0 / T, None, G, loss, hits, math="bf16x6"),
        "fused f32 MFMA: P.W2 + b2 -> softmax-CE, hits, dlogits":
            lambda: dense._fused(P, W_kc, b, y, 1.0 / T, None, G, loss, hits, math="f32"),
    }

    flops = 2.0 * T * K * C
    out = {"shape": f"{T} x {K} x {C}", "peak_TFLOPs": MFMA_F32_PEAK_TFLOPS,
           "bf16_peak_TFLOPs": MFMA_BF16_PEAK_TFLOPS,
           "note": "TFLOPs = useful f32 FLOP/s; frac against the f32 MFMA peak. gemm_nt (the "
                   "default, dense.NT_MATH), gemm_tn (dense.TN_MATH) and the fused layer run bf16x6: six bf16 plane products per f32 "
                   "product on the bf16 matrix cores (error vs float64 <= the f32 kernel's, "
                   "tests/test_dense_gpu.py); the bf16x6 forms split the weight's planes into a "
                   "workspace first, that launch inside the timed call; its frac = 6 x FLOP/s / the bf16 peak, "
                   "f32_equivalent_frac = FLOP/s / the f32 MFMA peak"}
    for name, fn in kernels.items():
        for _ in range(5):  # the first launches after a switch run while the clock ramps
            fn()
        ms = time_events(fn, reps, dev)
        tf = flops / (ms * 1e-3) / 1e12
        out[name] = {"ms": round(ms, 3), "TFLOPs": round(tf, 1),
                     "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 3)}
        if name.startswith(("gemm_nt:", "gemm_tn:", "fused:")):  # bf16x6: the bf16 pipe, 6 MFMA FLOP per FLOP
            out[name].update(math="bf16x6", frac=round(6 * tf / MFMA_BF16_PEAK_TFLOPS, 3),
                             f32_equivalent_frac=round(tf / MFMA_F32_PEAK_TFLOPS, 3))
    del P, G, dP, W_kc, W_ck
    return out


def spmm_mode_variant(A, H, K: int, mode: str, reps: int, dev) -> dict:
    """The headline SpMM (same graph, K) in another mode."""
    g = torch.Generator(device=dev).manual_seed(SEED)
    Z = gs.empty_dense(H.shape[0], K, dev).copy_(torch.randn((H.shape[0], K), generator=g, device=dev))
    Y = gs.empty_dense(H.shape[0], K, dev)
    gs.spmm(A, Z, out=Y, mode=mode)
    k_ms = time_events(lambda: gs.spmm(A, Z, out=Y, mode=mode), reps, dev)
    B = spmm_bytes(H.shape[0], H.nnz, K)
    gbs = B / (k_ms * 1e-3) / 1e9
    del Z, Y
    return {"graph": "powerlaw (the headline graph)", "mode": mode, "kernel_ms": round(k_ms, 3),
            "value": round(gbs, 1), "unit": "GB/s", "edges_per_s": round(H.nnz / (k_ms * 1e-3), 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": B}


def spmm_wide_variant(A, N: int, nnz: int, K: int, mode: str, reps: int, dev) -> dict:
    """the same World SpMM at a wider hidden size -- K = 500, main_mlpconv's
    default (tensormain.py:209), or 1500 (tensormain.py:398) -- on the headline graph already
    resident in HBM."""
    g = torch.Generator(device=dev).manual_seed(SEED + 13)
    Z = gs.empty_dense(N, K, dev).copy_(torch.randn((N, K), generator=g, device=dev))
    Y = gs.empty_dense(N, K, dev)
    gs.spmm(A, Z, out=Y, mode=mode)
    k_ms = time_events(lambda: gs.spmm(A, Z, out=Y, mode=mode), reps, dev)
    B = spmm_bytes(N, nnz, K)
    gbs = B / (k_ms * 1e-3) / 1e9
    del Z, Y
    return {"graph": "powerlaw (the headline graph)", "K": K, "mode": mode,
            "kernel_ms": round(k_ms, 3), "value": round(gbs, 1), "unit": "GB/s",
            "edges_per_s": round(nnz / (k_ms * 1e-3), 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": B}


def train_step_bench(steps: int, warmup: int, dev, config: str = "twitter-us") -> dict:
    """BASELINE config 3: one MLPCONV epoch (mlpconv.py:293-295 -> f_train: 2-layer GCN
    forward + backward + Lasagne Adam, tensormain.py:232-237) at Twitter-US scale on one GPU,
    in the reference's layer-2 order and the propagate-first order; plus each SpMM of the
    step timed alone (HIP events) with its edge-centric GB/s. Synthetic data (seed 77):
    power-law graph, 64-nnz/row BoW X, 60 % of nodes as train targets drawn with
    replacement (tensormain.py:226)."""
    from graphconvgeo_amd.mlpconv import LasagneAdam, MLPCONV
    from graphconvgeo_amd.synth import synthetic_features

    cfg = CONFIGS[config]
    t0 = time.perf_counter()
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges)
    X = synthetic_features(cfg.n_nodes, cfg.n_features, nnz_per_row=64)
    n, K, C = cfg.n_nodes, cfg.hidden, cfg.n_classes
    rng = np.random.default_rng(SEED)
    Y = rng.integers(0, C, size=n)
    n_tr = int(0.6 * n)
    train = rng.choice(n_tr, size=n_tr).astype(np.int32)
    dev_idx = np.arange(n_tr, int(0.8 * n), dtype=np.int32)
    test_idx = np.arange(int(0.8 * n), n, dtype=np.int32)
    t_gen = time.perf_counter() - t0
    out = {"config": cfg.name, "nodes": n, "edges": cfg.n_edges, "nnz_H": H.nnz, "nnz_X": X.nnz,
           "F": cfg.n_features, "K": K, "C": C, "train_rows": int(train.size),
           # the output layer runs on the distinct targets, weighted by multiplicity
           "train_rows_distinct": int(np.unique(train).size),
           "data": "synthetic", "data_gen_s": round(t_gen, 1), "steps": steps, "warmup": warmup}
    clf = None
    # MLPCONV's default (order "auto": propagate-first when C > K) as "default", then both
    # layer-2 orders explicitly, then the default captured as a HIP graph
    for order, graph in ((None, False), ("reference", False), ("propagate_first", False),
                         (None, True)):
        kw = {} if order is None else {"order": order}
        clf = MLPCONV(n_epochs=0, hidden_layer_size=K, device=dev, seed=1, use_graph=graph, **kw)
        clf.fit(X, train, dev_idx, test_idx, Y, H)  # builds layers, uploads H and X
        if order is None:
            out["default_order"] = f"{clf.order} -> {clf.l_out.order}"
            order = "default"
        y_train = torch.as_tensor(Y[train].astype(np.int32), device=dev)
        clf.n_epochs = 1  # lets _make_train_step capture the epoch when use_graph
        step = clf._make_train_step(LasagneAdam(clf.params), y_train)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(steps):
            loss, _acc = step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t1) / max(steps, 1) * 1e3
        out[order + ("_hip_graph" if graph else "")] = {"ms_per_step": round(ms, 3),
                                                          "loss": round(float(loss), 5)}
    # each SpMM of the step alone, on the last model's device operands
    A, Xd = clf.l_hid1.H, clf.Xd
    # the output layer runs on the distinct targets (RowSelection.distinct, weighted by
    # multiplicity), so its SpMMs are timed on those rows, as the training step runs them
    rows = clf.rows["train"]
    if rows.distinct() is not None:
        rows = rows.distinct()[0]
    n_t = rows.n
    g = torch.Generator(device=dev).manual_seed(SEED + 21)
    Z1 = gs.empty_dense(n, K, dev).copy_(torch.randn((n, K), generator=g, device=dev))
    G2 = gs.empty_dense(n_t, C, dev).copy_(torch.randn((n_t, C), generator=g, device=dev))
    W1 = clf.l_hid1.W.detach()
    b1 = clf.l_hid1.b.detach()
    gate = gs.empty_gate(n, K, dev)
    At = A.rows_transpose(rows)
    nnz_t = int(np.diff(H.indptr)[rows.host].sum())
    # X.W1 and X^T.g gather rows of a small dense operand (W1: F x K = 12 MB at Twitter-US) that
    # stays in L2 / the Infinity Cache: the edge-centric model counts every gathered row as an HBM
    # read; SURVEY.md §8d's K2 model counts W1 once -- 4(N+1) + 8 nnz_X + 4FK + 4NK (and, for
    # X^T.g, G read once and the F x K result written once). What bounds these kernels is neither
    # HBM figure but the L2 gather rate (16.8-18.8 TB/s, MI355X_MICROARCH.md §Indexed rows)
    k2 = {"X.W1 (mlpconv.py:71)": 4 * (n + 1) + 8 * X.nnz + 4 * cfg.n_features * K + 4 * n * K,
          "X^T.g (grad of mlpconv.py:71)": (4 * (cfg.n_features + 1) + 8 * X.nnz + 4 * n * K
                                            + 4 * cfg.n_features * K)}
    ops = {
        "X.W1 (mlpconv.py:71)": (lambda: gs.spmm(Xd, W1), spmm_bytes(n, X.nnz, K),
                                 "W1 (12 MB) cache-resident"),
        "rectify(H.Z1 + b1) + gate (mlpconv.py:73-77)": (
            lambda: gs.spmm(A, Z1, bias=b1, act="relu", gate=gate), spmm_bytes(n, H.nnz, K), ""),
        "(H.Z2 + b2)[train distinct], C wide (mlpconv.py:90-94)": (
            lambda: gs.spmm(A, Z1[:, :C], rows=rows), spmm_bytes(n_t, nnz_t, C), ""),
        "(H[train distinct])^T.G2, C wide (grad of mlpconv.py:90-94)": (
            lambda: gs.spmm(At, G2), spmm_bytes(n, nnz_t, C), ""),
        "H.g1 (grad of mlpconv.py:73)": (lambda: gs.spmm(A, Z1), spmm_bytes(n, H.nnz, K), ""),
        "X^T.g (grad of mlpconv.py:71)": (lambda: Xd.tmatmul(Z1), spmm_bytes(cfg.n_features, X.nnz, K),
                                          "dense Zipf-head columns on the MFMA GEMM"),
    }
    per = {}
    for name, (fn, nbytes, note) in ops.items():
        fn()
        k_ms = time_events(fn, max(steps, 5), dev)
        per[name] = {"ms": round(k_ms, 3), "GBps_edge_centric": round(nbytes / (k_ms * 1e-3) / 1e9, 1)}
        if name in k2:
            per[name].update(GBps_k2_model=round(k2[name] / (k_ms * 1e-3) / 1e9, 1),
                             k2_model_bytes=k2[name], bound="L2 gather rate (operand cache-"
                             "resident; neither byte model is an HBM bound here)")
        if note:
            per[name]["note"] = note
    out["spmm"] = per
    return out


def resolve_mode(A, mode: str) -> str:
    return mode if mode != "auto" else gs.resolve_auto(A)


def alternatives(H, rank, world, dev, part, Zl, K, B, eff, gen, timed, reps, args) -> dict:
    """Alternative strategies measured in the same N > 1 run: H replicated with Z split by columns
    (no exchange, distributed.FeatureParallelSpMM), and the exchange A/B --
    the same pipelined step with every exchange: RCCL all-gather (in place), a direct mesh of
    isend/irecv pairs (every xGMI link at once), the halo all-to-all of only the referenced rows
    -- and each exchange alone."""
    from graphconvgeo_amd.distributed import FeatureParallelSpMM
    N = H.shape[0]
    fp = FeatureParallelSpMM(H, rank, world, dev, K)
    Zc = torch.randn((N, fp.width), generator=gen, device=dev, dtype=torch.float32)
    Yc = gs.empty_dense(N, fp.width, dev)
    fp.spmm(Zc, out=Yc, mode=args.mode, task_nnz=args.task_nnz)
    for _ in range(args.warmup):
        fp.spmm(Zc, out=Yc, mode=args.mode, task_nnz=args.task_nnz)
    t_fp = timed(lambda: fp.spmm(Zc, out=Yc, mode=args.mode, task_nnz=args.task_nnz), args.steps)
    alt = {"feature_parallel": {"ms_per_step": round(t_fp, 4),
                                "value": round(B / (t_fp * 1e-3) / 1e9, 1), "unit": "GB/s",
                                "columns_per_gpu": fp.width, "exchange": "none",
                                "note": "H replicated (0.34 GB), Z/Y split by columns"}}
    del fp, Zc, Yc
    # The exchange A/B: the same pipelined step with every exchange --
    # RCCL all-gather (in place), a direct mesh of isend/irecv pairs (every xGMI link at
    # once), the halo all-to-all of only the referenced rows -- and each exchange alone.
    for m in ("allgather", "mesh", "halo"):
        try:
            alt.update(exchange_ab(H, rank, world, dev, part, Zl, K, B, eff, timed, reps, args, m))
        except Exception as exc:  # noqa: BLE001 -- one exchange failing keeps the others
            alt[f"exchange_{m}"] = {"error": f"{type(exc).__name__}: {exc}"[:500]}
        torch.cuda.empty_cache()
    return alt


def chunks_calibration(part, Zl, Y, K, chunks, ms, eff, timed, reps, args, t_comm, t_sp,
                       gathered) -> dict:
    """N > 1, in the headline line: the pipelined step at 1, 2 and 4 column chunks with the
    headline's own exchange (the same collectives, only narrower), beside what the chunk model
    predicts for each (distributed.pipeline_time on this run's measured exchange and local SpMM),
    and the inbound rate per xGMI link the exchange alone achieved -- so one scaling run fixes
    XGMI_LINK_GBPS and choose_chunks."""
    from graphconvgeo_amd.distributed import XGMI_LINK_GBPS, pipeline_time
    world = part.world
    links = min(world - 1, 7)
    ab, model = {}, {}
    for c in (1, 2, 4):
        model[str(c)] = round(pipeline_time(t_comm, t_sp, c), 4)
        if c == chunks:
            ab[str(c)] = round(ms, 4)  # the headline step itself
            continue
        if c > 1 and K // c < 16:
            continue
        part.chunk_buffers(K, c).fill(Zl)

        def step_c(c=c):
            part.spmm_pipelined(None, Y, n_chunks=c, mode=eff, task_nnz=args.task_nnz)
        step_c()
        ab[str(c)] = round(timed(step_c, reps), 4)
    best = min(ab, key=lambda k: ab[k])
    return {"chunks_ab": {"ms_per_step": ab, "model_ms": model, "best": int(best),
                          "chosen": chunks, "chosen_over_best": round(ab[str(chunks)] / ab[best], 4)
                          if str(chunks) in ab else None},
            "xgmi_links": links,
            "xgmi_link_GBps_fit": round(gathered / (t_comm * 1e-3) / links / 1e9, 2),
            "xgmi_link_GBps_model": XGMI_LINK_GBPS}


def exchange_ab(H, rank, world, dev, part, Zl, K, B, eff, timed, reps, args, m) -> dict:
    """One exchange of the A/B: the pipelined step with it, and the exchange alone."""
    from graphconvgeo_amd.distributed import RowPartitionedCSR
    alt = {}
    pm = part if m == part.exchange else RowPartitionedCSR(H, rank, world, dev, exchange=m,
                                                           plan=part.plan)
    cm = pm._n_chunks(args.chunks, K)
    pm.chunk_buffers(K, cm).fill(Zl)
    Ym = gs.empty_dense(pm.n_local, K, dev)

    def step_m():
        pm.spmm_pipelined(None, Ym, n_chunks=cm, mode=eff, task_nnz=args.task_nnz)
    for _ in range(max(args.warmup, 1)):
        step_m()
    t_m = timed(step_m, args.steps)
    b1 = pm.chunk_buffers(K, 1)
    b1.fill(Zl)
    t_x = timed(lambda: pm.layout.exchange(b1.chunks[0][2], async_op=False), reps)
    alt[f"exchange_{m}_ms"] = round(t_m, 4)
    alt[f"exchange_{m}"] = {"step_ms": round(t_m, 4), "exchange_alone_ms": round(t_x, 4),
                            "chunks": cm, "bytes_in_per_gpu": pm.exchange_bytes_per_row(K),
                            "value": round(B / (t_m * 1e-3) / 1e9, 1)}
    if pm is not part:
        del pm
    del Ym
    return alt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="twitter-world", choices=sorted(CONFIGS))
    ap.add_argument("--graph", default="powerlaw", choices=["powerlaw", "uniform"])
    ap.add_argument("--hidden", type=int, default=None, help="K (default: config hidden=300)")
    ap.add_argument("--mode", default="auto", choices=list(gs.MODES))
    ap.add_argument("--task-nnz", type=int, default=0)
    ap.add_argument("--ld", type=int, default=0,
                    help="row stride of Z/Y in floats (0 = the library's empty_dense layout)")
    ap.add_argument("--cpu-budget", type=float, default=30.0,
                    help="seconds of CPU baseline work: the scipy baseline (full graph while "
                         "it fits, else a row sample) and, up to 1/5 of it, the C-port extra")
    ap.add_argument("--no-live-pmc", dest="live_pmc", action="store_false",
                    help="N = 1: skip the live rocprofv3 PMC pass (traffic then comes from a "
                         "committed summary stamped with this library's source hash, if any)")
    ap.add_argument("--profile-dir", default="",
                    help="N = 1: keep the live kernel-trace stats CSVs there (e.g. gpurun_out/...)")
    ap.add_argument("--no-variants", dest="variants", action="store_false",
                    help="N = 1: skip the uniform-degree second run")
    ap.add_argument("--no-train-step", dest="train_step", action="store_false",
                    help="N = 1: skip the config-3 (Twitter-US) training-step measurement")
    ap.add_argument("--no-dense", dest="dense", action="store_false",
                    help="N = 1: skip timing the output layer's MFMA kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # auto chunks: the count minimising a pipeline model of this rank's exchange bytes over
    # xGMI against its local SpMM, each extra chunk costing the SpMM ~9 % (profiles/HISTORY.md §4)
    ap.add_argument("--chunks", type=int, default=0,
                    help="N > 1: column chunks of the exchange/SpMM pipeline (1 = no overlap; "
                         "0 = auto, RowPartitionedCSR.choose_chunks)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "allgather", "mesh", "halo"],
                    help="N > 1: all-gather every block, a direct isend/irecv mesh of whole "
                         "blocks, or send only the referenced halo rows")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 process-group backend (nccl = RCCL over xGMI; gloo only to "
                         "rehearse several ranks on one GPU)")
    ap.add_argument("--dist-timeout", type=float, default=180.0,
                    help="N > 1: seconds a collective may take before the process group "
                         "aborts and the run exits non-zero (distributed.init_process_group); "
                         "well inside the driver's 600 s bench limit")
    ap.add_argument("--exchange-ab", dest="alternatives", action="store_true",
                    help="N > 1: after the headline line, time the other exchanges (mesh / "
                         "halo / all-gather) and the feature-parallel alternative; printed as "
                         "one 'ALT {...}' line (off by default: the driver's scaling run runs "
                         "only the headline's own collectives)")
    ap.add_argument("--partitioned", action="store_true",
                    help="use the row-partitioned (all-gather) path even at N = 1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    cfg = CONFIGS[args.config]
    K = args.hidden or cfg.hidden
    t_gen = time.perf_counter()
    H = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind=args.graph)
    t_gen = time.perf_counter() - t_gen
    N, nnz = H.shape[0], H.nnz
    B = spmm_bytes(N, nnz, K)

    # Live PMC (N = 1): the headline launch's HBM-side bytes, measured by rocprofv3 child
    # processes before this process touches the GPU (and for the uniform second run's graph).
    single = world == 1 and not args.partitioned
    live = live_u = H_u = None
    if single and args.live_pmc and args.ld == 0 and args.steps > 0:
        if under_profiler():
            live = {"error": "skipped: this run is itself under rocprofv3"}
        else:
            live = live_traffic(H, K, host_mode(H, args.mode), keep_dir=args.profile_dir,
                                tag="headline", launches=args.steps, warmup=args.warmup)
            if args.variants:
                H_u = synthetic_graph(cfg.n_nodes, cfg.n_edges, kind="uniform")
                live_u = live_traffic(H_u, K, host_mode(H_u, args.mode),
                                      keep_dir=args.profile_dir, tag="uniform")

    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        import torch.distributed as dist

        from graphconvgeo_amd.distributed import init_process_group
        # explicit timeout + async error handling: a stuck collective ends the run non-zero
        init_process_group(args.dist_backend, dev if args.dist_backend == "nccl" else None,
                           timeout_s=args.dist_timeout)
        if dist.get_world_size() != world:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")

    gen = torch.Generator(device=dev)
    gen.manual_seed(SEED + rank)
    if world == 1 and not args.partitioned:
        A = gs.DeviceCSR.from_scipy(H, dev, symmetric=True)
        if args.ld == 0:  # the library's row layout (sparse.row_stride: K = 300 -> 304 floats)
            Z = gs.empty_dense(N, K, dev).copy_(
                torch.randn((N, K), generator=gen, device=dev, dtype=torch.float32))
            Y = gs.empty_dense(N, K, dev)
        else:
            ld = max(args.ld, K)
            Z = torch.randn((N, ld), generator=gen, device=dev, dtype=torch.float32)[:, :K]
            Y = torch.empty((N, ld), device=dev)[:, :K]
        gs.spmm(A, Z, out=Y, mode=args.mode, task_nnz=args.task_nnz)  # builds the plan
        eff = resolve_mode(A, args.mode)
        info = A.plan(None, eff == "ordered", args.task_nnz).info() if eff != "rowwise" else {}

        def step():
            gs.spmm(A, Z, out=Y, mode=args.mode, task_nnz=args.task_nnz)
    else:
        from graphconvgeo_amd.distributed import RowPartitionedCSR
        part = RowPartitionedCSR(H, rank, world, dev, exchange=args.exchange)
        # one mode for every rank and every N: the whole graph's (RowPartitionedCSR.resolve_mode)
        eff = part.resolve_mode(args.mode)
        chunks = part._n_chunks(args.chunks, K)  # 0 = auto: RowPartitionedCSR.choose_chunks
        Zl = gs.empty_dense(part.local_block_rows, K, dev).copy_(
            torch.randn((part.local_block_rows, K), generator=gen, device=dev))
        Y = gs.empty_dense(part.n_local, K, dev)
        if world > 1:
            # the producer's rows live in the exchange buffers' own slots: the step copies
            # nothing, it is the exchange pipelined with the local SpMM
            part.chunk_buffers(K, chunks).fill(Zl)
            step_z = None
        else:  # world 1: the local SpMM on Zl itself (no exchange, no copies)
            step_z = Zl
        part.spmm_pipelined(step_z, Y, n_chunks=chunks, mode=eff, task_nnz=args.task_nnz)
        info = part.A.plan(None, eff == "ordered", args.task_nnz).info() if eff != "rowwise" else {}

        def step():
            part.spmm_pipelined(step_z, Y, n_chunks=chunks, mode=eff, task_nnz=args.task_nnz)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    # HIP events on the SpMM's stream bracket the timed launches themselves: at N = 1 their
    # span / steps is the line's kernel time (the same launches the wall clock times)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3

    # Live per-launch kernel time with HIP events on the SpMM's own stream. N = 1: the whole
    # graph; N > 1: this rank's local SpMM on the gathered operand (local algorithmic bytes).
    roofline = None
    if args.steps > 0:
        if world == 1 and not args.partitioned:
            kstep, kbytes = None, B
            k_ms = ev0.elapsed_time(ev1) / args.steps
        else:
            full_k = part.all_gather(Zl)
            kbytes = spmm_bytes(part.n_local, part.nnz_local, K)

            def kstep():
                gs.spmm(part.A, full_k, out=Y, mode=eff, task_nnz=args.task_nnz)
            kstep()
            k_ms = time_events(kstep, args.steps, dev)
        traffic = traffic_src = None
        if kbytes == B:
            if live and "traffic" in live:
                traffic = live["traffic"]
                traffic_src = "live rocprofv3 --pmc pass of this run (bench.live_traffic)"
            else:
                traffic, traffic_src = load_traffic(f"{args.config}-{args.graph}-k{K}-{eff}", B)
        roofline = roofline_record(kbytes, k_ms, traffic, traffic_src,
                                   "spmm_rows_kernel (+ spmm_fixup_kernel)")
        if live:
            kt = live.pop("kernel_trace", None) or {}
            roofline["live_pmc"] = live
            if "avg_ms" in kt:
                # the same launch under rocprofv3 --kernel-trace, same box, same run, same loop
                # (warm-up + timed launches): backs the line's kernel time. A kernel cannot take
                # longer than the step that runs it -- compared without slack, against this
                # process's step and against the traced process's own step; their ratio is the
                # profiler's measured overhead
                roofline["kernel_trace_ms"] = kt["avg_ms"]
                roofline["kernel_trace"] = kt
                roofline["kernel_trace_vs_ms_per_step"] = round(kt["avg_ms"] / ms, 4)
                roofline["kernel_trace_le_step"] = bool(kt["avg_ms"] <= ms)
                tms = kt.get("traced_ms_per_step")
                if tms:
                    roofline["kernel_trace_le_traced_step"] = bool(kt["avg_ms"] <= tms)
                    roofline["profiler_overhead"] = round(tms / ms - 1.0, 4)
                    roofline["kernel_trace_note"] = (
                        "two processes, one box: the trace is bounded by the traced process's "
                        "own step (kernel_trace_le_traced_step); profiler_overhead = that step / "
                        "this step - 1 is the measured gap between the processes")
            elif kt:
                roofline["kernel_trace"] = kt
        # compulsory bytes (every array touched once) beside the edge-centric
        # count, so cache reuse on the gather is visible
        roofline["compulsory_bytes_per_launch"] = (
            compulsory_bytes(N, nnz, K, N) if kbytes == B else
            compulsory_bytes(part.n_local, part.nnz_local, K, part.operand_rows()))
        if 4 * K * N <= 256 * 2**20:  # the dense operand fits the Infinity Cache
            roofline["note"] = "cache-resident, not roofline-bound (Z fits the 256 MB Infinity Cache)"
        if kbytes != B:
            roofline["scope"] = f"rank {rank} local SpMM ({part.n_local} rows, {part.nnz_local} nnz)"

    # N > 1 (or --partitioned): the two phases alone, max over ranks, for the comm fraction.
    dist_info = None
    if world > 1 or args.partitioned:
        def timed(fn, reps):
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            barrier()
            dt = (time.perf_counter() - t0) / reps * 1e3
            if world > 1:
                import torch.distributed as dist
                tt = torch.tensor([dt], dtype=torch.float64, device=dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                dt = float(tt.item())
            return dt
        reps = max(args.steps // 2, 1)
        full = part.all_gather(Zl)
        t_comm = timed(lambda: part.all_gather(Zl), reps)
        t_sp = timed(lambda: gs.spmm(part.A, full, out=Y, mode=eff, task_nnz=args.task_nnz), reps)
        gathered = part.exchange_bytes_per_row(K)
        import torch.distributed as dist
        dist_info = {"world_size": dist.get_world_size() if world > 1 else 1,
                     "backend": dist.get_backend() if world > 1 else None,
                     "exchange": part.exchange, "halo_fraction": round(part.halo_fraction, 4),
                     "exchange_bytes_in_per_gpu": gathered,
                     "exchange_ms": round(t_comm, 4), "local_spmm_ms": round(t_sp, 4),
                     # the share of the pipelined step not covered by the
                     # local SpMM (exposed exchange + pipeline fill)
                     "exposed_comm_ms": round(max(ms - t_sp, 0.0), 4),
                     "comm_fraction": round(max(ms - t_sp, 0.0) / ms, 4) if ms > 0 else None,
                     "exchange_inbound_GBps_per_gpu": round(gathered / (t_comm * 1e-3) / 1e9, 1),
                     "chunks": chunks, "chunks_requested": args.chunks or "auto",
                     "rows_local": part.n_local,
                     "nnz_local": part.nnz_local, "block_rows": part.block_rows,
                     "spmm_only_aggregate_GBps": round(B / (t_sp * 1e-3) / 1e9, 1)}

        if world > 1:
            dist_info.update(chunks_calibration(part, Zl, Y, K, chunks, ms, eff, timed, reps,
                                                args, t_comm, t_sp, gathered))

    value = B / (ms * 1e-3) / 1e9
    rec = {
        "metric": "GCN SpMM fwd GB/s (achieved HBM) + edges/s, Twitter-World graph, 1/2/4/8 GPU",
        "value": round(value), "unit": "GB/s",
        # value = SURVEY.md §8d's edge-centric algorithmic bytes per step / step time (the
        # metric's model; it counts re-reads the Infinity Cache serves); the measured HBM-side
        # rate and its fraction of peak are roofline.achieved / roofline.frac
        "value_kind": "edge-centric", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "edges_per_s": round(nnz / (ms * 1e-3)),
        "config": {"workload": f"{cfg.name} H.Z SpMM fwd, {args.graph} degrees", "nodes": N,
                   "edges": cfg.n_edges, "nnz_H": nnz, "K": K, "mode": f"{args.mode}->{eff}",
                   "mode_resolution": ("the whole graph (RowPartitionedCSR.resolve_mode), the "
                                       "same at every N; each row block alone: " + ",".join(
                       getattr(part, "block_modes", [])) if (world > 1 or args.partitioned)
                                       else "the whole graph (sparse.resolve_auto)"),
                   "parallelism": f"row{world}" if world > 1 else "single",
                   "plan": info, "graph_gen_s": round(t_gen, 1)},
    }
    if roofline:
        rec["roofline"] = roofline
    if dist_info:
        rec["distributed"] = dist_info
    if world == 1 and not args.partitioned and args.variants:
        # SURVEY.md §8d second run: uniform degrees (no Infinity-Cache hub reuse)
        del Z, Y
        rec["variants"] = {"uniform": spmm_variant(cfg, "uniform", K, args.mode,
                                                   max(args.steps, 5), dev, H=H_u, live=live_u)}
        H_u = None
        if args.graph == "powerlaw":
            # the reference's other hidden sizes on the headline graph: main_mlpconv's default
            # hidden = 500 (tensormain.py:209) and the tuned 1500 (tensormain.py:398)
            for kk in (500, 1500):
                if kk != K:
                    rec["variants"][f"k{kk}"] = spmm_wide_variant(
                        A, N, nnz, kk, eff, max(args.steps // (2 if kk < 1000 else 4), 3), dev)
        if eff != "fast":
            # the same SpMM in 'fast' mode (hub rows split, within 1e-5): the N = 1 point of a
            # `--mode fast` scaling series (the default series runs the whole graph's mode,
            # 'ordered', at every N: RowPartitionedCSR.resolve_mode)
            rec["variants"]["fast"] = spmm_mode_variant(A, H, K, "fast", max(args.steps, 5), dev)
    if world == 1 and not args.partitioned and args.dense:
        rec["dense_kernels"] = dense_kernels_bench(max(args.steps // 2, 5), dev)
    if world == 1 and not args.partitioned and args.train_step:
        # BASELINE config 3: Twitter-US 2-layer fwd+bwd step (both layer-2 orders)
        rec["train_step"] = train_step_bench(max(args.steps // 2, 5), max(args.warmup, 2), dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = scipy_baseline(H, K, args.cpu_budget)
        rec["cpu_port"] = cpu_baseline(H, K, args.cpu_budget / 5)
        try:
            rec["cpu_multicore"] = cpu_multicore(H, K, min(args.cpu_budget, 5.0))
        except Exception as exc:  # informational only
            rec["cpu_multicore"] = {"error": repr(exc)[:200]}
    if rank == 0:
        print(json.dumps(rec), flush=True)  # the headline: printed before any extra
    # Opt-in extras (N > 1, --exchange-ab): the other exchanges (their collectives are not the
    # headline's) and the feature-parallel alternative, after the line is out: a failure or a
    # hang there (the process group's --dist-timeout ends it) cannot cost the headline.
    if world > 1 and args.alternatives:
        try:
            alt = alternatives(H, rank, world, dev, part, Zl, K, B, eff, gen, timed, reps, args)
        except Exception as exc:  # noqa: BLE001 -- the A/B is an extra
            # (raised on every rank alike -- a bad argument, an unsupported op -- so no rank is
            # left waiting in a collective)
            alt = {"error": f"{type(exc).__name__}: {exc}"[:500]}
        if rank == 0:
            print("ALT " + json.dumps(alt), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
