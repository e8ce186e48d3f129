#!/usr/bin/env python
"""Library A/B of the output layer's bf16x6 kernels at Twitter-World's shapes (840k x 300 x 930):
the fused layer (default tile), the NT projection and its input gradient, each timed with HIP
events (mean of 10 after 5 warm-ups). One process per library (GCG_LIB), alternated `--rounds`
times; prints one JSON line per (round, library).

  python tools/exp_dense_ab.py tools/varlibs/libgcg_base.so graphconvgeo_amd/libgcg_spmm.so
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, math, os, sys, torch
sys.path.insert(0, os.getcwd())
from graphconvgeo_amd import dense
from graphconvgeo_amd.sparse import empty_dense
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
T, K, C = 840_000, 300, 930
P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + C))
b = torch.randn(C, generator=g, device=dev) * 0.01
y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
W_kc = dense._WeightCache().get(W, False)
W_ck = dense._WeightCache().get(W, True)
G = empty_dense(T, C, dev); dP = empty_dense(T, K, dev)
loss = torch.empty(T, device=dev); hits = torch.empty(T, device=dev)
ks = {"fused": lambda: dense._fused(P, W_kc, b, y, 1.0 / T, None, G, loss, hits, math="bf16x6"),
      "nt_fwd": lambda: dense.gemm_nt(P, W_ck, bias=b, out=G, math="bf16x6"),
      "nt_dP": lambda: dense.gemm_nt(G, W_kc, out=dP, math="bf16x6")}
out = {}
for name, fn in ks.items():
    for _ in range(5): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): fn()
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    out[name] = {"ms": round(ms, 4), "TFLOPs": round(2.0 * T * K * C / (ms * 1e-3) / 1e12, 1)}
print("R " + json.dumps(out), flush=True)
'''


def main():
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = 3
    for a in sys.argv[1:]:
        if a.startswith("--rounds="):
            rounds = int(a.split("=")[1])
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, GCG_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                               timeout=300)
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("R ")), None)
            rec = {"round": r, "lib": lib}
            rec.update(json.loads(line[2:]) if line else {"error": (p.stderr or p.stdout)[-400:]})
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
