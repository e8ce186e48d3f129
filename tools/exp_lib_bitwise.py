#!/usr/bin/env python
"""Is a variant library bitwise the production one on the output layer? Runs the fused layer
(bf16x6 and f32 MFMA, with and without row weights, ragged N) once per library
(GCG_LIB, one child process each) on the same seeded inputs and compares every output byte.

  python tools/exp_lib_bitwise.py graphconvgeo_amd/libgcg_spmm.so tools/varlibs/libgcg_x.so
"""
import hashlib
import json
import os
import subprocess
import sys

CHILD = r'''
import hashlib, json, os, sys, torch
sys.path.insert(0, os.getcwd())
from graphconvgeo_amd import dense
from graphconvgeo_amd.sparse import empty_dense
dev = torch.device("cuda:0")
out = {}
for (T, K, C) in [(20_000, 300, 930), (5_003, 129, 257), (3_001, 64, 64)]:
    g = torch.Generator(device=dev).manual_seed(T)
    P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.3)
    W = torch.randn((K, C), generator=g, device=dev) * 0.1
    b = torch.randn(C, generator=g, device=dev) * 0.01
    y = torch.randint(0, C, (T,), generator=g, device=dev, dtype=torch.int32)
    rw = torch.rand(T, generator=g, device=dev)
    Wp = dense._WeightCache().get(W, False)
    for math in ("bf16x6", "f32"):
        for w in (None, rw):
            G = empty_dense(T, C, dev)
            loss = torch.empty(T, device=dev)
            hits = torch.empty(T, device=dev)
            dense._fused(P, Wp, b, y, 1.0 / T, None, G, loss, hits, row_weight=w, math=math)
            torch.cuda.synchronize()
            h = hashlib.sha256()
            for t in (G[:, :C], loss, hits):
                h.update(t.contiguous().cpu().numpy().tobytes())
            out[f"fused {T}x{K}x{C} {math} w={w is not None}"] = h.hexdigest()[:16]
print("R " + json.dumps(out), flush=True)
'''


def main():
    libs = [a for a in sys.argv[1:]]
    res = {}
    for lib in libs:
        env = dict(os.environ, GCG_LIB=os.path.abspath(lib))
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                           timeout=300)
        line = next((ln for ln in p.stdout.splitlines() if ln.startswith("R ")), None)
        if line is None:
            print(json.dumps({"lib": lib, "error": (p.stderr or p.stdout)[-600:]}))
            sys.exit(1)
        res[lib] = json.loads(line[2:])
    base = res[libs[0]]
    for lib in libs[1:]:
        diff = [k for k in base if res[lib].get(k) != base[k]]
        print(json.dumps({"lib": lib, "bitwise_equal": not diff, "differs": diff}))


if __name__ == "__main__":
    main()
