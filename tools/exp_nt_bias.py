import math, json, torch, numpy as np, sys, os
sys.path.insert(0, os.getcwd())
from graphconvgeo_amd import dense
from graphconvgeo_amd.sparse import empty_dense
dev = torch.device("cuda:0")
T, K, C = 840_000, 300, 930
g = torch.Generator(device=dev).manual_seed(98)
P = empty_dense(T, K, dev).copy_(torch.randn((T, K), generator=g, device=dev) * 0.1)
W = (torch.rand((K, C), generator=g, device=dev) * 2 - 1) * math.sqrt(6.0 / (K + C))
b = torch.randn(C, generator=g, device=dev) * 0.01
W_ck = dense._WeightCache().get(W, True)
G = empty_dense(T, C, dev)
flops = 2.0 * T * K * C
def per_launch(fn, reps=10):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        a.record(); fn(); e.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(e) for a, e in evs]
def agg(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
for name, fn in [("nobias", lambda: dense.gemm_nt(P, W_ck, out=G)), ("bias", lambda: dense.gemm_nt(P, W_ck, bias=b, out=G))]:
    fn(); torch.cuda.synchronize()
    for it in range(2):
        pl = per_launch(fn); ag = agg(fn)
        print(name, "per-launch", [round(flops/x/1e9,1) for x in pl], "agg", round(flops/ag/1e9,1), flush=True)
