"""Seeded synthetic inputs for the BASELINE.json configs.

There is no network and no Twitter data here, so every benchmark and large parity
case runs on synthetic data of the reference's shapes:

  * graph: symmetric, binary, exactly E undirected non-self edges, power-law degrees
    (Chung-Lu, exponent 2.1, expected degree capped at 0.01*N; node ids randomly
    permuted, since the reference numbers users in sorted-username order,
    data.py:280-297, which is uncorrelated with degree), or uniform random edges;
    then the normalized operator H = D^-1/2 (A+I) D^-1/2 (graph.csr_from_edges).
  * X: CSR N x F bag-of-words, `nnz_per_row` Zipf-distributed distinct columns,
    positive values, rows l2-normalized (TfidfVectorizer norm='l2', data.py:255).
  * dense operands ~ N(0,1) float32, weights Glorot-uniform (mlpconv.py:208).
Seed 77 everywhere (tensormain.py:35).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sps

from .graph import csr_from_edges

SEED = 77


@dataclass(frozen=True)
class GraphConfig:
    name: str
    n_nodes: int
    n_edges: int
    n_features: int
    hidden: int
    n_classes: int


# BASELINE.json configs (C = 129 / 256 are the datasets' usual region counts, 930 is
# hinted at tensormain.py:397).
CONFIGS = {
    "geotext": GraphConfig("geotext", 9_475, 80_000, 10_000, 300, 129),
    "twitter-us": GraphConfig("twitter-us", 450_000, 5_000_000, 10_000, 300, 256),
    "twitter-world": GraphConfig("twitter-world", 1_400_000, 20_000_000, 50_000, 300, 930),
}


def _unique_pairs(keys_parts):
    return np.unique(np.concatenate(keys_parts))


def powerlaw_edges(n: int, e: int, exponent: float = 2.1, max_deg_frac: float = 0.01,
                   seed: int = SEED):
    """Exactly `e` unique undirected edges (u < v) of a Chung-Lu power-law graph."""
    rng = np.random.default_rng(seed)
    if e > n * (n - 1) // 2:
        raise ValueError("too many edges for n")
    ranks = np.arange(1, n + 1, dtype=np.float64)
    w = ranks ** (-1.0 / (exponent - 1.0))
    cap = max(1.0, max_deg_frac * n)
    target = 2.0 * e
    scale = target / w.sum()
    for _ in range(50):  # fixed point: cap then rescale to keep sum(w) = 2E
        ww = np.minimum(w * scale, cap)
        s = ww.sum()
        if abs(s - target) < 1e-6 * target:
            break
        scale *= target / s
    ww = np.minimum(w * scale, cap)
    perm = rng.permutation(n)  # random node labels
    cdf = np.cumsum(ww)
    cdf /= cdf[-1]
    return _sample_edges(n, e, rng, lambda m: perm[np.searchsorted(cdf, rng.random(m), side="right").clip(0, n - 1)])


def uniform_edges(n: int, e: int, seed: int = SEED):
    """Exactly `e` unique undirected edges (u < v), endpoints uniform."""
    rng = np.random.default_rng(seed)
    return _sample_edges(n, e, rng, lambda m: rng.integers(0, n, size=m))


def _sample_edges(n, e, rng, draw):
    keys = np.empty(0, dtype=np.int64)
    m = int(e * 1.2) + 16
    while keys.size < e:
        a = draw(m).astype(np.int64)
        b = draw(m).astype(np.int64)
        ok = a != b
        a, b = a[ok], b[ok]
        lo = np.minimum(a, b)
        hi = np.maximum(a, b)
        keys = np.unique(np.concatenate([keys, lo * n + hi]))
        m = int((e - keys.size) * 1.5) + 1024
    if keys.size > e:
        keys = np.sort(rng.choice(keys, size=e, replace=False))
    return keys // n, keys % n


def synthetic_graph(n: int, e: int, kind: str = "powerlaw", seed: int = SEED,
                    dtype=np.float32) -> sps.csr_matrix:
    """H = D^-1/2 (A+I) D^-1/2 of a seeded synthetic graph (nnz = 2E + N)."""
    if kind == "powerlaw":
        u, v = powerlaw_edges(n, e, seed=seed)
    elif kind == "uniform":
        u, v = uniform_edges(n, e, seed=seed)
    else:
        raise ValueError(f"unknown graph kind {kind!r}")
    return csr_from_edges(n, u, v, dtype=dtype)


def synthetic_features(n: int, f: int, nnz_per_row: int = 64, seed: int = SEED,
                       zipf_a: float = 1.1, empty_frac: float = 0.0) -> sps.csr_matrix:
    """CSR N x F float32 bag-of-words: distinct Zipf columns per row, l2-normalized rows."""
    rng = np.random.default_rng(seed + 1)
    k = min(nnz_per_row, f)
    # Zipf-like column popularity over a random column permutation.
    pop = (np.arange(1, f + 1, dtype=np.float64)) ** (-zipf_a)
    pop = pop[rng.permutation(f)]
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]
    cols = np.searchsorted(cdf, rng.random((n, 2 * k)), side="right").clip(0, f - 1)
    cols.sort(axis=1)
    # drop duplicates inside each row, keep the first k distinct ones
    dup = np.zeros_like(cols, dtype=bool)
    dup[:, 1:] = cols[:, 1:] == cols[:, :-1]
    cols = np.where(dup, f, cols)  # push duplicates to the end
    cols.sort(axis=1)
    cols = cols[:, :k]
    valid = cols < f
    if empty_frac > 0:
        valid &= (rng.random(n) >= empty_frac)[:, None]
    counts = valid.sum(axis=1)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    indices = cols[valid].astype(np.int32)
    data = rng.random(indices.size).astype(np.float64) + 0.05
    x = sps.csr_matrix((data, indices, indptr.astype(np.int32)), shape=(n, f))
    norms = np.sqrt(np.asarray(x.multiply(x).sum(axis=1)).ravel())
    norms[norms == 0] = 1.0
    x = sps.diags(1.0 / norms) @ x
    x = sps.csr_matrix(x, dtype=np.float32)
    x.sort_indices()
    return x


def dense(n: int, k: int, seed: int = SEED, ld: int | None = None) -> np.ndarray:
    rng = np.random.default_rng(seed + 2)
    z = rng.standard_normal((n, k), dtype=np.float32)
    if ld is not None and ld > k:
        zp = np.zeros((n, ld), dtype=np.float32)
        zp[:, :k] = z
        return zp
    return z


def glorot_uniform(fan_in: int, fan_out: int, seed: int = SEED) -> np.ndarray:
    """lasagne.init.GlorotUniform (gain 1): U(-a, a), a = sqrt(6 / (fan_in + fan_out))."""
    rng = np.random.default_rng(seed + 3)
    a = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-a, a, size=(fan_in, fan_out)).astype(np.float32)
