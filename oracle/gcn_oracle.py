"""CPU oracle for the graphconvgeo hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline. The product path
(graphconvgeo_amd) never imports it.

Restates, with citations into /root/reference:
  * normalize_adjacency   tensormain.py:168-181 (H = D^-1/2 (A+I) D^-1/2, float64 -> float32)
  * spmm_f32              S.dot (mlpconv.py:71,73,90) = scipy csr_matvecs, via the C port in
                          spmm_oracle.c (bitwise scipy float32; pinned in tests/test_oracle.py)
  * gcn_forward           SparseConvolutionDenseLayer.get_output_for (mlpconv.py:66-77) and
                          ConvolutionDenseLayer.get_output_for (mlpconv.py:86-95)
  * gcn_loss              categorical CE mean + L1/L2 shares (mlpconv.py:228-245)
  * gcn_backward          Theano autodiff of the above (S.dot grad (gz.y^T, x^T.gz);
                          inc_subtensor for Y[target_indices]; relu grad 0.5*(1+sign(x)))
  * adam                  lasagne.updates.adam(lr=4e-3, .9, .999, 1e-8) (mlpconv.py:263)

Third-party algorithms restated here (not vendored in the reference, no version pinned
by it): Theano sparse Dot / nnet.relu / softmax, Lasagne GlorotUniform / adam /
regularization, scipy sparsetools csr_matvecs (scipy 1.15.3 in this image).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np
import scipy.sparse as sps

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle_spmm.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile spmm_oracle.c with gcc (make -C oracle)."""
    src = os.path.join(_HERE, "spmm_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        build()
        lib = C.CDLL(_LIB_PATH)
        i64, p = C.c_int64, C.c_void_p
        lib.oracle_spmm_f32.argtypes = [i64, p, p, p, p, i64, i64, p, i64, p, C.c_int, p, i64]
        lib.oracle_spmm_f64.argtypes = [i64, p, p, p, p, i64, i64, p, i64]
        lib.oracle_scatter_add_f32.argtypes = [i64, p, p, i64, i64, p, i64, i64]
        for f in (lib.oracle_spmm_f32, lib.oracle_spmm_f64, lib.oracle_scatter_add_f32):
            f.restype = C.c_int
        _lib = lib
    return _lib


def _csr_arrays(H):
    H = sps.csr_matrix(H)
    return (np.ascontiguousarray(H.indptr, dtype=np.int32),
            np.ascontiguousarray(H.indices, dtype=np.int32), H)


# ---------------------------------------------------------------------------------------
# tensormain.py:168-181
# ---------------------------------------------------------------------------------------
def normalize_adjacency(adj, out_dtype=np.float32):
    """H = D^-1/2 * (A with diag set to 1) * D^-1/2, float64 then cast (tensormain.py:172-180,
    main_mlpconv's H.astype('float32') tensormain.py:221). Entry (i, j) is
    fl64(d_i^-1/2 * d_j^-1/2) rounded to out_dtype; storage sorted by column."""
    A = sps.csr_matrix(adj, dtype=np.float64).tolil()
    A.setdiag(1)
    A = A.tocsr()
    A.sort_indices()
    d = np.asarray(A.sum(axis=1)).ravel()
    with np.errstate(divide="ignore"):
        dinv = 1.0 / np.sqrt(d)
    dinv[np.isinf(dinv)] = 0
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    data = (dinv[rows] * A.data) * dinv[A.indices]
    H = sps.csr_matrix((data, A.indices.copy(), A.indptr.copy()), shape=A.shape)
    return H.astype(out_dtype)


def row_normalize_l1(adj, out_dtype=np.float32):
    """The reference's NON-symmetric operator D^-1 (A+I) (main.py:451-456): adjacency with the
    diagonal set to 1, then sklearn normalize(axis=1, norm='l1') -- every row divided by the
    sum of its absolute values (in float64), then .astype('float32'). Storage sorted by column."""
    A = sps.csr_matrix(adj, dtype=np.float64).tolil()
    A.setdiag(1)
    A = A.tocsr()
    A.sort_indices()
    s = np.add.reduceat(np.abs(A.data), A.indptr[:-1])  # every row holds its diagonal 1
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    H = sps.csr_matrix((A.data / s[rows], A.indices.copy(), A.indptr.copy()), shape=A.shape)
    return H.astype(out_dtype)


# ---------------------------------------------------------------------------------------
# S.dot(H, Z) -> scipy csr_matvecs (mlpconv.py:71,73,90) + layer epilogue
# ---------------------------------------------------------------------------------------
def spmm_f32(H, Z, bias=None, act=None, rows=None):
    """act(H @ Z + bias)[rows] in float32, storage order, no FMA (bitwise scipy)."""
    indptr, indices, H = _csr_arrays(H)
    vals = np.ascontiguousarray(H.data, dtype=np.float32)
    Z = np.ascontiguousarray(Z, dtype=np.float32)
    K = Z.shape[1]
    rows_a = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    n_out = H.shape[0] if rows_a is None else rows_a.size
    Y = np.empty((n_out, K), dtype=np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    rc = _load().oracle_spmm_f32(H.shape[0], indptr.ctypes.data, indices.ctypes.data,
                                 vals.ctypes.data, Z.ctypes.data, K, K, Y.ctypes.data, K,
                                 None if b is None else b.ctypes.data,
                                 1 if act in ("relu", "rectify") else 0,
                                 None if rows_a is None else rows_a.ctypes.data, n_out)
    if rc != 0:
        raise IndexError("row index out of range")
    return Y


def spmm_f64(H, Z):
    """H @ Z in float64 (tolerance reference)."""
    indptr, indices, H = _csr_arrays(H)
    vals = np.ascontiguousarray(H.data, dtype=np.float64)
    Z = np.ascontiguousarray(Z, dtype=np.float64)
    K = Z.shape[1]
    Y = np.empty((H.shape[0], K), dtype=np.float64)
    _load().oracle_spmm_f64(H.shape[0], indptr.ctypes.data, indices.ctypes.data, vals.ctypes.data,
                            Z.ctypes.data, K, K, Y.ctypes.data, K)
    return Y


def scatter_add_f32(out, idx, src):
    """out[idx[i]] += src[i], i ascending (Theano inc_subtensor for Y[idx], mlpconv.py:94)."""
    out = np.ascontiguousarray(out, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    src = np.ascontiguousarray(src, dtype=np.float32)
    K = out.shape[1]
    rc = _load().oracle_scatter_add_f32(idx.size, idx.ctypes.data, src.ctypes.data, K, K,
                                        out.ctypes.data, K, out.shape[0])
    if rc != 0:
        raise IndexError("index out of range")
    return out


# ---------------------------------------------------------------------------------------
# mlpconv.py:66-95 forward, 228-245 loss, Theano autodiff backward, 263 adam
# ---------------------------------------------------------------------------------------
def relu(x):
    """theano.tensor.nnet.relu(x) with alpha=0: 0.5 * (x + abs(x))."""
    return x.dtype.type(0.5) * (x + np.abs(x))


def softmax(x):
    """theano.tensor.nnet.softmax, row-wise, max-shifted."""
    e = np.exp(x - x.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def softmax_xent_f64(logits, y=None, scale=None):
    """float64 restatement of the output-layer loss: softmax (mlpconv.py:95), per-row
    categorical cross-entropy -log softmax[i, y_i] (mlpconv.py:229), hit = argmax == y with
    numpy's first-index argmax (mlpconv.py:227,252), and the logits gradient of the mean
    loss, (softmax - onehot) * scale with scale = 1/M (Theano's crossentropy_softmax grad).
    Returns (probabilities, loss_rows, hits, grad); the last three are None without y."""
    x = np.asarray(logits, dtype=np.float64)
    P = softmax(x)
    if y is None:
        return P, None, None, None
    y = np.asarray(y)
    r = np.arange(x.shape[0])
    m = x.max(axis=1)
    loss = (m + np.log(np.exp(x - m[:, None]).sum(axis=1))) - x[r, y]
    hits = (x.argmax(axis=1) == y).astype(np.float64)
    G = P.copy()
    G[r, y] -= 1.0
    G *= (1.0 / max(x.shape[0], 1)) if scale is None else scale
    return P, loss, hits, G


def gcn_forward(X, H, W1, b1, W2, b2, idx, dtype=np.float64):
    """Returns dict of intermediates: Z1, pre1, h, Z2, pre2, logits (= pre2[idx]), P."""
    if dtype == np.float32:
        Z1 = spmm_f32(X, W1)                          # S.dot(input, W)   mlpconv.py:71
        pre1 = spmm_f32(H, Z1, bias=b1)               # S.dot(H, .) + b   mlpconv.py:73-76
        h = relu(pre1)                                # rectify           mlpconv.py:77
        Z2 = np.asarray(h @ W2.astype(np.float32), dtype=np.float32)   # T.dot  mlpconv.py:88
        pre2 = spmm_f32(H, Z2, bias=b2)               # S.dot(H, .) + b   mlpconv.py:90-93
    else:
        Xd = sps.csr_matrix(X, dtype=np.float64)
        Hd = sps.csr_matrix(H, dtype=np.float64)
        Z1 = Xd @ W1.astype(np.float64)
        pre1 = Hd @ Z1 + b1.astype(np.float64)
        h = relu(pre1)
        Z2 = h @ W2.astype(np.float64)
        pre2 = Hd @ Z2 + b2.astype(np.float64)
    logits = pre2[np.asarray(idx)]                    # [target_indices, :] mlpconv.py:94
    P = softmax(logits)                               # softmax           mlpconv.py:95
    return {"Z1": Z1, "pre1": pre1, "h": h, "Z2": Z2, "pre2": pre2, "logits": logits, "P": P}


def gcn_loss(P, y, W1, W2, regul_coefs=(5e-5, 5e-5)):
    """mean categorical CE + 0.5*c*L1 + 0.5*c*L2 on W only (mlpconv.py:228-245;
    lasagne l1 = sum|W|, l2 = sum W^2; biases are not regularizable)."""
    c_out, c_hid = regul_coefs
    ce = -np.log(P[np.arange(P.shape[0]), np.asarray(y)]).mean()
    pen = (np.abs(W2).sum() * c_out * 0.5 + (W2.astype(np.float64) ** 2).sum() * c_out * 0.5
           + np.abs(W1).sum() * c_hid * 0.5 + (W1.astype(np.float64) ** 2).sum() * c_hid * 0.5)
    return ce + pen


def gcn_backward(X, H, W1, W2, fwd, idx, y, regul_coefs=(5e-5, 5e-5)):
    """float64 gradients of gcn_loss w.r.t. W1, b1, W2, b2 (Theano autodiff rules)."""
    c_out, c_hid = regul_coefs
    Xd = sps.csr_matrix(X, dtype=np.float64)
    Hd = sps.csr_matrix(H, dtype=np.float64)
    W1 = W1.astype(np.float64)
    W2 = W2.astype(np.float64)
    idx = np.asarray(idx)
    T = idx.size
    g_logits = fwd["P"].astype(np.float64).copy()
    g_logits[np.arange(T), np.asarray(y)] -= 1.0
    g_logits /= T
    g_pre2 = np.zeros(fwd["pre2"].shape, dtype=np.float64)
    np.add.at(g_pre2, idx, g_logits)                  # grad of [target_indices] (duplicates add)
    g_b2 = g_pre2.sum(axis=0)
    g_Z2 = Hd.T @ g_pre2                              # grad of S.dot wrt dense: x^T . gz
    g_W2 = fwd["h"].astype(np.float64).T @ g_Z2 + c_out * 0.5 * np.sign(W2) + c_out * W2
    g_h = g_Z2 @ W2.T
    g_pre1 = g_h * 0.5 * (1.0 + np.sign(fwd["pre1"]))  # d relu = 0.5*(1+sign(x))
    g_b1 = g_pre1.sum(axis=0)
    g_Z1 = Hd.T @ g_pre1
    g_W1 = Xd.T @ g_Z1 + c_hid * 0.5 * np.sign(W1) + c_hid * W1
    return {"W1": g_W1, "b1": g_b1, "W2": g_W2, "b2": g_b2, "Z1": g_Z1, "pre1": g_pre1,
            "Z2": g_Z2, "pre2": g_pre2}


def adam_step(params, grads, state, lr=4e-3, beta1=0.9, beta2=0.999, eps=1e-8):
    """lasagne.updates.adam (mlpconv.py:263): t += 1; a = lr*sqrt(1-b2^t)/(1-b1^t);
    m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= a m / (sqrt(v) + eps)."""
    t = state.get("t", 0) + 1
    state["t"] = t
    a = lr * np.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
    out = {}
    for k, p in params.items():
        g = grads[k]
        m = state.setdefault("m_" + k, np.zeros_like(p))
        v = state.setdefault("v_" + k, np.zeros_like(p))
        m[...] = beta1 * m + (1 - beta1) * g
        v[...] = beta2 * v + (1 - beta2) * g * g
        out[k] = p - a * m / (np.sqrt(v) + eps)
    return out


def mlpconv_train(X, H, Y, train_idx, dev_idx, W1, b1, W2, b2, n_epochs, regul_coefs,
                  report_k_epoch=10):
    """float64 restatement of MLPCONV.fit's loop (mlpconv.py:288-309): one full-batch Adam step
    per epoch on mean CE + L1/L2 shares; dev loss every report_k_epoch epochs. Returns the
    per-epoch history and the final parameters (no early stopping / restore)."""
    params = {"W1": W1.astype(np.float64), "b1": b1.astype(np.float64),
              "W2": W2.astype(np.float64), "b2": b2.astype(np.float64)}
    Y = np.asarray(Y)
    state, hist = {}, []
    for n in range(n_epochs):
        f = gcn_forward(X, H, params["W1"], params["b1"], params["W2"], params["b2"], train_idx)
        y = Y[train_idx]
        loss = gcn_loss(f["P"], y, params["W1"], params["W2"], regul_coefs)
        acc = float((f["logits"].argmax(axis=1) == y).mean())
        g = gcn_backward(X, H, params["W1"], params["W2"], f, train_idx, y, regul_coefs)
        rec = {"epoch": n, "train_loss": float(loss), "train_acc": acc}
        params = adam_step(params, {k: g[k] for k in params}, state)
        if n % report_k_epoch == 0:
            # validation runs after the update, as f_val follows f_train (mlpconv.py:295-297)
            fv = gcn_forward(X, H, params["W1"], params["b1"], params["W2"], params["b2"], dev_idx)
            yd = Y[dev_idx]
            rec["val_loss"] = float(gcn_loss(fv["P"], yd, params["W1"], params["W2"], regul_coefs))
            rec["val_acc"] = float((fv["logits"].argmax(axis=1) == yd).mean())
        hist.append(rec)
    return hist, params


def project_mentions(n_users, n_nodes, a, b, celebrity_threshold=10):
    """Pure-Python restatement of get_graph's celebrity filter (data.py:364-370) and
    efficient_collaboration_weighted_projected_graph2 (data.py:226-250) on the incidence
    list: users carry self loops; a mention node survives iff 1 < degree <= threshold; every
    pair of user neighbours of a surviving node becomes an edge. Returns sorted (u < v) pairs."""
    adj = [set() for _ in range(n_nodes)]
    for x, y in zip(np.asarray(a).tolist(), np.asarray(b).tolist()):
        if x != y:
            adj[x].add(y)
            adj[y].add(x)
    dead = {m for m in range(n_users, n_nodes)
            if len(adj[m]) == 1 or len(adj[m]) > celebrity_threshold}
    edges = set()
    for m in range(n_nodes):
        if m in dead:
            continue
        T = sorted({t for t in adj[m] if t < n_users} | ({m} if m < n_users else set()))
        for i in range(len(T)):
            for j in range(i + 1, len(T)):
                edges.add((T[i], T[j]))
    return np.array(sorted(edges), dtype=np.int64).reshape(-1, 2)
