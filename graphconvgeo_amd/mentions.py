"""Mention graph: host-side parsing (stays on the host, per BASELINE north_star) + the
O(sum deg^2) projection on the GPU.

`mention_incidences` restates DataLoader.get_graph's parsing (data.py:302-362): users are
numbered train, dev, test in table order; every @mention (regex of data.py:311, lowercased)
that names a user maps to that user's id, any other name gets the next new id in order of
first appearance; each (mentioned id, user id) pair is one incidence.

`project_mentions` runs the celebrity filter (data.py:364-370) and the projection of
efficient_collaboration_weighted_projected_graph2 (data.py:226-250) on the GPU
(gcg_project_mention_graph) and returns the user-user edge list; `mention_graph_operator`
chains it into the normalized operator H (gcg_normalize_adjacency_f32).
"""
from __future__ import annotations

import ctypes as C
import re

import numpy as np
import torch

from ._native import call

MENTION_PATTERN = re.compile(r"(?<=^|(?<=[^a-zA-Z0-9-_\.]))@([A-Za-z]+[A-Za-z0-9_]+)")


def mention_incidences(df_train, df_dev, df_test):
    """(n_users, n_nodes, a, b) of the bipartite mention graph, as data.py:302-362 builds it.

    The frames are indexed by (lowercased, sorted) user name with a `text` column, as
    DataLoader.load_data leaves them (data.py:273-299)."""
    users = list(df_train.index) + list(df_dev.index) + list(df_test.index)
    node_id = {u: i for i, u in enumerate(users)}
    if len(node_id) != len(users):
        raise ValueError("duplicate target node")  # data.py:305
    a, b = [], []
    for df in (df_train, df_dev, df_test):
        texts = df["text"].tolist()
        for user, text in zip(df.index, texts):
            uid = node_id[user]
            ids = set()
            for m in MENTION_PATTERN.findall(text):
                m = m.lower()
                if m not in node_id:
                    node_id[m] = len(node_id)
                ids.add(node_id[m])
            for i in sorted(ids):
                a.append(i)
                b.append(uid)
    return len(users), len(node_id), np.asarray(a, np.int32), np.asarray(b, np.int32)


def project_mentions(n_users: int, n_nodes: int, a, b, celebrity_threshold: int = 10,
                     device="cuda"):
    """User-user edges (u < v, sorted, unique) of the projected mention graph, on the GPU."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("the projection runs on the GPU: device must be a CUDA (HIP) device")
    at = torch.as_tensor(np.asarray(a, np.int32)).to(dev)
    bt = torch.as_tensor(np.asarray(b, np.int32)).to(dev)
    if at.shape != bt.shape:
        raise ValueError("a and b must have the same length")
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ne = C.c_int64()
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    args = (int(n_users), int(n_nodes), int(at.numel()), C.c_void_p(at.data_ptr()),
            C.c_void_p(bt.data_ptr()), int(celebrity_threshold))
    with torch.cuda.device(dev):
        call("gcg_project_mention_graph", *args, None, None, 0, C.byref(ne),
             C.c_void_p(status.data_ptr()), stream)
        if int(status.item()) != 0:
            raise ValueError("incidence id out of range [0, n_nodes)")
        cap = max(ne.value, 1)
        u = torch.empty(cap, dtype=torch.int32, device=dev)
        v = torch.empty(cap, dtype=torch.int32, device=dev)
        call("gcg_project_mention_graph", *args, C.c_void_p(u.data_ptr()), C.c_void_p(v.data_ptr()),
             cap, C.byref(ne), C.c_void_p(status.data_ptr()), stream)
    return u[: ne.value], v[: ne.value]


def mention_graph_operator(df_train, df_dev, df_test, celebrity_threshold: int = 10,
                           device="cuda"):
    """H = D^-1/2 (A+I) D^-1/2 of the projected mention graph, built on the GPU
    (tensormain.py:168-181 over DataLoader.get_graph's graph)."""
    from .graph import normalize_edges_device

    n_users, n_nodes, a, b = mention_incidences(df_train, df_dev, df_test)
    u, v = project_mentions(n_users, n_nodes, a, b, celebrity_threshold, device)
    return normalize_edges_device(n_users, u.cpu().numpy(), v.cpu().numpy(), device)
