"""Seeded synthetic power-law graphs for the benchmark configs:
endpoints ~ Zipf(s=0.8) over their vertex range, ids randomly permuted,
weight 1.0.  Undirected lines are pushed as v1->v2 then v2->v1 (the reference
loader's order, src/proNet.cpp:208-215).  Generated natively
(smore_gen_powerlaw, multi-threaded, thread-count independent).
"""
import ctypes as C

import numpy as np

from . import _lib

CONFIGS = {
    # name: (kind, V or (users, items), lines, undirected, seed)
    "c2": ("powerlaw", 1_000_000, 20_000_000, True, 2),              # LINE-2 1M / 20M, d=64
    "c3": ("bipartite", (2_000_000, 1_000_000), 100_000_000, False, 3),  # BPR 2M x 1M / 100M, d=128
    "c4": ("powerlaw", 10_000_000, 200_000_000, True, 4),            # LINE-2 10M / 200M, d=64
    "c5": ("powerlaw", 1_134_890, 2_987_624, True, 5),              # Youtube-links-sized stand-in
    "small": ("powerlaw", 100_000, 2_000_000, True, 1),
}


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def powerlaw_edges(V, lines, undirected=True, seed=2, s=0.8):
    """(src, dst, w) directed edge slots in push order."""
    n = lines * (2 if undirected else 1)
    src = np.empty(n, np.int32)
    dst = np.empty(n, np.int32)
    rc = _lib.lib.smore_gen_powerlaw(int(V), int(lines), int(bool(undirected)), float(s), int(seed), _ptr(src),
                                     _ptr(dst))
    if rc != _lib.OK:
        raise _lib.SmoreError("smore_gen_powerlaw failed with status %d" % rc)
    return src, dst, np.ones(n, np.float64)


def bipartite_edges(users, items, lines, seed=3, s=0.8):
    """user -> item slots: users Zipf over [0, users), items Zipf over
    [users, users + items) (C3: 2M users x 1M items, directed)."""
    src, _, _ = powerlaw_edges(users, lines, False, seed * 2 + 1, s)
    _, dst, w = powerlaw_edges(items, lines, False, seed * 2 + 2, s)
    dst += users
    return src, dst, w


def config_edges(name):
    kind, V, lines, und, seed = CONFIGS[name]
    if kind == "bipartite":
        users, items = V
        return users + items, bipartite_edges(users, items, lines, seed)
    return V, powerlaw_edges(V, lines, und, seed)
