#!/usr/bin/env python3
"""Held-out skip-gram AUC of the walk models on the 1k-vertex golden graph,
per scatter mode and dimension: C++ DeepWalk and Go DeepWalk (the serial mode
is the oracle's order; the parallel modes must train like it).

    python tools/go_walk_check.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import smore_amd
    from oracle import oracle as orc
    path = os.path.join(ROOT, "tests", "golden", "pl1k.txt")
    g = orc.Graph.from_file(path, 1)
    rng = np.random.default_rng(3)
    src = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, 20000)
    negv, negc = rng.integers(0, g.V, 2000), rng.integers(0, g.V, 2000)

    def auc(W, C):
        pos = np.einsum("ij,ij->i", W[src[pick]], C[g.targets[pick]])
        neg = np.einsum("ij,ij->i", W[negv], C[negc])
        return float((pos[:, None] > neg[None, :]).mean())

    times = 4
    for sem in ("cpp", "go"):
        pn = smore_amd.ProNet(0)
        pn.LoadEdgeList(path, 1)
        if sem == "go":
            pn.set_semantics("go")
        order = smore_amd.deepwalk_order(g.V, times, 0)
        for dim in (32, 64):
            for mode in ("serial", "atomic", "hogwild", "hybrid"):
                pn.alloc_tables(dim, 2)
                pn.init_table_glibc(0, 0)
                pn.zero_table(1)
                pn.train_deepwalk(0, times * g.V, times, 20, 5, 5, 0.025, 777001, order, mode)
                W, C = pn.get_table(0), pn.get_table(1)
                print(json.dumps({"semantics": sem, "dim": dim, "mode": mode, "auc": round(auc(W, C), 4),
                                  "finite": bool(np.isfinite(W).all()), "wmax": float(np.abs(W).max())}), flush=True)


if __name__ == "__main__":
    main()
