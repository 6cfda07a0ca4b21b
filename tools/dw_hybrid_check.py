#!/usr/bin/env python3
"""Held-out AUC of DeepWalk and LINE-2 on the 920-vertex golden graph under the
scatter modes, with optional grid caps (SMORE_MAX_BLOCKS) -- the experiment
behind tests/test_gpu_configs.py::test_deepwalk_hybrid_mixed_tags_matches_atomic.

    python tools/dw_hybrid_check.py [--blocks 0 1 2] [--lib path/to/libsmore_hip.so]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--tau", type=float, default=0.3)
    args = ap.parse_args()
    import smore_amd
    from oracle import oracle as orc
    path = os.path.join(ROOT, "tests", "golden", "pl1k.txt")
    g = orc.Graph.from_file(path, 1)
    pn = smore_amd.ProNet(0)
    pn.LoadEdgeList(path, 1)
    rng = np.random.default_rng(3)
    src = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, 20000)
    negv, negc = rng.integers(0, g.V, 2000), rng.integers(0, g.V, 2000)

    def auc(W, C):
        pos = np.einsum("ij,ij->i", W[src[pick]], C[g.targets[pick]])
        neg = np.einsum("ij,ij->i", W[negv], C[negc])
        return float((pos[:, None] > neg[None, :]).mean())

    dim, K, times = 32, 5, 4
    order = smore_amd.deepwalk_order(g.V, times, 0)
    for nb in args.blocks:
        if nb > 0:
            os.environ["SMORE_MAX_BLOCKS"] = str(nb)
        else:
            os.environ.pop("SMORE_MAX_BLOCKS", None)
        for model in ("deepwalk", "line2"):
            for mode in ("serial", "atomic", "hybrid", "hogwild"):
                if model == "deepwalk" and mode == "serial" and nb not in (0,):
                    continue
                pn.alloc_tables(dim, 2)
                pn.init_table_glibc(0, 0)
                pn.zero_table(1)
                pn.set_hot_threshold(args.tau)
                if model == "deepwalk":
                    pn.train_deepwalk(0, times * g.V, times, 20, 5, K, 0.025, 7, order, mode)
                else:
                    total = 2 * 10 ** 6
                    pn.train_edges("line2", 0, total - 1, total, K, 0.025, 0.0, 7, mode)
                W, C = pn.get_table(0), pn.get_table(1)
                print(json.dumps({"blocks": nb, "model": model, "mode": mode, "auc": round(auc(W, C), 4),
                                  "finite": bool(np.isfinite(W).all() and np.isfinite(C).all())}), flush=True)


if __name__ == "__main__":
    main()
