#!/usr/bin/env python3
"""DeepWalk scatter-mode quality: held-out skip-gram AUC (positive edge vs
random pair) after training with each setting.  Prints one JSON line each.

    python tools/dw_quality.py --graph tests/golden/pl1k.txt --settings atomic hybrid:0.3:128:32
    python tools/dw_quality.py --config small --walk-times 2
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default=None)
    ap.add_argument("--config", default=None)
    ap.add_argument("--dim", type=int, default=32)
    ap.add_argument("--walk-times", type=int, default=4)
    ap.add_argument("--walk-steps", type=int, default=20)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--settings", nargs="+", default=["atomic", "hybrid:0.3:128:32", "hybrid:0.3:0:32",
                                                      "hybrid:1e30:0:32", "hogwild"])
    args = ap.parse_args()
    import smore_amd
    pn = smore_amd.ProNet(0)
    if args.graph:
        pn.LoadEdgeList(args.graph, 1)
    else:
        from smore_amd import graphgen
        V, (src, dst, w) = graphgen.config_edges(args.config)
        pn.set_graph_edges(V, src, dst, w)
    V = pn.MAX_vid
    off, tgt = pn.csr()
    rng = np.random.default_rng(3)
    srcv = np.repeat(np.arange(V), np.diff(off))
    pick = rng.integers(0, len(tgt), 20000)
    negv, negc = rng.integers(0, V, 2000), rng.integers(0, V, 2000)
    order = smore_amd.deepwalk_order(V, args.walk_times, 0)
    held = pn.sample_edges("line2", 1 << 40, 100_000, 5, 99)

    def loss_of(W, C):
        v, c, n = held[:, 0], held[:, 1], held[:, 2:]
        ok = c >= 0
        v, c, n = v[ok], c[ok], n[ok]
        Wv = W[v].astype(np.float64)
        l = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
        for k in range(n.shape[1]):
            l += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[n[:, k]].astype(np.float64)))
        return float(l.mean())
    for s in args.settings:
        parts = s.split(":")
        mode = parts[0]
        if mode == "hybrid":
            pn.set_hot_threshold(float(parts[1]))
            pn.set_write_combine(int(parts[2]), int(parts[3]))
        pn.alloc_tables(args.dim, 2)
        pn.init_table_glibc(0, 0)
        pn.zero_table(1)
        t0 = time.perf_counter()
        pn.train_deepwalk(0, args.walk_times * V, args.walk_times, args.walk_steps, args.window, 5, 0.025, 20251015,
                          order, mode)
        el = time.perf_counter() - t0
        W, C = pn.get_table(0), pn.get_table(1)
        pos = np.einsum("ij,ij->i", W[srcv[pick]], C[tgt[pick]])
        neg = np.einsum("ij,ij->i", W[negv], C[negc])
        auc = float((pos[:, None] > neg[None, :]).mean())
        print(json.dumps({"graph": args.graph or args.config, "setting": s, "auc": round(auc, 4),
                          "heldout_loss": round(loss_of(W, C), 5),
                          "wall_s": round(el, 3), "hot_rows": pn.hot_rows()}), flush=True)


if __name__ == "__main__":
    main()
