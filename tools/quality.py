#!/usr/bin/env python3
"""Embedding-quality check of the GPU scatter modes against the CPU Hogwild
oracle on a benchmark graph (the reference has no quality metric; this uses
the LINE-2 edge score W_v . C_c).

AUC = P(score(positive edge) > score(random pair)) over 20k x 2k pairs.

    python tools/quality.py --config c2 --samples 40000000 --modes hogwild atomic
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def auc(W, C, offsets, targets, rng, n=20000, m=2000):
    V = len(offsets) - 1
    E = len(targets)
    src = np.repeat(np.arange(V, dtype=np.int64), np.diff(offsets))
    pick = rng.integers(0, E, n)
    pos = np.einsum("ij,ij->i", W[src[pick]], C[targets[pick]])
    neg = np.einsum("ij,ij->i", W[rng.integers(0, V, m)], C[rng.integers(0, V, m)])
    return float((pos[:, None] > neg[None, :]).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--samples", type=int, default=40_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--modes", nargs="+", default=["hogwild", "atomic"])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges(args.config)
    res = {"config": args.config, "samples": args.samples, "dim": args.dim}
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    off, tgt = pn.csr()
    total = args.samples + 1
    for mode in args.modes:
        pn.alloc_tables(args.dim, 2)
        pn.init_table_uniform(0, 3)
        pn.zero_table(1)
        t = time.perf_counter()
        pn.train_edges("line2", 0, args.samples, total, 5, 0.025, 0.0, 11, mode)
        el = time.perf_counter() - t
        W, C = pn.get_table(0), pn.get_table(1)
        res[mode] = {"auc": auc(W, C, off, tgt, np.random.default_rng(0)), "seconds": el,
                     "Mups": args.samples / el / 1e6, "finite": bool(np.isfinite(W).all())}
        print(mode, res[mode], flush=True)
    if args.cpu:
        from oracle import oracle as orc
        g = orc.Graph(V, src, dst, w)
        pn.alloc_tables(args.dim, 2)
        pn.init_table_uniform(0, 3)
        W = pn.get_table(0)
        C = np.zeros_like(W)
        threads = min(16, os.cpu_count() or 1)
        t = time.perf_counter()
        orc.train_edge_f32(g, "line2", W, C, args.dim, 5, 0.025, 0.0, total, 0, args.samples, 11, threads)
        el = time.perf_counter() - t
        res["cpu"] = {"auc": auc(W, C, off, tgt, np.random.default_rng(0)), "seconds": el, "threads": threads,
                      "Mups": args.samples / el / 1e6}
        print("cpu", res["cpu"], flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
