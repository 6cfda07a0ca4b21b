#!/usr/bin/env python3
"""Embedding-quality check of the GPU scatter modes against the CPU Hogwild
oracle on a benchmark graph.  The reference has no quality metric; this uses
its own training objective on held-out draws (seed != training seed):
  loss  = mean over samples of -log s(W_v.C_c) - sum_k log s(-W_v.C_nk)
  auc   = P(W_v.C_c > W_v.C_n) for the sample's positive c vs its negatives n
with (v, c, n1..n5) drawn by the reference samplers (source alias, per-vertex
context alias, negative alias).

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


def objective(W, C, draws):
    v, c, n = draws[:, 0], draws[:, 1], draws[:, 2:]
    ok = c >= 0
    v, c, n = v[ok], c[ok], n[ok]
    pos = np.einsum("ij,ij->i", W[v], C[c])
    neg = np.einsum("ij,ikj->ik", W[v], C[n])
    ls = lambda x: -np.logaddexp(0.0, -x)  # log sigmoid
    loss = float(np.mean(-ls(pos) - ls(-neg).sum(1)))
    auc = float(np.mean(pos[:, None] > neg))
    return {"loss": round(loss, 5), "auc": round(auc, 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--samples", type=int, default=40_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--modes", nargs="+", default=["hogwild", "atomic"])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--semantics", default="cpp", choices=["cpp", "go"])
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges(args.config)
    res = {"config": args.config, "samples": args.samples, "dim": args.dim}
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    if args.semantics == "go":
        pn.set_semantics("go")
        res["semantics"] = "go"
    draws = pn.sample_edges("line2", 1 << 40, 200000, 5, 99991)   # held-out draws
    total = args.samples + 1
    for spec in args.modes:
        parts = spec.split(":")          # mode[:tau[:combine_rows[:flush_rounds]]]
        mode = parts[0]
        if len(parts) > 1:
            pn.set_hot_threshold(float(parts[1]))
        pn.set_write_combine(int(parts[2]) if len(parts) > 2 else 128, int(parts[3]) if len(parts) > 3 else 32)
        pn.alloc_tables(args.dim, 2)
        pn.init_table_uniform(0, 3)
        pn.zero_table(1)
        t = time.perf_counter()
        pn.train_edges("line2", 0, args.samples, total, 5, 0.025, 0.0, 11, mode)
        el = time.perf_counter() - t
        W, C = pn.get_table(0), pn.get_table(1)
        res[spec] = dict(objective(W, C, draws), seconds=round(el, 4), Mups=round(args.samples / el / 1e6, 2),
                         finite=bool(np.isfinite(W).all()))
        if mode == "hybrid":
            res[spec]["hot_rows_w_c"] = pn.hot_rows()
        print(spec, res[spec], flush=True)
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
        res["cpu"] = dict(objective(W, C, draws), seconds=round(el, 2), threads=threads,
                          Mups=round(args.samples / el / 1e6, 3))
        print("cpu", res["cpu"], flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
