#!/usr/bin/env python3
"""DeepWalk on one context, the same walks in calls of different sizes:
held-out loss / edge AUC per scatter mode and call size (does anything in a
call's setup or tail depend on its size?).  C5 stand-in graph, d=128.

    python tools/dw_calls_probe.py --calls 0 22856 5714 --modes hybrid atomic
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--calls", type=int, nargs="+", default=[0, 22856, 5714], help="walks per call (0: one call)")
    ap.add_argument("--modes", nargs="+", default=["hybrid", "atomic"])
    ap.add_argument("--walk-times", type=int, default=10)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--combine-rows", type=int, nargs="+", default=[None], help="hybrid: LDS write-combined rows")
    ap.add_argument("--hot-tau", type=float, nargs="+", default=[None])
    ap.add_argument("--flush", type=int, nargs="+", default=[0], help="hybrid: LDS drain interval (0: automatic)")
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    from replica_study import edge_auc, heldout_loss
    V, (src, dst, w) = graphgen.config_edges(args.config)
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    V = pn.MAX_vid
    held = pn.sample_edges("line2", (1 << 40) + 17, 100_000, 5, args.seed + 1)
    off, tgt = pn.csr()
    wt = args.walk_times
    order = smore_amd.deepwalk_order(V, wt, 0)
    pn.alloc_tables(args.dim, 2)
    import itertools
    for mode, per, rows, tau, fl in itertools.product(args.modes, args.calls, args.combine_rows, args.hot_tau,
                                                      args.flush):
        if mode != "hybrid" and (rows is not None or tau is not None or fl):
            continue
        pn.set_write_combine(128 if rows is None else rows, fl)
        pn.set_hot_threshold(-1 if tau is None else tau)
        if True:
            pn.init_table_glibc(0, 0)
            pn.init_table_glibc(1, V * args.dim)
            total = wt * V
            step = per or total
            t0 = time.perf_counter()
            for b in range(0, total, step):
                pn.train_deepwalk(b, min(total, b + step), wt, 40, 5, 5, 0.025, args.seed, order, mode)
            pn.synchronize()
            el = time.perf_counter() - t0
            W, C = pn.get_table(0), pn.get_table(1)
            print(json.dumps({"config": args.config, "mode": mode, "combine_rows": rows, "hot_tau": tau, "flush": fl,
                              "combine_info": pn.write_combine_info() if mode == "hybrid" else None,
                              "walks_per_call": step,
                              "calls": -(-total // step), "loss": round(heldout_loss(W, C, held), 5),
                              "auc": round(edge_auc(W, C, off, tgt), 5), "wall_s": round(el, 2)}), flush=True)


if __name__ == "__main__":
    main()
