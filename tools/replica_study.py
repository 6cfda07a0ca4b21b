#!/usr/bin/env python3
"""Multi-GPU replica quality through the library's own group driver
(smore_group_*, exchange.cpp), with N replicas on ONE GPU (the group's local
collectives): the same rounds, source partition, adaptive scales (row census
for the walk models) and one-late exchange as an N-GPU group, only the
all-reduce is a device pass.  DESIGN.md 10.

LINE-2 (`--model line2`, config c2 by default): held-out loss after T total
samples for 1 replica (the reference's one shared table) and for N replicas
at `--per-row` samples per row per replica per exchange (13.42 = the C4
bench's 2^27 samples per step over 10M rows), at several totals T, exchange
periods and c0.  Samples-to-loss: for each N-replica setting, the total it
needs to reach one replica's loss at T (log-linear interpolation over its
totals) gives the effective speed-up at N GPUs = N * T / T_N (before the
exchange's own cost).

DeepWalk (`--model deepwalk`, config c5 / a golden graph): held-out loss and
edge AUC after walk_times walks per vertex, 1 vs N replicas, walks per replica
per exchange from `--per-row` pair-updates per row.

One JSON line per run.

    python tools/replica_study.py --model line2 --config c2 --ranks 1 4 8 --totals 29 30 31 32 \
        --periods 1 0.5 0.25 --c0 1024 2048 4096
    python tools/replica_study.py --model deepwalk --config c5 --ranks 1 2 4 8 --c0 256 1024 4096
"""
import argparse
import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def heldout_loss(W, C, draws):
    v, c, negs = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = c >= 0
    v, c, negs = v[keep], c[keep], negs[keep]
    Wv = W[v].astype(np.float64)
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k]].astype(np.float64)))
    return float(loss.mean())


def edge_auc(W, C, off, tgt, seed=3):
    rng = np.random.default_rng(seed)
    V = len(off) - 1
    srcv = np.repeat(np.arange(V), np.diff(off))
    pick = rng.integers(0, len(tgt), 20000)
    nv, nc = rng.integers(0, V, 2000), rng.integers(0, V, 2000)
    pos = np.einsum("ij,ij->i", W[srcv[pick]].astype(np.float64), C[tgt[pick]].astype(np.float64))
    neg = np.einsum("ij,ij->i", W[nv].astype(np.float64), C[nc].astype(np.float64))
    return float((pos[:, None] > neg[None, :]).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="line2", choices=["line2", "deepwalk"])
    ap.add_argument("--config", default="c2")
    ap.add_argument("--graph", default=None, help="edge-list file instead of a config")
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--totals", type=float, nargs="+", default=[30],
                    help="line2: log2 of the total samples; deepwalk: walk_times")
    ap.add_argument("--periods", type=float, nargs="+", default=[1.0], help="exchange period x the --per-row period")
    ap.add_argument("--c0", type=float, nargs="+", default=[2048.0])
    ap.add_argument("--rules", nargs="+", default=["adaptive"])
    ap.add_argument("--per-row", type=float, default=13.42,
                    help="updates per row per replica per exchange (line2: samples; deepwalk: pairs)")
    ap.add_argument("--mode", default="hybrid")
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--no-partition", action="store_true")
    ap.add_argument("--walk-partition", action="store_true", help="walk models: W partitioned by walk center")
    ap.add_argument("--combine-rows", type=int, default=None, help="hybrid: LDS write-combined rows on every replica")
    ap.add_argument("--hot-exchange", type=int, default=None, help="sum rule: hub rows synced per launch (0: off)")
    ap.add_argument("--diag", action="store_true", help="largest rows of each table and their census rate rank")
    ap.add_argument("--hot-tau", type=float, default=None, help="hybrid: hot-row threshold on every replica")
    ap.add_argument("--schedule", default="replicas", choices=["replicas", "blocks"],
                    help="group schedule (blocks: --per-row = samples per row per replica per epoch for line2; "
                         "deepwalk: --walks-per-epoch)")
    ap.add_argument("--walks-per-epoch", type=int, default=0, help="blocks, deepwalk: walks per epoch (0: default)")
    ap.add_argument("--hubs", type=int, nargs="+", default=[-1],
                    help="blocks: hub C rows per setting (-1 the library's default, 0 none)")
    args = ap.parse_args()

    import smore_amd
    from smore_amd import graphgen

    if args.graph:
        src = dst = None
    else:
        V, (src, dst, w) = graphgen.config_edges(args.config)
    line = args.model == "line2"
    dim = args.dim or (64 if line else 128)
    K = 5
    groups = {}

    def group(n):
        if n not in groups:
            g = smore_amd.Group([0] * n)
            if args.graph:
                g.LoadEdgeList(args.graph, 1)
            else:
                g.set_graph_edges(V, src, dst, w)
            g.alloc_tables(dim, 2)
            g.set_partition(not args.no_partition)
            g.set_walk_partition(args.walk_partition)
            g.set_schedule(args.schedule)
            if args.hot_exchange is not None:
                g.set_hot_exchange(args.hot_exchange)
            for r in g.replicas:
                if args.combine_rows is not None:
                    r.set_write_combine(args.combine_rows)
                if args.hot_tau is not None:
                    r.set_hot_threshold(args.hot_tau)
            groups[n] = g
        return groups[n]

    g1 = group(1)
    Vn = g1.primary.MAX_vid
    held = g1.primary.sample_edges("line2", (1 << 40) + 17, 100_000, K, args.seed + 1)
    off, tgt = g1.primary.csr()
    pairs_per_walk = None
    for n, tot, period, c0, rule, hubs in itertools.product(args.ranks, args.totals, args.periods, args.c0,
                                                            args.rules, args.hubs):
        if n == 1 and (period != args.periods[0] or c0 != args.c0[0] or rule != args.rules[0] or
                       hubs != args.hubs[0]):
            continue
        # one replica at a time on the GPU: free the others' memory
        for m in [m for m in groups if m not in (1, n)]:
            groups.pop(m).close()
        g = group(n)
        g.set_adaptive(c0)
        for r in g.replicas:
            r.block_set_hubs(hubs)
        p = g.primary
        p.init_table_glibc(0, 0)
        p.zero_table(1)
        g.broadcast_tables()
        t0 = time.perf_counter()
        if line:
            T = int(2 ** tot)
            per = max(1, int(args.per_row * Vn * period)) if args.per_row > 0 else 0   # 0: the group default
            g.train_edges("line2", 0, T, T, K, 0.025, 0.0, args.seed, args.mode, per=per, mean=rule)
            row = {"model": "line2", "total": T, "log2_total": tot, "samples_per_exchange": per}
        else:
            wt = int(tot)
            order = smore_amd.deepwalk_order(Vn, wt, 0)
            if pairs_per_walk is None:
                p.census_begin()
                p.train_deepwalk(0, min(Vn, 1 << 16), wt, 40, 5, K, 0.025, args.seed, order, args.mode)
                p.census_end(min(Vn, 1 << 16))
                pairs_per_walk = float(p.row_rates("census", K, 0).sum())
            per = max(1, int(args.per_row * Vn * period / pairs_per_walk)) if args.per_row > 0 else 0
            if args.schedule == "blocks":
                per = args.walks_per_epoch
            g.train_deepwalk(0, wt * Vn, wt, 40, 5, K, 0.025, args.seed, order, args.mode, per=per, mean=rule)
            row = {"model": "deepwalk", "walk_times": wt, "walks_per_exchange": per,
                   "pairs_per_walk": round(pairs_per_walk, 2)}
        el = time.perf_counter() - t0
        W, C = p.get_table(0), p.get_table(1)
        spread = 0.0
        if n > 1:
            Cl = g.replicas[n - 1].get_table(1)
            spread = float(np.abs(Cl - C).max() / max(1e-30, np.abs(C).max()))
        if args.diag and (line or n > 1):
            # where a run went wrong: the largest rows of each table and their
            # rank in the census's touch rates (0 = the hottest row)
            for t, T in (("W", W), ("C", C)):
                nrm = np.sqrt((T.astype(np.float64) ** 2).sum(1))
                try:
                    rate = p.row_rates("census" if not line else "line2", K, 0 if t == "W" else 1)
                except smore_amd._lib.SmoreError:   # no census (the block schedule): the LINE-2 law
                    rate = p.row_rates("line2", K, 0 if t == "W" else 1)
                rank = np.empty(len(rate), np.int64)
                rank[np.argsort(-rate)] = np.arange(len(rate))
                top = np.argsort(-nrm)[:8]
                row["diag_" + t] = {"norm_p50": float(np.median(nrm)), "norm_p99": float(np.quantile(nrm, 0.99)),
                                    "top_norm": [round(float(nrm[i]), 3) for i in top],
                                    "top_rate_rank": [int(rank[i]) for i in top],
                                    "rows_norm_gt_10": int((nrm > 10).sum())}
        row.update({"config": args.graph or args.config, "ranks": n, "rule": rule if n > 1 else "one",
                    "schedule": args.schedule if n > 1 else "one",
                    "c0": c0, "period": period, "per_row": args.per_row, "mode": args.mode,
                    "combine_rows": args.combine_rows, "hot_tau": args.hot_tau, "hot_exchange": args.hot_exchange,
                    "walk_partition": args.walk_partition,
                    "hubs": int(p.block_hubs()[0]) if n > 1 and args.schedule == "blocks" else 0,
                    "neg_law": os.environ.get("SMORE_NEG_LAW", "1"), "hub_c0": os.environ.get("SMORE_HUB_C0", ""),
                    "hub_split": os.environ.get("SMORE_HUB_SPLIT", ""),
                    "local_serial": os.environ.get("SMORE_LOCAL_SERIAL", ""),
                    "finite": bool(np.isfinite(W).all() and np.isfinite(C).all()),
                    "loss": round(heldout_loss(W, C, held), 5), "auc": round(edge_auc(W, C, off, tgt), 5),
                    "replica_spread_rel": spread, "wall_s": round(el, 2)})
        print(json.dumps(row), flush=True)
    for g in groups.values():
        g.close()


if __name__ == "__main__":
    main()
