#!/usr/bin/env python3
"""What the replica exchange does to training at N GPUs, measured
on ONE GPU: N library contexts hold N replicas of a config's graph and tables,
each runs its own global-sample ranges exactly as bench.py's ranks do
(2^27 / 10 * V/1M samples per step per replica = the C4 bench's samples per
row per step), and after every step the snapshot-delta exchange runs with the
bench's one-exchange-late schedule (begin = [end of the previous exchange +]
D = T - S; R = D; S = T; the all-reduce is the sum of the replicas' R; end =
X = scale * R - D; T += X; S += X).  The replicas run one after another on the
GPU, which changes nothing in the arithmetic: each trains from its own state.

Reports the held-out LINE-2 loss of replica 0 after `--total` samples, against
one replica trained on the same total, for the sum and mean exchanges.

--sub k --hot H: every step runs as k launches, and after each one the H rows of
each table with the highest expected touch rate (the hub rows: source law for
W, context + K x negative law for C) are exchanged synchronously
(D' = T_h - S_h; R' = sum of the replicas' D'; T_h += R' - D'; S_h += R'),
composing with the one-late full exchange (no update counted twice).

    python tools/replica_sim.py --config c2 --ranks 1 2 4 8 --sync sum mean
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def heldout_loss(W, C, draws, dim):
    v, c, negs = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = c >= 0
    v, c, negs = v[keep], c[keep], negs[keep]
    Wv = W[v, :dim].astype(np.float64)
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c, :dim].astype(np.float64)))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k], :dim].astype(np.float64)))
    return float(loss.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--sync", nargs="+", default=["sum", "mean"])
    ap.add_argument("--total", type=int, default=1 << 30)
    ap.add_argument("--per-row", type=float, default=13.42, help="samples per vertex per step per replica")
    ap.add_argument("--mode", default="hybrid")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--sub", type=int, nargs="+", default=[1], help="launches (hot exchanges) per step")
    ap.add_argument("--hot", type=int, nargs="+", default=[0], help="hot rows per table exchanged per launch")
    ap.add_argument("--c0", type=float, nargs="+", default=[64.0],
                    help="adaptive: a row whose expected updates per exchange over all ranks, n*k, is at most c0 "
                         "is summed, a hotter one scaled by s + (1 - s)/n with s = c0/(n*k)")
    args = ap.parse_args()

    import torch
    import smore_amd
    from smore_amd import graphgen
    from smore_amd.dist import TorchPasses, table_tensor

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    V, (src, dst, w) = graphgen.config_edges(args.config)
    K, dim = 5, args.dim
    S = int(args.per_row * V)
    ctxs = []

    def ctx(i):
        while len(ctxs) <= i:
            pn = smore_amd.ProNet(0)
            pn.set_graph_edges(V, src, dst, w)
            pn.set_stream(stream.cuda_stream)
            pn.alloc_tables(dim, 2)
            ctxs.append(pn)
        return ctxs[i]

    heldout = ctx(0).sample_edges("line2", (1 << 40) + 17, 100_000, K, args.seed + 1)
    # expected touches per sample (unit weights): W rows by the source law
    # out_deg^0.75, C rows by the context law (source law / out-degree per
    # edge) plus K x the negative law (in + out)^0.75
    od = np.bincount(src, minlength=V).astype(np.float64)
    idg = np.bincount(dst, minlength=V).astype(np.float64)
    ps = od ** 0.75
    ps /= ps.sum()
    pn_ = (od + idg) ** 0.75
    pn_ /= pn_.sum()
    pc = np.bincount(dst, weights=(ps / np.maximum(od, 1))[src], minlength=V)
    rate = [ps, pc + K * pn_]
    order_by_rate = [torch.from_numpy(np.argsort(-r, kind="stable").astype(np.int64)).cuda() for r in rate]
    results = []
    import itertools
    syncs = [x for x in args.sync if x != "adaptive"] + ["adaptive:%g" % c for c in args.c0 if "adaptive" in args.sync]
    for n, sub, hot in itertools.product(args.ranks, args.sub, args.hot):
        if n == 1 and (sub != args.sub[0] or hot != args.hot[0]):
            continue
        for sync_spec in (syncs if n > 1 else ["none"]):
            # "<rule>+part": W partitioned by source (each replica draws its
            # sources from its part, smore_set_source_partition; only C exchanged)
            part = sync_spec.endswith("+part") and n > 1
            sync = sync_spec[:-5] if sync_spec.endswith("+part") else sync_spec
            tabs = [1] if part else [0, 1]
            reps = [ctx(i) for i in range(n)]
            for r, pn in enumerate(reps):
                pn.set_source_partition(n if part else 1, r if part else 0)
                pn.init_table_uniform(0, 5)
                pn.zero_table(1)
            T = [[table_tensor(pn, t) for t in (0, 1)] for pn in reps]
            Ss = [[t.clone() for t in ts] for ts in T]
            Ds = [[torch.zeros_like(t) for t in ts] for ts in T]
            Rs = [[torch.zeros_like(t) for t in ts] for ts in T]
            scale = 1.0 / n if sync == "mean" else 1.0
            if sync.startswith("adaptive"):
                # per-row scale of the summed deltas: sum for rows with few
                # updates per exchange, towards the mean for the hub rows
                c0 = float(sync.split(":")[1])
                scale = []
                for r_ in rate:
                    k = r_ * S * n
                    sv = np.minimum(1.0, c0 / np.maximum(k, 1e-30))
                    scale.append(torch.from_numpy((sv + (1.0 - sv) / n).astype(np.float32)).cuda().view(-1, 1))
            steps = max(1, args.total // (n * S))
            pending = False
            t0 = time.perf_counter()

            def reduce_all():
                for t in tabs:
                    tot = sum(Rs[r][t] for r in range(n))
                    for r in range(n):
                        Rs[r][t].copy_(tot)

            hidx = [o[:hot] for o in order_by_rate] if hot > 0 else None

            def hot_sync():
                for t in range(2):
                    idx = hidx[t]
                    Dh = [T[r][t][idx] - Ss[r][t][idx] for r in range(n)]
                    Rh = sum(Dh)
                    for r in range(n):
                        T[r][t][idx] += Rh - Dh[r]
                        Ss[r][t][idx] += Rh

            sub_n = S // sub
            for k in range(steps):
                for j in range(sub):
                    for r, pn in enumerate(reps):
                        pn.train_edges("line2", (k * n + r) * S + j * sub_n, sub_n if j + 1 < sub else S - j * sub_n,
                                       steps * n * S, K, 0.025, 0.0, args.seed, args.mode, sync=False)
                    if n > 1 and hidx is not None and sync == "sum":
                        hot_sync()
                if n > 1:
                    for r in range(n):
                        for t in tabs:
                            sc = scale[t] if isinstance(scale, list) else scale
                            if pending:
                                TorchPasses.cycle(T[r][t], Ss[r][t], Ds[r][t], Rs[r][t], sc)
                            else:
                                TorchPasses.begin(T[r][t], Ss[r][t], Ds[r][t], Rs[r][t])
                    reduce_all()       # the all-reduce of this exchange (lands before the next end)
                    pending = True
            if pending:
                for r in range(n):
                    for t in tabs:
                        TorchPasses.end(T[r][t], Ss[r][t], Ds[r][t], Rs[r][t],
                                        scale[t] if isinstance(scale, list) else scale)
            torch.cuda.synchronize()
            W0, C0 = reps[0].get_table(0), reps[0].get_table(1)
            spread = 0.0
            if part:
                # each W row from its owner
                b = reps[0].source_parts(n)
                for r in range(1, n):
                    W0[b[r]:b[r + 1]] = reps[r].get_table(0)[b[r]:b[r + 1]]
                spread = float(np.abs(reps[n - 1].get_table(1) - C0).max() / max(1e-30, np.abs(C0).max()))
                for pn in reps:
                    pn.set_source_partition(1, 0)
            elif n > 1:
                W1 = reps[n - 1].get_table(0)
                spread = float(np.abs(W1 - W0).max() / max(1e-30, np.abs(W0).max()))
            row = {"config": args.config, "ranks": n, "sync": sync_spec, "sub": sub, "hot_rows": hot, "steps": steps,
                   "samples_per_step": S,
                   "total": steps * n * S, "mode": args.mode, "finite": bool(np.isfinite(W0).all()),
                   "loss": round(heldout_loss(W0, C0, heldout, dim), 5), "replica_spread_rel": spread,
                   "wall_s": round(time.perf_counter() - t0, 1)}
            results.append(row)
            print(json.dumps(row), flush=True)
            del T, Ss, Ds, Rs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
