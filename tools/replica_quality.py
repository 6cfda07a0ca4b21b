#!/usr/bin/env python3
"""Held-out LINE-2 loss of `world` replicas (gloo ranks sharing cuda:0,
tests/helpers/replica_worker.py) per exchange rule, on the 1k-vertex golden
graph at the C4 bench's updates per row per exchange (12k samples per rank per
exchange over 920 rows), against one rank that ran all `total` samples and one
that ran total/world.  TEST INFRASTRUCTURE (reads the oracle's sampler).

    python tools/replica_quality.py --worlds 2 4 8 --rules sum mean adaptive:16 adaptive:64 adaptive:256
    python tools/replica_quality.py --model deepwalk --worlds 2 4 8 --rules mean adaptive:256 adaptive:1024

--model deepwalk: DeepWalk (40 steps, window 5, K 5) with `--walk-times` walks
per vertex, `--per` walks per rank per exchange (default: C5's ~54
pair-updates per row per rank per exchange at 2^18 walks), the adaptive
scales from a row census (the torch path: ReplicaSync(model="census")); the
held-out LINE-2 objective and the edge AUC.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 20251015


def run(tmp, world, total, steps, rule, model="line2"):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    worker = os.path.join(ROOT, "tests", "helpers", "replica_worker.py")
    run.n = getattr(run, "n", 0) + 1
    outs = [os.path.join(tmp, "c%d_w%d_r%d.npz" % (run.n, world, r)) for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-u", worker, str(r), str(world), str(port), str(total), str(steps),
                               outs[r], "0", "1", rule, model], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True)
             for r in range(world)]
    for p in procs:
        out, _ = p.communicate(timeout=600)
        if p.returncode != 0:
            raise RuntimeError(out[-3000:])
    res = []
    for o in outs:
        with np.load(o) as z:
            res.append({k: z[k] for k in z.files})
    return res


def heldout(W, C, draws):
    W = W.astype(np.float64)
    C = C.astype(np.float64)
    v, c, negs = draws
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", W[v], C[c]))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", W[v], C[negs[:, k]]))
    return float(loss.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rules", nargs="+", default=["sum", "mean", "adaptive:16", "adaptive:64", "adaptive:256"])
    ap.add_argument("--per", type=int, default=None, help="line2: samples / deepwalk: walks per rank per exchange")
    ap.add_argument("--total", type=int, default=4 * 10 ** 6)
    ap.add_argument("--model", default="line2", choices=["line2", "deepwalk"])
    ap.add_argument("--walk-times", type=int, default=20)
    args = ap.parse_args()
    from oracle import oracle as orc
    g = orc.Graph.from_file(os.path.join(ROOT, "tests", "golden", "pl1k.txt"), 1)
    h = orc.sample_line(g, SEED + 7, 0, 50_000, 5)
    h = h[h[:, 1] >= 0]
    draws = (h[:, 0], h[:, 1], h[:, 2:])
    if args.model == "deepwalk":
        deepwalk(args, g, draws)
        return
    args.per = args.per or 12_000
    with tempfile.TemporaryDirectory() as tmp:
        for world in args.worlds:
            steps = args.total // (world * args.per)
            one_all = run(tmp, 1, args.total, steps * world, "sum")[0]
            one_part = run(tmp, 1, args.total // world, steps, "sum")[0]
            base = {"world": world, "l1_total": heldout(one_all["W"], one_all["C"], draws),
                    "l1_part": heldout(one_part["W"], one_part["C"], draws)}
            print(json.dumps(dict(base, rule="1 rank")), flush=True)
            for rule in args.rules:
                outs = run(tmp, world, args.total, steps, rule)
                W, C = outs[0]["W"], outs[0]["C"]
                # (with "+part" the worker gathered W from the owners: every rank
                # holds all of it)
                spread = max(max(float(np.abs(o[k] - outs[0][k]).max()) for k in ("W", "C")) for o in outs)
                ok = bool(np.isfinite(W).all() and np.isfinite(C).all())
                ln = heldout(W, C, draws) if ok else float("nan")
                print(json.dumps(dict(base, rule=rule, loss=ln, finite=ok, spread=spread,
                                      vs_total=ln / base["l1_total"], vs_part=ln / base["l1_part"])), flush=True)


def edge_auc(W, C, g, seed=3):
    rng = np.random.default_rng(seed)
    srcv = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, 20000)
    nv, nc = rng.integers(0, g.V, 2000), rng.integers(0, g.V, 2000)
    pos = np.einsum("ij,ij->i", W[srcv[pick]].astype(np.float64), C[g.targets[pick]].astype(np.float64))
    neg = np.einsum("ij,ij->i", W[nv].astype(np.float64), C[nc].astype(np.float64))
    return float((pos[:, None] > neg[None, :]).mean())


def deepwalk(args, g, draws):
    """DeepWalk ranks (the worker's census + ReplicaSync path) vs one rank that
    walked every start: held-out loss and edge AUC."""
    total = args.walk_times * g.V
    # C5: 2^18 walks x ~232 pairs per replica per exchange over 1.13M rows =
    # ~54 pair-updates per row; here ~232 pairs per walk over 920 rows
    per = args.per or max(1, int(round(54 * g.V / 232)))
    with tempfile.TemporaryDirectory() as tmp:
        one = run(tmp, 1, total, max(1, total // per), "sum", "deepwalk")[0]
        l1, a1 = heldout(one["W"], one["C"], draws), edge_auc(one["W"], one["C"], g)
        print(json.dumps({"model": "deepwalk", "world": 1, "walks": total, "loss": l1, "auc": a1}), flush=True)
        for world in args.worlds:
            steps = max(1, total // (world * per))
            for rule in args.rules:
                outs = run(tmp, world, total, steps, rule, "deepwalk")
                W, C = outs[0]["W"], outs[0]["C"]
                spread = max(max(float(np.abs(o[k] - outs[0][k]).max()) for k in ("W", "C")) for o in outs)
                ok = bool(np.isfinite(W).all() and np.isfinite(C).all())
                ln = heldout(W, C, draws) if ok else float("nan")
                an = edge_auc(W, C, g) if ok else float("nan")
                print(json.dumps({"model": "deepwalk", "world": world, "rule": rule, "walks_per_exchange": per,
                                  "exchanges": steps, "loss": ln, "auc": an, "finite": ok, "spread": spread,
                                  "vs_one": ln / l1, "auc_vs_one": an - a1}), flush=True)


if __name__ == "__main__":
    main()
