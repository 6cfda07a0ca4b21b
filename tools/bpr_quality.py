#!/usr/bin/env python3
"""C3 BPR (2M users x 1M items / 100M edges, d=128, K=5): held-out BPR
objective and ranking accuracy after T samples, and the update time per 2^27
samples, per scatter: atomic, hybrid (no LDS combining, the default), hybrid
with the hub rows write-combined (SMORE_BPR_COMBINE=1).  TEST
INFRASTRUCTURE (reads the oracle's sampler).  DESIGN.md 8.

    python tools/bpr_quality.py --log2-total 28 [--variants atomic hybrid hybrid@3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 20251015


def bpr_objective(W, draws, dim):
    u, i, js = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = i >= 0
    u, i, js = u[keep], i[keep], js[keep]
    Wu = W[u, :dim].astype(np.float64)
    Wi = W[i, :dim].astype(np.float64)
    loss = np.zeros(len(u))
    hit = np.zeros(len(u))
    for k in range(js.shape[1]):
        x = np.einsum("ij,ij->i", Wu, Wi - W[js[:, k], :dim].astype(np.float64))
        loss += np.logaddexp(0.0, -x)
        hit += x > 0
    return float(loss.mean() / js.shape[1]), float(hit.mean() / js.shape[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2-total", type=int, default=28)
    ap.add_argument("--variants", nargs="+", default=["atomic", "hybrid", "hybrid+combine"])
    ap.add_argument("--dim", type=int, default=128)
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges("c3")
    pn = smore_amd.ProNet(0)
    pn.SetNegativeMethod("no_degrees")
    pn.set_graph_edges(V, src, dst, w)
    held = pn.sample_edges("bpr", 1 << 40, 100_000, 5, SEED + 1)
    total = 1 << args.log2_total
    step = 1 << 27
    for var in args.variants:
        # variant: mode[+combine][@tau] (tau: the hot-row threshold; default the library's)
        var, _, tau = var.partition("@")
        pn.set_hot_threshold(float(tau) if tau else -1.0)
        mode = var.split("+")[0]
        os.environ["SMORE_BPR_COMBINE"] = "1" if var.endswith("+combine") else "0"
        pn.alloc_tables(args.dim, 1)
        pn.init_table_uniform(0, 7)
        ms = []
        t0 = time.perf_counter()
        for b in range(0, total, step):
            pn.train_edges("bpr", b, min(step, total - b), total, 5, 0.025, 0.0, SEED, mode)
            ms.append(pn.last_kernel_ms())
        el = time.perf_counter() - t0
        loss, acc = bpr_objective(pn.get_table(0), held, args.dim)
        print(json.dumps({"config": "c3", "variant": var + ("@" + tau if tau else ""), "total": total, "loss": round(loss, 6),
                          "rank_acc": round(acc, 5), "call_ms_per_2^27": round(float(np.median(ms)), 2),
                          "wall_s": round(el, 2), "combine_info": pn.write_combine_info(),
                          "hot_rows": pn.hot_rows() if mode == "hybrid" else None}), flush=True)
    os.environ.pop("SMORE_BPR_COMBINE", None)


if __name__ == "__main__":
    main()
