#!/usr/bin/env python3
"""Throughput of the other configs of BASELINE.json on one MI355X (the
headline LINE-2 C4 number is bench.py's).  One JSON line per config:

  c2   LINE order 2, 1M vertices / 20M lines, d=64, K=5   (M edge-updates/s)
  c4   LINE order 2, 10M vertices / 200M lines (bench.py's headline config)
  c3   BPR (C++ rule: 5 rounds per sample), 2M users x 1M items / 100M edges,
       d=128, negatives uniform over items (BPR's "no_degrees")   (M BPR samples/s)
  c5   DeepWalk, Youtube-links-sized stand-in (1.13M vertices / 3M lines),
       d=128, walk_steps=40, window=5, K=5 (M skip-gram pair-updates/s, from the
       exact pairs-per-walk expectation of the window-shrink rule)

Timing: HIP events of the library (smore_last_kernel_ms) over `--steps`
calls after one warmup call, inputs resident in HBM.

    python tools/bench_models.py --configs c2 c3 c5 [--mode hybrid]
  c5go / c5n2v  Go DeepWalk / Go node2vec (p 0.5, q 2) on c5's graph
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pairs_per_walk(L, window):
    """E[# (i, j) pairs] of SkipGrams with the random shrink r ~ U{1..w}
    (src/proNet.cpp:769-809) on a walk of L vertices."""
    tot = 0.0
    for i in range(L):
        for r in range(1, window + 1):
            lo, hi = max(0, i - r), min(L - 1, i + r)
            tot += (hi - lo) / window
    return tot


def ran(pn):
    """The scatter the last call actually ran (smore_last_mode): "plain" for
    the plain-store kernel (C++ BPR's hybrid above the small-graph cap)."""
    m = pn.last_mode()
    return "plain" if m == "hogwild" else m


def run_edges(pn, model, S, steps, K, mode, seed=7):
    """mean ms per call, and the mean (draw, update) phase ms"""
    total = (steps + 1) * S
    ms, ph = [], []
    for k in range(steps + 1):
        pn.train_edges(model, k * S, S, total, K, 0.025, 0.0, seed, mode)
        if k:
            ms.append(pn.last_kernel_ms())
            ph.append(pn.last_phase_ms()[:2])
    return float(np.mean(ms)), [round(float(x), 3) for x in np.mean(ph, axis=0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c2", "c3", "c5"])
    ap.add_argument("--mode", default="hybrid")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    for cfg in args.configs:
        V, (src, dst, w) = graphgen.config_edges("c5" if cfg.startswith("c5") else cfg)
        pn = smore_amd.ProNet(0)
        t0 = time.perf_counter()
        if cfg == "c3":
            pn.SetNegativeMethod("no_degrees")       # BPR() (src/model/BPR.cpp:4-7)
        pn.set_graph_edges(V, src, dst, w)
        build = time.perf_counter() - t0
        out = {"config": cfg, "vertices": V, "edge_slots": pn.MAX_line, "mode": args.mode,
               "build_s": round(build, 1)}
        if cfg in ("c2", "c4"):
            S = 1 << 27
            pn.alloc_tables(64, 2)
            pn.init_table_uniform(0, 1)
            pn.zero_table(1)
            ms, ph = run_edges(pn, "line2", S, args.steps, 5, args.mode)
            out.update(model="line2", dim=64, K=5, samples_per_call=S, ms_per_call=round(ms, 3),
                       draw_update_ms=ph, value=round(S / ms / 1e3, 1), unit="M edge-updates/s")
        elif cfg == "c3":
            S = 1 << 26
            pn.alloc_tables(128, 1)
            pn.init_table_uniform(0, 1)
            ms, ph = run_edges(pn, "bpr", S, args.steps, 5, args.mode)
            out.update(model="bpr", dim=128, rounds=5, samples_per_call=S, ms_per_call=round(ms, 3),
                       draw_update_ms=ph,
                       value=round(S / ms / 1e3, 1), unit="M BPR samples/s (5 rounds each)")
        elif cfg == "c5":
            steps_, window, K, walk_times = 40, 5, 5, 1
            pn.alloc_tables(128, 2)
            pn.init_table_uniform(0, 1)
            pn.init_table_uniform(1, 2)
            order = smore_amd.deepwalk_order(V, walk_times + 1, 0)
            ms = []
            for k in range(args.steps + 1):
                pn.train_deepwalk(0, V, walk_times + 1, steps_, window, K, 0.025, 7 + k, order, args.mode)
                if k:
                    ms.append(pn.last_kernel_ms())
            ms = float(np.mean(ms))
            ppw = pairs_per_walk(steps_ + 1, window)
            out.update(model="deepwalk", dim=128, K=K, walk_steps=steps_, window=window, walks_per_call=V,
                       ms_per_call=round(ms, 3), pairs_per_walk=round(ppw, 1),
                       value=round(V * ppw / ms / 1e3, 1), unit="M pair-updates/s",
                       walks_per_s=round(V / ms * 1e3, 1))
        elif cfg in ("c5go", "c5n2v"):
            # Go DeepWalk / Go node2vec (p=0.5, q=2) on C5's graph, --mode scatter
            steps_, window, K = 40, 5, 5
            pn.set_semantics("go")
            pn.alloc_tables(128, 2)
            pn.init_table_uniform(0, 1)
            pn.init_table_uniform(1, 2)
            order = smore_amd.deepwalk_order(V, 2, 0)
            ms = []
            for k in range(args.steps + 1):
                if cfg == "c5go":
                    pn.train_deepwalk(0, V, 2, steps_, window, K, 0.025, 7 + k, order, args.mode)
                else:
                    pn.train_node2vec(0, V, 2, steps_, window, K, 0.025, 0.5, 2.0, 7 + k, order, args.mode)
                if k:
                    ms.append(pn.last_kernel_ms())
            ms = float(np.mean(ms))
            L = steps_ + 1
            ppw = sum(min(i + window, L - 1) - max(i - window, 0) for i in range(L))   # Go fixed window
            out.update(model="go_deepwalk" if cfg == "c5go" else "go_node2vec", dim=128, K=K, walk_steps=steps_,
                       window=window, walks_per_call=V, ms_per_call=round(ms, 3), pairs_per_walk=ppw,
                       value=round(V * ppw / ms / 1e3, 1), unit="M pair-updates/s",
                       walks_per_s=round(V / ms * 1e3, 1))
        out["scatter"] = ran(pn)       # what ran; "mode" is what was asked for
        print(json.dumps(out), flush=True)
        pn.close()


if __name__ == "__main__":
    main()
