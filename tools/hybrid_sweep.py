#!/usr/bin/env python3
"""Held-out LINE-2 loss and update time of scatter settings on a config graph
(the hybrid's quality/speed trade-off).  Prints one JSON line per setting.

    python tools/hybrid_sweep.py --config c2 --samples 268435456
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def loss_of(W, C, draws):
    v, c, n = draws[:, 0], draws[:, 1], draws[:, 2:]
    ok = c >= 0
    v, c, n = v[ok], c[ok], n[ok]
    Wv = W[v].astype(np.float64)
    l = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
    for k in range(n.shape[1]):
        l += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[n[:, k]].astype(np.float64)))
    return float(l.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--samples", type=int, default=1 << 28)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--settings", nargs="+", default=["atomic", "hybrid:0.3:128:0", "hybrid:0.3:128:32",
                                                      "hybrid:0.3:128:16", "hogwild"])
    args = ap.parse_args()
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges(args.config)
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    held = pn.sample_edges("line2", 1 << 40, 100_000, 5, 99)
    total = args.samples
    for s in args.settings:
        parts = s.split(":")
        mode = parts[0]
        if mode == "hybrid":
            pn.set_hot_threshold(float(parts[1]))
            pn.set_write_combine(int(parts[2]), int(parts[3]))
            if len(parts) > 4:          # staleness bound of the combined rows (expected updates per drain)
                os.environ["SMORE_SH_STALE"] = parts[4]
            else:
                os.environ.pop("SMORE_SH_STALE", None)
        pn.alloc_tables(args.dim, 2)
        pn.init_table_uniform(0, 5)
        pn.zero_table(1)
        t0 = time.perf_counter()
        pn.train_edges("line2", 0, total, total, 5, 0.025, 0.0, 20251015, mode)
        el = time.perf_counter() - t0
        ph = pn.last_phase_ms()
        out = {"config": args.config, "setting": s, "samples": total, "loss": round(loss_of(pn.get_table(0),
               pn.get_table(1), held), 5), "wall_s": round(el, 3), "draw_update_ms": ph, "hot_rows": pn.hot_rows(),
               "write_combine": pn.write_combine_info() if mode == "hybrid" else None}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
