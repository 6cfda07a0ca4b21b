#!/usr/bin/env python3
"""Caller pairs (smore_train_pairs) on the 920-vertex test graph: held-out
LINE-2 loss per scatter mode and hybrid knob (LDS write-combining rows, hot
threshold), C++ and Go rules.  The same setting as
tests/test_gpu_pairs.py::test_pairs_parallel_modes_train_like_serial.

    python tools/pairs_probe.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PL1K = os.path.join(ROOT, "tests", "golden", "pl1k.txt")
SEED = 20251015


def heldout(W, C, draws):
    v, c, negs = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = c >= 0
    v, c, negs = v[keep], c[keep], negs[keep]
    Wv = W[v].astype(np.float64)
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k]].astype(np.float64)))
    return float(loss.mean())


def main():
    import smore_amd
    variants = [("serial", None, None), ("atomic", None, None), ("hybrid", None, None), ("hybrid", 0, None),
                ("hybrid", None, 1.0), ("hybrid", 0, 1.0), ("hybrid", None, 1e9), ("hogwild", None, None)]
    for sem in ("cpp", "go"):
        for mode, rows, tau in variants:
            for rep in range(2):
                pn = smore_amd.ProNet(0)
                pn.LoadEdgeList(PL1K, 1)
                if sem == "go":
                    pn.set_semantics("go")
                d = pn.sample_edges("line2", 0, 400_000, 0, SEED)
                d = d[d[:, 1] >= 0]
                held = pn.sample_edges("line2", 1 << 40, 50_000, 5, SEED + 1)
                pn.alloc_tables(32, 2)
                pn.init_table_glibc(0, 0)
                pn.zero_table(1)
                if rows is not None:
                    pn.set_write_combine(rows)
                if tau is not None:
                    pn.set_hot_threshold(tau)
                pn.train_pairs(d[:, 0], d[:, 1], 5, 0.025, SEED, 5, mode)
                print(json.dumps({"sem": sem, "mode": mode, "combine_rows": rows, "tau": tau, "rep": rep,
                                  "loss": round(heldout(pn.get_table(0), pn.get_table(1), held), 5),
                                  "combine_info": pn.write_combine_info() if mode == "hybrid" else None}),
                      flush=True)
                pn.close()
                if mode == "serial":
                    break


if __name__ == "__main__":
    main()
