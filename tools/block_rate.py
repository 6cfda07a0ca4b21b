#!/usr/bin/env python3
"""One replica's compute in the 2-D block schedule, on one GPU.

A context set up as part r of N (smore_block_setup) runs one epoch of its
cells -- nb = 2N sub-rounds, cell (r, (2r + s) mod nb), the samples split by
the cells' mass -- back to back (no rotation: on N GPUs the transfers overlap
the next sub-round), against the one-GPU path over the same number of
samples.  Prints one JSON line per (config, N, part): the epoch's time, the
per-cell launch times, and the rate relative to one GPU, i.e. the measured
per-GPU factor of the predicted N-GPU speed-up.

    python tools/block_rate.py --model line2 --config c4 --nparts 2 4 8 --samples 134217728
    python tools/block_rate.py --model deepwalk --config c5 --nparts 2 4 8 --walks 262144
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="line2", choices=["line2", "deepwalk"])
    ap.add_argument("--config", default="c4")
    ap.add_argument("--nparts", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--parts", type=int, nargs="+", default=[0], help="which parts to time")
    ap.add_argument("--samples", type=int, default=1 << 27, help="line2: samples per epoch per GPU")
    ap.add_argument("--walks", type=int, default=1 << 18, help="deepwalk: walks per epoch")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="hybrid")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--hot-tau", type=float, default=None, help="hybrid: hot-row threshold")
    ap.add_argument("--combine-rows", type=int, default=None, help="hybrid: LDS write-combined rows (0: off)")
    ap.add_argument("--skip-one", action="store_true", help="no one-GPU reference (profiling the cells alone)")
    ap.add_argument("--hubs", type=int, default=-1, help="line2: hub C rows (-1 the library's default, 0 none)")
    ap.add_argument("--split", type=int, default=0,
                    help="line2: launches per cell (the hub slots' exchanges; 0: the library's default)")
    args = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime with torch, as bench.py)
    import smore_amd
    from smore_amd import graphgen

    V, (src, dst, w) = graphgen.config_edges(args.config)
    line = args.model == "line2"
    dim, K = (64, 5) if line else (128, 5)
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    pn.alloc_tables(dim, 2)
    if args.hot_tau is not None:
        pn.set_hot_threshold(args.hot_tau)
    if args.combine_rows is not None:
        pn.set_write_combine(args.combine_rows, 0)
    pn.init_table_glibc(0, 0)
    pn.zero_table(1)
    pn.block_set_hubs(args.hubs)
    S = args.samples
    total = S * 100
    wt, steps, window = 10, 40, 5
    order = smore_amd.deepwalk_order(V, wt, 0) if not line else None

    def timed(f):
        best = 1e30
        for _ in range(args.reps):
            pn.synchronize()
            t0 = time.perf_counter()
            f()
            pn.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    # the one-GPU path over the same work
    one_phase = None
    if args.skip_one:
        one, units = None, None
    elif line:
        one = timed(lambda: pn.train_edges("line2", 0, S, total, K, 0.025, 0.0, args.seed, args.mode, sync=False))
        units = S
        one_phase = [round(x, 3) for x in pn.last_phase_ms()[:2]]
    else:
        one = timed(lambda: pn.train_deepwalk(0, args.walks, wt, steps, window, K, 0.025, args.seed, order,
                                              args.mode))
        pn.census_begin()
        pn.train_deepwalk(0, args.walks, wt, steps, window, K, 0.025, args.seed, order, args.mode)
        pn.census_end(1.0)
        units = float(pn.row_rates("census", K, 0).sum())   # pairs of the walks
    if one is not None:
        print(json.dumps({"config": args.config, "model": args.model, "nparts": 1, "epoch_ms": round(one * 1e3, 3),
                          "units": units, "rate_M_per_s": round(units / one / 1e6, 2), "draw_update_ms": one_phase}),
              flush=True)
    for n in args.nparts:
        nb = 2 * n
        for r in args.parts:
            if r >= n:
                continue
            t0 = time.perf_counter()
            pn.block_setup("line2" if line else "census", n, r, K, args.mode)
            setup_s = time.perf_counter() - t0
            cells = []
            if line:
                cnt = pn.block_counts(S)      # weak scaling: S samples per GPU per epoch, as bench.py
                mine = S
                split = args.split or pn.block_cell_launches()

                def cell(b, b0, x, sync):
                    for q in range(split):      # the cell in `split` launches
                        lo, hi = x * q // split, x * (q + 1) // split
                        if hi > lo:
                            pn.block_train_edges(b, b0 + lo, hi - lo, total, K, 0.025, args.seed, args.mode,
                                                 sync=sync and q + 1 == split)

                def epoch():
                    b0 = 0
                    for s in range(nb):
                        b = (2 * r + s) % nb
                        if cnt[b]:
                            cell(b, b0, int(cnt[b]), False)
                        b0 += int(cnt[b])
                ep = timed(epoch)
                for s in range(nb):      # per-cell launch times (one pass, synchronised per cell)
                    b = (2 * r + s) % nb
                    if cnt[b]:
                        t1 = time.perf_counter()
                        cell(b, 0, int(cnt[b]), True)
                        ph = pn.last_phase_ms()
                        cells.append([b, int(cnt[b]), round((time.perf_counter() - t1) * 1e3, 3)] +
                                     ([round(ph[0], 3), round(ph[1], 3)] if ph else []))
                units_r = mine
            else:
                # walk-partitioned generation (the group default): this part walks
                # its 1/N of the round and buckets every walk's pairs; the other
                # slices' broadcast is block_sim's (walk_bytes over the link)
                # (the round buffer first holds every walk, as after the broadcast:
                # the emit then buckets the whole round, as in the group)
                def prep_split():
                    pn.block_walks_generate(0, args.walks, args.walks * r // n, args.walks * (r + 1) // n, wt, steps,
                                            window, K, 0.025, args.seed, order, args.mode)
                    pn.block_walks_emit()
                prep_all = timed(lambda: pn.block_prepare_walks(0, args.walks, wt, steps, window, K, 0.025, args.seed,
                                                                order, args.mode))
                prep = timed(prep_split)
                recs = [pn.block_walk_records(b) for b in range(nb)]

                L = pn.block_cell_launches()     # a cell in L launches (hub slots exchanged between)

                def wcell(b, sync):
                    for q in range(L):
                        pn.block_train_walks(b, sync=sync and q + 1 == L, part=q, parts=L)

                def epoch():
                    for s in range(nb):
                        wcell((2 * r + s) % nb, False)
                ep = timed(epoch)
                units_r = sum(recs)
                for s in range(nb):      # per-cell launch times (one pass, synchronised per cell)
                    b = (2 * r + s) % nb
                    t1 = time.perf_counter()
                    wcell(b, True)
                    cells.append([b, int(recs[b]), round((time.perf_counter() - t1) * 1e3, 3)])
            row = {"config": args.config, "model": args.model, "nparts": n, "part": r, "setup_s": round(setup_s, 2),
                   "hubs": int(pn.block_hubs()[0]), "split": split if line else pn.block_cell_launches(),
                   "epoch_ms": round(ep * 1e3, 3), "units": units_r,
                   "rate_M_per_s": round(units_r / ep / 1e6, 2),
                   "per_gpu_factor": round((units_r / ep) / (units / one), 4) if one else None,
                   "cells": cells}
            if not line:
                row["prepare_ms"] = round(prep * 1e3, 3)
                row["prepare_all_ms"] = round(prep_all * 1e3, 3)
                row["walk_bytes"] = args.walks * (steps + 2) * 4
                row["per_gpu_factor_with_prepare"] = round((units_r / (ep + prep)) / (units / one), 4) if one else None
            # the C block a rotation moves: its bytes (xGMI time is estimated in DESIGN.md 10)
            _, cb = pn.block_bounds()
            row["block_bytes_max"] = int(np.diff(cb).max()) * dim * 4
            print(json.dumps(row), flush=True)
    pn.block_setup("line2" if line else "census", 1, 0, K, args.mode)


if __name__ == "__main__":
    main()
