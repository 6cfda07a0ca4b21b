#!/usr/bin/env python3
"""Time the replica exchange's fused passes (replica_sync.hip) at the C4
bench's table size -- 10M rows x d 64, two tables -- on one GPU, with HIP
events on the context stream (run under rocprofv3 --kernel-trace --stats for
the per-kernel durations).  Prints one JSON line: ms per pass and per
exchange (the N > 1 bench runs one cycle pass per table per step).

    python tools/exchange_passes.py [--rows 10000000 --dim 64 --reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import smore_amd
    from smore_amd.dist import adaptive_scale, table_tensor
    pn = smore_amd.ProNet(0)
    V = args.rows
    src = np.arange(V, dtype=np.int32)
    dst = ((src.astype(np.int64) * 7 + 1) % V).astype(np.int32)
    pn.set_graph_edges(V, src, dst, np.ones(V))
    pn.alloc_tables(args.dim, 2)
    pn.init_table_uniform(0, 1)
    pn.init_table_uniform(1, 2)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    pn.set_stream(stream.cuda_stream)
    T = table_tensor(pn, 0)
    S, D, R = T.clone(), torch.zeros_like(T), torch.zeros_like(T)
    sc = torch.as_tensor(adaptive_scale(pn.row_rates("line2", 5, 1), 1 << 27, 8), device=T.device)
    rows, stride = T.shape
    n = T.numel()
    p = [x.data_ptr() for x in (T, S, D, R)]
    passes = {
        "begin": lambda: pn.delta_begin(*p, n),
        "end": lambda: pn.delta_end(*p, 0.125, n),
        "cycle": lambda: pn.delta_cycle(*p, 0.125, n),
        "end_rows": lambda: pn.delta_end_rows(*p, sc.data_ptr(), rows, stride),
        "cycle_rows": lambda: pn.delta_cycle_rows(*p, sc.data_ptr(), rows, stride),
    }
    streams = {"begin": 5, "end": 6, "cycle": 8, "end_rows": 6, "cycle_rows": 8}
    out = {"rows": rows, "dpad": stride, "table_gb": n * 4 / 1e9}
    for name, fn in passes.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        out[name + "_ms"] = round(ms, 3)
        out[name + "_gbs"] = round(streams[name] * n * 4 / ms / 1e6, 1)
    # the N > 1 bench: one cycle pass per table per exchange (two tables)
    out["exchange_ms_per_step"] = round(2 * out["cycle_rows_ms"], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
