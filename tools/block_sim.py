#!/usr/bin/env python3
"""Predicted N-GPU time of the 2-D block schedule from measured cell times.

Reads tools/block_rate.py output (one JSON line per (N, part) with "cells":
[block, units, ms] in sub-round order, plus the nparts=1 line) and replays
dist.BlockSync's dependencies on N GPUs:

    start(r, s) = max(end(r, s-1), xfer(r, s-2))
    end(r, s)   = start(r, s) + d(r, (2r + s) mod nb)
    xfer(r, s)  = max(end(r-1, s), end(r, s), end(r+1, s)) + bytes / link

(rank r's sub-round-s rotation sends its block to r-1 and receives from r+1;
both sides must have posted; the cell two sub-rounds later waits for it).
Cell times of parts not measured are taken from the measured part with the
same block (cells cost by block: the hub rows live in blocks).  Prints, per
N: the steady-state epoch time, the no-stall bound (the largest per-rank sum),
and the predicted speed-up over one GPU on the same per-GPU work (weak
scaling, as bench.py).

    python tools/block_sim.py gpurun_out/br_c4_all.jsonl --link-gbs 64
"""
import argparse
import json
from collections import defaultdict


def simulate(n, d, xfer_ms, epochs=4):
    """d[r][b]: ms of cell (r, b).  Returns the ms of the last epoch."""
    nb = 2 * n
    S = epochs * nb
    end = [[0.0] * S for _ in range(n)]
    xf = [[0.0] * S for _ in range(n)]
    for s in range(S):
        for r in range(n):
            t = end[r][s - 1] if s else 0.0
            if s >= 2:
                t = max(t, xf[r][s - 2])
            end[r][s] = t + d[r][(2 * r + s) % nb]
        for r in range(n):
            xf[r][s] = max(end[(r - 1) % n][s], end[r][s], end[(r + 1) % n][s]) + xfer_ms
    last = max(end[r][S - 1] for r in range(n))
    prev = max(end[r][S - nb - 1] for r in range(n))
    return last - prev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--link-gbs", type=float, default=64.0, help="xGMI GB/s per direction per link")
    args = ap.parse_args()
    one, rows = None, defaultdict(dict)
    for f in args.files:
        for line in open(f):
            d = json.loads(line)
            if d["nparts"] == 1:
                one = d
            elif d.get("cells") and isinstance(d["cells"][0], list):
                rows[d["nparts"]][d["part"]] = d
    for n in sorted(rows):
        nb = 2 * n
        meas = rows[n]
        by_block = defaultdict(list)
        for r, d in meas.items():
            for b, _, ms, *_ in d["cells"]:
                by_block[b].append(ms)
        dt = [[0.0] * nb for _ in range(n)]
        for r in range(n):
            for b in range(nb):
                if r in meas:
                    dt[r][b] = {c[0]: c[2] for c in meas[r]["cells"]}.get(b, 0.0)
                else:
                    v = by_block.get(b, [0.0])
                    dt[r][b] = sum(v) / len(v)
        any_row = next(iter(meas.values()))
        xfer = any_row["block_bytes_max"] / (args.link_gbs * 1e9) * 1e3
        # walks: every replica generates its slice of the round's walks and
        # receives the others' (walk_bytes (N-1)/N over the link) before its cells
        prep = sum(d.get("prepare_ms", 0.0) for d in meas.values()) / len(meas)
        wbytes = max(d.get("walk_bytes", 0) for d in meas.values())
        prep += wbytes * (n - 1) / n / (args.link_gbs * 1e9) * 1e3
        ep = simulate(n, dt, xfer) + prep
        bound = max(sum(dt[r]) for r in range(n)) + prep
        units = sum(d["units"] for d in meas.values()) / len(meas)
        one_rate = one["units"] / one["epoch_ms"]
        print(json.dumps({"config": any_row["config"], "model": any_row["model"], "nparts": n,
                          "parts_measured": sorted(meas), "xfer_ms": round(xfer, 3), "prepare_ms": round(prep, 3),
                          "epoch_ms_sim": round(ep, 3), "epoch_ms_no_stall": round(bound, 3),
                          "stall_frac": round(1 - bound / ep, 4),
                          "speedup_pred": round(n * units / ep / one_rate, 3),
                          "speedup_no_stall": round(n * units / bound / one_rate, 3)}))


if __name__ == "__main__":
    main()
