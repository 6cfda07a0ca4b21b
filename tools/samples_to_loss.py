#!/usr/bin/env python3
"""Samples-to-loss and the predicted effective multi-GPU speed-up from a
tools/replica_study.py LINE-2 sweep (JSON lines: ranks, c0, period,
log2_total, loss).  DESIGN.md 10.

For each N-replica setting and each target total T that one replica ran, the
total T_N the N replicas need to reach one replica's held-out loss at T
(log-linear interpolation over their totals; extrapolated one doubling past
the largest, marked) gives the sample efficiency T / T_N.  The effective
speed-up at N GPUs multiplies N by it and by the time efficiency of the
exchange at the C4 bench's rates: a step of 2^27 samples takes `--step-ms`,
an exchange pass over C costs `--exchange-ms` on the compute stream, and a
period p (x the 13.42 samples per row per rank of one exchange per step)
makes 1/p exchanges per step.

    python tools/samples_to_loss.py profiles/r04/replica/line2_c2_samples_to_loss.jsonl
"""
import argparse
import collections
import json
import math


def interp_log2_total(points, target):
    """log2 total at which the (log2 total, loss) curve reaches `target`."""
    pts = sorted(points)
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if (y0 - target) * (y1 - target) <= 0 and y0 != y1:
            return x0 + (y0 - target) / (y0 - y1) * (x1 - x0), False
    if len(pts) >= 2 and target < pts[-1][1]:     # past the largest total: extrapolate the last slope
        (x0, y0), (x1, y1) = pts[-2], pts[-1]
        if y0 > y1:
            return x1 + (y1 - target) / (y0 - y1) * (x1 - x0), True
    if target >= pts[0][1]:
        return pts[0][0], False
    return float("nan"), True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--step-ms", type=float, default=100.0, help="C4 bench step (2^27 samples), ms")
    ap.add_argument("--exchange-ms", type=float, default=3.9, help="C4 exchange pass over C, ms (DESIGN.md 10)")
    args = ap.parse_args()
    rows = [json.loads(l) for l in open(args.jsonl) if l.startswith("{")]
    one = {r["log2_total"]: r["loss"] for r in rows if r["ranks"] == 1}
    curves = collections.defaultdict(list)
    for r in rows:
        if r["ranks"] > 1:
            curves[(r["ranks"], r["c0"], r["period"])].append((r["log2_total"], r["loss"]))
    for (n, c0, period), pts in sorted(curves.items()):
        for t in sorted(one):
            if t >= max(x for x, _ in pts):
                continue
            xn, extra = interp_log2_total(pts, one[t])
            eff = 2.0 ** (t - xn) if math.isfinite(xn) else float("nan")
            time_eff = args.step_ms / (args.step_ms + args.exchange_ms / period)
            print(json.dumps({"ranks": n, "c0": c0, "period": period, "target_log2_total": t,
                              "one_rank_loss": one[t], "n_ranks_log2_total": round(xn, 3),
                              "extrapolated": extra, "sample_eff": round(eff, 3), "time_eff": round(time_eff, 3),
                              "effective_speedup": round(n * eff * time_eff, 2)}))


if __name__ == "__main__":
    main()
