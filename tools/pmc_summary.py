#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of the bench into profiles/: per-launch HBM
traffic of a kernel from separate FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE in KB, from the L2's
memory-side request counters, Infinity-Cache hits included) and the
kernel-trace average duration.

gfx950 correction, calibrated on this path's own access shape
(profiles/pmc_calibration.json: tools/probe_scatter's dword-per-lane gathers of
random 256-B rows from a 5-GB table, known byte counts): FETCH_SIZE reads
0.51 x the bytes fetched, WRITE_SIZE 1.000 x the bytes written (stores and
float atomics).  Fetched bytes are therefore FETCH_SIZE x 2.

    python tools/pmc_summary.py --fetch F.csv --write W.csv --stats S.csv \
        --config c4 --samples 134217728 --mode hybrid --out profiles/pmc_traffic.json \
        [--kernel edge_train_kernel] [--step draw_kernel --round r02]

With --step, the output holds the per-launch traffic of --kernel (the update
kernel) and of each --step kernel, and hbm_bytes_per_step = their sum: one
bench step launches each once (bench.py reads it as roofline.traffic).
"""
import argparse
import csv
import json


FETCH_CORRECTION = 2.0


def per_dispatch(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit("no %s dispatches in %s" % (kernel, path))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--kernel", default="edge_train_kernel")
    ap.add_argument("--config", required=True)
    ap.add_argument("--samples", type=int, required=True)
    ap.add_argument("--mode", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--step", nargs="*", default=[])
    ap.add_argument("--round", default="")
    a = ap.parse_args()
    one = summarize(a, a.kernel)
    if not a.step:
        json.dump(one, open(a.out, "w"), indent=1)
        print(json.dumps(one))
        return
    parts = {a.kernel: one}
    for k in a.step:
        parts[k] = summarize(a, k)
    out = {"round": a.round, "config": a.config, "samples": a.samples, "mode": a.mode,
           "hbm_bytes_per_step": sum(p["hbm_bytes_per_launch"] for p in parts.values()),
           "bytes_per_sample_step": sum(p["hbm_bytes_per_launch"] for p in parts.values()) / a.samples,
           "hbm_bytes_per_launch": one["hbm_bytes_per_launch"], "kernels": parts}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


def summarize(a, kernel):
    f, nf = per_dispatch(a.fetch, kernel)
    f_raw = f
    f = f * FETCH_CORRECTION
    w, nw = per_dispatch(a.write, kernel)
    stats = [r for r in csv.DictReader(open(a.stats)) if kernel in r["Name"]]
    avg_ns = float(stats[0]["AverageNs"]) if stats else None
    out = {
        "config": a.config, "samples": a.samples, "mode": a.mode,
        "kernel": stats[0]["Name"] if stats else kernel,
        "dispatches_fetch": nf, "dispatches_write": nw,
        "fetch_size_kb_raw": f_raw, "fetch_kb_corrected": f, "write_size_kb": w,
        "hbm_bytes_per_launch": (f + w) * 1024.0,
        "fetch_bytes_per_sample": f * 1024.0 / a.samples,
        "write_bytes_per_sample": w * 1024.0 / a.samples,
        "kernel_avg_ns": avg_ns,
        "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; units KB; "
                "fetch = FETCH_SIZE x 2 (gfx950 half-count, calibrated in profiles/pmc_calibration.json); "
                "includes Infinity-Cache hits",
    }
    return out


if __name__ == "__main__":
    main()
