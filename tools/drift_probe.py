#!/usr/bin/env python3
"""Per-step update-kernel time over a long run of the C4 bench step, to see
whether throughput drifts with time on the box (warm-up / clock ramp).
    python tools/drift_probe.py [seconds=90]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 90.0
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges("c4")
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    pn.alloc_tables(64, 2)
    pn.init_table_uniform(0, 1)
    pn.zero_table(1)
    S = 1 << 27
    total = 1 << 40
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < secs:
        pn.train_edges("line2", k * S, S, total, 5, 0.025, 0.0, 7, "hybrid")
        d, u, _ = pn.last_phase_ms()
        print(json.dumps({"t": round(time.perf_counter() - t0, 2), "step": k, "draw_ms": round(d, 2),
                          "update_ms": round(u, 2)}), flush=True)
        k += 1


if __name__ == "__main__":
    main()
