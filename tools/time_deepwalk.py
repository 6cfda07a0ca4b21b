#!/usr/bin/env python3
"""Time DeepWalk (walks -> pair records -> update kernel) on the C5 stand-in for a
few walk counts: python tools/time_deepwalk.py [hybrid|atomic|hogwild]."""
import sys, time, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import smore_amd
from smore_amd import graphgen
V, (src, dst, w) = graphgen.config_edges("c5")
pn = smore_amd.ProNet(0)
pn.set_graph_edges(V, src, dst, w)
pn.alloc_tables(128, 2)
pn.init_table_uniform(0, 1)
pn.init_table_uniform(1, 2)
order = smore_amd.deepwalk_order(V, 2, 0)
mode = sys.argv[1] if len(sys.argv) > 1 else "hybrid"
for n in (1 << 12, 1 << 16, 1 << 18, V):
    t = time.perf_counter()
    pn.train_deepwalk(0, n, 2, 40, 5, 5, 0.025, 7, order, mode)
    print(mode, n, "walks", round(time.perf_counter() - t, 3), "s", pn.last_kernel_ms(), "ms", flush=True)
