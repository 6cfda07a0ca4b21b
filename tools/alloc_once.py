#!/usr/bin/env python3
"""One table allocation, four C4 steps: the update-kernel time level of this
process (tools/alloc_probe.py shows it follows the tables' placement)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import smore_amd  # noqa: E402
from smore_amd import graphgen  # noqa: E402

V, (src, dst, w) = graphgen.config_edges("c4")
pn = smore_amd.ProNet(0)
pn.set_graph_edges(V, src, dst, w)
pn.alloc_tables(64, 2)
pn.init_table_uniform(0, 1)
pn.zero_table(1)
ms = []
for k in range(4):
    pn.train_edges("line2", k << 27, 1 << 27, 1 << 40, 5, 0.025, 0.0, 7, "hybrid")
    ms.append(round(pn.last_phase_ms()[1], 2))
print(json.dumps({"alloc": os.environ.get("SMORE_TABLE_ALLOC", "default"), "update_ms": ms}), flush=True)
