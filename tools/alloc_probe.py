#!/usr/bin/env python3
"""Update-kernel time of the C4 step after each of several table
(re)allocations in one process: does the time level follow the tables'
placement?   python tools/alloc_probe.py [reallocs=8]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    import smore_amd
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges("c4")
    pn = smore_amd.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    S, total = 1 << 27, 1 << 40
    keep = []
    for a in range(n):
        pn.alloc_tables(64, 2)
        pn.init_table_uniform(0, 1)
        pn.zero_table(1)
        ms = []
        for k in range(4):
            pn.train_edges("line2", k * S, S, total, 5, 0.025, 0.0, 7, "hybrid")
            ms.append(round(pn.last_phase_ms()[1], 2))
        ptr, _ = pn.table_device(0)
        ptr1, _ = pn.table_device(1)
        print(json.dumps({"alloc": a, "W": hex(ptr), "C": hex(ptr1), "update_ms": ms}), flush=True)
        if a % 3 == 1:   # perturb the allocator: hold a 3-GB block across the next allocations
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            q = ctypes.c_void_p()
            hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(3 << 30))
            keep.append(q)


if __name__ == "__main__":
    main()
