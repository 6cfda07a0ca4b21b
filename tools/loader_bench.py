#!/usr/bin/env python3
"""Edge-list loader timing: text parse (parallel) and cached
reload of a config's graph written as text, on a host-only context.

    tools/gen_edgelist 10000000 200000000 4 /tmp/c4.txt
    python tools/loader_bench.py /tmp/c4.txt --cache /tmp/smore_cache
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--cache", default=None)
    ap.add_argument("--undirected", type=int, default=1)
    args = ap.parse_args()
    import smore_amd
    if args.cache:
        os.makedirs(args.cache, exist_ok=True)
    for k in range(2 if args.cache else 1):
        pn = smore_amd.ProNet(-1)
        if args.cache:
            pn.set_load_cache(args.cache)
        t0 = time.perf_counter()
        pn.LoadEdgeList(args.path, args.undirected)
        el = time.perf_counter() - t0
        sec, threads, hit = pn.last_load_info()
        print(json.dumps({"file": args.path, "bytes": os.path.getsize(args.path), "pass": k, "cache_hit": hit,
                          "text_or_cache_s": round(sec, 2), "threads": threads,
                          "load_edgelist_total_s": round(el, 2), "V": pn.MAX_vid, "E": pn.MAX_line}), flush=True)
        pn.close()


if __name__ == "__main__":
    main()
