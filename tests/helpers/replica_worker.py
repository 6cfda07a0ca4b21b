"""One rank of the multi-process replica test (tests/test_gpu_multi.py): LINE-2
on the 1k-vertex golden graph on cuda:0, the table deltas exchanged through
smore_amd/dist.py ReplicaSync (the fused HIP passes of replica_sync.hip around a
torch.distributed all-reduce; gloo here, since every rank shares one GPU).
TEST INFRASTRUCTURE.

    python tests/helpers/replica_worker.py RANK WORLD PORT TOTAL STEPS OUT.npz [HOT_ROWS LAUNCHES [SYNC]]

HOT_ROWS > 0 (sum rule): the hub-row exchange after each of LAUNCHES
launches per step (ReplicaSync.hot).  SYNC: sum (default), mean, adaptive or
adaptive:C0 (bench.py's N > 1 default is adaptive:64); 0 / 1 = sum / mean.

MODEL deepwalk (argv 10): TOTAL walks of DeepWalk (walk_times = TOTAL / V,
40 steps, window 5, K 5) in STEPS exchanges per rank; the adaptive rule's row
rates come from a row census (smore_census_begin / _end) of the first
round's walks, ReplicaSync(model="census", updates = walks per rank per
exchange) -- DESIGN.md 10.  SYNC "...+part": the walk partition (every rank
runs every walk, trains the pairs of its own centers; only C exchanged).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, total, steps = (int(x) for x in sys.argv[1:6])
    out = sys.argv[6]
    hot_rows = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    launches = int(sys.argv[8]) if len(sys.argv) > 8 else 1
    spec = sys.argv[9] if len(sys.argv) > 9 else "sum"
    model = sys.argv[10] if len(sys.argv) > 10 else "line2"
    spec = {"0": "sum", "1": "mean"}.get(spec, spec)
    # "+part": W partitioned by source (ReplicaSync partition=True: each rank
    # draws sources from its own part of the vertex law, only C is exchanged,
    # W gathered from the owners at the end)
    spec, plus, opt = spec.partition("+")
    part = plus and opt == "part"
    rule, _, c0 = spec.partition(":")
    c0 = float(c0) if c0 else 64.0
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import smore_amd
    from smore_amd.dist import ReplicaSync
    pn = smore_amd.ProNet(0)
    pn.LoadEdgeList(os.path.join(ROOT, "tests", "golden", "pl1k.txt"), 1)
    pn.alloc_tables(32, 2)
    pn.init_table_glibc(0, 0)
    pn.zero_table(1)
    per = total // world // steps
    if model == "deepwalk":
        V = pn.MAX_vid
        wt = total // V
        order = smore_amd.deepwalk_order(V, wt, 0)
        sync = None
        if world > 1:
            units = min(total, max(per * world, 1 << 12))
            pn.census_begin()
            pn.train_deepwalk(0, units, wt, 40, 5, 5, 0.025, 20251015, order, "atomic")
            pn.census_end(units)
            sync = ReplicaSync(pn, sync=rule, model="census", K=5, updates=per, c0=c0, partition=part)
        for k in range(steps):
            # walk partition: every rank runs the step's walks (its pairs only)
            b = k * world * per if part else (k * world + rank) * per
            e = b + per * world if part else b + per
            pn.train_deepwalk(b, min(total, e), wt, 40, 5, 5, 0.025, 20251015, order, "atomic")
            if sync is not None:
                sync.begin()
        if sync is not None:
            sync.end()
        torch.cuda.synchronize()
        np.savez(out, W=pn.get_table(0), C=pn.get_table(1))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    sync = (ReplicaSync(pn, sync=rule, hot_rows=hot_rows, model="line2", K=5, updates=per, c0=c0,
                        partition=part)
            if world > 1 else None)
    nl = launches if (sync is not None and sync.hot_idx) else 1
    for k in range(steps):
        begin = (k * world + rank) * per
        sub = per // nl
        for j in range(nl):
            n = sub if j + 1 < nl else per - j * sub
            pn.train_edges("line2", begin + j * sub, n, total, 5, 0.025, 0.0, 20251015, "atomic", sync=False)
            if nl > 1:
                sync.hot()
        if sync is not None:
            sync.begin()
    if sync is not None:
        sync.end()
    torch.cuda.synchronize()
    np.savez(out, W=pn.get_table(0), C=pn.get_table(1))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
