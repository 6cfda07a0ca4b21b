#!/usr/bin/env python3
"""Benchmark: LINE order-2 edge-updates/s on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path over
`--samples` edge samples (default 2^27) of the synthetic power-law graph of
config c4 (10M vertices / 200M undirected lines = 400M directed slots, d=64,
K=5; the north star's 1/2/4/8-GPU graph), inputs resident in
HBM.  A step is the draw kernel (train_draw.hip) and the update kernel
(edge_kernels.h).  Default scatter: hybrid (atomic adds for the hot rows, the
128 hottest write-combined per workgroup in LDS, plain stores for the rest),
whose training objective matches the lossless atomic scatter.
One process per GPU.  With N > 1 the default is the 2-D block schedule
(smore_amd/dist.py BlockSync): rank r owns the W rows of part
r, the C table is cut into 2N blocks that rotate around the ring by send/recv
after each of a step's 2N sub-rounds, and nothing is all-reduced; each rank
draws S samples per step (weak scaling).  `--schedule replicas` keeps the
replicated tables with the adaptive delta all-reduce (dist.ReplicaSync).
Rank 0 prints one JSON line; n_gpus is the process group's world size.

    python bench.py [--gpus N --steps K --warmup W]
        (N > 1 without WORLD_SIZE: bench.py starts torch.distributed.run with
         N ranks as a child process, relays its output and exits with its
         status; nothing here touches the GPU first)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
        (WORLD_SIZE must equal --gpus)
"""
import argparse
import atexit
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def rec_width(K):
    """int32 words of a pre-drawn sample record (train_kernels.h rec_width)."""
    kmax = 5 if K <= 5 else 10 if K <= 10 else 20
    r = 4
    while r < 2 + kmax:
        r *= 2
    return r


def algorithmic_bytes(dim, K):
    """R = (2+K)*d*4 + 8 (vertex alias) + 16 (offset pair)
    + 8 (context alias) + 4 (target vid) + 8K (negative alias); W = (2+K)*d*4."""
    rows = (2 + K) * dim * 4
    return rows + 36 + 8 * K, rows


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--samples", type=int, default=1 << 27, help="edge samples per step per GPU")
    ap.add_argument("--mode", default="hybrid", choices=["hogwild", "atomic", "hybrid"],
                    help="scatter: hybrid (default), atomic (every row), hogwild (plain stores, loses updates)")
    ap.add_argument("--hot-tau", type=float, default=None, help="hybrid: hot-row threshold (default: the library's, 1.0)")
    ap.add_argument("--combine-rows", type=int, default=128, help="hybrid: LDS write-combined hottest rows")
    ap.add_argument("--combine-flush", type=int, default=0, help="hybrid: rounds between LDS drains (0: automatic)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal)")
    ap.add_argument("--schedule", default="blocks", choices=["blocks", "replicas"],
                    help="N > 1: blocks (default: the 2-D block schedule -- rank r owns W part r, the C table in 2N "
                         "blocks rotating around the ring by send/recv, one epoch of 2N sub-rounds per step, nothing "
                         "all-reduced; DESIGN.md 10) or replicas (replicated C, deltas all-reduced)")
    ap.add_argument("--sync-every", type=int, default=1)
    ap.add_argument("--exchanges-per-step", type=int, default=2,
                    help="N > 1: the step's samples in this many launches, an exchange after each (default 2: "
                         "6.7 samples per row per rank per exchange at C4, the best effective 8-GPU speed-up of "
                         "the C2-scale samples-to-loss study, DESIGN.md 10)")
    ap.add_argument("--sync", default="adaptive", choices=["sum", "mean", "adaptive"],
                    help="N > 1 exchange rule: adaptive (default: per row the sum for rows with few updates per "
                         "exchange, towards the mean for the hubs), mean (model averaging) or sum (every update "
                         "applied once; diverges at >= 4 ranks at this exchange period), DESIGN.md 10")
    ap.add_argument("--sync-c0", type=float, default=None,
                    help="adaptive rule: c0 (default 2048 with the source partition, 64 without)")
    ap.add_argument("--no-partition", action="store_true",
                    help="N > 1: replicate W too (default: W rows partitioned by source, only C exchanged)")
    ap.add_argument("--hot-rows", type=int, default=65536,
                    help="N > 1, --sync sum: hub rows per table exchanged after every launch")
    ap.add_argument("--launches", type=int, default=8,
                    help="N > 1: training launches per step, each followed by the hub-row exchange")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--semantics", default="cpp", choices=["cpp", "go"],
                    help="update rule: the C++ reference's (default) or the Go tree's (pkg/pronet)")
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"],
                    help="N=1: measure roofline.traffic with rocprofv3 --pmc in child runs of this config "
                         "before the timed run (off: the committed profiles/pmc_traffic.json)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    # exchanges inside a step assume one exchange period of S / n_ex samples;
    # with --sync-every > 1 the period would alternate between S / n_ex and S
    # while the adaptive scales assume one: not a valid combination
    if a.sync_every > 1 and a.exchanges_per_step > 1:
        ap.error("--sync-every > 1 needs --exchanges-per-step 1")
    return a


# gfx950: FETCH_SIZE counts half the bytes of these kernels' reads (calibrated on
# their own access shapes, profiles/pmc_calibration.json); WRITE_SIZE the bytes
FETCH_CORRECTION = 2.0
PMC_KERNELS = ("draw_kernel", "edge_train_kernel")


def pmc_per_launch(path, counter):
    """{kernel: bytes per dispatch} of PMC_KERNELS from a rocprofv3 --pmc
    counter_collection CSV (Counter_Value in KB, summed per dispatch, averaged
    over dispatches; FETCH_SIZE x FETCH_CORRECTION)."""
    per = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        for k in PMC_KERNELS:
            if k in row["Kernel_Name"]:
                d = per.setdefault(k, {})
                d[row["Dispatch_Id"]] = d.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    scale = 1024.0 * (FETCH_CORRECTION if counter == "FETCH_SIZE" else 1.0)
    return {k: sum(d.values()) / len(d) * scale for k, d in per.items() if d}


def pmc_traffic_live(args):
    """HBM traffic per step of this config, measured now: this script re-run for
    2 steps under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc
    WRITE_SIZE` (MI355X_MICROARCH.md: one counter group per pass), as child
    processes started before this process touches the GPU.  Returns
    ({kernel: bytes per launch}, note) or (None, reason)."""
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rocprof):
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "2", "--warmup", "0",
             "--config", args.config, "--dim", str(args.dim), "--negative", str(args.negative),
             "--samples", str(args.samples), "--mode", args.mode,
             "--combine-rows", str(args.combine_rows), "--combine-flush", str(args.combine_flush),
             "--semantics", args.semantics, "--seed", str(args.seed)]
    if args.hot_tau is not None:
        child += ["--hot-tau", str(args.hot_tau)]
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="smore_pmc_")
        try:
            r = subprocess.run([rocprof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--"]
                               + child, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=180)
            path = os.path.join(d, "run_counter_collection.csv")
            if r.returncode != 0 or not os.path.exists(path):
                return None, "rocprofv3 --pmc %s exited %d: %s" % (counter, r.returncode,
                                                                    r.stderr.decode(errors="replace")[-300:])
            per = pmc_per_launch(path, counter)
            for k in PMC_KERNELS:
                if k not in per:
                    return None, "no %s dispatches under --pmc %s" % (k, counter)
                vals[k] = vals.get(k, 0.0) + per[k]
        except (OSError, subprocess.SubprocessError, KeyError, ValueError) as e:
            return None, "rocprofv3 --pmc %s failed: %s" % (counter, e)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return vals, ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of this config, run by "
                  "bench.py in 2-step child runs before the timed run; FETCH_SIZE x 2 (gfx950 calibration), KB x 1024")


def cgroup_cpu_quota():
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max /
    v1 cfs quota), or None when unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // p))
    except (OSError, ValueError):
        pass
    return None


def host_cores():
    """(CPUs this process can actually use: its affinity mask capped by its
    cgroup's CPU quota; CPUs of the machine; the quota or None)."""
    try:
        mine = len(os.sched_getaffinity(0))
    except AttributeError:
        mine = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    return (min(mine, quota) if quota else mine), os.cpu_count() or mine, quota


def _cpu_rate(orc, g, W, C, K, seconds, threads):
    """LINE-2 samples/s of the oracle's fp64 OpenMP Hogwild loop on `threads`
    host threads, over >= `seconds` of training in 1M-sample chunks per thread."""
    total = 1 << 40
    chunk = 250_000 * threads
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.train_edge_f64(g, "line2", W, C, K, 0.025, 0.0, total, done, done + chunk, 7, threads)
        done += chunk
    return done, time.perf_counter() - t0


def cpu_baseline(V, src, dst, w, dim, K, seconds, config):
    """The reference's arithmetic and CPU structure -- fp64 rows, OpenMP Hogwild
    threads over contiguous sample blocks (src/model/LINE.cpp:160-191) -- as
    restated by the oracle (the reference sources do not travel to the GPU box),
    on the same graph, bounded in time: on every host CPU this process may run
    on (SURVEY.md 8d "threads = nproc") and on 1 thread."""
    from oracle import oracle as orc
    mine, machine, quota = host_cores()
    g = orc.Graph(V, src, dst, w)
    W = (np.random.default_rng(1).random((V, dim)) - 0.5) / dim
    C = np.zeros_like(W)
    n_all, t_all = _cpu_rate(orc, g, W, C, K, seconds, mine)
    n_one, t_one = _cpu_rate(orc, g, W, C, K, max(2.0, seconds / 2), 1)
    return {"value": round(n_all / t_all / 1e6, 4), "unit": "M edge-updates/s", "cores": mine, "kind": "port",
            "arithmetic": "f64 (the reference's)", "host_cpus_available": mine, "host_cpus_machine": machine,
            "value_1thread": round(n_one / t_one / 1e6, 4),
            "host_cpu_quota": quota,
            "sample": "LINE-2 (d=%d, K=%d) on the same %s graph, fp64 rows: %d samples on %d OpenMP Hogwild threads "
                      "(every CPU this process can use: affinity capped by the cgroup CPU quota %s; %d CPUs on the "
                      "machine) in %.1f s, and %d samples on 1 thread in %.1f s"
                      % (dim, K, config, n_all, mine, quota, machine, t_all, n_one, t_one)}


def graph_file(config):
    """Where rank 0 of a node leaves the built graph for the others: host
    memory (/dev/shm) when present; one name per job (the rendezvous port)."""
    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    return os.path.join(d, "smore_bench_%s_%s_%s.graph" % (config, os.environ.get("MASTER_PORT", "0"),
                                                            os.environ.get("TORCHELASTIC_RUN_ID", "x")))


def peak_rss_gb():
    """This process's peak resident host memory (GB)."""
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0 ** 2


def largest_remainder(samples, mass):
    """smore_block_counts restated: samples split by mass, largest remainder
    first (ties to the lower block)."""
    x = [samples * m for m in mass]
    c = [int(np.floor(v)) for v in x]
    rem = sorted(range(len(x)), key=lambda k: -(x[k] - np.floor(x[k])))
    for k in rem[:samples - sum(c)]:
        c[k] += 1
    return c


def block_schedule(count, per, world, rank, counts, part_mass=None):
    """exchange.cpp group_block_edges' split of samples [0, count) for replica
    `rank`: rounds (epochs) of per * world samples, each round's samples split
    over the replicas by their parts' source mass (largest remainder;
    part_mass None = equal parts), the rank's slice split over its 2N cells by
    counts(slice) in sub-round order.  Yields (sub-round, block, first sample,
    samples) -- zero-sample cells too: their rotation still happens."""
    nb = 2 * world
    pm = part_mass if part_mass is not None else [1.0 / world] * world
    rounds = 1 if per > count // world else -(-count // (per * world))
    for k in range(rounds):
        lo = count * k // rounds
        m = count * (k + 1) // rounds - lo
        share = largest_remainder(m, pm)
        cur = lo + sum(share[:rank])
        cnt = counts(share[rank])
        for s in range(nb):
            b = (2 * rank + s) % nb
            yield k * nb + s, b, cur, int(cnt[b])
            cur += int(cnt[b])


def run_block_step(pn, bsync, k, world, rank, S, total, K, seed, mode, cell_events=None):
    """One bench step in the block schedule: one epoch (2N sub-rounds) of the
    rank's samples [(k*world + rank)*S, +S), each sub-round one cell launch
    followed by its C block's rotation (dist.BlockSync).  cell_events: a list
    that gets a (start, end) CUDA event pair around each cell (read after the
    timed region, so no host wait inside it)."""
    import torch
    base = k * world * S
    L = pn.block_cell_launches()      # a cell in L launches, the hub slots exchanged after each
    for s, b, lo, n in block_schedule(world * S, S, world, rank, pn.block_counts, pn.block_part_mass()):
        assert bsync.block() == b

        def train(blk, q=0, lo=lo, n=n):
            x0, x1 = n * q // L, n * (q + 1) // L
            if x1 > x0:
                ev = None
                if cell_events is not None:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                pn.block_train_edges(blk, base + lo + x0, x1 - x0, total, K, 0.025, seed, mode, sync=False)
                if ev is not None:
                    ev[1].record()
                    cell_events.append(ev)
        bsync.sub_round(train, L)


def run_step(pn, sync, k, world, rank, S, n_launch, n_ex, total, K, seed, mode, sync_every, on_launch=None):
    """One bench step of rank `rank`: its global samples [(k*world + rank)*S, +S)
    in n_launch launches; with a replica exchange (N > 1) the hub-row exchange
    after every launch (sum rule), or an exchange begun after every launch but
    the last (--exchanges-per-step), and one begun at the end of every
    sync_every-th step, which overlaps the next step (dist.OverlapSync)."""
    begin = (k * world + rank) * S
    sub = S // n_launch
    for j in range(n_launch):
        n = sub if j + 1 < n_launch else S - j * sub
        pn.train_edges("line2", begin + j * sub, n, total, K, 0.025, 0.0, seed, mode, sync=False)
        if on_launch is not None:
            on_launch()
        if n_launch > 1 and sync.hot_idx:
            sync.hot()    # the hub rows of every rank, synchronously
        elif n_ex > 1 and j + 1 < n_launch:
            sync.begin()  # exchanges inside the step (--exchanges-per-step)
    if sync is not None and (k + 1) % sync_every == 0:
        sync.begin()      # folds the previous exchange in; this one overlaps the next step


def launch_ranks(args):
    """`--gpus N` (N > 1) outside a launcher: run this script under
    torch.distributed.run with N local ranks as a CHILD process (never exec:
    nothing in this process has touched the GPU, and must not), its output
    passed through, its exit status returned."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    print("[bench] --gpus %d: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def world_from_env(args):
    """The launcher's WORLD_SIZE, which must agree with --gpus: None when
    this process must start the ranks itself (--gpus N > 1, no launcher)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        return None if args.gpus > 1 else 1
    if int(ws) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s (the launcher's rank count); they must agree"
                         % (args.gpus, ws))
    return int(ws)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    world = world_from_env(args)
    if world is None:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # live PMC traffic (N=1): child runs under rocprofv3, before this process
    # initialises the GPU
    pmc_live, pmc_note = None, "off"
    # (not when this run is itself under a profiler: no nested rocprofv3)
    profiled = any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)
    if world == 1 and not args.pmc_child and args.pmc == "auto" and not profiled:
        pmc_live, pmc_note = pmc_traffic_live(args)
        print("[bench] pmc: %s" % (pmc_note if pmc_live is None else
                                   {k: round(v / args.samples, 1) for k, v in pmc_live.items()}),
              file=sys.stderr, flush=True)
    import torch
    dist = None
    node_rank = local                       # this process's index on the node (the graph builder is 0)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    import smore_amd
    from smore_amd import graphgen
    from smore_amd.dist import BlockSync, ReplicaSync, block_hubs, table_tensor

    t_gen = time.perf_counter()
    pn = smore_amd.ProNet(local)
    src = dst = w = None
    if world == 1:
        V, (src, dst, w) = graphgen.config_edges(args.config)
        t_build = time.perf_counter()
        pn.set_graph_edges(V, src, dst, w)
    else:
        # one process per node generates and builds the graph and writes it
        # (smore_save_graph); the others read it (smore_load_graph) instead of
        # generating and building 400M slots each under a shared CPU quota
        path = graph_file(args.config)
        if node_rank == 0:
            V, (src, dst, w) = graphgen.config_edges(args.config)
            t_build = time.perf_counter()
            pn.set_graph_edges(V, src, dst, w)
            pn.save_graph(path)
            # a run that fails before the removal below must not leave a
            # multi-GB file in host memory (/dev/shm)
            atexit.register(lambda p=path: os.path.exists(p) and os.remove(p))
            src = dst = w = None
        dist.barrier()
        t_build = time.perf_counter() if node_rank != 0 else t_build
        if node_rank != 0:
            pn.load_graph(path)
        V = pn.MAX_vid
        dist.barrier()
        if node_rank == 0:
            os.remove(path)
    t_ready = time.perf_counter()
    setup = {"rank": rank, "setup_s": round(t_ready - t_gen, 2), "graph_s": round(t_ready - t_build, 2),
             "peak_rss_gb": round(peak_rss_gb(), 2)}
    if rank == 0:
        print("[bench] %s: graph ready in %.1f s (generated %.1f s, built / read + uploaded %.1f s)"
              % (args.config, t_ready - t_gen, t_build - t_gen, t_ready - t_build), file=sys.stderr, flush=True)
    E = pn.MAX_line
    if args.semantics == "go":
        pn.set_semantics("go")
    if args.hot_tau is not None:
        pn.set_hot_threshold(args.hot_tau)
    pn.set_write_combine(args.combine_rows, args.combine_flush)
    pn.alloc_tables(args.dim, 2)
    pn.init_table_uniform(0, args.seed)     # W ~ (u-0.5)/d, as the reference Init law
    pn.zero_table(1)                        # C = 0 (src/model/LINE.cpp:92)
    stream = torch.cuda.Stream()             # a real stream: the default one is the null stream
    torch.cuda.set_stream(stream)
    pn.set_stream(stream.cuda_stream)
    # N > 1: each rank draws its sources from its own part of the vertex ids
    # (equal source mass), so W rows are owned and only C is exchanged; the
    # adaptive rule scales C's summed deltas per row
    blocks = world > 1 and args.schedule == "blocks"
    partition = world > 1 and not args.no_partition and not blocks
    c0 = args.sync_c0 if args.sync_c0 is not None else (2048.0 if partition else 64.0)
    n_ex = max(1, args.exchanges_per_step) if world > 1 and args.sync != "sum" and not blocks else 1
    sync = (ReplicaSync(pn, sync=args.sync, hot_rows=args.hot_rows, model="line2", K=args.negative,
                        updates=args.samples * args.sync_every // n_ex, c0=c0, partition=partition)
            if world > 1 and not blocks else None)
    bsync = None
    if blocks:
        # the 2-D block schedule: this rank's cells' draw tables (W part r,
        # 2N C blocks), the rotation over torch.distributed
        t_bs = time.perf_counter()
        pn.block_setup("line2", world, rank, args.negative, args.mode)
        setup["block_setup_s"] = round(time.perf_counter() - t_bs, 2)
        wb, cb = pn.block_bounds()
        # the hub C rows' slots: every cell trains them, exchanged after every
        # sub-round (S / 2N samples per rank)
        hubs = block_hubs(pn, args.samples / (2 * world) / pn.block_cell_launches())
        setup["hubs"] = int(pn.block_hubs()[0])
        bsync = BlockSync(table_tensor(pn, 0), table_tensor(pn, 1), wb, cb, hubs=hubs)
        if rank == 0:
            print("[bench] block schedule set up in %.1f s" % (time.perf_counter() - t_bs), file=sys.stderr,
                  flush=True)
    n_launch = max(1, args.launches) if (sync is not None and sync.hot_idx) else n_ex
    phase = [0.0, 0.0, 0]     # exposed draw ms, update ms, update launches (timed steps)
    cell_events = []          # block schedule: (start, end) events of the timed steps' cells

    S, K = args.samples, args.negative
    total = (args.warmup + args.steps) * S * world     # alpha schedule over the whole job

    def step(k, timed=False):
        if bsync is not None:
            run_block_step(pn, bsync, k, world, rank, S, total, K, args.seed, args.mode,
                           cell_events if timed else None)
            return

        def on_launch():
            if timed:
                ph = pn.last_phase_ms()      # waits for this launch's events (a few us of host gap)
                if ph is not None:
                    phase[0] += ph[0]
                    phase[1] += ph[1]
                    phase[2] += ph[2]
        run_step(pn, sync, k, world, rank, S, n_launch, n_ex, total, K, args.seed, args.mode, args.sync_every,
                 on_launch)

    if args.pmc_child:      # the profiled child of pmc_traffic_live: the steps only
        for k in range(args.steps):
            step(k)
        torch.cuda.synchronize()
        return
    for k in range(args.warmup):
        step(k)
    if sync is not None:
        sync.end()
    if bsync is not None:
        bsync.finish(gather=False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.warmup, args.warmup + args.steps):
        step(k, timed=True)
    draw_ms, upd_ms, launches = phase
    if sync is not None:
        sync.end()            # the last exchange lands inside the timed region
    if bsync is not None:
        bsync.finish(gather=True)   # the last rotations and the W / C gather inside the timed region
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if cell_events:           # block schedule: the cells (draw + update kernels) as the "update" time
        upd_ms = sum(a.elapsed_time(b) for a, b in cell_events)
        launches = len(cell_events)
    if dist:
        assert dist.get_world_size() == world
        t = torch.tensor([el], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    skipped = pn.skipped()
    ran_mode = pn.last_mode()       # the scatter the timed launches ran (smore_last_mode)
    setup["peak_rss_gb"] = round(peak_rss_gb(), 2)
    setups = [setup]
    if dist:
        setups = [None] * world
        dist.all_gather_object(setups, setup)

    updates = S * args.steps * world
    R, Wb = algorithmic_bytes(args.dim, K)
    step_s = gpu_ms / 1e3 / args.steps              # avg per-step time on the launch stream
    # dominant kernel = the update kernel (gather/update/scatter); its algorithmic
    # reads are the K+2 rows plus the 32-B pre-drawn record of each sample
    rec_b = 4 * rec_width(K)
    R_upd = (2 + K) * args.dim * 4 + rec_b
    upd_s = upd_ms / 1e3 / args.steps if upd_ms > 0 else step_s       # update-kernel time per step
    launch_s = upd_ms / 1e3 / launches if launches else step_s         # per update launch (rocprof average)
    achieved = R_upd * S / upd_s / 1e9
    # PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_summary.py) of this
    # config from a committed rocprofv3 --pmc run: per step (draw + update
    # kernel, one launch each) and per update launch
    traffic = traffic_upd = traffic_src = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if pmc_live is not None and n_launch == 1:
        traffic = sum(pmc_live.values())
        traffic_upd = pmc_live["edge_train_kernel"]
        traffic_src = pmc_note
    elif os.path.exists(pmc):
        p = json.load(open(pmc))
        if p.get("config") == args.config and p.get("samples") == S and p.get("mode") == args.mode:
            traffic = p.get("hbm_bytes_per_step", p.get("hbm_bytes_per_launch"))
            traffic_upd = p.get("hbm_bytes_per_launch")
            traffic_src = ("profiles/pmc_traffic.json: rocprofv3 --pmc of this config (%s)%s"
                           % (p.get("round", ""), "" if pmc_note == "off" else "; live measurement: " + pmc_note))
    copy_peak = pn.copy_bandwidth(4 << 30, 5) if rank == 0 else 0.0   # membw.hip float4 copy
    Wt = pn.get_table(0)
    assert np.isfinite(Wt).all(), "non-finite embeddings"

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.cpu_baseline_seconds > 0:
            cpu = cpu_baseline(V, src, dst, w, args.dim, K, args.cpu_baseline_seconds, args.config)
        out = {
            "metric": "M edge-updates/sec (d=64, neg=5)",
            "value": round(updates / el / 1e6, 3),
            "unit": "M edge-updates/s",
            "n_gpus": dist.get_world_size() if dist else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic power-law (Zipf 0.8 endpoints, seeded), random-init tables",
            "config": {"workload": "LINE order-2 sampled negative-sampling SGD, config %s%s"
                                   % (args.config, "" if args.semantics == "cpp" else ", Go rules (pkg/pronet)"),
                       "vertices": V, "edge_slots": E, "dim": args.dim, "negative": K,
                       "samples_per_step_per_gpu": S,
                       "scatter": {"hogwild": "plain"}.get(ran_mode, ran_mode), "scatter_asked": args.mode,
                       "sync": (("blocks: 2-D block schedule, rank r owns W part r, C in %d blocks rotated to "
                                 "rank r-1 (send/recv) after each of %d sub-rounds per step; the %d hub C rows "
                                 "trained in every cell on per-rank slots, their deltas all-reduced after each "
                                 "sub-round (adaptive scales); W parts and C blocks gathered at the end"
                                 % (2 * world, 2 * world, setup.get("hubs", 0))) if blocks else
                                "%s%s every %s%s%s" % (
                           args.sync, " c0=%g" % c0 if args.sync == "adaptive" else "",
                           "%d steps" % args.sync_every if n_ex == 1 else "1/%d step" % n_ex,
                           ", W partitioned by source (C exchanged, W gathered at the end)" if partition else "",
                           ", %d hub rows per table after each of %d launches per step"
                           % (args.hot_rows, n_launch) if sync is not None and sync.hot_idx else ""))
                               if world > 1 else "none",
                       "parallelism": ("blocks%d" if blocks else "replicas%d") % world},
            # achieved = updates/s x 1868 B (the whole path's algorithmic
            # reads) over the 8 TB/s HBM read roofline; the dominant kernel's own
            # figure (its per-launch time, as rocprof reports it) is "kernel"
            "roofline": {"bound": "hbm", "achieved": round(R * S / step_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(R * S / step_s / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "bytes_per_update_read": R, "bytes_per_update_write": Wb,
                         "ms_per_step": round(step_s * 1e3, 3),
                         "traffic_per_algorithmic": (round(traffic / ((R + Wb) * S), 3) if traffic else None),
                         "measured_peak": {"copy_GBs": round(copy_peak, 1),
                                           "frac": round((R + Wb) * S / step_s / 1e9 / copy_peak, 4),
                                           "note": "the path's algorithmic read+write bytes per second over the "
                                                   "library's float4 device copy (membw.hip, 4 GiB, best of "
                                                   "default / non-temporal policy and 4 / 8 blocks per CU)"},
                         "kernel": {"name": ("block cells: block_draw_kernel + edge_train_kernel per cell"
                                             if blocks else "edge_train_kernel (gather/update/scatter)"),
                                    "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                                    "bytes_per_update_read": R_upd, "bytes_per_update_write": Wb,
                                    "achieved_rw": round((R_upd + Wb) * S / upd_s / 1e9, 1),
                                    "ms_per_launch": round(launch_s * 1e3, 3),
                                    "launches_per_step": round(launches / args.steps, 2),
                                    "update_ms_per_step": round(upd_s * 1e3, 3),
                                    "exposed_draw_ms_per_step": round(draw_ms / args.steps, 3),
                                    "traffic": traffic_upd}},
            "cpu_baseline": cpu,
            "skipped_samples": int(skipped),
            # per rank: graph generation / build (local rank 0) or read (the
            # others), block-table setup, peak host RSS
            "setup": {"max_setup_s": max(x["setup_s"] for x in setups),
                      "max_peak_rss_gb": max(x["peak_rss_gb"] for x in setups), "ranks": setups},
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
