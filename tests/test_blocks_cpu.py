"""The 2-D block schedule's rotation (smore_amd/dist.py BlockSync) on CPU with
gloo, world size 2 and 3: every rank trains its cells in sub-round order on
the C blocks it holds, blocks move to rank r - 1 after each sub-round, and
after finish() every rank holds exactly the tables of ONE shared table pair
trained cell by cell in the same order -- the schedule is the reference's
single table (src/model/LINE.cpp:160-191) with the samples grouped by cell.
Also the group driver's sample split: rounds, replica slices and the
largest-remainder cell counts (exchange.cpp group_block_edges)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

V, D = 48, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bounds(world):
    wb = [V * p // world for p in range(world + 1)]
    nb = 2 * world
    cb = [V * b // nb for b in range(nb + 1)]
    return wb, cb


def _cell(W, C, wb, cb, r, b, s):
    """A deterministic, order-dependent update touching W part r and C block
    b only (the shape of a LINE-2 cell launch)."""
    w = W[wb[r]:wb[r + 1]]
    c = C[cb[b]:cb[b + 1]]
    g = torch.tanh(w.sum(0) * 0.1 + c.mean(0))
    c.mul_(0.99).add_(g * (0.01 * (r + 1)) + 0.001 * s)
    w.add_(c.mean(0) * 0.05 - 0.002 * b)


def _reference(world, subrounds):
    torch.manual_seed(0)
    W, C = torch.randn(V, D), torch.randn(V, D)
    wb, cb = _bounds(world)
    nb = 2 * world
    for s in range(subrounds):
        for r in range(world):
            _cell(W, C, wb, cb, r, (2 * r + s) % nb, s)
    return W, C


def _worker(rank, world, port, subrounds, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smore_amd.dist import BlockSync
    torch.manual_seed(0)
    W, C = torch.randn(V, D), torch.randn(V, D)
    wb, cb = _bounds(world)
    # rows this rank must not read stale: poison everything it does not own
    # at the start except the two blocks it trains first (they are its own)
    bs = BlockSync(W, C, wb, cb)
    for b in range(2 * world):
        if b not in (bs.block(0), bs.block(1)):
            C[cb[b]:cb[b + 1]] = float("nan")
    for p in range(world):
        if p != rank:
            W[wb[p]:wb[p + 1]] = float("nan")
    for _ in range(subrounds):
        s = bs.s
        bs.sub_round(lambda b: _cell(W, C, wb, cb, rank, b, s))
    bs.finish(gather=True)
    RW, RC = _reference(world, subrounds)
    out[rank] = int(torch.equal(W, RW) and torch.equal(C, RC))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,subrounds", [(2, 4), (2, 11), (3, 6), (3, 17), (4, 8), (8, 21)])
def test_block_rotation_gloo(world, subrounds):
    """Whole epochs and a partial one: the holder of every block after the
    drain is ((b - s) mod 2N) // 2 and no rank ever trains a stale block."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, subrounds, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world


def test_group_block_split():
    """exchange.cpp group_block_edges' split restated (bench.py reuses it):
    the rounds tile [0, count), every replica's slice is split over its cells
    exactly, in sub-round order, with consecutive sample ranges."""
    from bench import block_schedule, largest_remainder
    mass = [[0.1, 0.2, 0.3, 0.15, 0.25, 0.0], [0.5, 0.1, 0.1, 0.1, 0.1, 0.1], [1 / 6] * 6]
    for (count, per), pm in zip(((10_000, 1000), (9_999, 5000), (7, 100), (10_000, 1000)),
                                (None, None, None, [0.6, 0.3, 0.1])):
        seen = []
        per_rank = [0, 0, 0]
        for r, m in enumerate(mass):
            subs = list(block_schedule(count, per, 3, r, lambda x, m=m: largest_remainder(x, m), pm))
            assert [s for s, _, _, _ in subs] == list(range(len(subs))) and len(subs) % 6 == 0
            for s, b, lo, n in subs:
                assert b == (2 * r + s) % 6
                if n:
                    seen.append((lo, n))
                    per_rank[r] += n
        if pm is not None:      # a skewed partition: replicas get their parts' share of every round
            assert per_rank == [6000, 3000, 1000]
        seen.sort()
        pos = 0
        for lo, n in seen:
            assert lo == pos
            pos += n
        assert pos == count


def test_part_mass_split_on_a_skewed_graph(tmp_path):
    """smore_block_part_mass on a graph whose parts cannot have equal source
    mass: the part holding the most has that share, the group's round
    split (largest remainder over the part masses) gives it that
    share of every round's samples, and the union of the parts' laws is the
    global source law (needs no GPU: the host side of smore_block_setup is
    restated by tests/block_spec.py)."""
    import numpy as np
    from tests.block_spec import part_masses
    from bench import largest_remainder
    from tests.block_spec import skewed_graph_lines
    f = tmp_path / "skewed.txt"
    f.write_text(skewed_graph_lines())
    for world in (2, 4, 8):
        pm, wb = part_masses(str(f), world, undirected=0)
        assert abs(sum(pm) - 1.0) < 1e-12
        assert max(pm) > 1.1 / world            # a part far off 1/N
        share = largest_remainder(1 << 20, pm)
        assert sum(share) == 1 << 20
        for r in range(world):
            assert abs(share[r] - pm[r] * (1 << 20)) <= 1


def _neg_law_check(g, world, tag):
    import numpy as np
    from tests.block_spec import cell_masses, negative_marginal
    wb, cb, m, pnb, pn = cell_masses(g, world)
    share = m / m.sum(axis=1, keepdims=True)
    w = (pnb[None, :] / np.where(share > 0, share, 1.0)).astype(np.float32).astype(np.float64)
    raw, _ = negative_marginal(cb, m, pnb, pn, np.ones_like(m))
    fix, parts = negative_marginal(cb, m, pnb, pn, w)
    nz = pn > 0
    raw_dev = raw[nz] / pn[nz]
    fix_dev = fix[nz] / pn[nz]
    # per block (the granularity the uncorrected schedule gets wrong)
    blk_raw = np.array([raw[cb[k]:cb[k + 1]].sum() / pnb[k] for k in range(2 * world)])
    print("%s N=%d: uncorrected block marginal %.3f..%.3f, corrected rows %.6f..%.6f"
          % (tag, world, blk_raw.min(), blk_raw.max(), fix_dev.min(), fix_dev.max()))
    assert np.abs(fix_dev - 1.0).max() < 0.01          # within 1 % of NegativeSample's law, every row
    for f in parts:                                      # and every part's own epoch
        assert np.abs(f[nz] / pn[nz] - 1.0).max() < 0.01
    return blk_raw


@pytest.mark.parametrize("world", [2, 4, 8])
def test_block_negative_law_pl1k(world):
    """the epoch marginal of the block schedule's negatives
    against NegativeSample's law (src/proNet.cpp:623-633).  Without a
    correction, block b's negatives come 2N m_ctx(b) times as often as the law
    says; with blocks.cpp's per-cell weight pn(b) / m(r, b) on the negative
    steps every row's expected negative updates are the law's (to fp32
    rounding of the weight)."""
    from oracle import oracle as orc
    from tests.conftest import GOLDEN
    g = orc.Graph.from_file(os.path.join(GOLDEN, "pl1k.txt"), 1)
    blk_raw = _neg_law_check(g, world, "pl1k")
    assert blk_raw.max() > 1.05 or blk_raw.min() < 0.95    # the uncorrected law is off


def test_block_negative_law_c2():
    """The same on config C2's graph (1M vertices / 40M slots)."""
    from oracle import oracle as orc
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges("c2")
    g = orc.Graph(V, src, dst, w)
    for world in (2, 4, 8):
        _neg_law_check(g, world, "c2")


# ---- the hub slots in BlockSync (dist.py): every cell also trains this
# rank's copy of H hub rows (slots V .. V + H of C), exchanged one late after
# every sub-round with per-slot scales (OverlapSync over the slots, TorchPasses)
HUBS = 3


def _hub_scale():
    return torch.tensor([1.0, 0.75, 0.5])


def _cell_hubs(W, C, wb, cb, r, b, s, q=0):
    """A launch (part q of a cell) that touches W part r, C block b and the hub
    slots (the shape of a LINE-2 cell with hub atoms and hub negatives)."""
    _cell(W, C, wb, cb, r, b, s + 7 * q)
    h = C[V:V + HUBS]
    w = W[wb[r]:wb[r + 1]]
    h.mul_(0.995).add_(torch.tanh(w.mean(0) + h) * (0.01 * (r + 1)) + 0.0005 * (b + s + q))
    w.add_(h.mean(0) * 0.01)


def _reference_hubs(world, subrounds, hub_rows, parts=1):
    """BlockSync with hubs restated in one process: per-rank tables, cells in
    sub-round order, after each sub-round the slots' begin / cycle passes and
    the summed deltas, then the rotation; at the end the last exchange's end,
    the slots into the hub rows and the gather."""
    torch.manual_seed(0)
    W0, C0 = torch.randn(V, D), torch.randn(V, D)
    wb, cb = _bounds(world)
    nb = 2 * world
    Ws = [W0.clone() for _ in range(world)]
    Cs = [torch.cat([C0, C0[hub_rows]]) for _ in range(world)]
    S = [c[V:].clone() for c in Cs]
    Dd = [torch.zeros(HUBS, D) for _ in range(world)]
    R = [torch.zeros(HUBS, D) for _ in range(world)]
    sc = _hub_scale().view(-1, 1)
    pending = False
    for s in range(subrounds):
        for q in range(parts):
            for r in range(world):
                _cell_hubs(Ws[r], Cs[r], wb, cb, r, (2 * r + s) % nb, s, q)
            for r in range(world):
                T = Cs[r][V:]
                if pending:                       # TorchPasses.cycle: end, then begin
                    R[r].mul_(sc).sub_(Dd[r])
                    T.add_(R[r])
                    S[r].add_(R[r])
                torch.sub(T, S[r], out=Dd[r])
                R[r].copy_(Dd[r])
                S[r].copy_(T)
            tot = R[0].clone()
            for r in range(1, world):
                tot += R[r]
            R = [tot.clone() for _ in range(world)]
            pending = True
        moved = [Cs[r][cb[(2 * r + s) % nb]:cb[(2 * r + s) % nb + 1]].clone() for r in range(world)]
        for r in range(world):
            b = (2 * r + s) % nb
            Cs[(r - 1) % world][cb[b]:cb[b + 1]] = moved[r]
    for r in range(world):
        R[r].mul_(sc).sub_(Dd[r])
        Cs[r][V:].add_(R[r])
        Cs[r][hub_rows] = Cs[r][V:].clone()
    W, C = W0.clone(), C0.clone()
    for p in range(world):
        W[wb[p]:wb[p + 1]] = Ws[p][wb[p]:wb[p + 1]]
    for b in range(nb):
        holder = ((b - subrounds) % nb) // 2
        C[cb[b]:cb[b + 1]] = Cs[holder][cb[b]:cb[b + 1]]
    return W, C


def _worker_hubs(rank, world, port, subrounds, out, parts=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smore_amd.dist import BlockSync, TorchPasses
    hub_rows = torch.tensor([5, 17, 40])
    torch.manual_seed(0)
    W, C0 = torch.randn(V, D), torch.randn(V, D)
    C = torch.cat([C0, torch.zeros(HUBS, D)])
    wb, cb = _bounds(world)

    def load():
        C[V:] = C[hub_rows].clone()

    def store():
        C[hub_rows] = C[V:].clone()
    hubs = {"slots": C[V:], "scale": _hub_scale(), "passes": TorchPasses(), "load": load, "store": store}
    bs = BlockSync(W, C[:V], wb, cb, hubs=hubs)
    for _ in range(subrounds):
        s = bs.s
        if parts == 1:
            bs.sub_round(lambda b: _cell_hubs(W, C, wb, cb, rank, b, s))
        else:
            bs.sub_round(lambda b, q: _cell_hubs(W, C, wb, cb, rank, b, s, q), parts)
    bs.finish(gather=True)
    RW, RC = _reference_hubs(world, subrounds, hub_rows, parts)
    exact = world == 2            # sums of 2 are order-free; gloo's ring may add 3+ in another order
    if exact:
        ok = torch.equal(W, RW) and torch.equal(C[:V], RC)
    else:
        ok = torch.allclose(W, RW, atol=1e-5, rtol=1e-5) and torch.allclose(C[:V], RC, atol=1e-5, rtol=1e-5)
    ok = ok and torch.equal(C[hub_rows], C[V:])
    out[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,subrounds,parts", [(2, 4, 1), (2, 9, 4), (3, 7, 1), (4, 8, 4)])
def test_block_rotation_with_hubs_gloo(world, subrounds, parts):
    """BlockSync with hub slots over gloo (cells in 1 or 4 launches, the slots
    exchanged after each) equals its one-process restatement (bit for bit at
    2 ranks), and every rank ends with the hub rows equal to the exchanged
    slots."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_worker_hubs, args=(r, world, port, subrounds, out, parts)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world
