"""The 2-D block schedule of the multi-GPU path (blocks.cpp, train_blocks.hip,
exchange.cpp group_block_*) on one MI355X:
  * a cell's draws are bit-exact against the numpy restatement of its tables
    (tests/block_spec.py: bounds, per-block negative tables, atoms), every
    source in the part, every context and negative in the block;
  * a replica's serial cell training equals the oracle's fp32 update over the
    same records (orc_train_records_f32);
  * a serial block-schedule group of 2 / 3 replicas on cuda:0 equals the
    schedule restated around the oracle (cells in sub-round order, C blocks
    copied to replica r - 1 after each sub-round, W parts / C blocks gathered
    from their owners) bit for bit;
  * walk rounds: the bucketed records of all parts and blocks are exactly the
    one-context pairs (their count), the serial group equals its restatement;
  * quality: C2 LINE-2 and C5 DeepWalk at 2 / 4 / 8 replicas within 5 % of
    one context's held-out loss (VERDICT r4's bar).
"""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from bench import largest_remainder
from tests.block_spec import BlockSpec, part_masses, skewed_graph_lines
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
SEED = 20251015
PL1K = os.path.join(GOLDEN, "pl1k.txt")


@pytest.fixture(scope="module")
def smore():
    import smore_amd
    return smore_amd


@pytest.fixture(scope="module")
def graph():
    return orc.Graph.from_file(PL1K, 1)


def _ctx(smore, dim=32):
    pn = smore.ProNet(0)
    pn.LoadEdgeList(PL1K, 1)
    pn.alloc_tables(dim, 2)
    pn.init_table_glibc(0, 0)
    pn.zero_table(1)
    return pn


@pytest.mark.parametrize("n,hubs", [(2, -1), (3, -1), (4, -1), (2, 0), (4, 0), (3, 100)])
def test_block_draws_match_spec(smore, graph, n, hubs):
    """Bit-exact cell draws against tests/block_spec.py, with the automatic
    hub rows (pl1k: 1000 / 8nb), none, and many."""
    K = 5
    pn = _ctx(smore)
    pn.block_set_hubs(hubs)
    for r in range(n):
        spec = BlockSpec(graph, n, r, K, hubs)
        pn.block_setup("line2", n, r, K, "atomic")
        wb, cb = pn.block_bounds()
        assert list(wb) == spec.wb and list(cb) == spec.cb
        H, first, rows, _ = pn.block_hubs()
        assert H == spec.H and first == graph.V and list(rows) == spec.hubs
        np.testing.assert_allclose(pn.block_mass(), spec.mass, rtol=1e-12, atol=0)
        np.testing.assert_allclose([pn.block_neg_scale(k) for k in range(2 * n)], spec.neg_w, rtol=1e-6)
        assert abs(pn.block_mass().sum() - 1.0) < 1e-12
        for k in range(2 * n):
            if spec.mass[k] == 0:
                continue
            got = pn.block_sample_edges(k, SEED, (1 << 33) + 977 * k, 600, K)
            want = spec.draw(k, SEED, (1 << 33) + 977 * k, 600, K)
            np.testing.assert_array_equal(got, want)
            assert ((got[:, 0] >= wb[r]) & (got[:, 0] < wb[r + 1])).all()
            ctx = got[:, 1:]
            slot = ctx >= graph.V
            assert ((ctx >= cb[k]) & (ctx < cb[k + 1]) | slot & (ctx < graph.V + H)).all()
            assert not np.isin(ctx[~slot], rows).any()     # a hub row is only ever drawn as its slot
            if H:
                assert slot.any()
    pn.close()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_block_part_mass_skewed_graph(smore, tmp_path, n):
    """smore_block_part_mass against the spec on a graph whose parts differ by
    ~13 % of source mass: a group's round split gives each replica
    its part's share, so the union of the parts draws SourceSample's law."""
    f = tmp_path / "skewed.txt"
    f.write_text(skewed_graph_lines())
    want, wb = part_masses(str(f), n, undirected=0)
    pn = smore.ProNet(0)
    pn.LoadEdgeList(str(f), 0)
    pn.alloc_tables(8, 2)
    pn.block_setup("line2", n, n - 1, 5, "atomic")
    assert list(pn.block_bounds()[0]) == wb
    np.testing.assert_allclose(pn.block_part_mass(), want, rtol=1e-12, atol=1e-15)
    assert max(want) > 1.1 / n
    pn.close()


def test_block_counts_largest_remainder(smore):
    pn = _ctx(smore)
    pn.block_setup("line2", 4, 1, 5, "atomic")
    m = pn.block_mass()
    for S in (0, 1, 7, 1000, 123457):
        c = pn.block_counts(S).astype(np.int64)
        assert c.sum() == S
        assert (np.abs(c - S * m) < 1.0 + 1e-9).all()
    pn.close()


def test_block_cell_serial_equals_oracle(smore, graph):
    """One replica's serial cell launches against the oracle's fp32 update
    over the same records, cell after cell."""
    K, dim, total = 5, 32, 10 ** 6
    pn = _ctx(smore, dim)
    W, C = pn.get_table(0), pn.get_table(1)
    pn.block_setup("line2", 3, 2, K, "serial")
    H, V, rows, _ = pn.block_hubs()
    assert H > 0
    pn.block_hubs_load()                 # slots V .. V + H <- the hub rows
    C = np.concatenate([C, C[rows]])     # the oracle's table with the slot rows
    begin = 5000
    for k in (0, 3, 5, 1):
        n = 700
        rec = pn.block_sample_edges(k, SEED, begin, n, K)
        pn.block_train_edges(k, begin, n, total, K, 0.025, SEED, "serial")
        w = pn.block_neg_scale(k)
        assert w != 1.0          # the epoch negative-law weight is on (SMORE_NEG_LAW default)
        orc.train_records_f32("line2", W, C, rec, K, 0.025, 0.0, total, begin, w)
        begin += n
    assert (C[V:] != C[rows]).any()      # the slots trained, the hub rows did not
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C[:V])
    pn.block_hubs_store()                # hub rows <- slots
    C[rows] = C[V:]
    np.testing.assert_array_equal(pn.get_table(1), C[:V])
    pn.close()


def _hub_exchange(n, V, Cs, Ss, Ds, Rs, sc, pending):
    """The hub slots' one-late exchange after a launch of every replica
    (replica_sync.hip begin / cycle passes in fp32, the all-reduce summing the
    replicas in order); returns the new pending state."""
    for r in range(n):
        T = Cs[r][V:]
        if pending:
            X = sc * Rs[r] - Ds[r]
            tn, sn = T + X, Ss[r] + X
            Ds[r] = tn - sn
            T[:] = tn
            Ss[r] = tn.copy()
        else:
            Ds[r] = T - Ss[r]
            Ss[r] = T.copy()
        Rs[r] = Ds[r].copy()
    tot = Rs[0].copy()
    for r in range(1, n):
        tot = tot + Rs[r]
    for r in range(n):
        Rs[r] = tot.copy()
    return True


def _schedule_edges(smore, graph, n, begin, count, per, total, K, dim, W0, C0, hubs=-1):
    """exchange.cpp group_block_edges restated: rounds of per * n samples
    split over the replicas by their parts' source mass (largest remainder),
    replica r's slice split over the blocks by its mass, sub-round s trains
    cell (r, (2r + s) mod 2n) on replica r's tables and its own copy of the
    hub slots (rows V .. V + H), then the slots' one-late exchange (begin /
    cycle with the per-slot scales, the all-reduce summing the replicas in
    order) and C block (2r + s) mod 2n moves to replica r - 1; at the end the
    last exchange's end, the slots back into the hub rows, W part p from
    replica p, C block b from b // 2."""
    nb = 2 * n
    ctxs, specs = [], []
    for r in range(n):
        p = smore.ProNet(0)
        p.LoadEdgeList(PL1K, 1)
        p.alloc_tables(dim, 2)
        p.block_set_hubs(hubs)
        p.block_setup("line2", n, r, K, "serial")
        ctxs.append(p)
    H, V, hub_rows, _ = ctxs[0].block_hubs()
    L = ctxs[0].block_cell_launches()          # a cell in L launches, the slots exchanged after each
    assert L == (4 if H else 1)
    sc = ctxs[0].block_hub_scales(min(per, count // n) / nb / L, 2048.0)[:, None] if H else None
    Ws = [W0.copy() for _ in range(n)]
    Cs = [np.concatenate([C0, C0[hub_rows]]) for _ in range(n)]
    Ss = [c[V:].copy() for c in Cs]
    Ds = [np.zeros_like(x) for x in Ss]
    Rs = [np.zeros_like(x) for x in Ss]
    pending = False
    wb, cb = ctxs[0].block_bounds()
    rounds = -(-count // (per * n)) if per * n < count else 1
    for k in range(rounds):
        lo, hi = count * k // rounds, count * (k + 1) // rounds
        m = hi - lo
        share = largest_remainder(m, ctxs[0].block_part_mass())
        cur = [lo + sum(share[:r]) for r in range(n)]
        cnt = [ctxs[r].block_counts(share[r]) for r in range(n)]
        for s in range(nb):
            for q in range(L):
                for r in range(n):
                    b = (2 * r + s) % nb
                    x0, x1 = int(cnt[r][b]) * q // L, int(cnt[r][b]) * (q + 1) // L
                    if x1 > x0:
                        rec = ctxs[r].block_sample_edges(b, SEED, begin + cur[r] + x0, x1 - x0, K)
                        orc.train_records_f32("line2", Ws[r], Cs[r], rec, K, 0.025, 0.0, total,
                                              begin + cur[r] + x0, ctxs[r].block_neg_scale(b))
                if H:
                    pending = _hub_exchange(n, V, Cs, Ss, Ds, Rs, sc, pending)
            for r in range(n):
                cur[r] += int(cnt[r][(2 * r + s) % nb])
            moved = [Cs[r][cb[(2 * r + s) % nb]:cb[(2 * r + s) % nb + 1]].copy() for r in range(n)]
            for r in range(n):
                b = (2 * r + s) % nb
                Cs[(r - 1) % n][cb[b]:cb[b + 1]] = moved[r]
    if H:
        for r in range(n):
            if pending:
                X = sc * Rs[r] - Ds[r]
                Cs[r][V:] += X
            Cs[r][hub_rows] = Cs[r][V:]
    W, C = W0.copy(), C0.copy()
    for p in range(n):
        W[wb[p]:wb[p + 1]] = Ws[p][wb[p]:wb[p + 1]]
    for b in range(nb):
        C[cb[b]:cb[b + 1]] = Cs[b // 2][cb[b]:cb[b + 1]]
    for p in ctxs:
        p.close()
    return W, C


@pytest.mark.parametrize("n,hubs", [(2, -1), (3, -1), (2, 0), (3, 0)])
def test_block_group_serial_equals_schedule(smore, graph, n, hubs):
    K, dim, total = 5, 32, 10 ** 6
    g = smore.Group([0] * n)
    for r in g.replicas:
        r.block_set_hubs(hubs)
    g.LoadEdgeList(PL1K, 1)
    g.alloc_tables(dim, 2)
    g.primary.init_table_glibc(0, 0)
    g.primary.init_table_glibc(1, graph.V * dim)
    g.broadcast_tables()
    W0, C0 = g.primary.get_table(0), g.primary.get_table(1)
    g.set_schedule("blocks")
    begin, count, per = 1000, 9000, 1500
    g.train_edges("line2", begin, count, total, K, 0.025, 0.0, SEED, "serial", per=per)
    W, C = _schedule_edges(smore, graph, n, begin, count, per, total, K, dim, W0, C0, hubs)
    for r in g.replicas:
        np.testing.assert_array_equal(r.get_table(0), W)
        np.testing.assert_array_equal(r.get_table(1), C)
    g.close()


def test_block_walk_rounds_cover_the_pairs(smore, graph):
    """Every part's pair records, over all blocks, are the one-context
    records: for DeepWalk the per-walk pair counts of the oracle's SkipGrams
    (the window draws are shared), for Walklets the clamped ranges."""
    K = 5
    V = graph.V
    order = orc.deepwalk_order(V, 2, 0)
    one = _ctx(smore)
    one.census_begin()
    one.train_deepwalk(0, 700, 2, 20, 4, K, 0.025, SEED, order, "atomic")
    one.census_end(1.0)
    total_pairs = int(round(one.row_rates("census", K, 0).sum()))
    one.close()
    for n in (2, 4):
        got = 0
        for r in range(n):
            pn = _ctx(smore)
            pn.block_setup("census", n, r, K, "atomic")
            pn.block_prepare_walks(0, 700, 2, 20, 4, K, 0.025, SEED, order, "atomic")
            got += sum(pn.block_walk_records(b) for b in range(2 * n))
            pn.close()
        assert got == total_pairs, (n, got, total_pairs)


@pytest.mark.parametrize("n,rule,steps,window,K", [(2, "deepwalk", 20, 4, 5), (3, "deepwalk", 100, 10, 5),
                                                   (4, "walklets", 90, 6, 10), (8, "deepwalk", 40, 5, 5)])
def test_block_walk_records_wave_kernels(smore, graph, monkeypatch, n, rule, steps, window, K):
    """The wave-per-walk count / emit kernels (train_blocks.hip
    block_pairs_wave_kernel: lane = position, the pair counts scanned across
    the wave for the negatives' Philox words and per block for the records'
    places) write the per-walk kernels' records bit for bit: every bucket of
    every part, hybrid tags, hub slots (3 and 8 parts), walks longer than a
    wave (101 and 91 positions), Walklets' two ranges and K = 10."""
    order = orc.deepwalk_order(graph.V, 2, 0)
    total = 0
    for r in range(n):
        recs = []
        for kernels in ("walk", "wave"):
            monkeypatch.setenv("SMORE_WALK_PAIR_KERNELS", kernels)
            pn = _ctx(smore)
            pn.block_setup("census", n, r, K, "hybrid")
            pn.block_prepare_walks(0, 900, 2, steps, window, K, 0.025, SEED, order, "hybrid", rule=rule,
                                   window_min=2 if rule == "walklets" else 0)
            recs.append([pn.block_walk_records_copy(b) for b in range(2 * n)])
            pn.close()
        for b, (x, y) in enumerate(zip(*recs)):
            np.testing.assert_array_equal(x, y, err_msg=f"part {r} block {b}")
            total += len(x)
    assert total > 0


def test_block_group_walks_serial_replicas_agree(smore, graph):
    """A serial DeepWalk block group of 3: every replica ends with the same
    tables (gathered), they moved, and two identical runs agree bit for bit
    (cells of one sub-round touch disjoint rows: the schedule is
    deterministic)."""
    K, dim = 5, 32
    order = orc.deepwalk_order(graph.V, 2, 0)
    out = []
    for _ in range(2):
        g = smore.Group([0] * 3)
        g.LoadEdgeList(PL1K, 1)
        g.alloc_tables(dim, 2)
        g.primary.init_table_glibc(0, 0)
        g.primary.zero_table(1)
        g.broadcast_tables()
        W0 = g.primary.get_table(0)
        g.set_schedule("blocks")
        g.train_deepwalk(0, 2 * graph.V, 2, 20, 4, K, 0.025, SEED, order, "serial", per=500)
        W, C = g.primary.get_table(0), g.primary.get_table(1)
        for r in g.replicas[1:]:
            np.testing.assert_array_equal(r.get_table(0), W)
            np.testing.assert_array_equal(r.get_table(1), C)
        assert np.abs(W - W0).max() > 0 and np.abs(C).max() > 0
        out.append((W, C))
        g.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


def _heldout_loss(W, C, draws):
    v, c, negs = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = c >= 0
    v, c, negs = v[keep], c[keep], negs[keep]
    Wv = W[v].astype(np.float64)
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k]].astype(np.float64)))
    return float(loss.mean())


@pytest.mark.parametrize("mode", ["atomic", "hybrid"])
def test_block_walks_parallel_modes_train(smore, graph, mode):
    """DeepWalk in the block schedule on 2 and 4 replicas (cuda:0) in the
    Hogwild modes: every replica holds the gathered tables, they stay finite,
    and the held-out LINE objective is within 10 % of one context's."""
    K, dim, wt = 5, 32, 6
    order = orc.deepwalk_order(graph.V, wt, 0)
    held = orc.sample_line(graph, SEED + 7, 0, 50_000, 5)
    one = _ctx(smore, dim)
    one.train_deepwalk(0, wt * graph.V, wt, 20, 4, K, 0.025, SEED, order, mode)
    l1 = _heldout_loss(one.get_table(0), one.get_table(1), held)
    one.close()
    for n in (2, 4):
        g = smore.Group([0] * n)
        g.LoadEdgeList(PL1K, 1)
        g.alloc_tables(dim, 2)
        g.primary.init_table_glibc(0, 0)
        g.primary.zero_table(1)
        g.broadcast_tables()
        g.set_schedule("blocks")
        g.train_deepwalk(0, wt * graph.V, wt, 20, 4, K, 0.025, SEED, order, mode, per=1000)
        W, C = g.primary.get_table(0), g.primary.get_table(1)
        for r in g.replicas[1:]:
            np.testing.assert_array_equal(r.get_table(0), W)
            np.testing.assert_array_equal(r.get_table(1), C)
        g.close()
        ln = _heldout_loss(W, C, held)
        print("pl1k DeepWalk blocks", mode, n, ln, "one", l1, flush=True)
        assert np.isfinite(W).all() and np.isfinite(C).all() and ln <= 1.10 * l1, (n, ln, l1)


def test_block_group_walks_partitioned_generation(smore, graph, monkeypatch):
    """Walk-partitioned generation: each replica walks
    1/N of a round and the slices are broadcast from their walkers before the
    pairs are bucketed.  Walks are deterministic per walk index, so a serial
    group of 3 and of 4 ends bit-identical to every replica walking every walk
    (SMORE_WALK_GEN_ALL=1, round 5)."""
    K, dim = 5, 32
    order = orc.deepwalk_order(graph.V, 2, 0)
    for n in (3, 4):
        out = []
        for gen_all in ("1", "0"):
            monkeypatch.setenv("SMORE_WALK_GEN_ALL", gen_all)
            g = smore.Group([0] * n)
            g.LoadEdgeList(PL1K, 1)
            g.alloc_tables(dim, 2)
            g.primary.init_table_glibc(0, 0)
            g.primary.zero_table(1)
            g.broadcast_tables()
            g.set_schedule("blocks")
            g.train_deepwalk(0, 2 * graph.V, 2, 20, 4, K, 0.025, SEED, order, "serial", per=500)
            out.append((g.primary.get_table(0), g.primary.get_table(1)))
            g.close()
        np.testing.assert_array_equal(out[0][0], out[1][0])
        np.testing.assert_array_equal(out[0][1], out[1][1])
