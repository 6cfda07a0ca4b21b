"""Parity at the benchmark configurations' sizes and shapes:
C2 (LINE-2, 1M vertices / 20M lines; also Walklets, APP, HPE on that graph), C3 (BPR, 2M x 1M / 100M edges, d=128),
C5 (DeepWalk d=128, 40 steps, window 5, K=5), the full-grid default hybrid
scatter, the replica-exchange kernels with R != D, and DeepWalk context-buffer
reuse.  Needs an MI355X.

Tolerances:
  * draws, serial mode vs the oracle's fp32 spec      : bit-exact
  * d=128 DeepWalk end to end vs the reference (fp64) : 2e-3 max / 2e-4 median abs
  * exchange kernels vs numpy float32 (same op order) : bit-exact
  * hybrid scatter vs atomic (held-out LINE-2 loss)   : within 1 % relative
The big graphs are generated natively (smore_gen_powerlaw) and the SAME edge
arrays are handed to the oracle's graph builder.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests.test_gpu_parity import SEED, gold, make_pair, padded, rand_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def smore():
    import smore_amd
    return smore_amd


def _config_pair(smore, name, vm="out_degrees", nm="degrees"):
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges(name)
    g = orc.Graph(V, src, dst, w, vm, nm)
    pn = smore.ProNet(0)
    pn.SetVertexMethod(vm)
    pn.SetNegativeMethod(nm)
    pn.set_graph_edges(V, src, dst, w)
    return g, pn


@pytest.fixture(scope="module")
def c2(smore):
    return _config_pair(smore, "c2")


def _heldout_loss(W, C, draws, dim):
    """LINE-2 objective on held-out draws: -log s(W_v.C_c) - sum_k log s(-W_v.C_nk)."""
    v, c, negs = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = c >= 0
    v, c, negs = v[keep], c[keep], negs[keep]
    Wv = W[v, :dim].astype(np.float64)
    pos = np.einsum("ij,ij->i", Wv, C[c, :dim].astype(np.float64))
    loss = np.logaddexp(0.0, -pos)
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k], :dim].astype(np.float64)))
    return float(loss.mean())


# ---------------------------------------------------------------- C2 / C3 at full size
def test_c2_draws_bit_exact(c2):
    g, pn = c2
    assert g.V == 1_000_000 and g.E == 40_000_000
    for begin in (0, (1 << 33) + 12345):
        np.testing.assert_array_equal(pn.sample_edges("line2", begin, 100_000, 5, SEED),
                                      orc.sample_line(g, SEED, begin, 100_000, 5))


def test_c2_serial_bit_exact(c2):
    g, pn = c2
    dim, K, total = 64, 5, 20 * 10 ** 9
    W0, C0 = rand_tables(g.V, dim, 2, 31)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    begin = 7 * 10 ** 9 + 3
    pn.train_edges("line2", begin, 20_000, total, K, 0.025, 0.0, SEED, "serial")
    orc.train_edge_f32(g, "line2", W0, C0, dim, K, 0.025, 0.0, total, begin, begin + 20_000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W0)
    np.testing.assert_array_equal(pn.get_table(1), C0)


def test_c2_walklets_app_hpe_serial_bit_exact(c2):
    """The other UpdatePair consumers (Walklets, APP, HPE) on the C2 graph
    (1M vertices / 40M slots, d=64, K=5): serial mode bit-exact vs the oracle's
    fp32 spec over ranges far from the start."""
    import smore_amd
    g, pn = c2
    dim, K = 64, 5
    W0, C0 = rand_tables(g.V, dim, 2, 77)
    # Walklets: walks [500_000, 501_000) of walk_times 2, 40 steps, windows 1..5
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    W, C = W0.copy(), C0.copy()
    pn.train_walklets(500_000, 501_000, 2, 40, 1, 5, K, 0.025, SEED, "serial")
    orc.train_walklets_f32(g, W, C, dim, 2, 40, 1, 5, K, 0.025, SEED, 500_000, 501_000)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)
    # APP: units [3_000_000, 3_005_000) of walk_times 1, 10 samples per start
    order = smore_amd.deepwalk_order(g.V, 1, 2 * g.V * dim)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    W, C = W0.copy(), C0.copy()
    pn.train_app(3_000_000, 3_005_000, 1, 10, 0.15, K, 0.025, SEED, order, "serial")
    orc.train_app_f32(g, W, C, dim, 1, 10, 0.15, K, 0.025, SEED, order, 3_000_000, 3_005_000)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)
    # HPE: samples [10^9, 10^9 + 5000) of 2 * 10^9, walk_steps 5
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    W, C = W0.copy(), C0.copy()
    total = 2 * 10 ** 9
    pn.train_hpe(10 ** 9, 5000, total, 5, K, 0.01, 0.025, SEED, "serial")
    orc.train_hpe_f32(g, W, C, dim, 5, K, 0.01, 0.025, total, 10 ** 9, 10 ** 9 + 5000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)


def test_c2_full_grid_hybrid_matches_atomic(c2):
    """The bench's default scatter on a full grid (no V/16 cap at V=1M): 2^28
    samples, hybrid (the defaults: tau 1.0, 128 LDS write-combined rows,
    automatic drain) vs the lossless atomic scatter, held-out LINE-2 loss
    within 1.5 % (measured 0.9 %; tau 0.3: 0.7 %, profiles/r03/tau)."""
    g, pn = c2
    dim, K, total = 64, 5, 1 << 28
    heldout = orc.sample_line(g, SEED + 1, 0, 100_000, K)
    res = {}
    for mode in ("atomic", "hybrid"):
        pn.alloc_tables(dim, 2)
        pn.init_table_uniform(0, 5)
        pn.zero_table(1)
        pn.set_hot_threshold(1.0)
        pn.set_write_combine(128, 0)     # the defaults: 128 rows, automatic drain interval
        pn.train_edges("line2", 0, total, total, K, 0.025, 0.0, SEED, mode)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[mode] = _heldout_loss(W, C, heldout, dim)
        if mode == "hybrid":
            hw, hc = pn.hot_rows()
            assert hw > 0 and hc > 0, (hw, hc)
    init = np.log(2.0) * (1 + K)          # C = 0: every logit is 0
    assert res["atomic"] < 0.9 * init, res
    assert abs(res["hybrid"] - res["atomic"]) <= 0.015 * res["atomic"], res


# ---------------------------------------------------------------- C4: the north-star graph
# 10M vertices / 200M undirected lines = 400M directed slots: E above 2^28, the
# 6.4-GB packed context table (ct16, u32 offsets), 33-bit sample indices and
# the hybrid scatter's hot tags at V = 10M (src/model/LINE.cpp:160-191).  The
# oracle graph build is the slow part (about a minute), so one fixture serves
# every C4 test.
@pytest.fixture(scope="module")
def c4(smore):
    return _config_pair(smore, "c4")


@pytest.mark.timeout(600)
def test_c4_draws_bit_exact(c4):
    g, pn = c4
    assert g.V == 10_000_000 and g.E == 400_000_000
    for begin in (0, (1 << 33) + 4321):
        np.testing.assert_array_equal(pn.sample_edges("line2", begin, 100_000, 5, SEED),
                                      orc.sample_line(g, SEED, begin, 100_000, 5))


@pytest.mark.timeout(600)
def test_c4_serial_bit_exact(c4):
    g, pn = c4
    dim, K, total = 64, 5, 40 * 10 ** 9
    W0, C0 = rand_tables(g.V, dim, 2, 44)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    begin = (1 << 34) + 77
    pn.train_edges("line2", begin, 20_000, total, K, 0.025, 0.0, SEED, "serial")
    orc.train_edge_f32(g, "line2", W0, C0, dim, K, 0.025, 0.0, total, begin, begin + 20_000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W0)
    np.testing.assert_array_equal(pn.get_table(1), C0)


@pytest.mark.timeout(600)
def test_c4_full_grid_hybrid_matches_atomic(c4):
    """The bench's workload and default scatter: full-grid hybrid launches of
    2^27 samples are finite and tag hot rows at V = 10M; after 2^31 samples
    (~215 per vertex) the held-out LINE-2 loss of the hybrid scatter is within
    1 % of the lossless atomic scatter's (measured with the default tau 1.0:
    2.5585 vs 2.5509, 0.3 %; tau 0.3: 0.2 %, profiles/r03/tau)."""
    g, pn = c4
    dim, K, launch, total = 64, 5, 1 << 27, 1 << 31
    heldout = orc.sample_line(g, SEED + 1, 0, 100_000, K)
    res = {}
    for mode in ("atomic", "hybrid"):
        pn.alloc_tables(dim, 2)
        pn.init_table_uniform(0, 5)
        pn.zero_table(1)
        pn.set_hot_threshold(1.0)
        pn.set_write_combine(128, 0)
        for b in range(0, total, launch):
            pn.train_edges("line2", b, launch, total, K, 0.025, 0.0, SEED, mode)
            if mode == "hybrid" and b == 0:
                assert np.isfinite(pn.get_table(0)).all()
                hw, hc = pn.hot_rows()
                assert hw > 0 and hc > 0, (hw, hc)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[mode] = _heldout_loss(W, C, heldout, dim)
        del W, C
    assert pn.skipped() == 0
    init = np.log(2.0) * (1 + K)
    assert res["atomic"] < 0.9 * init, res
    assert res["hybrid"] <= 1.01 * res["atomic"], res


@pytest.fixture(scope="module")
def c3(smore):
    return _config_pair(smore, "c3", nm="no_degrees")


def test_c3_draws_bit_exact(c3):
    g, pn = c3
    assert g.V == 3_000_000 and g.E == 100_000_000
    for begin in (0, (1 << 34) + 99):
        np.testing.assert_array_equal(pn.sample_edges("bpr", begin, 100_000, 5, SEED),
                                      orc.sample_bpr(g, SEED, begin, 100_000))


def test_c3_bpr_serial_bit_exact(c3):
    g, pn = c3
    dim, total = 128, 5 * 10 ** 8
    (W0,) = rand_tables(g.V, dim, 1, 41)
    pn.alloc_tables(dim, 1)
    pn.set_table(0, W0)
    begin = 123_456_789
    pn.train_edges("bpr", begin, 20_000, total, 5, 0.025, 0.0, SEED, "serial")
    orc.train_bpr_f32(g, W0, dim, 0.025, total, begin, begin + 20_000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W0)


def _bpr_objective(W, draws, dim):
    """BPR objective on held-out draws {u, i, j0..j4} (UpdateBPRPair's rounds,
    src/proNet.cpp:1406-1455): mean over rounds of -log s(W_u.(W_i - W_j)),
    and the fraction of rounds ranking i above j."""
    u, i, js = draws[:, 0], draws[:, 1], draws[:, 2:]
    keep = i >= 0
    u, i, js = u[keep], i[keep], js[keep]
    Wu = W[u, :dim].astype(np.float64)
    Wi = W[i, :dim].astype(np.float64)
    loss = np.zeros(len(u))
    hit = np.zeros(len(u))
    for k in range(js.shape[1]):
        x = np.einsum("ij,ij->i", Wu, Wi - W[js[:, k], :dim].astype(np.float64))
        loss += np.logaddexp(0.0, -x)
        hit += x > 0
    return float(loss.mean() / js.shape[1]), float(hit.mean() / js.shape[1])


def test_c3_full_grid_hybrid_matches_atomic(c3):
    """C3 BPR asked for the hybrid scatter on the full grid (d=128, 2^28
    samples) vs the lossless atomic scatter.  Above the small-graph cap, C++
    BPR's "hybrid" runs the PLAIN-STORE kernel (capi.cpp: its ~170 hot rows are
    hub items drawn as positives; smore_last_mode says "hogwild"), so this
    pins the plain stores' loss: held-out BPR objective within 1 % and the
    held-out ranking accuracy within 0.5 points (VERDICT r3 weak 5, r5 weak 6;
    measured in DESIGN.md 8)."""
    g, pn = c3
    dim, total = 128, 1 << 28
    held = orc.sample_bpr(g, SEED + 1, 0, 100_000)
    res = {}
    for mode in ("atomic", "hybrid"):
        pn.alloc_tables(dim, 1)
        pn.init_table_uniform(0, 7)
        pn.train_edges("bpr", 0, total, total, 5, 0.025, 0.0, SEED, mode)
        assert pn.last_mode() == {"atomic": "atomic", "hybrid": "hogwild"}[mode]
        W = pn.get_table(0)
        assert np.isfinite(W).all()
        res[mode] = _bpr_objective(W, held, dim)
        del W
    print("C3 BPR held-out (loss, rank acc):", res)
    assert res["atomic"][0] < 0.95 * np.log(2.0), res        # trained away from the initial log 2
    assert res["hybrid"][0] <= 1.01 * res["atomic"][0], res
    assert res["hybrid"][1] >= res["atomic"][1] - 0.005, res


def test_bpr_small_parallel_modes_vs_serial(smore):
    """On the golden bipartite graph (300 vertices: the V/16 concurrency cap
    applies) the atomic and hybrid BPR scatters train like the serial order:
    held-out BPR objective within 2 % after 2 x 10^6 samples."""
    import os
    from tests.conftest import GOLDEN
    path = os.path.join(GOLDEN, "bip.txt")
    g = orc.Graph.from_file(path, 0, "out_degrees", "no_degrees")
    held = orc.sample_bpr(g, SEED + 1, 0, 50_000)
    dim, total = 32, 2 * 10 ** 6
    res = {}
    for mode in ("serial", "atomic", "hybrid"):
        pn = smore.ProNet(0)
        pn.SetNegativeMethod("no_degrees")
        pn.LoadEdgeList(path, 0)
        pn.alloc_tables(dim, 1)
        pn.init_table_uniform(0, 7)
        pn.train_edges("bpr", 0, total, total, 5, 0.025, 0.0, SEED, mode)
        res[mode] = _bpr_objective(pn.get_table(0), held, dim)
    assert res["serial"][0] < 0.95 * np.log(2.0), res
    for mode in ("atomic", "hybrid"):
        assert res[mode][0] <= 1.02 * res["serial"][0], res


# ---------------------------------------------------------------- C5 shape: DeepWalk d=128
def test_c5_deepwalk_serial_bit_exact(smore):
    """Config 5's model on config 5's stand-in graph (1.13M vertices / 3M
    lines): d=128, walk_steps 40, window 5, K 5, a range of 300 walks of the
    fourth walk_time, serial mode vs the oracle's fp32 spec."""
    g, pn = _config_pair(smore, "c5")
    dim, K, window, steps, times = 128, 5, 5, 40, 10
    W0, C0 = rand_tables(g.V, dim, 2, 51)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = smore.deepwalk_order(g.V, times, 2 * g.V * dim)
    b = 3 * g.V + 17
    pn.train_deepwalk(b, b + 300, times, steps, window, K, 0.025, SEED, order, "serial")
    orc.train_deepwalk_f32(g, W0, C0, dim, times, steps, window, K, 0.025, SEED, order, b, b + 300)
    np.testing.assert_array_equal(pn.get_table(0), W0)
    np.testing.assert_array_equal(pn.get_table(1), C0)


def test_deepwalk_d128_serial_bit_exact_small(smore):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    dim, K, window, steps = 128, 5, 5, 40
    W0, C0 = rand_tables(g.V, dim, 2, 52)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 2, 5)
    pn.train_deepwalk(0, 2 * g.V, 2, steps, window, K, 0.025, SEED, order, "serial")
    orc.train_deepwalk_f32(g, W0, C0, dim, 2, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W0)
    np.testing.assert_array_equal(pn.get_table(1), C0)


def test_deepwalk_d128_end_to_end_vs_reference(smore):
    """DeepWalk::Train of the compiled reference at config 5's model shape
    (d=128, 40 steps, window 5, K 5; src/model/DeepWalk.cpp:98-155)."""
    z = gold("e2e_deepwalk_d128_pl100w")
    _, pn = make_pair(smore, "pl100w.txt", 1)
    V, dim = z["W0"].shape
    pn.alloc_tables(dim, 2)
    pn.init_table_glibc(0, 0)
    pn.init_table_glibc(1, V * dim)
    np.testing.assert_array_equal(pn.get_table(0), z["W0"].astype(np.float32))
    order = smore.deepwalk_order(V, 1, 2 * V * dim)
    pn.train_deepwalk(0, V, 1, 40, 5, 5, 0.025, SEED, order, "serial")
    for t, key in ((0, "W"), (1, "C")):
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 2e-3 and np.median(d) < 2e-4, (key, d.max(), np.median(d))


# ---------------------------------------------------------------- DeepWalk buffer reuse
def test_deepwalk_buffers_reused_across_shapes(smore):
    """One context, two calls: few walks with many steps, then more walks
    with few steps (the walk-length buffer must grow with the walk count,
    not with walks x steps), then a third call whose start order array is
    a different array with new contents: every call serial bit-exact."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    dim, K = 16, 3
    W0, C0 = rand_tables(g.V, dim, 2, 61)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    W, C = padded(W0, dim), padded(C0, dim)
    times = 3
    order = orc.deepwalk_order(g.V, times, 0)
    calls = [(10, 20, 80, 2), (100, 300, 3, 2), (300, 800, 6, 3)]
    for i, (b, e, steps, window) in enumerate(calls):
        o = order if i < 2 else np.ascontiguousarray(order[::-1])
        pn.train_deepwalk(b, e, times, steps, window, K, 0.025, SEED, o, "serial")
        orc.train_deepwalk_f32(g, W, C, dim, times, steps, window, K, 0.025, SEED, o, b, e)
        np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
        np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_deepwalk_hybrid_mixed_tags_matches_atomic(smore):
    """Hybrid DeepWalk with a threshold that leaves some rows hot as W rows
    and cold as C rows (and the reverse): every pair's W row carries the W
    tag and its C row the C tag, so no update is dropped; training quality
    (held-out skip-gram AUC) matches the atomic scatter."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    dim, K, times = 32, 5, 4
    order = smore.deepwalk_order(g.V, times, 0)
    rng = np.random.default_rng(3)
    src = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, 20000)
    negv, negc = rng.integers(0, g.V, 2000), rng.integers(0, g.V, 2000)

    def auc(W, C):
        pos = np.einsum("ij,ij->i", W[src[pick]], C[g.targets[pick]])
        neg = np.einsum("ij,ij->i", W[negv], C[negc])
        return (pos[:, None] > neg[None, :]).mean()

    res = {}
    for mode in ("atomic", "hybrid"):
        pn.alloc_tables(dim, 2)
        pn.init_table_glibc(0, 0)
        pn.zero_table(1)
        pn.set_hot_threshold(0.3)      # ~19 hot W rows, ~400 hot C rows of 920
        pn.train_deepwalk(0, times * g.V, times, 20, 5, K, 0.025, SEED, order, mode)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[mode] = auc(W, C)
        if mode == "hybrid":
            hw, hc = pn.hot_rows()
            assert 0 < hw < g.V and 0 < hc < g.V and hw != hc, (hw, hc)
    assert res["atomic"] > 0.7, res
    assert abs(res["hybrid"] - res["atomic"]) < 0.02, res


# ---------------------------------------------------------------- replica exchange kernels
@pytest.mark.parametrize("scale", [1.0, 0.125])
def test_exchange_kernels_r_ne_d(smore, scale):
    """delta_begin / delta_end / delta_cycle (replica_sync.hip) on device
    buffers with R != D (what a world-size > 1 all-reduce leaves), bit for
    bit against numpy float32 in the kernels' operation order."""
    import torch
    _, pn = make_pair(smore, "toy.txt", 1)
    n = 4 * 40_001
    rng = np.random.default_rng(int(scale * 8))
    T, S, D, R = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in range(4)]
    dev = [torch.from_numpy(x.copy()).cuda() for x in (T, S, D, R)]
    p = [t.data_ptr() for t in dev]
    sc = np.float32(scale)

    def host():
        return [t.cpu().numpy() for t in dev]

    # begin: D = T - S; R = D; S = T
    pn.delta_begin(*p, n)
    torch.cuda.synchronize()
    D1 = T - S
    t, s, d, r = host()
    np.testing.assert_array_equal(d, D1)
    np.testing.assert_array_equal(r, D1)
    np.testing.assert_array_equal(s, T)
    np.testing.assert_array_equal(t, T)
    # what the other ranks' deltas add: R != D
    R2 = (D1 + (rng.standard_normal(n) * 0.05).astype(np.float32)).astype(np.float32)
    dev[3].copy_(torch.from_numpy(R2))
    T2 = (T + (rng.standard_normal(n) * 0.01).astype(np.float32)).astype(np.float32)   # training since begin
    dev[0].copy_(torch.from_numpy(T2))
    # end: X = scale*R - D; T += X; S += X
    pn.delta_end(*p, float(scale), n)
    torch.cuda.synchronize()
    X = sc * R2 - D1
    T3, S3 = T2 + X, T + X
    t, s, d, r = host()
    np.testing.assert_array_equal(t, T3)
    np.testing.assert_array_equal(s, S3)
    np.testing.assert_array_equal(d, D1)
    # cycle = end of one exchange fused with the next begin
    R4 = (rng.standard_normal(n) * 0.05).astype(np.float32)
    dev[3].copy_(torch.from_numpy(R4))
    pn.delta_cycle(*p, float(scale), n)
    torch.cuda.synchronize()
    X = sc * R4 - D1
    Tn, Sn = T3 + X, S3 + X
    Dn = Tn - Sn
    t, s, d, r = host()
    np.testing.assert_array_equal(t, Tn)
    np.testing.assert_array_equal(s, Tn)
    np.testing.assert_array_equal(d, Dn)
    np.testing.assert_array_equal(r, Dn)


@pytest.mark.parametrize("stride", [4, 64])
def test_exchange_row_kernels_r_ne_d(smore, stride):
    """delta_end_rows / delta_cycle_rows (the adaptive rule's per-row scale,
    replica_sync.hip) with R != D, bit for bit against numpy float32: row i of
    `stride` floats uses scale[i]."""
    import torch
    _, pn = make_pair(smore, "toy.txt", 1)
    rows = 20_003
    n = rows * stride
    rng = np.random.default_rng(stride)
    T, S, D, R = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in range(4)]
    sc = (0.125 + 0.875 * rng.random(rows)).astype(np.float32)
    dev = [torch.from_numpy(x.copy()).cuda() for x in (T, S, D, R)]
    dsc = torch.from_numpy(sc).cuda()
    p = [t.data_ptr() for t in dev]
    scn = np.repeat(sc, stride)

    def host():
        return [t.cpu().numpy() for t in dev]

    # end: X = scale[row]*R - D; T += X; S += X
    pn.delta_end_rows(*p, dsc.data_ptr(), rows, stride)
    torch.cuda.synchronize()
    X = scn * R - D
    T1, S1 = T + X, S + X
    t, s, d, r = host()
    np.testing.assert_array_equal(t, T1)
    np.testing.assert_array_equal(s, S1)
    np.testing.assert_array_equal(d, D)
    np.testing.assert_array_equal(r, R)
    # cycle: the end fused with the next begin
    R2 = (rng.standard_normal(n) * 0.05).astype(np.float32)
    dev[3].copy_(torch.from_numpy(R2))
    pn.delta_cycle_rows(*p, dsc.data_ptr(), rows, stride)
    torch.cuda.synchronize()
    X = scn * R2 - D
    Tn, Sn = T1 + X, S1 + X
    Dn = Tn - Sn
    t, s, d, r = host()
    np.testing.assert_array_equal(t, Tn)
    np.testing.assert_array_equal(s, Tn)
    np.testing.assert_array_equal(d, Dn)
    np.testing.assert_array_equal(r, Dn)
    with pytest.raises(Exception):
        pn.delta_end_rows(*p, dsc.data_ptr(), rows, 6)    # stride % 4 != 0
