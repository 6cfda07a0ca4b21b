"""Go-semantics mode (pkg/pronet + internal/models
rules) of the HIP path against the oracle's orc_go_* functions, themselves
pinned against an independent restatement of the Go source
(tests/test_go_semantics.py).  Needs an MI355X.

Tolerances: draws and serial mode bit-exact; one atomic sample 1e-6; a
serial run vs the fp64 oracle 2e-3 max / 2e-4 median (as the C++ path)."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEED = 777001


@pytest.fixture(scope="module")
def smore():
    import smore_amd
    return smore_amd


def pair(smore, fname, und):
    path = os.path.join(GOLDEN, fname)
    g = orc.GoGraph.from_file(path, und)
    pn = smore.ProNet(0)
    pn.LoadEdgeList(path, und)
    pn.set_semantics("go")
    return g, pn


def tables(V, dim, seed):
    rng = np.random.default_rng(seed)
    return [(rng.random((V, dim), dtype=np.float32) - 0.5) for _ in range(2)]


def padded(T, dim):
    out = np.zeros((T.shape[0], (dim + 3) // 4 * 4), np.float32)
    out[:, :dim] = T
    return out


@pytest.mark.parametrize("fname,und,model,K", [("pl100w.txt", 1, "line2", 5), ("pl1k.txt", 1, "line2", 10),
                                               ("toy.txt", 0, "line2", 3), ("bip.txt", 0, "bpr", 1)])
def test_go_draws_bit_exact(smore, fname, und, model, K):
    g, pn = pair(smore, fname, und)
    got = pn.sample_edges(model, 31, 50000, K, SEED)
    np.testing.assert_array_equal(got, orc.go_sample(g, SEED, 31, 50000, K))


@pytest.mark.parametrize("model,dim,K", [("line2", 8, 5), ("line2", 64, 5), ("line2", 300, 10), ("line2", 128, 7),
                                         ("line1", 20, 5), ("line1", 64, 10), ("bpr", 16, 1), ("bpr", 128, 1)])
def test_go_serial_bit_exact_vs_oracle(smore, model, dim, K):
    fname, und = ("bip.txt", 0) if model == "bpr" else ("pl100w.txt", 1)
    g, pn = pair(smore, fname, und)
    W0, C0 = tables(g.V, dim, dim + K)
    ntab = 1 if model == "line1" else 2
    pn.alloc_tables(dim, ntab)
    pn.set_table(0, W0)
    if ntab == 2:
        pn.set_table(1, C0)
    lam = 0.01 if model == "bpr" else 0.0
    total, begin, n = 10 ** 6, 9000, 20000                  # crosses an alpha step
    pn.train_edges(model, begin, n, total, K, 0.025, lam, SEED, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.go_train_f32(g, model, W, C, dim, K, 0.025, lam, total, begin, begin + n, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    if ntab == 2:
        np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_go_serial_skips_dead_ends(smore):
    g, pn = pair(smore, "toy.txt", 0)
    W0, C0 = tables(g.V, 8, 3)
    pn.alloc_tables(8, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    pn.train_edges("line2", 0, 30000, 50000, 2, 0.025, 0.0, SEED, "serial")
    W, C = padded(W0, 8), padded(C0, 8)
    orc.go_train_f32(g, "line2", W, C, 8, 2, 0.025, 0.0, 50000, 0, 30000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)


@pytest.mark.parametrize("dim,K,window,steps", [(16, 5, 2, 10), (64, 5, 5, 40), (100, 10, 3, 20)])
def test_go_deepwalk_serial_bit_exact(smore, dim, K, window, steps):
    g, pn = pair(smore, "pl100w.txt", 1)
    W0, C0 = tables(g.V, dim, dim)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 2, 5)
    pn.train_deepwalk(0, 2 * g.V, 2, steps, window, K, 0.025, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.go_deepwalk_f32(g, W, C, dim, 2, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_go_deepwalk_directed_dead_ends(smore):
    g, pn = pair(smore, "toy.txt", 0)
    W0, C0 = tables(g.V, 8, 1)
    pn.alloc_tables(8, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 3, 0)
    pn.train_deepwalk(0, 3 * g.V, 3, 8, 2, 3, 0.025, SEED, order, "serial")
    W, C = padded(W0, 8), padded(C0, 8)
    orc.go_deepwalk_f32(g, W, C, 8, 3, 8, 2, 3, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)


def test_go_deepwalk_parallel_modes_train_like_serial(smore):
    """Go DeepWalk's parallel modes on the record path (go_pair_emit_kernel ->
    go_rec.h go_pair_kernel, concurrency capped at V/16 groups as the C++
    walks): atomic and hybrid reach the serial order's held-out skip-gram AUC
    (within 0.02).  Plain stores (hogwild) lose context-row updates on this
    920-vertex graph -- C++ DeepWalk's hogwild sits at the same level
    (tools/go_walk_check.py: 0.78 vs 0.87) -- but W_v's run gradient is added,
    not stored, so it still trains (> 0.75)."""
    g, pn = pair(smore, "pl1k.txt", 1)
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
    for mode in ("serial", "atomic", "hybrid", "hogwild"):
        pn.alloc_tables(dim, 2)
        pn.init_table_glibc(0, 0)
        pn.zero_table(1)
        pn.train_deepwalk(0, times * g.V, times, 20, 5, K, 0.025, SEED, order, mode)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[mode] = auc(W, C)
    assert res["serial"] > 0.85, res
    assert abs(res["atomic"] - res["serial"]) < 0.02, res
    assert abs(res["hybrid"] - res["serial"]) < 0.02, res
    assert res["hogwild"] > 0.75, res


@pytest.mark.parametrize("model", ["line2", "line1", "bpr"])
def test_go_atomic_single_sample(smore, model):
    fname, und = ("bip.txt", 0) if model == "bpr" else ("pl100w.txt", 1)
    g, pn = pair(smore, fname, und)
    W0, C0 = tables(g.V, 64, 9)
    ntab = 1 if model == "line1" else 2
    pn.alloc_tables(64, ntab)
    K = 1 if model == "bpr" else 5
    for s in (5, 99, 12345):
        pn.set_table(0, W0)
        if ntab == 2:
            pn.set_table(1, C0)
        pn.train_edges(model, s, 1, 10 ** 6, K, 0.025, 0.01, SEED, "atomic")
        W, C = W0.copy(), C0.copy()
        orc.go_train_f32(g, model, W, C, 64, K, 0.025, 0.01, 10 ** 6, s, s + 1, SEED)
        np.testing.assert_allclose(pn.get_table(0), W, atol=1e-6, rtol=0)
        if ntab == 2:
            np.testing.assert_allclose(pn.get_table(1), C, atol=1e-6, rtol=0)


@pytest.mark.parametrize("model", ["line2", "bpr"])
def test_go_serial_close_to_fp64(smore, model):
    """fp32 HIP path vs the fp64 Go rules over 2*10^5 dependent updates."""
    fname, und = ("bip.txt", 0) if model == "bpr" else ("pl1k.txt", 1)
    g, pn = pair(smore, fname, und)
    dim = 32
    W0, C0 = tables(g.V, dim, 2)
    W0 *= 0.1
    C0 *= 0.1
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    total = 200000
    K = 1 if model == "bpr" else 5
    pn.train_edges(model, 0, total, total, K, 0.025, 0.001, SEED, "serial")
    W, C = W0.astype(np.float64), C0.astype(np.float64)
    orc.go_train_f64(g, model, W, C, K, 0.025, 0.001, total, 0, total, SEED)
    for got, want in ((pn.get_table(0), W), (pn.get_table(1), C)):
        err = np.abs(got - want)
        assert err.max() < 2e-3 and np.median(err) < 2e-4, (err.max(), np.median(err))


def test_go_rejects_mf(smore):
    g, pn = pair(smore, "bip.txt", 0)
    pn.alloc_tables(8, 2)
    with pytest.raises(smore._lib.SmoreError):
        pn.train_edges("mf", 0, 10, 10, 5, 0.025, 0.0, SEED, "atomic")


def test_go_model_drivers(smore, tmp_path):
    """internal/models/{line,bpr,deepwalk,node2vec} mirrors: Go totals and Go save format."""
    from smore_amd import go_models
    path = os.path.join(GOLDEN, "pl1k.txt")
    m = go_models.LINE.New()
    m.LoadEdgeList(path, True)
    assert m.MaxLine * 2 == m.pnet.MAX_line
    m.Init(16, go_models.LINE.Second)
    m.Train(2, 5, 0.025, 4)
    out = tmp_path / "line.txt"
    m.SaveWeights(str(out))
    lines = out.read_text().splitlines()
    assert len(lines) == m.pnet.MAX_vid + 1
    assert np.isfinite(m.w_vertex).all() and np.abs(m.w_vertex).max() > 0
    b = go_models.BPR.New()
    b.LoadEdgeList(os.path.join(GOLDEN, "bip.txt"), False)
    b.Init(8)
    b.Train(3, 0.025, 0.001, 1)
    assert np.isfinite(b.w_vertex).all()
    d = go_models.DeepWalk.New()
    d.LoadEdgeList(path, True)
    d.Init(8)
    d.Train(1, 10, 2, 3, 0.025, 1)
    assert np.isfinite(d.w_context).all()
    n = go_models.Node2Vec.New()
    n.LoadEdgeList(path, True)
    n.Init(8, 0.5, 2.0)
    n.Train(1, 10, 2, 3, 0.025, 1)
    assert np.isfinite(n.w_context).all() and np.abs(n.w_vertex).max() > 0


@pytest.mark.parametrize("fname,und,p,q,dim,K,window,steps",
                         [("pl100w.txt", 1, 0.25, 4.0, 16, 5, 2, 10), ("pl1k.txt", 1, 2.0, 0.5, 64, 5, 5, 40),
                          ("toy.txt", 0, 0.5, 2.0, 8, 3, 2, 8), ("pl100w.txt", 1, 1.0, 1.0, 100, 10, 3, 20)])
def test_go_node2vec_serial_bit_exact(smore, fname, und, p, q, dim, K, window, steps):
    """(*Node2Vec).Train (internal/models/node2vec/node2vec.go:178-258) on the GPU
    vs the oracle's fp32 spec of it (parity unpinned vs Go: no Go toolchain)."""
    g, pn = pair(smore, fname, und)
    W0, C0 = tables(g.V, dim, dim + 1)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 2, 3)
    half = g.V   # two calls: the second starts mid-order
    pn.train_node2vec(0, half, 2, steps, window, K, 0.025, p, q, SEED, order, "serial")
    pn.train_node2vec(half, 2 * g.V, 2, steps, window, K, 0.025, p, q, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.go_node2vec_f32(g, W, C, dim, 2, steps, window, K, 0.025, p, q, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_go_node2vec_parallel_and_rejects(smore):
    g, pn = pair(smore, "pl1k.txt", 1)
    W0, C0 = tables(g.V, 32, 7)
    pn.alloc_tables(32, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 4, 0)
    with pytest.raises(smore._lib.SmoreError):
        pn.train_node2vec(0, 4 * g.V, 4, 20, 3, 5, 0.025, 0.0, 1.0, SEED, order, "atomic")   # p <= 0
    pn.train_node2vec(0, 4 * g.V, 4, 20, 3, 5, 0.025, 0.5, 2.0, SEED, order, "atomic")
    W = pn.get_table(0)
    assert np.isfinite(W).all() and np.abs(W - W0).max() > 1e-3
    pn.set_semantics("cpp")
    with pytest.raises(smore._lib.SmoreError):
        pn.train_node2vec(0, g.V, 1, 20, 3, 5, 0.025, 0.5, 2.0, SEED, order, "atomic")   # Go model only


def _hetero_pair(smore, und):
    from smore_amd.go_models import load_hetero
    names, ntype, tkeys, s, d, w = load_hetero(os.path.join(GOLDEN, "hetero.txt"), und)
    g = orc.GoGraph(len(names), s, d, w, names)
    prob, alias = orc.go_uniform_negatives(g)
    pn = smore.ProNet(0)
    pn.set_graph_edges(len(names), s, d, w)
    pn.set_semantics("go")
    pn.set_node_types(ntype, len(tkeys))
    pn.set_alias(smore._lib.AT_NEGATIVE, prob, alias)
    U, I, C_ = (tkeys.index(x) for x in ("User", "Item", "Category"))
    return g, pn, ntype, [[U, I, U], [I, C_, I], [U, I, C_, I, U]]


@pytest.mark.parametrize("und,dim,K,window,steps", [(1, 16, 5, 2, 10), (1, 64, 5, 5, 40), (0, 8, 3, 2, 8)])
def test_go_metapath2vec_serial_bit_exact(smore, und, dim, K, window, steps):
    """(*Metapath2Vec).Train (internal/models/metapath2vec/metapath2vec.go:106-200)
    on the GPU vs the oracle's fp32 spec (parity unpinned vs Go: no Go toolchain)."""
    g, pn, ntype, paths = _hetero_pair(smore, und)
    W0, C0 = tables(g.V, dim, dim + 3)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 2, 1)
    pn.train_metapath2vec(0, g.V + 7, 2, steps, window, K, 0.025, paths, SEED, order, "serial")
    pn.train_metapath2vec(g.V + 7, 2 * g.V, 2, steps, window, K, 0.025, paths, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.go_metapath_f32(g, ntype, paths, W, C, dim, 2, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_go_metapath2vec_model_driver(smore, tmp_path):
    from smore_amd import go_models
    m = go_models.Metapath2Vec.New(mode="atomic")
    m.LoadEdgeList(os.path.join(GOLDEN, "hetero.txt"), True)
    with pytest.raises(ValueError):
        m.AddMetaPath("User Nope")
    m.AddMetaPath("User Item User")
    m.AddMetaPath("Item Category Item")
    m.Init(16)
    m.Train(3, 10, 2, 5, 0.025, 4)
    W = m.w_vertex
    assert np.isfinite(W).all() and np.abs(W).max() > 0
    out = tmp_path / "mp.txt"
    m.SaveEmbeddings(str(out))
    lines = out.read_text().splitlines()
    assert lines[0] == "%d 16" % len(m.names) and lines[1].split()[0].endswith("]")


def _ctdne_pair(smore):
    from smore_amd.go_models import load_temporal
    names, s, d, ts = load_temporal(os.path.join(GOLDEN, "temporal.txt"))
    g = orc.GoGraph(len(names), s, d, np.ones(len(s)), names)
    pn = smore.ProNet(0)
    pn.set_graph_edges(len(names), s, d, np.ones(len(s)))
    pn.set_semantics("go")
    pn.set_temporal_edges(s, d, ts)
    return g, pn, s, d, ts


@pytest.mark.parametrize("window,dim,K,win,steps", [(30.0, 16, 5, 2, 10), (8.0, 64, 5, 5, 40), (0.0, 8, 3, 2, 8)])
def test_go_ctdne_serial_bit_exact(smore, window, dim, K, win, steps):
    """(*CTDNE).Train (internal/models/ctdne/ctdne.go:80-200) on the GPU vs the
    oracle's fp32 spec (parity unpinned vs Go: no Go toolchain).  window 0:
    the library's default, 0.1 x the time span."""
    g, pn, s, d, ts = _ctdne_pair(smore)
    W0, C0 = tables(g.V, dim, dim + 5)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(g.V, 2, 2)
    pn.train_ctdne(0, g.V - 3, 2, steps, win, K, 0.025, window, SEED, order, "serial")
    pn.train_ctdne(g.V - 3, 2 * g.V, 2, steps, win, K, 0.025, window, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    eff = window if window > 0 else (ts.max() - ts.min()) * 0.1
    orc.go_ctdne_f32(g, s, d, ts, eff, W, C, dim, 2, steps, win, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_go_ctdne_model_driver(smore, tmp_path):
    from smore_amd import go_models
    m = go_models.CTDNE.New(mode="atomic")
    m.LoadEdgeList(os.path.join(GOLDEN, "temporal.txt"))
    m.Init(16, 0.0)
    m.Train(3, 10, 2, 5, 0.025, 4)
    W = m.w_vertex
    assert np.isfinite(W).all() and np.abs(W).max() > 0
    out = tmp_path / "ct.txt"
    m.SaveEmbeddings(str(out))
    lines = out.read_text().splitlines()
    assert lines[0] == "%d 16" % len(m.names) and len(lines) == len(m.names) + 1


def test_go_c2_full_grid_hybrid_matches_atomic(smore):
    """The Go rules on the record path at full grid (config 2's graph, 2^28
    samples, d=64, K=5): the hybrid scatter (hot rows by atomic add, the
    hottest context rows write-combined in LDS; W rows are not combined by
    default) trains like the lossless atomic
    scatter -- held-out Go LINE-2 loss within 1 % -- and Go BPR's hybrid run on
    the same graph is finite."""
    from smore_amd import graphgen
    V, (src, dst, w) = graphgen.config_edges("c2")
    pn = smore.ProNet(0)
    pn.set_graph_edges(V, src, dst, w)
    pn.set_semantics("go")
    dim, K, total = 64, 5, 1 << 28
    held = pn.sample_edges("line2", 1 << 40, 100_000, K, SEED + 1)
    res = {}
    for mode in ("atomic", "hybrid"):
        W0, C0 = [(t / dim).astype(np.float32) for t in tables(V, dim, 5)]
        pn.alloc_tables(dim, 2)
        pn.set_table(0, W0)
        pn.set_table(1, C0)
        pn.set_hot_threshold(0.3)
        pn.set_write_combine(128, 0)
        pn.train_edges("line2", 0, total, total, K, 0.025, 0.0, SEED, mode)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        v, c, negs = held[:, 0], held[:, 1], held[:, 2:]
        keep = c >= 0
        v, c, negs = v[keep], c[keep], negs[keep]
        Wv = W[v].astype(np.float64)
        loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[c].astype(np.float64)))
        for k in range(K):
            loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k]].astype(np.float64)))
        res[mode] = float(loss.mean())
        if mode == "hybrid":
            hw, hc = pn.hot_rows()
            assert hw > 0 and hc > 0, (hw, hc)
    assert res["atomic"] < 0.9 * np.log(2.0) * (1 + K), res
    assert abs(res["hybrid"] - res["atomic"]) <= 0.01 * res["atomic"], res
    pn.train_edges("bpr", 0, 1 << 26, 1 << 26, 1, 0.025, 0.001, SEED, "hybrid")
    assert np.isfinite(pn.get_table(0)).all() and np.isfinite(pn.get_table(1)).all()
