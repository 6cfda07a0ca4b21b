"""Go-semantics mode of the oracle, pinned against an
independent line-by-line Python restatement of the Go source
(tests/go_semantics_ref.py).  CPU only; no Go toolchain exists here, so this
mode's parity is "pinned by restatement" (DESIGN.md 6)."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests import go_semantics_ref as ref
from tests.conftest import GOLDEN

SEED = 4242


def graphs(name, und):
    names, s, d, w = orc.read_edgelist(os.path.join(GOLDEN, name), und)
    return orc.GoGraph(len(names), s, d, w, names), ref.ProNet(names, s, d, w)


@pytest.mark.parametrize("dist,power", [([3.0, 1.0, 0.0, 2.0, 2.0], 1.0), ([0.0] * 4, 0.75), ([5.0], 1.0),
                                        (list(np.random.default_rng(1).random(200) * 7), 0.75)])
def test_go_alias_rule(dist, power):
    p, a = orc.alias_go(dist, power)
    rp, ra = ref.build_alias(dist, power)
    np.testing.assert_array_equal(p, rp)
    np.testing.assert_array_equal(a, ra)


@pytest.mark.parametrize("name,und", [("pl100w.txt", 1), ("bip.txt", 0)])
def test_go_draws(name, und):
    g, pn = graphs(name, und)
    got = orc.go_sample(g, SEED, 17, 3000, 4)
    for t in range(3000):
        rng = ref.Rng(SEED, 0, 17 + t, 11)
        v = pn.source(rng)
        c = pn.target(v, rng)
        negs = [pn.negative(rng) for _ in range(4)]
        assert list(got[t]) == [v, c] + negs, t


def _tables(V, dim, seed):
    rng = np.random.default_rng(seed)
    return rng.random((V, dim)) - 0.5, rng.random((V, dim)) - 0.5


@pytest.mark.parametrize("model,name,und", [("line2", "pl100w.txt", 1), ("line1", "pl100w.txt", 1),
                                            ("bpr", "bip.txt", 0)])
def test_go_train_f64_equals_restatement(model, name, und):
    g, pn = graphs(name, und)
    W0, C0 = _tables(g.V, 8, 3)
    W, Cc = W0.copy(), C0.copy()
    total = 50000
    orc.go_train_f64(g, model, W, Cc, 5, 0.05, 0.001, total, 9990, 10990, SEED)   # crosses an alpha step
    Wl, Cl = [list(r) for r in W0], [list(r) for r in C0]
    ref.train(pn, model, Wl, Cl, 5, 0.05, 0.001, total, 9990, 10990, SEED)
    np.testing.assert_array_equal(W, np.array(Wl))
    np.testing.assert_array_equal(Cc, np.array(Cl))


def test_go_deepwalk_f64_equals_restatement():
    g, pn = graphs("pl100w.txt", 1)
    W0, C0 = _tables(g.V, 8, 4)
    order = orc.deepwalk_order(g.V, 1, 0)
    W, Cc = W0.copy(), C0.copy()
    orc.go_deepwalk_f64(g, W, Cc, 1, 6, 2, 3, 0.025, SEED, order)
    Wl, Cl = [list(r) for r in W0], [list(r) for r in C0]
    ref.deepwalk(pn, Wl, Cl, 1, 6, 2, 3, 0.025, SEED, order)
    np.testing.assert_array_equal(W, np.array(Wl))
    np.testing.assert_array_equal(Cc, np.array(Cl))


@pytest.mark.parametrize("model,name,und", [("line2", "pl100w.txt", 1), ("line1", "pl100w.txt", 1),
                                            ("bpr", "bip.txt", 0)])
def test_go_fp32_spec_close_to_fp64(model, name, und):
    g, _ = graphs(name, und)
    W0, C0 = _tables(g.V, 16, 5)
    for s in (3, 77, 12345):                        # one sample: 1e-5 (north-star criterion)
        W, Cc = W0.copy(), C0.copy()
        orc.go_train_f64(g, model, W, Cc, 5, 0.025, 0.001, 10 ** 6, s, s + 1, SEED)
        W32, C32 = W0.astype(np.float32), C0.astype(np.float32)
        orc.go_train_f32(g, model, W32, C32, 16, 5, 0.025, 0.001, 10 ** 6, s, s + 1, SEED)
        np.testing.assert_allclose(W32, W, atol=1e-5, rtol=0)
        np.testing.assert_allclose(C32, Cc, atol=1e-5, rtol=0)


def test_go_semantics_differ_from_cpp():
    """The Go rule really is different: skip-not-redraw duplicates, deferred
    positive context, power-1 source sampling."""
    g, _ = graphs("pl100w.txt", 1)
    gc = orc.Graph.from_file(os.path.join(GOLDEN, "pl100w.txt"), 1)
    assert not np.array_equal(g.vprob, gc.vprob)           # out_deg^1 vs ^0.75
    np.testing.assert_array_equal(g.offsets, gc.offsets)
    W0, C0 = _tables(g.V, 8, 6)
    a, b = W0.copy(), C0.copy()
    orc.go_train_f64(g, "line2", a, b, 5, 0.025, 0.0, 10 ** 6, 0, 2000, SEED)
    c, d = W0.copy(), C0.copy()
    orc.train_edge_f64(gc, "line2", c, d, 5, 0.025, 0.0, 10 ** 6, 0, 2000, SEED)
    assert not np.allclose(a, c)


@pytest.mark.parametrize("name,und,p,q", [("pl100w.txt", 1, 0.25, 4.0), ("pl100w.txt", 1, 2.0, 0.5),
                                          ("bip.txt", 0, 1.0, 1.0), ("pl1k.txt", 1, 0.5, 2.0)])
def test_go_node2vec_walk_equals_restatement(name, und, p, q):
    """The C oracle's node2vec walk vs the literal Python restatement of
    internal/models/node2vec/node2vec.go:82-175 (parity unpinned vs Go itself)."""
    g, pn = graphs(name, und)
    for unit in range(0, 400):
        start = unit % g.V
        got = orc.go_node2vec_walk(g, p, q, SEED, unit, start, 12)
        want = ref.node2vec_walk(pn, start, 12, p, q, ref.Rng(SEED, 1, unit, 64))
        assert list(got) == want, (unit, list(got), want)


def test_go_node2vec_unbiased_equals_deepwalk_walks():
    """p = q = 1: every bias is 1, so the biased scan is
    the plain TargetSample scan and node2vec trains exactly as Go DeepWalk."""
    g, _ = graphs("pl100w.txt", 1)
    W0, C0 = _tables(g.V, 8, 5)
    order = orc.deepwalk_order(g.V, 1, 0)
    Wa, Ca = W0.astype(np.float32), C0.astype(np.float32)
    Wb, Cb = Wa.copy(), Ca.copy()
    orc.go_deepwalk_f32(g, Wa, Ca, 8, 1, 6, 2, 3, 0.025, SEED, order)
    orc.go_node2vec_f32(g, Wb, Cb, 8, 1, 6, 2, 3, 0.025, 1.0, 1.0, SEED, order)
    np.testing.assert_array_equal(Wa, Wb)
    np.testing.assert_array_equal(Ca, Cb)


def _hetero(und):
    from smore_amd.go_models import load_hetero   # host-side parser (no GPU call)
    names, ntype, tkeys, s, d, w = load_hetero(os.path.join(GOLDEN, "hetero.txt"), und)
    return names, ntype, tkeys, s, d, w


def test_hetero_loader_first_appearance():
    names, ntype, tkeys, s, d, w = _hetero(True)
    assert tkeys[:2] == ["User", "Item"] and set(tkeys) == {"User", "Item", "Category"}
    first = {}
    with open(os.path.join(GOLDEN, "hetero.txt")) as f:
        for line in f:
            p = line.split()
            for nm, ty in ((p[0], p[1]), (p[2], p[3])):
                first.setdefault(nm, ty)
    assert names == list(first)
    assert [tkeys[t] for t in ntype] == [first[n] for n in names]
    assert len(s) == 2 * 214 and s[0] == d[1] and d[0] == s[1]


@pytest.mark.parametrize("und", [1, 0])
def test_go_metapath_walk_equals_restatement(und):
    names, ntype, tkeys, s, d, w = _hetero(und)
    g = orc.GoGraph(len(names), s, d, w, names)
    graph = {v: [] for v in range(g.V)}
    for a, b in zip(s, d):
        graph[int(a)].append(int(b))
    U, I, C_ = (tkeys.index(x) for x in ("User", "Item", "Category"))
    paths = [[U, I, U], [I, C_, I], [U, I, C_, I, U], [C_]]
    for unit in range(600):
        start = unit % g.V
        got = orc.go_metapath_walk(g, ntype, paths, SEED, unit, start, 9)
        rng = ref.Rng(SEED, 1, unit, 64)
        mp = paths[rng.intn(len(paths))]
        want = ref.metapath_walk(graph, ntype, start, mp, 9, rng)
        assert list(got) == want, unit


def test_go_uniform_negative_table():
    """metapath2vec.go:140-145: BuildAliasMethod(ones, 0.75) is {prob 1, alias i}
    exactly (what smore_amd.go_models.Metapath2Vec injects)."""
    p, a = orc.alias_go(np.ones(101), 0.75)
    np.testing.assert_array_equal(p, np.ones(101))
    np.testing.assert_array_equal(a, np.arange(101))


def _temporal():
    from smore_amd.go_models import load_temporal   # host-side parser (no GPU call)
    return load_temporal(os.path.join(GOLDEN, "temporal.txt"))


def test_temporal_loader_skips_malformed():
    names, s, d, ts = _temporal()
    assert len(s) == 600 and len(names) <= 80 and np.isfinite(ts).all()


@pytest.mark.parametrize("window", [5.0, 40.0, 0.5])
def test_go_ctdne_walk_equals_restatement(window):
    names, s, d, ts = _temporal()
    V = len(names)
    out = {v: [] for v in range(V)}
    for a, b, t in zip(s, d, ts):
        out[int(a)].append((int(b), float(t)))
    for v in out:
        out[v].sort(key=lambda e: e[1])
    tmin, tmax = {}, {}
    for a, b, t in zip(s, d, ts):
        for v in (int(a), int(b)):
            tmin[v] = min(tmin.get(v, np.inf), t)
            tmax[v] = max(tmax.get(v, -np.inf), t)
    tmin = [tmin.get(v, 0.0) for v in range(V)]
    tmax = [tmax.get(v, 0.0) for v in range(V)]
    for unit in range(400):
        start = unit % V
        got = orc.go_ctdne_walk(V, s, d, ts, window, SEED, unit, start, 15)
        want = ref.ctdne_walk(out, tmin, tmax, float(ts.max()), window, start, 15, ref.Rng(SEED, 1, unit, 64))
        assert list(got) == want, unit


def test_go_ctdne_negative_table_is_activity():
    """ctdne.go:119-131: BuildAliasMethod(out+in edge counts, 0.75) equals the Go
    negative table of the temporal edges with unit weights."""
    names, s, d, ts = _temporal()
    V = len(names)
    g = orc.GoGraph(V, s, d, np.ones(len(s)), names)
    act = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
    p, a = orc.alias_go(np.where(act > 0, act, 1).astype(np.float64), 0.75)
    np.testing.assert_array_equal(g.nprob, p)
    np.testing.assert_array_equal(g.nalias, a)
