"""The Go drop-in's call sequence through the C ABI (go/pkg/pronet/hip.go,
replayed by the C program tests/c/go_shape.c, since this image has no Go
toolchain): adjacency of pn.Graph in vertex order -> smore_group_set_graph_edges,
Go semantics, pn.NegativeAT injected, fp64 tables flattened to fp32, chunked
training with total = sample_times * MaxLine, tables copied back.  In serial
mode the result is bit-exact with the oracle's Go-rule fp32 spec
(orc_go_*_f32; parity against Go itself is unpinned: no Go toolchain).
Needs an MI355X."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tests", "c", "go_shape")
SEED = 4242
SERIAL, ATOMIC = 2, 1
MODEL = {"line2": 0, "line1": 1, "bpr": 3, "deepwalk": -1, "node2vec": -2, "metapath2vec": -3, "ctdne": -4,
         "pairs": -5}


def _shim_inputs(g):
    """What NewHIP flattens: the directed slots of pn.Graph in vertex order."""
    src = np.repeat(np.arange(g.V, dtype=np.int32), np.diff(g.offsets)).astype(np.int32)
    dst = g.targets[:g.E].astype(np.int32)
    w = g.weights[:g.E].astype(np.float64)
    return src, dst, w


def _run(tmp_path, g, model, dim, K, total, mode, alpha, lam, W0, C0, walk=None, neg=None, extra=b""):
    src, dst, w = _shim_inputs(g)
    nprob, nalias = neg if neg is not None else (g.nprob, g.nalias)
    p_in, p_out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    with open(p_in, "wb") as f:
        f.write(struct.pack("<8q", g.V, g.E, dim, MODEL[model], K, total, 1, mode))
        f.write(struct.pack("<2dQ", alpha, lam, SEED))
        for a in (src, dst, w, np.asarray(nprob, np.float64), np.asarray(nalias, np.int64),
                  W0.astype(np.float64), C0.astype(np.float64)):
            f.write(np.ascontiguousarray(a).tobytes())
        if walk is not None:
            times, steps, window, order = walk[:4]
            f.write(struct.pack("<4q", times, steps, window, len(order)))
            f.write(np.ascontiguousarray(order, np.int64).tobytes())
            if model == "node2vec":
                f.write(struct.pack("<2d", *walk[4]))
        f.write(extra)
    r = subprocess.run([BIN, p_in, p_out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = np.fromfile(p_out, np.float64).reshape(2, g.V, dim)
    return out[0], out[1]


def _tables(V, dim, seed):
    rng = np.random.default_rng(seed)
    return [(rng.random((V, dim), dtype=np.float32) - 0.5) for _ in range(2)]


def _padded(T, dim):
    out = np.zeros((T.shape[0], (dim + 3) // 4 * 4), np.float32)
    out[:, :dim] = T
    return out


def test_go_shape_binary_built():
    assert os.access(BIN, os.X_OK), "build it with `make goshape`"


@pytest.mark.parametrize("model,fname,und,dim,K,lam", [("line2", "pl100w.txt", 1, 64, 5, 0.0),
                                                       ("line1", "pl100w.txt", 1, 20, 5, 0.0),
                                                       ("bpr", "bip.txt", 0, 16, 1, 0.001)])
def test_go_shim_sequence_serial_bit_exact(tmp_path, model, fname, und, dim, K, lam):
    g = orc.GoGraph.from_file(os.path.join(GOLDEN, fname), und)
    max_line = g.E // 2 if und else g.E            # Go's MaxLine counts input lines
    total = 3 * max_line                           # sample_times = 3
    W0, C0 = _tables(g.V, dim, dim + K)
    W, C = _run(tmp_path, g, model, dim, K, total, SERIAL, 0.025, lam, W0, C0)
    Wr, Cr = _padded(W0, dim), _padded(C0, dim)
    orc.go_train_f32(g, model, Wr, Cr, dim, K, 0.025, lam, total, 0, total, SEED)
    np.testing.assert_array_equal(W.astype(np.float32), Wr[:, :dim])
    if model != "line1":
        np.testing.assert_array_equal(C.astype(np.float32), Cr[:, :dim])


def test_go_shim_deepwalk_serial_bit_exact(tmp_path):
    g = orc.GoGraph.from_file(os.path.join(GOLDEN, "pl100w.txt"), 1)
    dim, K, times, steps, window = 32, 5, 2, 10, 3
    order = np.concatenate([np.random.default_rng(t).permutation(g.V) for t in range(times)]).astype(np.int64)
    W0, C0 = _tables(g.V, dim, 9)
    W, C = _run(tmp_path, g, "deepwalk", dim, K, 0, SERIAL, 0.025, 0.0, W0, C0, (times, steps, window, order))
    Wr, Cr = _padded(W0, dim), _padded(C0, dim)
    orc.go_deepwalk_f32(g, Wr, Cr, dim, times, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(W.astype(np.float32), Wr[:, :dim])
    np.testing.assert_array_equal(C.astype(np.float32), Cr[:, :dim])


def test_go_shim_atomic_trains(tmp_path):
    """The shim's default scatter (atomic) on the 1k-vertex graph: finite, and
    positive edges score above random pairs."""
    g = orc.GoGraph.from_file(os.path.join(GOLDEN, "pl1k.txt"), 1)
    dim = 32
    W0, C0 = _tables(g.V, dim, 3)
    W0 /= dim
    C0 /= dim
    W, C = _run(tmp_path, g, "line2", dim, 5, 200 * (g.E // 2), ATOMIC, 0.025, 0.0, W0, C0)
    assert np.isfinite(W).all() and np.isfinite(C).all()
    rng = np.random.default_rng(0)
    src = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, 5000)
    pos = np.einsum("ij,ij->i", W[src[pick]], C[g.targets[pick]])
    neg = np.einsum("ij,ij->i", W[rng.integers(0, g.V, 5000)], C[rng.integers(0, g.V, 5000)])
    assert (pos[:, None] > neg[None, :1000]).mean() > 0.75


def test_go_shim_node2vec_serial_bit_exact(tmp_path):
    """(*HIP).TrainNode2Vec's call sequence (go/pkg/pronet/hip.go) vs the oracle."""
    g = orc.GoGraph.from_file(os.path.join(GOLDEN, "pl1k.txt"), 1)
    dim, K, times, steps, window = 16, 5, 2, 12, 3
    order = np.concatenate([np.random.default_rng(t + 3).permutation(g.V) for t in range(times)]).astype(np.int64)
    W0, C0 = _tables(g.V, dim, 10)
    W, C = _run(tmp_path, g, "node2vec", dim, K, 0, SERIAL, 0.025, 0.0, W0, C0,
                (times, steps, window, order, (0.25, 4.0)))
    Wr, Cr = _padded(W0, dim), _padded(C0, dim)
    orc.go_node2vec_f32(g, Wr, Cr, dim, times, steps, window, K, 0.025, 0.25, 4.0, SEED, order)
    np.testing.assert_array_equal(W.astype(np.float32), Wr[:, :dim])
    np.testing.assert_array_equal(C.astype(np.float32), Cr[:, :dim])


def test_go_shim_metapath2vec_serial_bit_exact(tmp_path):
    """metapath2vec_hip.go's call sequence (NewHIPEdges with hg.Edges in vertex
    order and Train's BuildAliasMethod(ones, 0.75), SetNodeTypes,
    TrainMetapath2Vec) vs the oracle's Go-rule fp32 spec."""
    from smore_amd.go_models import load_hetero
    names, ntype, tkeys, s, d, w = load_hetero(os.path.join(GOLDEN, "hetero.txt"), True)
    g = orc.GoGraph(len(names), s, d, w, names)
    U, I, Cat = (tkeys.index(x) for x in ("User", "Item", "Category"))
    paths = [[U, I, U], [I, Cat, I], [U, I, Cat, I, U]]
    dim, K, times, steps, window = 16, 5, 2, 10, 2
    order = np.concatenate([np.random.default_rng(t + 7).permutation(g.V) for t in range(times)]).astype(np.int64)
    W0, C0 = _tables(g.V, dim, 21)
    flat = np.concatenate([np.array(p, np.int32) for p in paths])
    extra = (struct.pack("<q", len(tkeys)) + np.asarray(ntype, np.int32).tobytes() +
             struct.pack("<2q", len(paths), len(flat)) + np.array([len(p) for p in paths], np.int32).tobytes() +
             flat.tobytes())
    neg = orc.go_uniform_negatives(g)
    W, C = _run(tmp_path, g, "metapath2vec", dim, K, 0, SERIAL, 0.025, 0.0, W0, C0, (times, steps, window, order),
                neg=neg, extra=extra)
    Wr, Cr = _padded(W0, dim), _padded(C0, dim)
    orc.go_metapath_f32(g, ntype, paths, Wr, Cr, dim, times, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(W.astype(np.float32), Wr[:, :dim])
    np.testing.assert_array_equal(C.astype(np.float32), Cr[:, :dim])


def test_go_shim_ctdne_serial_bit_exact(tmp_path):
    """ctdne_hip.go's call sequence (tg.OutEdges in vertex order, each sorted
    by timestamp as pkg/temporal's loader leaves them, as the graph with unit
    weights and as the temporal edges; Train's BuildAliasMethod(activity,
    0.75); TrainCTDNE) vs the oracle's Go-rule fp32 spec."""
    from smore_amd.go_models import load_temporal
    names, s, d, ts = load_temporal(os.path.join(GOLDEN, "temporal.txt"))
    V = len(names)
    o = np.lexsort((ts, s))                       # OutEdges[v] sorted by timestamp, v in order
    so, do, tso = s[o], d[o], ts[o]
    g = orc.GoGraph(V, so, do, np.ones(len(so)), names)   # Go table of activity = in + out counts
    act = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
    assert (act > 0).all()
    dim, K, times, steps, window = 16, 5, 2, 10, 2
    twin = 30.0
    order = np.concatenate([np.random.default_rng(t + 9).permutation(V) for t in range(times)]).astype(np.int64)
    W0, C0 = _tables(V, dim, 23)
    extra = (struct.pack("<dq", twin, len(so)) + so.astype(np.int32).tobytes() + do.astype(np.int32).tobytes() +
             tso.astype(np.float64).tobytes())
    W, C = _run(tmp_path, g, "ctdne", dim, K, 0, SERIAL, 0.025, 0.0, W0, C0, (times, steps, window, order),
                extra=extra)
    Wr, Cr = _padded(W0, dim), _padded(C0, dim)
    orc.go_ctdne_f32(g, s, d, ts, twin, Wr, Cr, dim, times, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(W.astype(np.float32), Wr[:, :dim])
    np.testing.assert_array_equal(C.astype(np.float32), Cr[:, :dim])


@pytest.mark.parametrize("mode", [SERIAL, ATOMIC])
def test_go_shim_update_pairs(tmp_path, mode):
    """(*ProNet).UpdatePairs under -tags smore_hip (hip.go updatePairsHIP ->
    PairsRows = smore_pairs_rows, gather the touched rows, smore_train_pairs_rows,
    scatter them back; rows no pair touches never move): in serial mode bit-exact
    with the oracle's Go UpdatePair over the caller's pairs (negatives skipped
    when equal to the context, deferred context); atomic mode (Hogwild order,
    ~240 updates per row of a 98-vertex graph, so the tables themselves differ
    from the serial order's by tens of %) finite and training like it: the
    pairs' logistic loss against fixed uniform negatives within 3 % of the
    serial run's, and below the initial tables'."""
    g = orc.GoGraph.from_file(os.path.join(GOLDEN, "pl100w.txt"), 1)
    dim, K, unit = 24, 5, 1 << 40
    rng = np.random.default_rng(5)
    v = np.repeat(rng.integers(0, g.V, 1000), 4).astype(np.int32)
    c = rng.integers(0, g.V, 4000).astype(np.int32)
    c[::17] = v[::17]
    W0, C0 = _tables(g.V, dim, 77)
    extra = struct.pack("<qQ", len(v), unit) + v.tobytes() + c.tobytes()
    W, C = _run(tmp_path, g, "pairs", dim, K, 0, mode, 0.025, 0.0, W0, C0, extra=extra)
    Wo, Co = _padded(W0, dim), _padded(C0, dim)
    orc.update_pairs_f32(g, Wo, Co, dim, v, c, K, 0.025, SEED, unit, go=True)
    if mode == SERIAL:
        np.testing.assert_array_equal(W.astype(np.float32), Wo[:, :dim])
        np.testing.assert_array_equal(C.astype(np.float32), Co[:, :dim])
    else:
        assert np.isfinite(W).all() and np.isfinite(C).all()
        negs = np.random.default_rng(6).integers(0, g.V, (len(v), K))

        def loss(Wt, Ct):
            Wv = Wt[v].astype(np.float64)
            out = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, Ct[c].astype(np.float64)))
            for k in range(K):
                out += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, Ct[negs[:, k]].astype(np.float64)))
            return float(out.mean())

        l_par, l_ser, l_0 = loss(W, C), loss(Wo[:, :dim], Co[:, :dim]), loss(W0, C0)
        assert l_ser < l_0 and l_par <= 1.03 * l_ser, (l_par, l_ser, l_0)
