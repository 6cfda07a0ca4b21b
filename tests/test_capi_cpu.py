"""C-ABI library checks that need no GPU: every declared symbol is exported,
and the product's host graph/alias construction equals the reference (golden
fixtures) and the oracle."""
import os
import re

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "smore_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(smore_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from smore_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 29
    for s in syms:
        assert hasattr(_lib.lib, s), s
    # and the ctypes table covers them all
    assert set(syms) == set(_lib.lib._signatures)


def test_version():
    from smore_amd import _lib
    assert b"gfx950" in _lib.lib.smore_version()


def gold(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def names_of(z):
    raw = bytes(z["names"])
    off = z["name_off"]
    return [raw[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]


CASES = [("graph_toy_undir", "toy.txt"), ("graph_toy_dir_nodeg", "toy.txt"), ("graph_pl100w", "pl100w.txt"),
         ("graph_pl1k", "pl1k.txt"), ("graph_bip_indeg", "bip.txt"), ("graph_bip_nodeg", "bip.txt")]


@pytest.mark.parametrize("name,fname", CASES)
def test_host_loader_and_alias_match_reference(name, fname):
    from smore_amd import ProNet
    from smore_amd import _lib
    z = gold(name)
    pn = ProNet(device=-1)
    pn.SetVertexMethod(bytes(z["meta_vertex_method"]).decode())
    pn.SetNegativeMethod(bytes(z["meta_negative_method"]).decode())
    pn.LoadEdgeList(os.path.join(GOLDEN, fname), int(z["meta_undirected"]))
    assert pn.names == names_of(z)
    off, tgt = pn.csr()
    np.testing.assert_array_equal(off[:-1], z["offset"])
    np.testing.assert_array_equal(np.diff(off), z["branch"])
    np.testing.assert_array_equal(tgt, z["ctx_vid"])
    for which, pk, ak in ((_lib.AT_VERTEX, "vprob", "valias"), (_lib.AT_NEGATIVE, "nprob", "nalias"),
                          (_lib.AT_CONTEXT, "cprob", "calias")):
        p, a = pn.alias(which)
        np.testing.assert_array_equal(p, z[pk])
        np.testing.assert_array_equal(a, z[ak])


def test_encoded_alias_matches_oracle():
    from oracle import oracle as orc
    from smore_amd import ProNet
    from smore_amd import _lib
    g = orc.Graph.from_file(os.path.join(GOLDEN, "pl1k.txt"), 1)
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "pl1k.txt"), 1)
    for which, t, a in ((_lib.AT_VERTEX, g.vthr, g.valias_enc), (_lib.AT_NEGATIVE, g.nthr, g.nalias_enc),
                        (_lib.AT_CONTEXT, g.cthr[:g.E], g.calias_enc[:g.E])):
        tt, aa = pn.alias_encoded(which)
        np.testing.assert_array_equal(tt, t)
        np.testing.assert_array_equal(aa, a)


def test_set_graph_edges_equals_loader():
    from oracle import oracle as orc
    from smore_amd import ProNet
    names, s, d, w = orc.read_edgelist(os.path.join(GOLDEN, "pl100w.txt"), True)
    a = ProNet(device=-1)
    a.set_graph_edges(len(names), s, d, w)
    b = ProNet(device=-1)
    b.LoadEdgeList(os.path.join(GOLDEN, "pl100w.txt"), 1)
    for x, y in zip(a.csr(), b.csr()):
        np.testing.assert_array_equal(x, y)
    assert a.vertex_name(0) is None and b.vertex_name(0) == names[0]


def test_set_alias_injection_roundtrip():
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "pl100w.txt"), 1)
    V = pn.MAX_vid
    prob = np.linspace(0, 1, V)
    alias = np.arange(V)[::-1].copy()
    pn.set_alias(_lib.AT_NEGATIVE, prob, alias)
    p, a = pn.alias(_lib.AT_NEGATIVE)
    np.testing.assert_array_equal(p, prob)
    np.testing.assert_array_equal(a, alias)
    with pytest.raises(_lib.SmoreError):
        pn.set_alias(_lib.AT_NEGATIVE, prob[:-1], alias[:-1])


def test_bad_edges_rejected():
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    with pytest.raises(_lib.SmoreError):
        pn.set_graph_edges(3, [0, 5], [1, 2], [1.0, 1.0])
    with pytest.raises(_lib.SmoreError):
        pn.LoadEdgeList("/nonexistent/file.txt", 1)


def test_deepwalk_order_matches_oracle():
    from oracle import oracle as orc
    from smore_amd import deepwalk_order
    np.testing.assert_array_equal(deepwalk_order(137, 3, 999), orc.deepwalk_order(137, 3, 999))


def test_host_only_context_has_no_gpu_state():
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "toy.txt"), 1)
    with pytest.raises(_lib.SmoreError):
        pn.alloc_tables(8, 2)


@pytest.mark.parametrize("fname,und", [("pl1k.txt", 1), ("bip.txt", 0)])
def test_go_semantics_tables_match_oracle(fname, und):
    """smore_set_semantics(GO) rebuilds VertexAT (power 1) / NegativeAT (power
    0.75, Go alias rule); switching back restores the C++ tables."""
    from oracle import oracle as orc
    from smore_amd import ProNet
    from smore_amd import _lib
    path = os.path.join(GOLDEN, fname)
    gg = orc.GoGraph.from_file(path, und)
    gc = orc.Graph.from_file(path, und)
    pn = ProNet(device=-1)
    pn.LoadEdgeList(path, und)
    pn.set_semantics("go")
    for which, t, a in ((_lib.AT_VERTEX, gg.vthr, gg.valias_enc), (_lib.AT_NEGATIVE, gg.nthr, gg.nalias_enc)):
        tt, aa = pn.alias_encoded(which)
        np.testing.assert_array_equal(tt, t)
        np.testing.assert_array_equal(aa, a)
    pn.set_semantics("cpp")
    for which, t, a in ((_lib.AT_VERTEX, gc.vthr, gc.valias_enc), (_lib.AT_NEGATIVE, gc.nthr, gc.nalias_enc)):
        tt, aa = pn.alias_encoded(which)
        np.testing.assert_array_equal(tt, t)
        np.testing.assert_array_equal(aa, a)


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_source_parts_are_contiguous_equal_mass(nparts):
    """smore_source_parts (host only): bounds 0 .. V, non-empty contiguous parts,
    each vertex in the part that holds the midpoint of its source mass (the
    exact vertex-table marginals), so every part's mass is within one vertex's
    mass of 1/nparts; the row rates of W under LINE-2 are that law."""
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "pl1k.txt"), 1)
    V = pn.MAX_vid
    b = pn.source_parts(nparts)
    assert b[0] == 0 and b[-1] == V and (np.diff(b) > 0).all()
    ps = pn.row_rates("line2", 5, 0)
    assert abs(ps.sum() - 1.0) < 1e-9
    # the exact marginal of the encoded vertex table
    t, a = pn.alias_encoded(_lib.AT_VERTEX)
    acc = t.astype(np.float64) / 2.0 ** 32
    law = acc.copy()
    np.add.at(law, a, 1.0 - acc)
    np.testing.assert_allclose(ps, law / V, rtol=1e-9, atol=1e-15)
    cum = np.concatenate([[0.0], np.cumsum(ps)])
    mid = (cum[:-1] + 0.5 * ps) / cum[-1]
    owner = np.minimum(np.floor(mid * nparts).astype(np.int64), nparts - 1)
    for p in range(nparts):
        assert (owner[b[p]:b[p + 1]] == p).all()
        assert abs(ps[b[p]:b[p + 1]].sum() - 1.0 / nparts) <= ps.max() + 1e-12
    with pytest.raises(_lib.SmoreError):
        pn.source_parts(V + 1)


def test_walk_owner_arguments():
    """smore_set_walk_owner / smore_walk_parts host checks (no GPU): ranges
    inside [0, V], hi < 0 = every pair, and parts only after a row census."""
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "pl1k.txt"), 1)
    V = pn.MAX_vid
    pn.set_walk_owner(0, V)
    pn.set_walk_owner(V // 3, V // 2)
    pn.set_walk_owner(0, -1)
    for lo, hi in ((5, 3), (-1, 4), (0, V + 1)):
        with pytest.raises(_lib.SmoreError):
            pn.set_walk_owner(lo, hi)
    with pytest.raises(_lib.SmoreError):
        pn.walk_parts(4)                      # no census yet


@pytest.mark.parametrize("call", ["train_pairs", "pairs_rows", "get_rows", "set_rows", "train_pairs_rows"])
@pytest.mark.parametrize("bad", [2 ** 32 + 5, 2 ** 31, -1, 1 << 40])
def test_ids_checked_before_narrowing(call, bad):
    """Every binding that narrows vertex ids to int32 range-checks them first
    (ADVICE r5): 2^32 + 5 must not become row 5 and pass the C side's check."""
    from smore_amd import ProNet
    from smore_amd import _lib
    pn = ProNet(device=-1)
    pn.LoadEdgeList(os.path.join(GOLDEN, "toy.txt"), 1)
    ids = np.array([0, bad], np.int64)
    ok = np.array([0, 1], np.int64)
    rows = np.zeros((2, 4), np.float32)
    with pytest.raises(_lib.SmoreError, match="out of range"):
        if call == "train_pairs":
            pn.train_pairs(ids, ok, 5, 0.025, 1)
        elif call == "pairs_rows":
            pn.pairs_rows(ok, ids, 5, 1)
        elif call == "get_rows":
            pn.get_rows(1, ids)
        elif call == "set_rows":
            pn.set_rows(0, ids, rows)
        else:
            pn.train_pairs_rows(ok, ok, 5, 0.025, 1, 0, "hogwild", ids, rows, ok, rows)
