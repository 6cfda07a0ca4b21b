"""The parallel edge-list loader and its binary cache (smore_amd/csrc/loader.cpp,
SURVEY.md 8f-1) on a host-only context (no GPU): vertex ids in order of first
appearance and directed slots in the reference's push order
(src/proNet.cpp:115-236), checked against the oracle's sequential restatement
(oracle/oracle.py read_edgelist) on the golden edge lists and on a generated
file large enough to be cut into many chunks, with ragged lines."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import GOLDEN


def _load(path, und, cache=None, threads=None):
    import smore_amd
    if threads:
        os.environ["SMORE_LOAD_THREADS"] = str(threads)
    try:
        pn = smore_amd.ProNet(-1)
        if cache:
            pn.set_load_cache(cache)
        pn.LoadEdgeList(path, und)
        info = pn.last_load_info()
        off, tgt = pn.csr()
        return pn.names, off, tgt, info
    finally:
        os.environ.pop("SMORE_LOAD_THREADS", None)


def _expected(path, und):
    names, s, d, w = orc.read_edgelist(path, und)
    g = orc.Graph(len(names), s, d, w)
    return names, g.offsets, g.targets[:g.E]


@pytest.mark.parametrize("fname,und", [("toy.txt", 1), ("toy.txt", 0), ("pl1k.txt", 1), ("bip.txt", 0),
                                       ("pl100w.txt", 1)])
def test_golden_edge_lists(fname, und):
    path = os.path.join(GOLDEN, fname)
    names, off, tgt, _ = _load(path, und)
    en, eo, et = _expected(path, und)
    assert names == en
    np.testing.assert_array_equal(off, eo)
    np.testing.assert_array_equal(tgt, et)


def _ragged_file(path, lines=1_000_000, seed=5):
    """Zipf-ish ids, mixed separators, \\r\\n, short and malformed lines, no
    trailing newline."""
    rng = np.random.default_rng(seed)
    a = (rng.zipf(1.6, lines) % 50_000).astype(np.int64)
    b = (rng.zipf(1.6, lines) % 50_000).astype(np.int64)
    w = rng.integers(1, 5, lines)
    out = []
    for i in range(lines):
        r = i % 97
        if r == 13:
            out.append("lonely%d 7" % a[i])                       # 2 fields: skipped
        elif r == 29:
            out.append("u%d\tv%d\tnotanumber" % (a[i], b[i]))     # bad weight: skipped
        elif r == 41:
            out.append("")                                         # empty line
        elif r == 53:
            out.append("  u%d   v%d  %d.5 extra fields\r" % (a[i], b[i], w[i]))
        else:
            out.append("u%d v%d %d" % (a[i], b[i], w[i]))
    with open(path, "w") as f:
        f.write("\n".join(out))                                    # no newline at the end


@pytest.mark.parametrize("und,threads", [(1, 8), (0, 3), (1, 1)])
def test_parallel_loader_matches_sequential(tmp_path, und, threads):
    path = str(tmp_path / "ragged.txt")
    _ragged_file(path)
    names, off, tgt, info = _load(path, und, threads=threads)
    en, eo, et = _expected(path, und)
    assert info[1] == min(threads, os.path.getsize(path) // (1 << 20) + 1)   # >= 1 MiB of text per thread
    assert names == en
    np.testing.assert_array_equal(off, eo)
    np.testing.assert_array_equal(tgt, et)


def test_directory_input(tmp_path):
    d = tmp_path / "parts"
    d.mkdir()
    for k in range(3):
        _ragged_file(str(d / ("p%d.txt" % k)), lines=20_000, seed=k)
    names, off, tgt, _ = _load(str(d), 1, threads=4)
    # readdir order (the reference's opendir/readdir loop, src/proNet.cpp:124-134)
    files = [str(d / e) for e in os.listdir(str(d))]
    en, s, dd, w = [], [], [], []
    ids = {}
    for fn in files:
        nm, s1, d1, w1 = orc.read_edgelist(fn, 1)
        remap = []
        for n in nm:
            if n not in ids:
                ids[n] = len(en)
                en.append(n)
            remap.append(ids[n])
        remap = np.array(remap, np.int32)
        s.append(remap[s1]); dd.append(remap[d1]); w.append(w1)
    g = orc.Graph(len(en), np.concatenate(s), np.concatenate(dd), np.concatenate(w))
    assert names == en
    np.testing.assert_array_equal(off, g.offsets)
    np.testing.assert_array_equal(tgt, g.targets[:g.E])


def test_binary_cache_roundtrip(tmp_path):
    path = str(tmp_path / "g.txt")
    _ragged_file(path, lines=100_000)
    cache = str(tmp_path / "cache")
    os.makedirs(cache)
    n1, o1, t1, i1 = _load(path, 1, cache=cache)
    assert not i1[2]
    assert len([f for f in os.listdir(cache) if f.endswith(".smorelc")]) == 1
    n2, o2, t2, i2 = _load(path, 1, cache=cache)
    assert i2[2], "second load not served from the cache"
    assert n1 == n2
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(t1, t2)
    # the undirected flag and the content are part of the key
    _, _, _, i3 = _load(path, 0, cache=cache)
    assert not i3[2]
    with open(path, "a") as f:
        f.write("\nnewa newb 1\n")
    n4, _, _, i4 = _load(path, 1, cache=cache)
    assert not i4[2] and n4[-2:] == ["newa", "newb"]


def test_built_graph_cache(tmp_path):
    """A second load of the same input with the same sampling methods reads the
    built graph (CSR, degrees, every alias table) back: identical to a fresh
    build; other methods fall back to the cached edge slots and build."""
    import smore_amd
    path = str(tmp_path / "g.txt")
    _ragged_file(path, lines=50_000)
    cache = str(tmp_path / "cache")
    os.makedirs(cache)

    def load(vm, nm):
        pn = smore_amd.ProNet(-1)
        pn.set_load_cache(cache)
        pn.SetVertexMethod(vm)
        pn.SetNegativeMethod(nm)
        pn.LoadEdgeList(path, 1)
        tabs = [pn.alias(w) + pn.alias_encoded(w) for w in range(3)]
        return pn.last_load_info()[2], pn.names, pn.csr(), tabs

    h1, n1, c1, t1 = load("out_degrees", "degrees")
    assert h1 == 0 and len([f for f in os.listdir(cache) if f.endswith(".smoregc")]) == 1
    h2, n2, c2, t2 = load("out_degrees", "degrees")
    assert h2 == 2, "second load did not read the built graph"
    h3, n3, c3, t3 = load("degrees", "in_degrees")
    assert h3 == 1 and len([f for f in os.listdir(cache) if f.endswith(".smoregc")]) == 2
    assert n1 == n2 == n3
    for a, b in zip(c1 + c3, c2 + c3):
        np.testing.assert_array_equal(a, b)
    for x, y in zip(t1, t2):
        for a, b in zip(x, y):
            np.testing.assert_array_equal(a, b)
    # the methods matter: the negative tables differ between the two builds
    assert not np.array_equal(t1[1][0], t3[1][0])


def test_cache_key_independent_of_threads(tmp_path):
    """The cache key is a function of the input bytes only: a file above one
    hash piece's worth of threads (> 4 MiB) cached by a 1-thread load is found
    by an 8-thread load (the key used to depend on the thread count)."""
    path = str(tmp_path / "g.txt")
    _ragged_file(path, lines=700_000)
    assert os.path.getsize(path) > (5 << 20)
    cache = str(tmp_path / "cache")
    os.makedirs(cache)
    _, _, _, i1 = _load(path, 1, cache=cache, threads=1)
    assert not i1[2]
    _, _, _, i2 = _load(path, 1, cache=cache, threads=8)
    assert i2[2], "8-thread load missed the 1-thread cache"


def test_corrupt_graph_cache_is_rebuilt(tmp_path):
    """A built-graph cache whose CSR targets were overwritten with an id >= V
    is rejected by the read-back checks and the graph is built again (same
    result as a fresh build), never uploaded as read."""
    import smore_amd
    path = str(tmp_path / "g.txt")
    _ragged_file(path, lines=20_000)
    cache = str(tmp_path / "cache")
    os.makedirs(cache)

    def load():
        pn = smore_amd.ProNet(-1)
        pn.set_load_cache(cache)
        pn.LoadEdgeList(path, 1)
        return pn.last_load_info()[2], pn.csr()

    h1, c1 = load()
    gc = [f for f in os.listdir(cache) if f.endswith(".smoregc")]
    assert h1 == 0 and len(gc) == 1
    fn = os.path.join(cache, gc[0])
    V = len(c1[0]) - 1
    hdr = 8 + 9 * 8
    with open(fn, "r+b") as f:
        f.seek(hdr)
        nb = int(np.frombuffer(open(fn, "rb").read(hdr)[8 + 5 * 8:8 + 6 * 8], np.uint64)[0])
        f.seek(hdr + nb + (V + 1) * 8 + 4 * 10)          # the 11th CSR target
        f.write(np.array([V + 7], np.int32).tobytes())
    h2, c2 = load()
    assert h2 != 2, "corrupt graph cache was used"
    np.testing.assert_array_equal(c1[0], c2[0])
    np.testing.assert_array_equal(c1[1], c2[1])


@pytest.mark.parametrize("weighted", [False, True])
def test_graph_file_round_trip(tmp_path, weighted):
    """smore_save_graph / smore_load_graph (bench.py's build-once start-up and
    the loader cache): the file holds the CSR, weights and the vertex / negative
    tables; the per-edge context tables are rebuilt on load
    (build_ctx_tables) and equal the built graph's bit for bit, in both the
    (prob, alias) and the encoded device form."""
    import smore_amd
    rng = np.random.default_rng(3)
    V, E = 5000, 60_000
    src = (rng.zipf(1.5, E) % V).astype(np.int32)
    dst = rng.integers(0, V, E).astype(np.int32)
    w = rng.integers(1, 7, E).astype(np.float64) if weighted else None
    a = smore_amd.ProNet(-1)
    a.set_graph_edges(V, src, dst, w)
    path = str(tmp_path / "g.graph")
    a.save_graph(path)
    b = smore_amd.ProNet(-1)
    b.load_graph(path)
    for x, y in zip(a.csr(), b.csr()):
        np.testing.assert_array_equal(x, y)
    assert a.names == b.names
    for which in (0, 1, 2):
        for x, y in zip(a.alias(which), b.alias(which)):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a.alias_encoded(which), b.alias_encoded(which)):
            np.testing.assert_array_equal(x, y)
    # the context tables are not stored: 24 -> 4 (+8 weighted) bytes per slot
    assert os.path.getsize(path) < (4 + (8 if weighted else 0)) * 2 * E + 200 * V
