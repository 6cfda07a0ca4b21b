"""Benchmark-input generator and the parallel CSR build (host code, CPU)."""
import numpy as np

from smore_amd import graphgen


def test_powerlaw_deterministic_and_undirected_order():
    a = graphgen.powerlaw_edges(50_000, 300_000, True, 9)
    b = graphgen.powerlaw_edges(50_000, 300_000, True, 9)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    src, dst, w = a
    np.testing.assert_array_equal(src[0::2], dst[1::2])
    np.testing.assert_array_equal(src[1::2], dst[0::2])
    assert src.min() >= 0 and src.max() < 50_000 and (w == 1.0).all()
    c = graphgen.powerlaw_edges(50_000, 300_000, True, 10)[0]
    assert (c != src).mean() > 0.9


def test_powerlaw_is_zipf():
    V, n = 10_000, 2_000_000
    src, _, _ = graphgen.powerlaw_edges(V, n, False, 5)
    cnt = np.sort(np.bincount(src, minlength=V))[::-1].astype(np.float64)
    ranks = np.arange(1, V + 1, dtype=np.float64)
    p = ranks ** -0.8
    p /= p.sum()
    # top ranks within 3% of the law (sampling noise ~0.7%), log-log slope ~ -0.8 over ranks 10..1000
    np.testing.assert_allclose(cnt[:5] / n, p[:5], rtol=0.03)
    slope = np.polyfit(np.log(ranks[10:1000]), np.log(cnt[10:1000]), 1)[0]
    assert abs(slope + 0.8) < 0.05, slope


def test_bipartite_ranges():
    src, dst, _ = graphgen.bipartite_edges(3000, 1000, 100_000, 3)
    assert src.min() >= 0 and src.max() < 3000
    assert dst.min() >= 3000 and dst.max() < 4000


def test_parallel_csr_is_stable_counting_sort():
    """build_graph's radix CSR (threads over > 2^16 slots) equals a stable
    sort by source: per source, targets in push order."""
    from smore_amd import ProNet
    V = 70_000
    src, dst, w = graphgen.powerlaw_edges(V, 400_000, True, 11)
    w = np.random.default_rng(0).random(len(src)) + 0.5
    pn = ProNet(device=-1)
    pn.set_graph_edges(V, src, dst, w)
    off, tgt = pn.csr()
    order = np.argsort(src, kind="stable")
    np.testing.assert_array_equal(tgt, dst[order])
    np.testing.assert_array_equal(off, np.concatenate([[0], np.cumsum(np.bincount(src, minlength=V))]))
