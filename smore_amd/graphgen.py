"""Seeded synthetic power-law graphs for the benchmark configs:
both endpoints ~ Zipf(s=0.8) over V, ids randomly permuted, weight 1.0.
Undirected lines are pushed as v1->v2 then v2->v1 (the reference loader's
order, src/proNet.cpp:208-215)."""
import numpy as np

CONFIGS = {
    # name: (V, lines, undirected, seed)
    "c2": (1_000_000, 20_000_000, True, 2),      # LINE-2 1M / 20M, d=64
    "c4": (10_000_000, 200_000_000, True, 4),    # LINE-2 10M / 200M, d=64
    "small": (100_000, 2_000_000, True, 1),
}


def zipf_endpoints(V, n, seed, s=0.8, chunk=1 << 24):
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(1.0 / np.arange(1, V + 1, dtype=np.float64) ** s)
    cdf /= cdf[-1]
    perm = rng.permutation(V).astype(np.int32)
    out = np.empty(n, np.int32)
    for b in range(0, n, chunk):
        e = min(n, b + chunk)
        idx = np.searchsorted(cdf, rng.random(e - b), side="right")
        np.minimum(idx, V - 1, out=idx)
        out[b:e] = perm[idx]
    return out


def powerlaw_edges(V, lines, undirected=True, seed=2):
    """(src, dst, w) directed edge slots in push order."""
    a = zipf_endpoints(V, lines, seed * 2 + 1)
    b = zipf_endpoints(V, lines, seed * 2 + 2)
    if undirected:
        src = np.empty(2 * lines, np.int32)
        dst = np.empty(2 * lines, np.int32)
        src[0::2], src[1::2] = a, b
        dst[0::2], dst[1::2] = b, a
    else:
        src, dst = a, b
    return src, dst, np.ones(len(src), np.float64)


def config_edges(name):
    V, lines, und, seed = CONFIGS[name]
    return V, powerlaw_edges(V, lines, und, seed)
