"""Parity of the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.  Needs an MI355X.

Tolerances (DESIGN.md "Parity"):
  * draws (source/target/negatives)            : bit-exact
  * serial mode vs oracle fp32 spec            : bit-exact
  * one sample vs the reference (fp64)         : 1e-5 absolute (north star)
  * atomic scatter (serial) vs oracle fp32     : 1e-6 absolute
  * 10^6-sample end-to-end vs reference (fp64) : 2e-3 max / 2e-4 median abs
    (fp32 rounding plus fastSigmoid bucket flips accumulated over 10^6
    dependent updates; measured 4.3e-4 / 4.6e-5 for the CPU fp32 spec)
"""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEED = 20251015


def gold(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="module")
def smore():
    import smore_amd
    return smore_amd


def make_pair(smore, fname, und, vm="out_degrees", nm="degrees"):
    g = orc.Graph.from_file(os.path.join(GOLDEN, fname), und, vm, nm)
    pn = smore.ProNet(0)
    pn.SetVertexMethod(vm)
    pn.SetNegativeMethod(nm)
    pn.LoadEdgeList(os.path.join(GOLDEN, fname), und)
    return g, pn


def rand_tables(V, dim, n, seed):
    rng = np.random.default_rng(seed)
    return [(rng.random((V, dim), dtype=np.float32) - 0.5) for _ in range(n)]


def padded(T, dim):
    dpad = (dim + 3) // 4 * 4
    out = np.zeros((T.shape[0], dpad), np.float32)
    out[:, :dim] = T
    return out


# ---------------------------------------------------------------- draws
@pytest.mark.parametrize("fname,und,nm,model,K", [("pl1k.txt", 1, "degrees", "line2", 5),
                                                 ("pl100w.txt", 1, "degrees", "line2", 13),
                                                 ("bip.txt", 0, "no_degrees", "bpr", 5),
                                                 ("toy.txt", 0, "no_degrees", "mf", 1)])
def test_sampler_draws_bit_exact(smore, fname, und, nm, model, K):
    g, pn = make_pair(smore, fname, und, nm=nm)
    for begin in (0, (1 << 33) + 12345):
        got = pn.sample_edges(model, begin, 50000, K, SEED)
        want = orc.sample_bpr(g, SEED, begin, 50000) if model == "bpr" else orc.sample_line(g, SEED, begin, 50000, K)
        np.testing.assert_array_equal(got, want)


# ---------------------------------------------------------------- serial == fp32 spec
@pytest.mark.parametrize("model,dim,K", [("line2", 16, 5), ("line2", 64, 5), ("line2", 5, 3), ("line2", 128, 5),
                                         ("line2", 300, 2), ("line2", 64, 0), ("line2", 32, 9), ("line2", 8, 17),
                                         ("line2", 100, 5), ("line2", 20, 4), ("line2", 512, 1), ("line2", 200, 2), ("mf", 36, 3),
                                         ("line1", 16, 5), ("line1", 64, 5), ("mf", 12, 5), ("mf", 64, 5)])
def test_serial_bit_exact_vs_oracle(smore, model, dim, K):
    fname, und, nm = ("bip.txt", 0, "no_degrees") if model == "mf" else ("pl100w.txt", 1, "degrees")
    g, pn = make_pair(smore, fname, und, nm=nm)
    V = g.V
    W0, C0 = rand_tables(V, dim, 2, dim * 7 + K)
    ntab = 2 if model == "line2" else 1
    pn.alloc_tables(dim, ntab)
    pn.set_table(0, W0)
    if ntab == 2:
        pn.set_table(1, C0)
    total, begin, n = 10 ** 6, 12345, 20000
    reg = 0.01 if model == "mf" else 0.0
    pn.train_edges(model, begin, n, total, K, 0.025, reg, SEED, "serial")
    W = padded(W0, dim)
    C = padded(C0, dim) if ntab == 2 else W
    orc.train_edge_f32(g, model, W, C, dim, K, 0.025, reg, total, begin, begin + n, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    if ntab == 2:
        np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


@pytest.mark.parametrize("dim", [8, 20, 64, 128, 300])
def test_serial_bpr_bit_exact_vs_oracle(smore, dim):
    g, pn = make_pair(smore, "bip.txt", 0, nm="no_degrees")
    (W0,) = rand_tables(g.V, dim, 1, dim)
    pn.alloc_tables(dim, 1)
    pn.set_table(0, W0)
    total, begin, n = 10 ** 6, 777, 20000
    pn.train_edges("bpr", begin, n, total, 5, 0.05, 0.0, SEED, "serial")
    W = padded(W0, dim)
    orc.train_bpr_f32(g, W, dim, 0.05, total, begin, begin + n, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])


def test_serial_alpha_schedule_and_skips(smore):
    """Crosses several 10^4 alpha steps with a small total so alpha decays to
    its floor; a directed graph has sources without out-edges -> skips."""
    g, pn = make_pair(smore, "toy.txt", 0)
    (W0, C0) = rand_tables(g.V, 8, 2, 5)
    pn.alloc_tables(8, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    total, n = 50000, 60000
    pn.train_edges("line2", 0, n, total, 2, 0.025, 0.0, SEED, "serial")
    W, C = padded(W0, 8), padded(C0, 8)
    skipped = orc.train_edge_f32(g, "line2", W, C, 8, 2, 0.025, 0.0, total, 0, n, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :8])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :8])
    assert pn.skipped() == skipped


def test_atomic_scatter_single_sample(smore):
    """One sample in atomic mode (a single group): W_v gets W_v + e exactly,
    context rows get orig + (new - orig), within 1 ulp-ish of the spec."""
    g, pn = make_pair(smore, "pl100w.txt", 1)
    W0, C0 = rand_tables(g.V, 64, 2, 11)
    pn.alloc_tables(64, 2)
    for s in (5, 99, 12345):
        pn.set_table(0, W0)
        pn.set_table(1, C0)
        pn.train_edges("line2", s, 1, 10 ** 6, 5, 0.025, 0.0, SEED, "atomic")
        W, C = padded(W0, 64), padded(C0, 64)
        orc.train_edge_f32(g, "line2", W, C, 64, 5, 0.025, 0.0, 10 ** 6, s, s + 1, SEED)
        np.testing.assert_array_equal(pn.get_table(0), W)
        np.testing.assert_allclose(pn.get_table(1), C, atol=1e-6, rtol=0)


# ---------------------------------------------------------------- vs the reference
def _updates_case(name):
    z = gold(name)
    und, dim, K, seed, first, n = (int(x) for x in z["meta"])
    alpha, reg = (float(x) for x in z["meta_f"])
    model = bytes(z["meta_model"]).decode()
    return z, und, dim, K, seed, first, n, alpha, reg, model


@pytest.mark.parametrize("name", ["updates_line2", "updates_line1", "updates_line2_d5", "updates_mf", "updates_bpr"])
def test_single_sample_vs_reference_1e5(smore, name):
    """North-star criterion: one sampled update matches the reference C++
    (fp64) within 1e-5."""
    z, und, dim, K, seed, first, n, alpha, reg, model = _updates_case(name)
    fname, nm = ("bip.txt", "no_degrees") if model in ("mf", "bpr") else ("pl100w.txt", "degrees")
    _, pn = make_pair(smore, fname, und, nm=nm)
    V = z["W0"].shape[0]
    ntab = 2 if model == "line2" else 1
    pn.alloc_tables(dim, ntab)
    Wref = np.repeat(z["W0"][None], n, 0)
    Cref = np.repeat(z["C0"][None], n, 0)
    for (t, r), v in zip(z["W_idx"], z["W_val"]):
        Wref[t, r] = v
    for (t, r), v in zip(z["C_idx"], z["C_val"]):
        Cref[t, r] = v
    for t in range(n):
        s = int(z["trial"][t, 0])
        pn.set_table(0, z["W0"].astype(np.float32))
        if ntab == 2:
            pn.set_table(1, z["C0"].astype(np.float32))
        pn.train_edges(model, s, 1, 10 ** 9, K, alpha, reg, seed, "serial")
        np.testing.assert_allclose(pn.get_table(0), Wref[t], atol=1e-5, rtol=0, err_msg="%s W trial %d" % (name, t))
        if ntab == 2:
            np.testing.assert_allclose(pn.get_table(1), Cref[t], atol=1e-5, rtol=0)
    assert V == pn.MAX_vid


@pytest.mark.parametrize("name,fname,und,nm,model,K,reg,n_off", [
    ("e2e_line2_pl1k", "pl1k.txt", 1, "degrees", "line2", 5, 0.0, 1),
    ("e2e_line1_pl100w", "pl100w.txt", 1, "degrees", "line1", 5, 0.0, 1),
    ("e2e_mf_toy", "toy.txt", 0, "no_degrees", "mf", 5, 0.01, 0),
    ("e2e_bpr_bip", "bip.txt", 0, "no_degrees", "bpr", 5, 0.0, 0)])
def test_end_to_end_vs_reference(smore, name, fname, und, nm, model, K, reg, n_off):
    """10^6-sample 1-thread runs of the reference (interposed RNG, glibc Init)."""
    z = gold(name)
    _, pn = make_pair(smore, fname, und, nm=nm)
    V, dim = z["W0"].shape
    ntab = 2 if model == "line2" else 1
    pn.alloc_tables(dim, ntab)
    pn.init_table_glibc(0, 0)                      # the reference's own Init
    np.testing.assert_array_equal(pn.get_table(0), z["W0"].astype(np.float32))
    if ntab == 2:
        pn.zero_table(1)
    total = 10 ** 6
    pn.train_edges(model, 0, total - n_off, total, K, 0.025, reg, SEED, "serial")
    for t, key in ((0, "W"), (1, "C")):
        if t >= ntab:
            break
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 2e-3 and np.median(d) < 2e-4, (key, d.max(), np.median(d))


# ---------------------------------------------------------------- DeepWalk
@pytest.mark.parametrize("dim,K,window,steps", [(8, 2, 3, 10), (64, 5, 5, 40), (20, 1, 2, 7)])
def test_deepwalk_serial_bit_exact_vs_oracle(smore, dim, K, window, steps):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V = g.V
    W0, C0 = rand_tables(V, dim, 2, dim + K)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(V, 2, 77)
    pn.train_deepwalk(0, 2 * V, 2, steps, window, K, 0.025, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.train_deepwalk_f32(g, W, C, dim, 2, steps, window, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_deepwalk_end_to_end_vs_reference(smore):
    z = gold("e2e_deepwalk_pl100w")
    _, pn = make_pair(smore, "pl100w.txt", 1)
    V, dim = z["W0"].shape
    pn.alloc_tables(dim, 2)
    pn.init_table_glibc(0, 0)
    pn.init_table_glibc(1, V * dim)
    np.testing.assert_array_equal(pn.get_table(1), z["C0"].astype(np.float32))
    order = smore.deepwalk_order(V, 2, 2 * V * dim)
    pn.train_deepwalk(0, 2 * V, 2, 10, 3, 2, 0.025, SEED, order, "serial")
    for t, key in ((0, "W"), (1, "C")):
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 2e-3 and np.median(d) < 2e-4, (key, d.max(), np.median(d))


@pytest.mark.parametrize("mode", ["atomic", "hogwild"])
def test_deepwalk_parallel_runs(smore, mode):
    g, pn = make_pair(smore, "pl1k.txt", 1)
    pn.alloc_tables(32, 2)
    pn.init_table_glibc(0, 0)
    pn.init_table_glibc(1, g.V * 32)
    order = smore.deepwalk_order(g.V, 3, 2 * g.V * 32)
    pn.train_deepwalk(0, 3 * g.V, 3, 20, 5, 5, 0.025, SEED, order, mode)
    assert np.isfinite(pn.get_table(0)).all() and np.isfinite(pn.get_table(1)).all()


# ---------------------------------------------------------------- Hogwild quality
def _auc(W, C, g, rng, n=20000):
    src = np.repeat(np.arange(g.V), np.diff(g.offsets))
    pick = rng.integers(0, g.E, n)
    pos = np.einsum("ij,ij->i", W[src[pick]], C[g.targets[pick]])
    neg = np.einsum("ij,ij->i", W[rng.integers(0, g.V, n)], C[rng.integers(0, g.V, n)])
    return (pos[:, None] > neg[None, :2000]).mean()


@pytest.mark.parametrize("mode", ["atomic", "hybrid"])
def test_hogwild_quality_matches_serial(smore, mode):
    """The lossless scatters (atomic, hybrid) train as well as the serial
    order.  Plain-store Hogwild is NOT in this list: on a 1k-vertex graph the
    ~20k samples a full GPU keeps in flight rewrite the same rows and lose
    most updates (DESIGN.md "Scatter modes"); test_hogwild_store_runs covers it."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    total = 2 * 10 ** 6
    res = {}
    for m in ("serial", mode):
        pn.alloc_tables(32, 2)
        pn.init_table_glibc(0, 0)
        pn.zero_table(1)
        pn.train_edges("line2", 0, total - 1, total, 5, 0.025, 0.0, SEED, m)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[m] = _auc(W, C, g, np.random.default_rng(0))
    assert res["serial"] > 0.8
    assert abs(res[mode] - res["serial"]) < 0.02, res


def test_hogwild_store_runs(smore):
    """Plain-store Hogwild on a tiny graph: finite, and trains at all (the
    lost updates make it worse than serial, by design of that mode)."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    total = 2 * 10 ** 6
    pn.alloc_tables(32, 2)
    pn.init_table_glibc(0, 0)
    pn.zero_table(1)
    pn.train_edges("line2", 0, total - 1, total, 5, 0.025, 0.0, SEED, "hogwild")
    W, C = pn.get_table(0), pn.get_table(1)
    assert np.isfinite(W).all() and np.isfinite(C).all()
    assert _auc(W, C, g, np.random.default_rng(0)) > 0.55


def test_glibc_init_matches_reference(smore):
    z = gold("e2e_line2_pl1k")
    _, pn = make_pair(smore, "pl1k.txt", 1)
    pn.alloc_tables(16, 2)
    pn.init_table_glibc(0, 0)
    pn.init_table_glibc(1, 1000 * 16)
    np.testing.assert_array_equal(pn.get_table(0), z["W0"].astype(np.float32))
    assert not np.array_equal(pn.get_table(1), pn.get_table(0))


def test_save_weights_format(smore, tmp_path):
    _, pn = make_pair(smore, "toy.txt", 1)
    pn.alloc_tables(5, 1)
    pn.init_table_glibc(0, 0)
    p = str(tmp_path / "rep.txt")
    pn.save_weights(0, p, 0)
    lines = open(p).read().splitlines()
    assert lines[0] == "6 5"
    assert lines[1].split()[0] == "userA" and len(lines[1].split()) == 6
    W = pn.get_table(0)
    np.testing.assert_allclose([float(x) for x in lines[1].split()[1:]], W[0], rtol=1e-5)


def test_replica_sync_rccl_single_rank(smore):
    """RCCL all-reduce path of smore_amd/dist.py (fused HIP passes,
    replica_sync.hip) on the context's own device tables (zero-copy views),
    world size 1: W_snap + sum(delta) == W, synchronous and overlapped."""
    import socket

    import torch
    import torch.distributed as dist
    from smore_amd.dist import ReplicaSync, table_tensor
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        _, pn = make_pair(smore, "pl1k.txt", 1)
        pn.alloc_tables(64, 2)
        pn.init_table_glibc(0, 0)
        pn.zero_table(1)
        sync = ReplicaSync(pn)
        t = table_tensor(pn, 0)
        assert t.data_ptr() == pn.table_device(0)[0]
        pn.train_edges("line2", 0, 100000, 10 ** 6, 5, 0.025, 0.0, SEED, "atomic")
        before = [pn.get_table(0), pn.get_table(1)]
        sync.allreduce()
        torch.cuda.synchronize()
        np.testing.assert_allclose(pn.get_table(0), before[0], atol=1e-6)
        np.testing.assert_allclose(pn.get_table(1), before[1], atol=1e-6)
        assert torch.equal(sync.S[0][:, :64].cpu(), torch.from_numpy(pn.get_table(0)))
        # overlapped schedule: a step runs while the exchange is in flight
        pn.train_edges("line2", 100000, 100000, 10 ** 6, 5, 0.025, 0.0, SEED, "atomic", sync=False)
        sync.begin()
        torch.cuda.synchronize()
        at_begin = pn.get_table(1)
        np.testing.assert_array_equal(sync.S[1][:, :64].cpu().numpy(), at_begin)
        pn.train_edges("line2", 200000, 100000, 10 ** 6, 5, 0.025, 0.0, SEED, "atomic", sync=False)
        sync.end()             # world 1: adds (R - D) = 0 to T and S
        torch.cuda.synchronize()
        assert np.isfinite(pn.get_table(0)).all()
        np.testing.assert_array_equal(sync.S[1][:, :64].cpu().numpy(), at_begin)
        assert not np.array_equal(pn.get_table(1), at_begin)
        # begin() while an exchange is in flight: the fused end+begin pass
        sync.begin()
        pn.train_edges("line2", 300000, 100000, 10 ** 6, 5, 0.025, 0.0, SEED, "atomic", sync=False)
        sync.begin()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(sync.S[0][:, :64].cpu().numpy(), pn.get_table(0))
        sync.end()
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------- hybrid scatter (tagged ids)
def test_hybrid_tags_keep_draws_and_serial_bit_exact(smore):
    """A hybrid run tags hot rows in the device graph's id words; draws and
    every other mode must be unaffected (tags are split off before use)."""
    g, pn = make_pair(smore, "pl100w.txt", 1)
    W0, C0 = rand_tables(g.V, 64, 2, 21)
    pn.alloc_tables(64, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    pn.set_hot_threshold(1e-3)                     # many hot rows
    pn.train_edges("line2", 0, 200000, 10 ** 6, 5, 0.025, 0.0, SEED, "hybrid")
    hw, hc = pn.hot_rows()
    assert 0 < hw <= g.V and 0 < hc <= g.V
    assert np.isfinite(pn.get_table(0)).all()
    np.testing.assert_array_equal(pn.sample_edges("line2", 7, 20000, 5, SEED), orc.sample_line(g, SEED, 7, 20000, 5))
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    pn.train_edges("line2", 12345, 20000, 10 ** 6, 5, 0.025, 0.0, SEED, "serial")
    W, C = padded(W0, 64), padded(C0, 64)
    orc.train_edge_f32(g, "line2", W, C, 64, 5, 0.025, 0.0, 10 ** 6, 12345, 12345 + 20000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W)
    np.testing.assert_array_equal(pn.get_table(1), C)


@pytest.mark.parametrize("tau", [0.0, 1e30])
def test_hybrid_single_sample(smore, tau):
    """tau 0: every row hot (atomic deltas); tau huge: no row hot (stores)."""
    g, pn = make_pair(smore, "pl100w.txt", 1)
    W0, C0 = rand_tables(g.V, 64, 2, 12)
    pn.alloc_tables(64, 2)
    pn.set_hot_threshold(tau)
    for s in (5, 99, 12345):
        pn.set_table(0, W0)
        pn.set_table(1, C0)
        pn.train_edges("line2", s, 1, 10 ** 6, 5, 0.025, 0.0, SEED, "hybrid")
        W, C = padded(W0, 64), padded(C0, 64)
        orc.train_edge_f32(g, "line2", W, C, 64, 5, 0.025, 0.0, 10 ** 6, s, s + 1, SEED)
        np.testing.assert_allclose(pn.get_table(0), W, atol=1e-6, rtol=0)
        np.testing.assert_allclose(pn.get_table(1), C, atol=1e-6, rtol=0)


def test_hybrid_deepwalk_and_bpr_run(smore):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    pn.alloc_tables(32, 2)
    pn.init_table_uniform(0, 1)
    pn.zero_table(1)
    pn.set_hot_threshold(1e-3)
    order = orc.deepwalk_order(g.V, 1, 0)
    pn.train_deepwalk(0, g.V, 1, 20, 3, 5, 0.025, SEED, order, "hybrid")
    assert np.isfinite(pn.get_table(0)).all() and np.isfinite(pn.get_table(1)).all()
    gb, pb = make_pair(smore, "bip.txt", 0, nm="no_degrees")
    pb.alloc_tables(16, 1)
    pb.init_table_uniform(0, 1)
    pb.set_hot_threshold(1e-3)
    pb.train_edges("bpr", 0, 100000, 100000, 5, 0.05, 0.0, SEED, "hybrid")
    assert np.isfinite(pb.get_table(0)).all()


def test_chunked_overlapped_draws(smore):
    """Calls larger than one record chunk: the draws of chunk k+1 run on a
    second stream during the update of chunk k (double-buffered records).
    Serial mode is unaffected (one chunk); a chunked atomic run trains as
    well as an unchunked one and leaves finite tables."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    total = 2 * 10 ** 6
    res = {}
    for chunk in (None, "65536"):
        if chunk:
            os.environ["SMORE_DRAW_CHUNK"] = chunk
        try:
            pn.alloc_tables(32, 2)
            pn.init_table_glibc(0, 0)
            pn.zero_table(1)
            pn.train_edges("line2", 0, total - 1, total, 5, 0.025, 0.0, SEED, "atomic")
            ph = pn.last_phase_ms()
            W, C = pn.get_table(0), pn.get_table(1)
        finally:
            os.environ.pop("SMORE_DRAW_CHUNK", None)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        assert ph is not None and ph[2] == (1 if chunk is None else -(-(total - 1) // int(chunk)))
        res[chunk] = _auc(W, C, g, np.random.default_rng(0))
    assert abs(res[None] - res["65536"]) < 0.02, res


@pytest.mark.parametrize("fmt,spec", [(0, "%g"), (1, "%.6f")])
def test_save_weights_parallel_text_is_exact(smore, tmp_path, fmt, spec):
    """The multi-threaded saver writes exactly the sequential printf text
    (C++ ostream default / Go %.6f), over more rows than one thread block."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    dim = 7
    pn.alloc_tables(dim, 1)
    W0 = (np.random.default_rng(4).standard_normal((g.V, dim)) * 10.0 ** np.random.default_rng(5).integers(
        -6, 4, (g.V, dim))).astype(np.float32)
    pn.set_table(0, W0)
    p = str(tmp_path / "rep.txt")
    os.environ["SMORE_SAVE_THREADS"] = "3"
    try:
        pn.save_weights(0, p, fmt)
    finally:
        del os.environ["SMORE_SAVE_THREADS"]
    expect = ["%d %d" % (g.V, dim)]
    for v in range(g.V):
        expect.append(g.names[v] + "".join(" " + spec % float(x) for x in W0[v]))
    assert open(p).read() == "\n".join(expect) + "\n"


def test_save_weights_raw_roundtrip(smore, tmp_path):
    """fmt 2: raw fp32 dump, read back bit-exactly by load_pretrain."""
    _, pn = make_pair(smore, "pl100w.txt", 1)
    dim = 13
    pn.alloc_tables(dim, 2)
    W0 = np.random.default_rng(9).standard_normal((pn.MAX_vid, dim)).astype(np.float32)
    pn.set_table(0, W0)
    p = str(tmp_path / "w.raw")
    pn.save_weights(0, p, 2)
    assert os.path.getsize(p) == 24 + 4 * W0.size
    pn.zero_table(1)
    pn.load_pretrain(1, p)
    np.testing.assert_array_equal(pn.get_table(1), W0)
