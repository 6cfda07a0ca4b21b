"""Walklets, APP and HPE on the GPU (other UpdatePair consumers
on the pair-record path).  Needs an MI355X.

Tolerances:
  * serial mode vs the oracle's fp32 spec                 : bit-exact
  * serial mode vs the reference's 1-thread fp64 run      : 1e-5 absolute (north star)
  * Hogwild modes vs serial (held-out training loss)      : within 2 %
  * HPE 10^6-sample run vs the reference (fp64)          : 2e-3 max / 2e-4 median
    (accumulated fp32 rounding, as DeepWalk's end-to-end test)
The reference fixtures (tests/golden/e2e_{walklets,app,hpe}_pl100w.npz) come
from oracle/_ref/ref_harness, the reference's Walklets.cpp / APP.cpp / HPE.cpp
compiled unmodified (oracle/gen_golden.py).
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as orc
from tests.conftest import GOLDEN, ROOT
from tests.test_gpu_parity import SEED, gold, make_pair, padded, rand_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def smore():
    import smore_amd
    return smore_amd


# ---------------------------------------------------------------- Walklets
@pytest.mark.parametrize("dim,K,wmin,wmax,steps", [(8, 2, 2, 4, 10), (64, 5, 2, 5, 40), (20, 1, 0, 3, 7),
                                                  (128, 5, 1, 1, 12), (32, 0, 3, 6, 5)])
def test_walklets_serial_bit_exact_vs_oracle(smore, dim, K, wmin, wmax, steps):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V = g.V
    W0, C0 = rand_tables(V, dim, 2, dim + K + wmin)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    pn.train_walklets(0, 2 * V, 2, steps, wmin, wmax, K, 0.025, SEED, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.train_walklets_f32(g, W, C, dim, 2, steps, wmin, wmax, K, 0.025, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_walklets_split_calls_equal_one_call(smore):
    """Walk ranges are independent units: [0, a) then [a, n) == [0, n) (serial)."""
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V, dim = g.V, 16
    W0, C0 = rand_tables(V, dim, 2, 5)
    res = []
    for cuts in ([0, 2 * V], [0, 37, V + 5, 2 * V]):
        pn.alloc_tables(dim, 2)
        pn.set_table(0, W0)
        pn.set_table(1, C0)
        for a, b in zip(cuts[:-1], cuts[1:]):
            pn.train_walklets(a, b, 2, 10, 2, 4, 3, 0.025, SEED, "serial")
        res.append((pn.get_table(0), pn.get_table(1)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_walklets_end_to_end_vs_reference(smore):
    z = gold("e2e_walklets_pl100w")
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V, dim = z["W0"].shape
    pn.alloc_tables(dim, 2)
    pn.set_table(0, z["W0"].astype(np.float32))
    pn.set_table(1, z["C0"].astype(np.float32))
    pn.train_walklets(0, 2 * V, 2, 10, 2, 4, 2, 0.025, SEED, "serial")
    for t, key in ((0, "W"), (1, "C")):
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 1e-5, (key, d.max())


# ---------------------------------------------------------------- APP
@pytest.mark.parametrize("dim,K,jump,st", [(8, 2, 0.15, 3), (64, 5, 0.15, 10), (20, 1, 0.5, 1), (128, 5, 1.0, 2),
                                           (32, 0, 0.05, 4)])
def test_app_serial_bit_exact_vs_oracle(smore, dim, K, jump, st):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V = g.V
    W0, C0 = rand_tables(V, dim, 2, dim + K + st)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    order = orc.deepwalk_order(V, 2, 91)
    pn.train_app(0, 2 * V * st, 2, st, jump, K, 0.025, SEED, order, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.train_app_f32(g, W, C, dim, 2, st, jump, K, 0.025, SEED, order)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_app_end_to_end_vs_reference(smore):
    z = gold("e2e_app_pl100w")
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V, dim = z["W0"].shape
    order = orc.deepwalk_order(V, 2, 2 * V * dim)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, z["W0"].astype(np.float32))
    pn.set_table(1, z["C0"].astype(np.float32))
    pn.train_app(0, 2 * V * 3, 2, 3, 0.15, 2, 0.025, SEED, order, "serial")
    for t, key in ((0, "W"), (1, "C")):
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 1e-5, (key, d.max())


def test_app_rejects_zero_jump(smore):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    pn.alloc_tables(8, 2)
    order = orc.deepwalk_order(g.V, 1, 0)
    with pytest.raises(Exception):
        pn.train_app(0, g.V, 1, 1, 0.0, 2, 0.025, SEED, order, "serial")


# ---------------------------------------------------------------- HPE
@pytest.mark.parametrize("dim,K,ws,reg", [(8, 2, 3, 0.01), (64, 5, 5, 0.01), (20, 1, 1, 0.0), (128, 5, 2, 0.1),
                                          (32, 0, 4, 0.01)])
def test_hpe_serial_bit_exact_vs_oracle(smore, dim, K, ws, reg):
    g, pn = make_pair(smore, "pl100w.txt", 1)
    V = g.V
    W0, C0 = rand_tables(V, dim, 2, dim + K + ws)
    pn.alloc_tables(dim, 2)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    total = 10 ** 6
    pn.train_hpe(1000, 20000, total, ws, K, reg, 0.025, SEED, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    orc.train_hpe_f32(g, W, C, dim, ws, K, reg, 0.025, total, 1000, 21000, SEED)
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_hpe_directed_bipartite_serial(smore):
    """A directed bipartite graph (items are sinks: community walks end early);
    serial bit-exact, skipped-sample count equal to the oracle's."""
    g, pn = make_pair(smore, "bip.txt", 0)
    dim = 8
    pn.alloc_tables(dim, 2)
    W0, C0 = rand_tables(g.V, dim, 2, 3)
    pn.set_table(0, W0)
    pn.set_table(1, C0)
    before = pn.skipped()
    pn.train_hpe(0, 30000, 10 ** 6, 3, 2, 0.01, 0.025, SEED, "serial")
    W, C = padded(W0, dim), padded(C0, dim)
    sk = orc.train_hpe_f32(g, W, C, dim, 3, 2, 0.01, 0.025, 10 ** 6, 0, 30000, SEED)
    assert pn.skipped() - before == sk
    np.testing.assert_array_equal(pn.get_table(0), W[:, :dim])
    np.testing.assert_array_equal(pn.get_table(1), C[:, :dim])


def test_hpe_end_to_end_vs_reference(smore):
    z = gold("e2e_hpe_pl100w")
    g, pn = make_pair(smore, "pl100w.txt", 1)
    pn.alloc_tables(z["W0"].shape[1], 2)
    pn.set_table(0, z["W0"].astype(np.float32))
    pn.set_table(1, z["C0"].astype(np.float32))
    total = 10 ** 6
    pn.train_hpe(0, total, total, 3, 2, 0.01, 0.025, SEED, "serial")
    for t, key in ((0, "W"), (1, "C")):
        d = np.abs(pn.get_table(t) - z[key])
        assert d.max() < 2e-3 and np.median(d) < 2e-4, (key, d.max(), np.median(d))


# ---------------------------------------------------------------- Hogwild modes
def _heldout(g, model, order, K):
    """Held-out training pairs of the model with K negatives from the negative
    sampler: Walklets -- graph edges (its distance-1 pairs); APP -- (start,
    jumping-walk end) pairs drawn with another seed."""
    draws = orc.sample_line(g, SEED + 7, 0, 20000, K)
    negs = draws[:, 2:]
    if model == "walklets":
        keep = draws[:, 1] >= 0
        return draws[keep, 0], draws[keep, 1], negs[keep]
    if model == "hpe":   # UpdatePair(v2, v1): the reversed edges
        keep = draws[:, 1] >= 0
        return draws[keep, 1], draws[keep, 0], negs[keep]
    vc = orc.app_pairs(g, 4, 50, 0.15, SEED + 1, order, 0, 20000)
    return vc[:, 0], vc[:, 1], negs


def _loss(W, C, pv, pc, negs):
    """The models' own objective: -log s(W_v.C_c) - sum_k log s(-W_v.C_nk)."""
    Wv = W[pv].astype(np.float64)
    loss = np.logaddexp(0.0, -np.einsum("ij,ij->i", Wv, C[pc].astype(np.float64)))
    for k in range(negs.shape[1]):
        loss += np.logaddexp(0.0, np.einsum("ij,ij->i", Wv, C[negs[:, k]].astype(np.float64)))
    return float(loss.mean())


@pytest.mark.parametrize("model", ["walklets", "app", "hpe"])
def test_parallel_modes_train_like_serial(smore, model):
    """atomic and hybrid (tau 0.3: a mix of hot and cold rows) reach the serial
    order's held-out loss within 2 %; plain-store Hogwild runs and stays finite."""
    g, pn = make_pair(smore, "pl1k.txt", 1)
    dim, K = 32, 5
    order = orc.deepwalk_order(g.V, 4, 0)
    held = _heldout(g, model, order, K)
    res = {}
    for mode in ("serial", "atomic", "hybrid", "hogwild"):
        pn.alloc_tables(dim, 2)
        pn.init_table_glibc(0, 0)
        pn.init_table_glibc(1, g.V * dim)   # both tables random (DeepWalk/APP Init)
        pn.set_hot_threshold(0.3)
        if model == "walklets":
            pn.train_walklets(0, 4 * g.V, 4, 20, 1, 4, K, 0.025, SEED, mode)
        elif model == "hpe":
            pn.train_hpe(0, 10 ** 6, 10 ** 6, 3, K, 0.01, 0.025, SEED, mode)
        else:
            pn.train_app(0, 4 * g.V * 50, 4, 50, 0.15, K, 0.025, SEED, order, mode)
        W, C = pn.get_table(0), pn.get_table(1)
        assert np.isfinite(W).all() and np.isfinite(C).all()
        res[mode] = _loss(W, C, *held)
    assert res["serial"] < 0.9 * (1 + K) * np.log(2.0), res   # well below the untrained loss
    for mode in ("atomic", "hybrid"):
        assert abs(res[mode] - res["serial"]) <= 0.02 * res["serial"], res


# ---------------------------------------------------------------- CLIs
BIN = os.path.join(ROOT, "smore_amd", "bin")


def _run(tool, *args):
    r = subprocess.run([os.path.join(BIN, tool)] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _read_rep(path):
    lines = open(path).read().splitlines()
    n, d = map(int, lines[0].split())
    vals = np.array([[float(x) for x in ln.split()[1:]] for ln in lines[1:]])
    assert vals.shape == (n, d)
    return vals


@pytest.mark.parametrize("tool,args,fixture", [
    ("walklets", ["-walk_times", 2, "-walk_steps", 10, "-window_min", 2, "-window_max", 4, "-negative_samples", 2],
     "e2e_walklets_pl100w"),
    ("app", ["-walk_times", 2, "-sample_times", 3, "-jump", 0.15, "-negative_samples", 2], "e2e_app_pl100w"),
    ("hpe", ["-sample_times", 1, "-walk_steps", 3, "-negative_samples", 2, "-reg", 0.01], "e2e_hpe_pl100w"),
])
def test_cli_vs_reference(tmp_path, tool, args, fixture):
    z = gold(fixture)
    out = str(tmp_path / "rep.txt")
    log = _run(tool, "-train", os.path.join(GOLDEN, "pl100w.txt"), "-save", out, "-undirected", 1,
               "-dimensions", 8, "-alpha", 0.025, "-threads", 1, "-seed", SEED, "-mode", "serial", *args)
    assert "Start Training:" in log
    d = np.abs(_read_rep(out) - z["W"])
    if tool == "hpe":   # 10^6 samples: accumulated fp32 rounding (as DeepWalk's CLI test)
        assert d.max() < 2e-3 and np.median(d) < 2e-4, (d.max(), np.median(d))
    else:
        assert d.max() < 2e-5, d.max()   # 1e-5 arithmetic + the 6-significant-digit text format
