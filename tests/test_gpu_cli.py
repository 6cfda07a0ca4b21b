"""The flag-compatible C++ CLIs (smore_amd/bin/*) end to end on the GPU,
against the reference's own 1-thread runs (golden fixtures)."""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "smore_amd", "bin")
SEED = "20251015"


def run(tool, *args):
    r = subprocess.run([os.path.join(BIN, tool)] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def read_rep(path):
    lines = open(path).read().splitlines()
    n, d = map(int, lines[0].split())
    names, vals = [], []
    for ln in lines[1:]:
        p = ln.split()
        names.append(p[0])
        vals.append([float(x) for x in p[1:]])
    assert len(names) == n and all(len(v) == d for v in vals)
    return names, np.array(vals)


def names_of(z):
    raw = bytes(z["names"])
    off = z["name_off"]
    return [raw[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]


def check(z, key, path, tol_max=2e-3, tol_med=2e-4):
    names, W = read_rep(path)
    assert names == names_of(z)
    d = np.abs(W - z[key])
    assert d.max() < tol_max and np.median(d) < tol_med, (d.max(), np.median(d))


def test_cli_line_vs_reference(tmp_path):
    z = np.load(os.path.join(GOLDEN, "e2e_line2_pl1k.npz"))
    out = str(tmp_path / "rep.txt")
    log = run("line", "-train", os.path.join(GOLDEN, "pl1k.txt"), "-save", out, "-undirected", 1, "-order", 2,
              "-dimensions", 16, "-sample_times", 1, "-negative_samples", 5, "-alpha", 0.025, "-threads", 1,
              "-seed", SEED, "-mode", "serial")
    assert "Start Training:" in log and "Save to <" in log
    check(z, "W", out)


def test_cli_mf_toy_config1(tmp_path):
    """BASELINE config 1: README toy, MF d=5."""
    z = np.load(os.path.join(GOLDEN, "e2e_mf_toy.npz"))
    out = str(tmp_path / "rep.txt")
    run("mf", "-train", os.path.join(GOLDEN, "toy.txt"), "-save", out, "-dimensions", 5, "-sample_times", 1,
        "-negative_samples", 5, "-alpha", 0.025, "-reg", 0.01, "-seed", SEED, "-mode", "serial")
    check(z, "W", out, 1e-4, 2e-5)


def test_cli_bpr_vs_reference(tmp_path):
    z = np.load(os.path.join(GOLDEN, "e2e_bpr_bip.npz"))
    out = str(tmp_path / "rep.txt")
    run("bpr", "-train", os.path.join(GOLDEN, "bip.txt"), "-save", out, "-dimensions", 8, "-sample_times", 1,
        "-alpha", 0.025, "-seed", SEED, "-mode", "serial")
    check(z, "W", out, 5e-3, 5e-4)


def test_cli_deepwalk_vs_reference(tmp_path):
    z = np.load(os.path.join(GOLDEN, "e2e_deepwalk_pl100w.npz"))
    out = str(tmp_path / "rep.txt")
    run("deepwalk", "-train", os.path.join(GOLDEN, "pl100w.txt"), "-save", out, "-undirected", 1, "-dimensions", 8,
        "-walk_times", 2, "-walk_steps", 10, "-window_size", 3, "-negative_samples", 2, "-alpha", 0.025,
        "-seed", SEED, "-mode", "serial")
    check(z, "W", out)


def test_cli_deepwalk_warm_start(tmp_path):
    """-load_v overwrites matching rows before training (walk_times 0 -> no
    updates), so the saved table equals the warm-start file."""
    z = np.load(os.path.join(GOLDEN, "e2e_deepwalk_pl100w.npz"))
    warm = str(tmp_path / "warm.txt")
    names = names_of(z)
    rng = np.random.default_rng(5)
    vals = rng.random((len(names), 8)) - 0.5
    with open(warm, "w") as f:
        f.write("%d 8\n" % len(names))
        for n, v in zip(names, vals):
            f.write(n + " " + " ".join("%.6f" % x for x in v) + "\n")
    out = str(tmp_path / "rep.txt")
    run("deepwalk", "-train", os.path.join(GOLDEN, "pl100w.txt"), "-save", out, "-dimensions", 8,
        "-walk_times", 1, "-walk_steps", 0, "-window_size", 1, "-negative_samples", 0, "-alpha", 0.0,
        "-load_v", warm, "-mode", "serial")
    got_names, W = read_rep(out)
    assert got_names == names
    np.testing.assert_allclose(W, vals, atol=2e-6)


def test_cli_usage_banner():
    for tool in ("line", "mf", "bpr", "deepwalk"):
        r = subprocess.run([os.path.join(BIN, tool)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and "Usage:" in r.stdout
