#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE C++.

TEST INFRASTRUCTURE.  Runs oracle/_ref/ref_harness (the reference compiled
unmodified from /root/reference/src by `make -C oracle ref`, with the seeded
random_gen interposed) and stores its outputs as .npz (no pickles) next to the
synthetic edge lists it was run on.  Re-run only in a container that has
/root/reference; the committed fixtures are what the tests read.

    python oracle/gen_golden.py            # regenerate everything
    python oracle/gen_golden.py --only e2e_deepwalk_d128_pl100w   # one end-to-end fixture
"""
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")
TMP = os.path.join(HERE, "_ref", "tmp")

DT = {b"d": np.float64, b"q": np.int64, b"i": np.int32, b"b": np.uint8}


def read_smrf(path):
    out = {}
    with open(path, "rb") as f:
        assert f.read(4) == b"SMRF"
        while True:
            h = f.read(4)
            if not h:
                break
            (nl,) = struct.unpack("<I", h)
            name = f.read(nl).decode()
            dt = DT[f.read(1)]
            (nd,) = struct.unpack("<I", f.read(4))
            shape = struct.unpack("<%dQ" % nd, f.read(8 * nd))
            n = int(np.prod(shape)) if nd else 1
            out[name] = np.frombuffer(f.read(n * np.dtype(dt).itemsize), dtype=dt).reshape(shape).copy()
    return out


def run(*args):
    cmd = [HARNESS] + [str(a) for a in args]
    r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    if r.returncode != 0:
        raise RuntimeError("harness failed: %s\n%s" % (" ".join(cmd), r.stderr.decode()))


def zipf_graph(path, n_vertices, n_lines, seed, weighted, s=0.8):
    """Synthetic power-law edge list (SURVEY.md section 6 law: both endpoints
    ~ Zipf(s) over V, ids randomly permuted, text "v<a> v<b> w")."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, n_vertices + 1) ** s
    p /= p.sum()
    perm = rng.permutation(n_vertices)
    a = perm[rng.choice(n_vertices, n_lines, p=p)]
    b = perm[rng.choice(n_vertices, n_lines, p=p)]
    w = rng.integers(1, 6, n_lines) * 0.5 if weighted else np.ones(n_lines)
    with open(path, "w") as f:
        for x, y, z in zip(a, b, w):
            f.write("v%d v%d %g\n" % (x, y, z))


def bipartite_graph(path, n_users, n_items, n_edges, seed, s=0.8):
    rng = np.random.default_rng(seed)
    pu = 1.0 / np.arange(1, n_users + 1) ** s
    pi = 1.0 / np.arange(1, n_items + 1) ** s
    u = rng.permutation(n_users)[rng.choice(n_users, n_edges, p=pu / pu.sum())]
    i = rng.permutation(n_items)[rng.choice(n_items, n_edges, p=pi / pi.sum())]
    w = rng.integers(1, 6, n_edges).astype(np.float64)
    with open(path, "w") as f:
        for x, y, z in zip(u, i, w):
            f.write("u%d i%d %g\n" % (x, y, z))


TOY = "userA itemA 3\nuserA itemC 5\nuserB itemA 1\nuserB itemB 5\nuserC itemA 4\n"  # README.md:50-56


def changed_rows(T0, T):
    """(trial, row) pairs whose row differs from the starting table."""
    idx, vals = [], []
    for t in range(T.shape[0]):
        rows = np.nonzero(np.any(T[t] != T0, axis=1))[0]
        for r in rows:
            idx.append((t, r))
            vals.append(T[t, r])
    return np.array(idx, dtype=np.int64).reshape(-1, 2), np.array(vals).reshape(len(idx), T0.shape[1])


def main():
    os.makedirs(GOLD, exist_ok=True)
    os.makedirs(TMP, exist_ok=True)
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")

    # ---- edge lists (data fixtures) ---------------------------------------
    graphs = {
        "toy": os.path.join(GOLD, "toy.txt"),
        "pl1k": os.path.join(GOLD, "pl1k.txt"),
        "pl100w": os.path.join(GOLD, "pl100w.txt"),
        "bip": os.path.join(GOLD, "bip.txt"),
    }
    with open(graphs["toy"], "w") as f:
        f.write(TOY)
    zipf_graph(graphs["pl1k"], 1000, 3000, seed=11, weighted=False)
    zipf_graph(graphs["pl100w"], 100, 400, seed=12, weighted=True)
    bipartite_graph(graphs["bip"], 200, 100, 2000, seed=13)
    only = sys.argv[sys.argv.index("--only") + 1:] if "--only" in sys.argv else None
    if only:
        gen_e2e(graphs, 20251015, only)
        gen_pairs(graphs, 20251015, only)
        return

    # ---- G1: AliasMethod on hand-made distributions (src/proNet.cpp:544-620)
    rng = np.random.default_rng(21)
    cases = {
        "single": [3.0],
        "pair": [1.0, 3.0],
        "equal": [2.0] * 7,
        "ties": [1, 1, 2, 2, 4, 4, 8, 8],
        "spike": [0.0] * 9 + [5.0],
        "zeros_mixed": [0, 3, 0, 1, 0, 0, 7, 2, 0, 1],
        "all_zero": [0.0] * 5,
        "random": list(rng.random(257) * 10),
        "powerlaw": list(1.0 / np.arange(1, 2001) ** 0.8 * 1000),
    }
    alias = {}
    for name, d in cases.items():
        fn = os.path.join(TMP, "dist.f64")
        np.asarray(d, dtype=np.float64).tofile(fn)
        run("alias", fn, os.path.join(TMP, "alias.bin"))
        o = read_smrf(os.path.join(TMP, "alias.bin"))
        alias[name + "/dist"] = np.asarray(d, dtype=np.float64)
        alias[name + "/prob"] = o["prob"]
        alias[name + "/alias"] = o["alias"]
    np.savez_compressed(os.path.join(GOLD, "alias_cases.npz"), **alias)

    # ---- G3: fastSigmoid at bucket edges (src/proNet.cpp:52-71) --------------
    edges = np.array([i * 2.0 * 8.0 / 1000 - 8.0 for i in range(1001)])
    xs = np.concatenate([edges, np.nextafter(edges, -np.inf), np.nextafter(edges, np.inf),
                         [-8.0, 8.0, -9.0, 9.0, 0.0, np.nextafter(8.0, 9.0), np.nextafter(-8.0, -9.0)],
                         rng.uniform(-8.5, 8.5, 2000)])
    fn = os.path.join(TMP, "x.f64")
    xs.astype(np.float64).tofile(fn)
    run("sigmoid", fn, os.path.join(TMP, "sig.bin"))
    o = read_smrf(os.path.join(TMP, "sig.bin"))
    np.savez_compressed(os.path.join(GOLD, "sigmoid.npz"), x=o["x"], y=o["y"])

    # ---- G2: graph build + alias tables (src/proNet.cpp:115-236, 410-542) ---
    gcases = [
        ("graph_toy_undir", graphs["toy"], 1, "out_degrees", "degrees"),
        ("graph_toy_dir_nodeg", graphs["toy"], 0, "out_degrees", "no_degrees"),
        ("graph_pl100w", graphs["pl100w"], 1, "out_degrees", "degrees"),
        ("graph_pl1k", graphs["pl1k"], 1, "out_degrees", "degrees"),
        ("graph_bip_indeg", graphs["bip"], 0, "no_degrees", "in_degrees"),
        ("graph_bip_nodeg", graphs["bip"], 0, "out_degrees", "no_degrees"),
    ]
    for name, path, und, vm, nm in gcases:
        out = os.path.join(TMP, name + ".bin")
        run("graph", path, und, vm, nm, out)
        o = read_smrf(out)
        o["meta_undirected"] = np.array(und)
        o["meta_vertex_method"] = np.frombuffer(vm.encode(), np.uint8)
        o["meta_negative_method"] = np.frombuffer(nm.encode(), np.uint8)
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **o)

    # ---- G4: single-sample updates ------------------------------------------
    seed = 20251015
    ucases = [
        ("updates_line2", graphs["pl100w"], 1, "line2", 16, 5, 0.025, 0.0),
        ("updates_line1", graphs["pl100w"], 1, "line1", 16, 5, 0.025, 0.0),
        ("updates_line2_d5", graphs["pl100w"], 1, "line2", 5, 3, 0.05, 0.0),
        ("updates_mf", graphs["bip"], 0, "mf", 12, 5, 0.025, 0.01),
        ("updates_bpr", graphs["bip"], 0, "bpr", 12, 5, 0.025, 0.01),
    ]
    for name, path, und, model, dim, K, alpha, reg in ucases:
        out = os.path.join(TMP, name + ".bin")
        run("updates", path, und, model, dim, K, alpha, reg, seed, 1000, 48, out)
        o = read_smrf(out)
        rec = {k: o[k] for k in ("W0", "C0", "trial", "names", "name_off")}
        rec["W_idx"], rec["W_val"] = changed_rows(o["W0"], o["W"])
        rec["C_idx"], rec["C_val"] = changed_rows(o["C0"], o["C"])
        rec["meta"] = np.array([und, dim, K, seed, 1000, 48], dtype=np.int64)
        rec["meta_f"] = np.array([alpha, reg])
        rec["meta_model"] = np.frombuffer(model.encode(), np.uint8)
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **rec)

    gen_e2e(graphs, seed, None)
    gen_pairs(graphs, seed, None)
    print("golden fixtures written to", GOLD)


def gen_e2e(graphs, seed, only):
    # ---- G5: end-to-end 1-thread runs ----------------------------------------
    e2e = [
        ("e2e_mf_toy", ["mf", graphs["toy"], 5, 1, 5, 0.025, 0.01, seed]),         # config 1
        ("e2e_line2_pl1k", ["line", graphs["pl1k"], 1, 2, 16, 1, 5, 0.025, seed]),
        ("e2e_line1_pl100w", ["line", graphs["pl100w"], 1, 1, 8, 1, 5, 0.025, seed]),
        ("e2e_bpr_bip", ["bpr", graphs["bip"], 8, 1, 0.025, 0.01, seed]),
        ("e2e_deepwalk_pl100w", ["deepwalk", graphs["pl100w"], 1, 8, 2, 10, 3, 2, 0.025, seed]),
        # config 5's model shape: d=128, walk_steps 40, window 5, K 5
        ("e2e_deepwalk_d128_pl100w", ["deepwalk", graphs["pl100w"], 1, 128, 1, 40, 5, 5, 0.025, seed]),
        # Walklets (src/model/Walklets.cpp): window_min 2, window_max 4
        ("e2e_walklets_pl100w", ["walklets", graphs["pl100w"], 1, 8, 2, 10, 2, 4, 2, 0.025, seed]),
        # APP (src/model/APP.cpp): 3 jumping walks per start, jump 0.15
        ("e2e_app_pl100w", ["app", graphs["pl100w"], 1, 8, 2, 3, 0.15, 2, 0.025, seed]),
        # HPE (src/model/HPE.cpp): 10^6 samples, walk_steps 3, K 2, reg 0.01
        ("e2e_hpe_pl100w", ["hpe", graphs["pl100w"], 1, 8, 1, 3, 2, 0.01, 0.025, seed]),
    ]
    for name, args in e2e:
        if only and name not in only:
            continue
        out = os.path.join(TMP, name + ".bin")
        run(*(args + [out]))
        o = read_smrf(out)
        o["meta_args"] = np.frombuffer(" ".join(str(a) for a in args[:1] + args[2:]).encode(), np.uint8)
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **o)


def gen_pairs(graphs, seed, only):
    # ---- caller-supplied pairs: proNet::UpdatePairs (src/proNet.cpp:2741-2753)
    # from fixed starting tables; pairs mix runs of one vertex (the pair kernel
    # keeps W_v in registers over a run), v == c, and uniform ids
    cases = [("pairs_pl100w", 16, 5, 0.025, 7, 3000, 31), ("pairs_pl100w_d7", 7, 3, 0.05, 1 << 33, 1500, 32)]
    for name, dim, K, alpha, unit, n, rs in cases:
        if only and name not in only:
            continue
        rng = np.random.default_rng(rs)
        with open(graphs["pl100w"]) as f:
            V = len({x for line in f for x in line.split()[:2]})
        v = np.empty(n, np.int64)
        c = rng.integers(0, V, n)
        i = 0
        while i < n:
            run_len = int(rng.integers(1, 12))
            v[i:i + run_len] = rng.integers(0, V)
            i += run_len
        same = rng.random(n) < 0.05
        c[same] = v[same]
        fn = os.path.join(TMP, name + ".i64")
        np.stack([v, c], 1).astype(np.int64).tofile(fn)
        out = os.path.join(TMP, name + ".bin")
        run("pairs", graphs["pl100w"], 1, dim, K, alpha, seed, unit, fn, out)
        o = read_smrf(out)
        o["meta"] = np.array([dim, K, seed, unit], dtype=np.uint64)
        o["meta_f"] = np.array([alpha])
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **o)


if __name__ == "__main__":
    main()
