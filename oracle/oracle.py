"""ctypes front-end of the CPU oracle (oracle/smore_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the smore_amd product package.

Also holds a tiny pure-Python edge-list reader that restates the reference
loader's id assignment (src/proNet.cpp:115-236: vertex ids in first-appearance
order, directed edge slots pushed per line as v1->v2 then v2->v1 when
undirected), used to build test graphs for the oracle.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

VM = {"out_degrees": 0, "no_degrees": 1, "degrees": 2}
NM = {"degrees": 0, "in_degrees": 1, "no_degrees": 2}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


P = C.c_void_p
i64, u64, i32, u32, dbl = C.c_int64, C.c_uint64, C.c_int32, C.c_uint32, C.c_double


def _declare(L):
    L.orc_philox4x32_10.argtypes = [P, P, P]
    L.orc_word.restype = u32
    L.orc_word.argtypes = [u64, u32, u64, u32]
    L.orc_words.argtypes = [u64, u32, u64, u32, P]
    L.orc_glibc_rand_fill.argtypes = [u32, P, i64]
    L.orc_alias_cpp.argtypes = [P, i64, P, P]
    L.orc_alias_go.argtypes = [P, i64, dbl, P, P]
    L.orc_alias_encode.argtypes = [P, P, i64, P, P, P]
    L.orc_build_graph.restype = C.c_int
    L.orc_build_graph.argtypes = [i64, i64, P, P, P, C.c_int, C.c_int] + [P] * 10
    L.orc_sample_line.argtypes = [P, u64, u64, u64, C.c_int, P]
    L.orc_sample_bpr.argtypes = [P, u64, u64, u64, P]
    L.orc_sigmoid_table.argtypes = [P]
    L.orc_fast_sigmoid.restype = dbl
    L.orc_fast_sigmoid.argtypes = [dbl]
    L.orc_alpha_line.restype = dbl
    L.orc_alpha_line.argtypes = [u64, dbl, u64]
    L.orc_alpha_walk.restype = dbl
    L.orc_alpha_walk.argtypes = [u64, dbl, u64]
    L.orc_train_edge_f64.restype = C.c_int
    L.orc_train_edge_f64.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64]
    L.orc_train_edge_f64_mt.restype = C.c_int
    L.orc_train_edge_f64_mt.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64, C.c_int]
    L.orc_train_bpr_f64.restype = C.c_int
    L.orc_train_bpr_f64.argtypes = [P, P, C.c_int, dbl, u64, u64, u64, u64]
    L.orc_train_deepwalk_f64.restype = C.c_int
    L.orc_train_deepwalk_f64.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, u64, P]
    L.orc_train_records_f32.restype = C.c_int
    L.orc_train_records_f32.argtypes = [C.c_int, P, P, C.c_int, P, i64, C.c_int, dbl, dbl, u64, u64, C.c_float]
    L.orc_train_edge_f32.restype = C.c_int
    L.orc_train_edge_f32.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64, C.c_int]
    L.orc_train_bpr_f32.restype = C.c_int
    L.orc_train_bpr_f32.argtypes = [P, P, C.c_int, C.c_int, dbl, u64, u64, u64, u64, C.c_int]
    L.orc_train_deepwalk_f32.restype = C.c_int
    L.orc_train_deepwalk_f32.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, u64, P, u64, u64]
    L.orc_lane_width.restype = C.c_int
    L.orc_lane_width.argtypes = [C.c_int]
    L.orc_train_walklets_f64.restype = C.c_int
    L.orc_train_walklets_f64.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, u64]
    L.orc_train_walklets_f32.restype = C.c_int
    L.orc_train_walklets_f32.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl,
                                         u64, u64, u64]
    L.orc_train_app_f64.restype = C.c_int
    L.orc_train_app_f64.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, dbl, C.c_int, dbl, u64, P]
    L.orc_train_app_f32.restype = C.c_int
    L.orc_train_app_f32.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, dbl, C.c_int, dbl, u64, P, u64, u64]
    L.orc_train_hpe_f64.restype = C.c_int
    L.orc_train_hpe_f64.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64]
    L.orc_train_hpe_f32.restype = C.c_int
    L.orc_train_hpe_f32.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64]
    L.orc_app_pairs.restype = None
    L.orc_app_pairs.argtypes = [P, C.c_int, C.c_int, dbl, u64, P, u64, u64, P]
    L.orc_update_pairs_f64.restype = C.c_int
    L.orc_update_pairs_f64.argtypes = [P, P, P, C.c_int, P, P, i64, C.c_int, dbl, u64, u64, C.c_int]
    L.orc_update_pairs_f32.restype = C.c_int
    L.orc_update_pairs_f32.argtypes = [P, P, P, C.c_int, C.c_int, P, P, i64, C.c_int, dbl, u64, u64, C.c_int]


def ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


# --------------------------------------------------------------------- RNG
def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(ptr(c), ptr(k), ptr(o))
    return o


def words(seed, stream, unit, nslots):
    o = np.zeros(nslots, np.uint32)
    lib().orc_words(seed, stream, unit, nslots, ptr(o))
    return o


def glibc_rand(n, seed=1):
    o = np.zeros(n, np.int32)
    lib().orc_glibc_rand_fill(seed, ptr(o), n)
    return o


# --------------------------------------------------------------------- alias
def alias_cpp(dist):
    d = np.ascontiguousarray(dist, dtype=np.float64)
    p = np.zeros(len(d))
    a = np.zeros(len(d), np.int64)
    lib().orc_alias_cpp(ptr(d), len(d), ptr(p), ptr(a))
    return p, a


def alias_go(dist, power):
    d = np.ascontiguousarray(dist, dtype=np.float64)
    p = np.zeros(len(d))
    a = np.zeros(len(d), np.int64)
    lib().orc_alias_go(ptr(d), len(d), power, ptr(p), ptr(a))
    return p, a


def alias_encode(prob, alias, self_ids=None):
    prob = np.ascontiguousarray(prob, np.float64)
    alias = np.ascontiguousarray(alias, np.int64)
    t = np.zeros(len(prob), np.uint32)
    a = np.zeros(len(prob), np.int32)
    s = None if self_ids is None else np.ascontiguousarray(self_ids, np.int32)
    lib().orc_alias_encode(ptr(prob), ptr(alias), len(prob), ptr(s), ptr(t), ptr(a))
    return t, a


# --------------------------------------------------------------------- graph
def read_edgelist(path, undirected):
    """Reference id assignment and edge push order (src/proNet.cpp:165-216)."""
    ids, names = {}, []
    src, dst, w = [], [], []
    with open(path, "rb") as f:
        for line in f:
            parts = line.split()
            if len(parts) < 3:
                continue
            a, b = parts[0].decode(), parts[1].decode()
            try:
                x = float(parts[2])
            except ValueError:       # unparsable weight: skipped (pkg/pronet/pronet.go:139-143)
                continue
            for n in (a, b):
                if n not in ids:
                    ids[n] = len(names)
                    names.append(n)
            src.append(ids[a]); dst.append(ids[b]); w.append(x)
            if undirected:
                src.append(ids[b]); dst.append(ids[a]); w.append(x)
    return names, np.array(src, np.int32), np.array(dst, np.int32), np.array(w, np.float64)


class Graph:
    """CSR + alias tables built by the oracle, encoded like the HIP path."""

    def __init__(self, V, src, dst, w, vertex_method="out_degrees", negative_method="degrees", names=None):
        self.V, self.E = V, len(src)
        self.names = names
        V, E = self.V, self.E
        self.offsets = np.zeros(V + 1, np.int64)
        self.targets = np.zeros(max(E, 1), np.int32)
        self.out_deg = np.zeros(V); self.in_deg = np.zeros(V)
        self.vprob = np.zeros(V); self.valias = np.zeros(V, np.int64)
        self.nprob = np.zeros(V); self.nalias = np.zeros(V, np.int64)
        self.cprob = np.zeros(max(E, 1)); self.calias = np.zeros(max(E, 1), np.int64)
        src = np.ascontiguousarray(src, np.int32); dst = np.ascontiguousarray(dst, np.int32)
        w = np.ascontiguousarray(w, np.float64)
        rc = lib().orc_build_graph(V, E, ptr(src), ptr(dst), ptr(w), VM[vertex_method], NM[negative_method],
                                   ptr(self.offsets), ptr(self.targets), ptr(self.out_deg), ptr(self.in_deg),
                                   ptr(self.vprob), ptr(self.valias), ptr(self.nprob), ptr(self.nalias),
                                   ptr(self.cprob), ptr(self.calias))
        if rc != 0:
            raise ValueError("bad edge list")
        self.vthr, self.valias_enc = alias_encode(self.vprob, self.valias)
        self.nthr, self.nalias_enc = alias_encode(self.nprob, self.nalias)
        self.cthr, self.calias_enc = alias_encode(self.cprob, self.calias, self.targets)
        self._struct = _OrcGraph(V, E, ptr(self.offsets), ptr(self.targets), ptr(self.vthr), ptr(self.valias_enc),
                                 ptr(self.nthr), ptr(self.nalias_enc), ptr(self.cthr), ptr(self.calias_enc))

    @classmethod
    def from_file(cls, path, undirected, vertex_method="out_degrees", negative_method="degrees"):
        names, s, d, w = read_edgelist(path, undirected)
        return cls(len(names), s, d, w, vertex_method, negative_method, names)

    @property
    def ref(self):
        return C.byref(self._struct)


class _OrcGraph(C.Structure):
    _fields_ = [("V", i64), ("E", i64), ("offsets", P), ("targets", P), ("vthr", P), ("valias", P),
                ("nthr", P), ("nalias", P), ("cthr", P), ("calias", P)]


def sample_line(g, seed, begin, count, K):
    o = np.zeros((count, 2 + K), np.int32)
    lib().orc_sample_line(g.ref, seed, begin, count, K, ptr(o))
    return o


def sample_bpr(g, seed, begin, count):
    o = np.zeros((count, 7), np.int32)
    lib().orc_sample_bpr(g.ref, seed, begin, count, ptr(o))
    return o


def sigmoid_table():
    t = np.zeros(1001)
    lib().orc_sigmoid_table(ptr(t))
    return t


def fast_sigmoid(x):
    return lib().orc_fast_sigmoid(float(x))


def alpha_line(c, alpha0, total):
    return lib().orc_alpha_line(c, alpha0, total)


def lane_width(dpad):
    return lib().orc_lane_width(dpad)


MODEL = {"line2": 0, "line1": 1, "mf": 2}


def train_edge_f64(g, model, W, C_, K, alpha0, reg, total, begin, end, seed, threads=1):
    dim = W.shape[1]
    if threads > 1:
        return lib().orc_train_edge_f64_mt(g.ref, MODEL[model], ptr(W), ptr(C_), dim, K, alpha0, reg, total, begin,
                                           end, seed, threads)
    return lib().orc_train_edge_f64(g.ref, MODEL[model], ptr(W), ptr(C_), dim, K, alpha0, reg, total, begin, end, seed)


def train_edge_f32(g, model, W, C_, dim, K, alpha0, reg, total, begin, end, seed, threads=1):
    dpad = W.shape[1]
    return lib().orc_train_edge_f32(g.ref, MODEL[model], ptr(W), ptr(C_), dim, dpad, K, alpha0, reg, total,
                                    begin, end, seed, threads)


def train_records_f32(model, W, C_, rec, K, alpha0, reg, total, begin, neg_scale=1.0):
    """The fp32 update over explicit records {v, c, n_1..n_K} in order
    (orc_train_records_f32); record i has the rate of sample begin + i; the
    negatives step with alpha * neg_scale (a block cell's weight, fp32)."""
    rec = np.ascontiguousarray(rec, np.int32)
    return lib().orc_train_records_f32(MODEL[model], ptr(W), ptr(C_), W.shape[1], ptr(rec), len(rec), K, alpha0, reg,
                                       total, begin, float(neg_scale))


def train_bpr_f64(g, W, alpha0, total, begin, end, seed):
    return lib().orc_train_bpr_f64(g.ref, ptr(W), W.shape[1], alpha0, total, begin, end, seed)


def train_bpr_f32(g, W, dim, alpha0, total, begin, end, seed, threads=1):
    return lib().orc_train_bpr_f32(g.ref, ptr(W), dim, W.shape[1], alpha0, total, begin, end, seed, threads)


def deepwalk_order(V, walk_times, rand_calls_before):
    """Walk start order of DeepWalk::Train (src/model/DeepWalk.cpp:122-131):
    per walk_time a Fisher-Yates pass with glibc rand(), continuing the rand()
    stream after Init consumed `rand_calls_before` values."""
    r = glibc_rand(rand_calls_before + walk_times * V)[rand_calls_before:]
    order = np.zeros(walk_times * V, np.int64)
    k = 0
    for t in range(walk_times):
        keys = np.arange(V, dtype=np.int64)
        for vid in range(V):
            rdx = vid + int(r[k]) % (V - vid)
            k += 1
            keys[vid], keys[rdx] = keys[rdx], keys[vid]
        order[t * V:(t + 1) * V] = keys
    return order


def train_deepwalk_f64(g, W, C_, walk_times, walk_steps, window, K, alpha0, seed, order):
    order = np.ascontiguousarray(order, np.int64)
    return lib().orc_train_deepwalk_f64(g.ref, ptr(W), ptr(C_), W.shape[1], walk_times, walk_steps, window, K,
                                        alpha0, seed, ptr(order))


def train_deepwalk_f32(g, W, C_, dim, walk_times, walk_steps, window, K, alpha0, seed, order, begin=0, end=None):
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V
    return lib().orc_train_deepwalk_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], walk_times, walk_steps, window,
                                        K, alpha0, seed, ptr(order), begin, end)


def train_walklets_f64(g, W, C_, walk_times, walk_steps, wmin, wmax, K, alpha0, seed):
    """Walklets::Train (src/model/Walklets.cpp:24-63), 1 worker, fp64."""
    return lib().orc_train_walklets_f64(g.ref, ptr(W), ptr(C_), W.shape[1], walk_times, walk_steps, wmin, wmax, K,
                                        alpha0, seed)


def train_walklets_f32(g, W, C_, dim, walk_times, walk_steps, wmin, wmax, K, alpha0, seed, begin=0, end=None):
    if end is None:
        end = walk_times * g.V
    return lib().orc_train_walklets_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], walk_times, walk_steps, wmin, wmax,
                                        K, alpha0, seed, begin, end)


def train_app_f64(g, W, C_, walk_times, sample_times, jump, K, alpha0, seed, order):
    """APP::Train (src/model/APP.cpp:59-120), 1 worker, fp64."""
    order = np.ascontiguousarray(order, np.int64)
    return lib().orc_train_app_f64(g.ref, ptr(W), ptr(C_), W.shape[1], walk_times, sample_times, jump, K, alpha0,
                                   seed, ptr(order))


def train_app_f32(g, W, C_, dim, walk_times, sample_times, jump, K, alpha0, seed, order, begin=0, end=None):
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V * sample_times
    return lib().orc_train_app_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], walk_times, sample_times, jump, K,
                                   alpha0, seed, ptr(order), begin, end)


def train_hpe_f64(g, W, C_, walk_steps, K, reg, alpha0, total, begin, end, seed):
    """HPE::Train (src/model/HPE.cpp:94-150), 1 worker, fp64; returns skipped samples."""
    return lib().orc_train_hpe_f64(g.ref, ptr(W), ptr(C_), W.shape[1], walk_steps, K, reg, alpha0, total, begin, end,
                                   seed)


def train_hpe_f32(g, W, C_, dim, walk_steps, K, reg, alpha0, total, begin, end, seed):
    return lib().orc_train_hpe_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], walk_steps, K, reg, alpha0, total, begin,
                                   end, seed)


def app_pairs(g, walk_times, sample_times, jump, seed, order, begin, end):
    """(start, walk end) of APP units [begin, end)."""
    order = np.ascontiguousarray(order, np.int64)
    out = np.zeros((end - begin, 2), np.int32)
    lib().orc_app_pairs(g.ref, walk_times, sample_times, jump, seed, ptr(order), begin, end, ptr(out))
    return out


PAIR_BLOCK = 1 << 20


def update_pairs_f64(g, W, C_, v, c, K, alpha, seed, unit, go=False):
    """UpdatePairs (src/proNet.cpp:2741-2753; Go pkg/pronet/optimizer.go:8-18) over
    caller pairs, fp64; negatives from stream 3, unit + i // PAIR_BLOCK."""
    v = np.ascontiguousarray(v, np.int32)
    c = np.ascontiguousarray(c, np.int32)
    return lib().orc_update_pairs_f64(g.ref, ptr(W), ptr(C_), W.shape[1], ptr(v), ptr(c), len(v), K, alpha, seed,
                                      unit, int(go))


def update_pairs_f32(g, W, C_, dim, v, c, K, alpha, seed, unit, go=False):
    v = np.ascontiguousarray(v, np.int32)
    c = np.ascontiguousarray(c, np.int32)
    return lib().orc_update_pairs_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], ptr(v), ptr(c), len(v), K, alpha,
                                      seed, unit, int(go))


# --------------------------------------------------------------------- Go semantics
class _OrcGoGraph(C.Structure):
    _fields_ = [("base", _OrcGraph), ("tcum", P)]


class GoGraph:
    """Graph with the Go rules (pkg/pronet/pronet.go:191-249): VertexAT power 1,
    NegativeAT power 0.75 (Go alias rule), CDF target sampling."""

    def __init__(self, V, src, dst, w, names=None):
        self.V, self.E, self.names = V, len(src), names
        base = Graph(V, src, dst, w)               # CSR + degrees (same as C++)
        self.offsets, self.targets = base.offsets, base.targets
        self.out_deg, self.in_deg = base.out_deg, base.in_deg
        self.weights = np.zeros(max(self.E, 1))
        # CSR weights in push order
        order = np.argsort(np.asarray(src), kind="stable")
        self.weights[:self.E] = np.asarray(w, np.float64)[order]
        self.vprob, self.valias = alias_go(self.out_deg, 1.0)
        self.nprob, self.nalias = alias_go(self.in_deg + self.out_deg, 0.75)
        self.vthr, self.valias_enc = alias_encode(self.vprob, self.valias)
        self.nthr, self.nalias_enc = alias_encode(self.nprob, self.nalias)
        self.tcum = np.zeros(max(self.E, 1))
        lib().orc_go_cumsum(ptr(self.offsets), V, ptr(self.weights), ptr(self.tcum))
        b = _OrcGraph(V, self.E, ptr(self.offsets), ptr(self.targets), ptr(self.vthr), ptr(self.valias_enc),
                      ptr(self.nthr), ptr(self.nalias_enc), None, None)
        self._struct = _OrcGoGraph(b, ptr(self.tcum))
        self._keep = base

    @classmethod
    def from_file(cls, path, undirected):
        names, s, d, w = read_edgelist(path, undirected)
        return cls(len(names), s, d, w, names)

    @property
    def ref(self):
        return C.byref(self._struct)


GO_MODEL = {"line2": 0, "line1": 1, "bpr": 3}


def _declare_go(L):
    L.orc_go_cumsum.argtypes = [P, i64, P, P]
    L.orc_go_sample.argtypes = [P, u64, u64, u64, C.c_int, P]
    L.orc_go_train_f64.restype = C.c_int
    L.orc_go_train_f64.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64]
    L.orc_go_train_f32.restype = C.c_int
    L.orc_go_train_f32.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, C.c_int, dbl, dbl, u64, u64, u64, u64]
    L.orc_go_deepwalk_f32.restype = C.c_int
    L.orc_go_deepwalk_f32.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, u64, P,
                                      u64, u64]
    L.orc_go_ctdne_walk.restype = C.c_int
    L.orc_go_ctdne_walk.argtypes = [i64, i64, P, P, P, dbl, u64, u64, C.c_int32, C.c_int, P]
    L.orc_go_ctdne_f32.restype = C.c_int
    L.orc_go_ctdne_f32.argtypes = [P, i64, P, P, P, dbl, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, dbl, u64, P, u64, u64]
    L.orc_go_metapath_walk.restype = C.c_int
    L.orc_go_metapath_walk.argtypes = [P, P, P, P, C.c_int, u64, u64, C.c_int32, C.c_int, P]
    L.orc_go_metapath_f32.restype = C.c_int
    L.orc_go_metapath_f32.argtypes = [P, P, P, P, C.c_int, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, dbl, u64, P, u64, u64]
    L.orc_go_node2vec_walk.restype = C.c_int
    L.orc_go_node2vec_walk.argtypes = [P, P, dbl, dbl, u64, u64, C.c_int32, C.c_int, P]
    L.orc_go_node2vec_f32.restype = C.c_int
    L.orc_go_node2vec_f32.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, dbl,
                                      dbl, u64, P, u64, u64]
    L.orc_go_deepwalk_f64.restype = C.c_int
    L.orc_go_deepwalk_f64.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, dbl, u64, P]


_orig_declare = _declare


def _declare(L):  # noqa: F811
    _orig_declare(L)
    _declare_go(L)


def go_sample(g, seed, begin, count, K):
    o = np.zeros((count, 2 + K), np.int32)
    lib().orc_go_sample(g.ref, seed, begin, count, K, ptr(o))
    return o


def go_train_f64(g, model, W, C_, K, alpha0, lam, total, begin, end, seed):
    return lib().orc_go_train_f64(g.ref, GO_MODEL[model], ptr(W), ptr(C_), W.shape[1], K, alpha0, lam, total,
                                  begin, end, seed)


def go_train_f32(g, model, W, C_, dim, K, alpha0, lam, total, begin, end, seed):
    return lib().orc_go_train_f32(g.ref, GO_MODEL[model], ptr(W), ptr(C_), dim, W.shape[1], K, alpha0, lam, total,
                                  begin, end, seed)


def go_deepwalk_f32(g, W, C_, dim, walk_times, walk_steps, window, K, alpha0, seed, order, begin=0, end=None):
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V
    return lib().orc_go_deepwalk_f32(g.ref, ptr(W), ptr(C_), dim, W.shape[1], walk_times, walk_steps, window, K,
                                     alpha0, seed, ptr(order), begin, end)


def go_deepwalk_f64(g, W, C_, walk_times, walk_steps, window, K, alpha0, seed, order):
    order = np.ascontiguousarray(order, np.int64)
    return lib().orc_go_deepwalk_f64(g.ref, ptr(W), ptr(C_), W.shape[1], walk_times, walk_steps, window, K, alpha0,
                                     seed, ptr(order))


def go_node2vec_walk(g, p, q, seed, unit, start, steps):
    """internal/models/node2vec/node2vec.go:82-164 (one walk)."""
    out = np.zeros(steps + 1, np.int32)
    L = lib().orc_go_node2vec_walk(g.ref, ptr(g.weights), p, q, seed, unit, start, steps, ptr(out))
    return out[:L].copy()


def go_node2vec_f32(g, W, C_, dim, walk_times, walk_steps, window, K, alpha0, p, q, seed, order, begin=0, end=None):
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V
    return lib().orc_go_node2vec_f32(g.ref, ptr(g.weights), ptr(W), ptr(C_), dim, W.shape[1], walk_times,
                                     walk_steps, window, K, alpha0, p, q, seed, ptr(order), begin, end)


def _paths(paths):
    flat = np.ascontiguousarray([t for p in paths for t in p] or [0], np.int32)
    off = np.ascontiguousarray(np.concatenate([[0], np.cumsum([len(p) for p in paths])]), np.int32)
    return flat, off


def go_uniform_negatives(g):
    """metapath2vec's NegativeAT = BuildAliasMethod(ones, 0.75) (metapath2vec.go:140-145),
    written into the graph's negative table in place."""
    prob, alias = alias_go(np.ones(g.V), 0.75)
    thr, al = alias_encode(prob, alias)
    g.nthr[:] = thr
    g.nalias_enc[:] = al
    return prob, alias


def go_metapath_walk(g, ntype, paths, seed, unit, start, steps):
    ntype = np.ascontiguousarray(ntype, np.int32)
    flat, off = _paths(paths)
    out = np.zeros(steps + 1, np.int32)
    L = lib().orc_go_metapath_walk(g.ref, ptr(ntype), ptr(flat), ptr(off), len(paths), seed, unit, start, steps,
                                   ptr(out))
    return out[:L].copy()


def go_metapath_f32(g, ntype, paths, W, C_, dim, walk_times, walk_steps, window, K, alpha0, seed, order, begin=0,
                    end=None):
    ntype = np.ascontiguousarray(ntype, np.int32)
    flat, off = _paths(paths)
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V
    return lib().orc_go_metapath_f32(g.ref, ptr(ntype), ptr(flat), ptr(off), len(paths), ptr(W), ptr(C_), dim,
                                     W.shape[1], walk_times, walk_steps, window, K, alpha0, seed, ptr(order),
                                     begin, end)


def go_ctdne_walk(V, src, dst, ts, window, seed, unit, start, steps):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    ts = np.ascontiguousarray(ts, np.float64)
    out = np.zeros(steps + 1, np.int32)
    L = lib().orc_go_ctdne_walk(V, len(src), ptr(src), ptr(dst), ptr(ts), window, seed, unit, start, steps, ptr(out))
    return out[:L].copy()


def go_ctdne_f32(g, src, dst, ts, window, W, C_, dim, walk_times, walk_steps, win, K, alpha0, seed, order, begin=0,
                 end=None):
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    ts = np.ascontiguousarray(ts, np.float64)
    order = np.ascontiguousarray(order, np.int64)
    if end is None:
        end = walk_times * g.V
    return lib().orc_go_ctdne_f32(g.ref, len(src), ptr(src), ptr(dst), ptr(ts), window, ptr(W), ptr(C_), dim,
                                  W.shape[1], walk_times, walk_steps, win, K, alpha0, seed, ptr(order), begin, end)
