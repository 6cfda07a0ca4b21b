"""ProNet: host-side mirror of the reference proNet core (src/proNet.h:109-269,
Go pkg/pronet/pronet.go:47-74) backed by one libsmore_hip context (one GPU).

Method names follow the reference (SetNegativeMethod, LoadEdgeList,
SourceSample/TargetSample/NegativeSample as batch samplers, ...).  All work
happens in the C ABI; this module only marshals numpy buffers.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib, ptr


class ProNet:
    """Graph + alias tables + embedding tables on one GPU.

    device=-1 gives a host-only context (graph and alias building, no GPU)."""

    def __init__(self, device=0, _ctx=None):
        self.ctx = C.c_void_p()
        self._owned = _ctx is None
        if _ctx is not None:          # a replica of a Group (owned by the group)
            self.ctx = C.c_void_p(_ctx)
        else:
            rc = lib.smore_create(int(device), C.byref(self.ctx))
            if rc != _lib.OK:
                raise _lib.SmoreError("smore_create(device=%d) failed with status %d" % (device, rc))
        self.device = device
        self.vertex_method = "out_degrees"    # src/proNet.cpp:9
        self.negative_method = "degrees"      # src/proNet.cpp:11
        self.dim = 0

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if self.ctx and self._owned:
            lib.smore_destroy(self.ctx)
        self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        check(self.ctx, rc, what)

    # ---------------------------------------------------------------- methods
    def SetNegativeMethod(self, method):
        if method not in _lib.NM:
            raise ValueError(method)
        self.negative_method = method

    def SetVertexMethod(self, method):
        if method not in _lib.VM:
            raise ValueError(method)
        self.vertex_method = method

    # ---------------------------------------------------------------- graph
    def LoadEdgeList(self, filename, undirect):
        """proNet::LoadEdgeList (src/proNet.cpp:115-236)."""
        self._chk(lib.smore_load_edgelist(self.ctx, filename.encode(), int(bool(undirect)),
                                          _lib.VM[self.vertex_method], _lib.NM[self.negative_method]),
                  "LoadEdgeList(%s)" % filename)

    def set_load_cache(self, directory):
        """Binary edge-list cache directory for LoadEdgeList (None: off)."""
        self._chk(lib.smore_set_load_cache(self.ctx, directory.encode() if directory else None), "set_load_cache")

    def last_load_info(self):
        """(seconds, parser threads, cache hit: 0 none, 1 edge slots, 2 the built graph)
        of the last LoadEdgeList."""
        sec, th, hit = C.c_double(), C.c_int(), C.c_int()
        self._chk(lib.smore_last_load_info(self.ctx, C.byref(sec), C.byref(th), C.byref(hit)), "last_load_info")
        return sec.value, th.value, hit.value

    def set_graph_edges(self, V, src, dst, w):
        """Graph from ids: directed edge slots src->dst (weight w) in push order."""
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        # w None: unit weights (np.ascontiguousarray(None) would be one NaN)
        w = np.ones(len(src)) if w is None else np.ascontiguousarray(w, np.float64)
        if len(dst) != len(src) or len(w) != len(src):
            raise ValueError("set_graph_edges: src, dst and w need one entry per edge slot")
        self._chk(lib.smore_set_graph_edges(self.ctx, int(V), len(src), ptr(src), ptr(dst), ptr(w),
                                            _lib.VM[self.vertex_method], _lib.NM[self.negative_method]),
                  "set_graph_edges")

    def _info(self):
        V, E = C.c_int64(), C.c_int64()
        self._chk(lib.smore_graph_info(self.ctx, C.byref(V), C.byref(E)), "graph_info")
        return V.value, E.value

    @property
    def MAX_vid(self):
        return self._info()[0]

    @property
    def MAX_line(self):
        return self._info()[1]

    def vertex_name(self, vid):
        n = lib.smore_vertex_name(self.ctx, int(vid))
        return None if n is None else n.decode()

    @property
    def names(self):
        return [self.vertex_name(v) for v in range(self.MAX_vid)]

    def csr(self):
        V, E = self._info()
        off = np.zeros(V + 1, np.int64)
        tgt = np.zeros(max(E, 1), np.int32)
        self._chk(lib.smore_get_csr(self.ctx, ptr(off), ptr(tgt)), "get_csr")
        return off, tgt[:E]

    def alias(self, which):
        """(prob, alias) of vertex_AT / negative_AT / context_AT."""
        V, E = self._info()
        n = E if which == _lib.AT_CONTEXT else V
        p = np.zeros(n)
        a = np.zeros(n, np.int64)
        self._chk(lib.smore_get_alias(self.ctx, which, ptr(p), ptr(a), n), "get_alias")
        return p, a

    def alias_encoded(self, which):
        V, E = self._info()
        n = E if which == _lib.AT_CONTEXT else V
        t = np.zeros(n, np.uint32)
        a = np.zeros(n, np.int32)
        self._chk(lib.smore_get_alias_encoded(self.ctx, which, ptr(t), ptr(a), n), "get_alias_encoded")
        return t, a

    def set_alias(self, which, prob, alias):
        """Inject an alias table (Go CTDNE assigns ProNet.NegativeAT directly)."""
        prob = np.ascontiguousarray(prob, np.float64)
        alias = np.ascontiguousarray(alias, np.int64)
        self._chk(lib.smore_set_alias(self.ctx, which, ptr(prob), ptr(alias), len(prob)), "set_alias")

    # ---------------------------------------------------------------- samplers
    def sample_edges(self, model, begin, count, K, seed):
        """Draws of samples [begin, begin+count): rows {v, c, n1..nK} (BPR: {u, i, j0..j4};
        Go semantics BPR: {u, i, j})."""
        go = getattr(self, "semantics", "cpp") == "go"
        width = (3 if go else 7) if model == "bpr" else 2 + K
        out = np.zeros((count, width), np.int32)
        self._chk(lib.smore_sample_edges(self.ctx, _lib.MODEL[model], begin, count, K, seed, ptr(out)),
                  "sample_edges")
        return out

    # ---------------------------------------------------------------- tables
    def alloc_tables(self, dim, ntables):
        self._chk(lib.smore_alloc_tables(self.ctx, int(dim), int(ntables)), "alloc_tables")
        self.dim = dim

    def init_table_glibc(self, which, skip=0):
        self._chk(lib.smore_init_table_glibc(self.ctx, which, int(skip)), "init_table_glibc")

    def init_table_uniform(self, which, seed):
        self._chk(lib.smore_init_table_uniform(self.ctx, which, int(seed)), "init_table_uniform")

    def zero_table(self, which):
        self._chk(lib.smore_zero_table(self.ctx, which), "zero_table")

    def set_table(self, which, host):
        host = np.ascontiguousarray(host, np.float32)
        self._chk(lib.smore_set_table(self.ctx, which, ptr(host), host.shape[0], host.shape[1]), "set_table")

    def get_table(self, which):
        V = self.MAX_vid
        out = np.zeros((V, self.dim), np.float32)
        self._chk(lib.smore_get_table(self.ctx, which, ptr(out), V, self.dim), "get_table")
        return out

    def table_device(self, which):
        p, s = C.c_void_p(), C.c_int64()
        self._chk(lib.smore_table_device(self.ctx, which, C.byref(p), C.byref(s)), "table_device")
        return p.value, s.value

    # ---------------------------------------------------------------- training
    def set_stream(self, stream_handle):
        self._chk(lib.smore_set_stream(self.ctx, C.c_void_p(stream_handle) if stream_handle else None),
                  "set_stream")

    def train_edges(self, model, begin, count, total, K, alpha0, reg=0.0, seed=1, mode="hogwild", sync=True):
        fn = lib.smore_train_edges if sync else lib.smore_train_edges_async
        self._chk(fn(self.ctx, _lib.MODEL[model], int(begin), int(count), int(total), int(K), float(alpha0),
                     float(reg), int(seed), _lib.MODE[mode]), "train_edges")

    def train_deepwalk(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, seed, order,
                       mode="hogwild"):
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_train_deepwalk(self.ctx, int(walk_begin), int(walk_end), int(walk_times),
                                           int(walk_steps), int(window), int(K), float(alpha0), int(seed),
                                           ptr(order), _lib.MODE[mode]), "train_deepwalk")

    def _ids(self, ids, what):
        """Vertex ids as contiguous int32, range-checked against MAX_vid BEFORE
        the narrowing: an id of 2^31 or more (e.g. 2^32 + 5) must not wrap to a
        valid small one and reach the C side's own range check as a legal row."""
        a = np.asarray(ids)
        if a.size:
            if not (np.issubdtype(a.dtype, np.integer) or a.dtype == np.bool_):
                raise TypeError("%s: vertex ids must be integers, got %s" % (what, a.dtype))
            if int(a.min()) < 0 or int(a.max()) >= self.MAX_vid:
                raise _lib.SmoreError("%s: vertex id out of range [0, %d)" % (what, self.MAX_vid))
        return np.ascontiguousarray(a, np.int32)

    def train_pairs(self, v, c, K, alpha, seed, unit=0, mode="hogwild"):
        """UpdatePairs (src/proNet.cpp:2741-2753; Go pkg/pronet/optimizer.go:8-18)
        over caller-supplied pairs (v[i], c[i]) in order, fixed alpha; pair i's
        negatives from stream 3, unit `unit` + i // 2^20 (smore_train_pairs).
        Ids are range-checked before they are narrowed to int32 (an id of 2^31
        or more must not wrap to a valid small one; the reference panics)."""
        v, c = self._ids(v, "train_pairs"), self._ids(c, "train_pairs")
        if v.shape != c.shape:
            raise ValueError("v and c must have the same length")
        self._chk(lib.smore_train_pairs(self.ctx, ptr(v), ptr(c), len(v), int(K), float(alpha), int(seed), int(unit),
                                        _lib.MODE[mode]), "train_pairs")

    # ---- 2-D block schedule, one replica's side (smore_block_*)
    def save_graph(self, path):
        """The built graph to a binary file (smore_save_graph)."""
        self._chk(lib.smore_save_graph(self.ctx, path.encode()), "save_graph")

    def load_graph(self, path, vertex_method="out_degrees", negative_method="degrees"):
        """A graph written by save_graph (smore_load_graph), uploaded."""
        self._chk(lib.smore_load_graph(self.ctx, path.encode(), _lib.VM[vertex_method], _lib.NM[negative_method]),
                  "load_graph")

    def block_setup(self, model, nparts, part, K, mode="hybrid"):
        """This context as part `part` of `nparts`: W part bounds, 2 nparts C
        blocks and the cells' draw tables (smore_block_setup; model "line2" or
        "census" for the C++ walk models)."""
        self._chk(lib.smore_block_setup(self.ctx, _lib.MODEL[model], int(nparts), int(part), int(K),
                                        _lib.MODE[mode]), "block_setup")

    def block_bounds(self):
        """(W part bounds [N + 1], C block bounds [2N + 1]) of the block setup."""
        n, r, nb = C.c_int(), C.c_int(), C.c_int()
        lib.smore_block_info(self.ctx, C.byref(n), C.byref(r), C.byref(nb))
        wb = np.zeros(n.value + 1, np.int64)
        cb = np.zeros(nb.value + 1, np.int64)
        self._chk(lib.smore_block_bounds(self.ctx, ptr(wb), ptr(cb)), "block_bounds")
        return wb, cb

    def block_mass(self):
        """LINE-2: this part's sample mass per C block (sums to 1)."""
        _, cb = self.block_bounds()
        m = np.zeros(len(cb) - 1, np.float64)
        self._chk(lib.smore_block_mass(self.ctx, ptr(m)), "block_mass")
        return m

    def block_part_mass(self):
        """LINE-2: every part's share of the global source law (sums to 1)."""
        wb, _ = self.block_bounds()
        m = np.zeros(len(wb) - 1, np.float64)
        self._chk(lib.smore_block_part_mass(self.ctx, ptr(m)), "block_part_mass")
        return m

    def block_neg_scale(self, block):
        """LINE-2: the negative-step weight of cell (part, block) (fp32 value)."""
        w = C.c_double()
        self._chk(lib.smore_block_neg_scale(self.ctx, int(block), C.byref(w)), "block_neg_scale")
        return w.value

    def block_set_hubs(self, hubs):
        """LINE-2 hub C rows of the next block_setup (-1 automatic, 0 none)."""
        self._chk(lib.smore_block_set_hubs(self.ctx, int(hubs)), "block_set_hubs")

    def block_hubs(self):
        """(H, first slot row V, hub C rows [H] int32, expected touches per sample [H])."""
        h, first = C.c_int64(), C.c_int64()
        self._chk(lib.smore_block_hubs(self.ctx, C.byref(h), C.byref(first), None, None), "block_hubs")
        rows = np.zeros(max(1, h.value), np.int32)
        rates = np.zeros(max(1, h.value), np.float64)
        self._chk(lib.smore_block_hubs(self.ctx, None, None, ptr(rows), ptr(rates)), "block_hubs")
        return h.value, first.value, rows[:h.value].copy(), rates[:h.value].copy()

    def block_hubs_load(self):
        self._chk(lib.smore_block_hubs_load(self.ctx), "block_hubs_load")

    def block_hubs_store(self):
        self._chk(lib.smore_block_hubs_store(self.ctx), "block_hubs_store")

    def block_cell_launches(self):
        """LINE-2: launches per cell (the hub slots exchanged after each)."""
        return int(lib.smore_block_cell_launches(self.ctx))

    def block_hub_scales(self, samples, c0):
        h = self.block_hubs()[0]
        out = np.zeros(max(1, h), np.float32)
        self._chk(lib.smore_block_hub_scales(self.ctx, float(samples), float(c0), ptr(out)), "block_hub_scales")
        return out[:h].copy()

    def block_counts(self, samples):
        """LINE-2: `samples` split over the C blocks by mass (largest remainder)."""
        _, cb = self.block_bounds()
        out = np.zeros(len(cb) - 1, np.uint64)
        self._chk(lib.smore_block_counts(self.ctx, int(samples), ptr(out)), "block_counts")
        return out

    def block_train_edges(self, block, begin, count, total, K, alpha0, seed, mode="hybrid", sync=True):
        """LINE-2 samples [begin, begin + count) of cell (part, block)."""
        self._chk(lib.smore_block_train_edges_async(self.ctx, int(block), int(begin), int(count), int(total), int(K),
                                                    float(alpha0), int(seed), _lib.MODE[mode]), "block_train_edges")
        if sync:
            self.synchronize()

    def block_sample_edges(self, block, seed, begin, count, K):
        out = np.zeros((int(count), 2 + int(K)), np.int32)
        self._chk(lib.smore_block_sample_edges(self.ctx, int(block), int(seed), int(begin), int(count), int(K),
                                               ptr(out)), "block_sample_edges")
        return out

    def block_prepare_walks(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, seed, order=None,
                            mode="hybrid", rule="deepwalk", window_min=0):
        """A round of walks -> this part's pair records bucketed by C block."""
        if order is not None:
            order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_block_prepare_walks(self.ctx, 0 if rule == "deepwalk" else 1, int(walk_begin),
                                                int(walk_end), int(walk_times), int(walk_steps), int(window),
                                                int(window_min), int(K), float(alpha0), int(seed),
                                                ptr(order) if order is not None else None, 0, _lib.MODE[mode]),
                  "block_prepare_walks")

    def block_walks_generate(self, walk_begin, walk_end, gen_lo, gen_hi, walk_times, walk_steps, window, K, alpha0,
                             seed, order=None, mode="hybrid", rule="deepwalk", window_min=0):
        """Walk only [gen_lo, gen_hi) of the round [walk_begin, walk_end)
        (walk-partitioned generation); smore_block_walks_emit buckets the pairs."""
        if order is not None:
            order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_block_walks_generate(self.ctx, 0 if rule == "deepwalk" else 1, int(walk_begin),
                                                 int(walk_end), int(gen_lo), int(gen_hi), int(walk_times),
                                                 int(walk_steps), int(window), int(window_min), int(K), float(alpha0),
                                                 int(seed), ptr(order) if order is not None else None, 0,
                                                 _lib.MODE[mode]), "block_walks_generate")

    def block_walks_emit(self):
        self._chk(lib.smore_block_walks_emit(self.ctx), "block_walks_emit")

    def block_train_walks(self, block, sync=True, part=0, parts=1):
        """Train cell (part, block)'s bucket of the prepared round (or one of
        `parts` consecutive parts of it)."""
        self._chk(lib.smore_block_train_walks_part_async(self.ctx, int(block), int(part), int(parts)),
                  "block_train_walks")
        if sync:
            self.synchronize()

    def block_walk_records(self, block):
        n = C.c_uint64()
        self._chk(lib.smore_block_walk_records(self.ctx, int(block), C.byref(n)), "block_walk_records")
        return n.value

    def block_walk_records_copy(self, block):
        """A bucket's records, int32 [n, width] (parity tests)."""
        n, w = C.c_uint64(), C.c_int32()
        self._chk(lib.smore_block_walk_records_copy(self.ctx, int(block), None, 0, C.byref(n), C.byref(w)),
                  "block_walk_records_copy")
        out = np.zeros((n.value, w.value), np.int32)
        self._chk(lib.smore_block_walk_records_copy(self.ctx, int(block), out.ctypes.data_as(C.c_void_p), n.value,
                                                    C.byref(n), C.byref(w)), "block_walk_records_copy")
        return out

    def pairs_rows(self, v, c, K, seed, unit=0):
        """(W row ids, C row ids) a train_pairs batch touches: its vertices, and
        its contexts plus the K negatives it will draw (smore_pairs_rows)."""
        v, c = self._ids(v, "pairs_rows"), self._ids(c, "pairs_rows")
        w_ids = np.zeros(max(1, len(v)), np.int32)
        c_ids = np.zeros(max(1, len(v) * (int(K) + 1)), np.int32)
        nw, nc = C.c_int64(), C.c_int64()
        self._chk(lib.smore_pairs_rows(self.ctx, ptr(v), ptr(c), len(v), int(K), int(seed), int(unit), ptr(w_ids),
                                       C.byref(nw), ptr(c_ids), C.byref(nc)), "pairs_rows")
        return w_ids[:nw.value].copy(), c_ids[:nc.value].copy()

    def set_rows(self, which, ids, rows):
        ids = self._ids(ids, "set_rows")
        rows = np.ascontiguousarray(rows, np.float32)
        self._chk(lib.smore_set_rows(self.ctx, int(which), ptr(ids), len(ids), ptr(rows)), "set_rows")

    def get_rows(self, which, ids):
        ids = self._ids(ids, "get_rows")
        out = np.zeros((len(ids), self.dim), np.float32)
        self._chk(lib.smore_get_rows(self.ctx, int(which), ptr(ids), len(ids), ptr(out)), "get_rows")
        return out

    def train_pairs_rows(self, v, c, K, alpha, seed, unit, mode, w_ids, w_rows, c_ids, c_rows):
        """smore_train_pairs_rows: the touched rows up, the pairs, the rows back
        (w_rows / c_rows float32 [n][dim], updated in place)."""
        v, c = self._ids(v, "train_pairs_rows"), self._ids(c, "train_pairs_rows")
        w_ids, c_ids = self._ids(w_ids, "train_pairs_rows"), self._ids(c_ids, "train_pairs_rows")
        assert w_rows.dtype == np.float32 and w_rows.flags.c_contiguous and c_rows.dtype == np.float32
        assert c_rows.flags.c_contiguous
        self._chk(lib.smore_train_pairs_rows(self.ctx, ptr(v), ptr(c), len(v), int(K), float(alpha), int(seed),
                                             int(unit), _lib.MODE[mode], ptr(w_ids), len(w_ids), ptr(w_rows),
                                             ptr(c_ids), len(c_ids), ptr(c_rows)), "train_pairs_rows")

    def train_pairs_rows_mt(self, v, c, K, alpha, seed, unit, mode, w_ids, w_rows, c_ids, c_rows):
        """smore_train_pairs_rows_mt: as train_pairs_rows, safe from concurrent
        threads (their calls are combined into one device call)."""
        v, c = self._ids(v, "train_pairs_rows_mt"), self._ids(c, "train_pairs_rows_mt")
        w_ids, c_ids = self._ids(w_ids, "train_pairs_rows_mt"), self._ids(c_ids, "train_pairs_rows_mt")
        assert w_rows.dtype == np.float32 and w_rows.flags.c_contiguous and c_rows.dtype == np.float32
        assert c_rows.flags.c_contiguous
        self._chk(lib.smore_train_pairs_rows_mt(self.ctx, ptr(v), ptr(c), len(v), int(K), float(alpha), int(seed),
                                                int(unit), _lib.MODE[mode], ptr(w_ids), len(w_ids), ptr(w_rows),
                                                ptr(c_ids), len(c_ids), ptr(c_rows)), "train_pairs_rows_mt")

    def census_begin(self):
        """Row census: the following walk-model calls count the rows their
        records would update instead of training (smore_census_begin)."""
        self._chk(lib.smore_census_begin(self.ctx), "census_begin")

    def census_end(self, units):
        """End the census: counts / units = row_rates("census", ...)."""
        self._chk(lib.smore_census_end(self.ctx, float(units)), "census_end")

    def set_temporal_edges(self, src, dst, ts):
        """Timestamped edges (pkg/temporal OutEdges) for CTDNE."""
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        ts = np.ascontiguousarray(ts, np.float64)
        self._chk(lib.smore_set_temporal_edges(self.ctx, len(src), ptr(src), ptr(dst), ptr(ts)), "set_temporal_edges")

    def train_ctdne(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, time_window, seed, order,
                    mode="hogwild"):
        """(*CTDNE).Train (Go, internal/models/ctdne/ctdne.go:80-200) over walks [walk_begin, walk_end)."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_train_ctdne(self.ctx, int(walk_begin), int(walk_end), int(walk_times), int(walk_steps),
                                        int(window), int(K), float(alpha0), float(time_window), int(seed),
                                        ptr(order), _lib.MODE[mode]), "train_ctdne")

    def set_node_types(self, node_type, ntypes):
        """Node types of a heterogeneous graph (pkg/hetero NodeTypes) for metapath2vec."""
        node_type = np.ascontiguousarray(node_type, np.int32)
        self._chk(lib.smore_set_node_types(self.ctx, ptr(node_type), int(ntypes)), "set_node_types")

    def train_metapath2vec(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, paths, seed,
                           order, mode="hogwild"):
        """(*Metapath2Vec).Train (Go, internal/models/metapath2vec/metapath2vec.go:106-200)
        over walks [walk_begin, walk_end); paths = list of meta-paths (lists of type ids)."""
        order = np.ascontiguousarray(order, np.int64)
        flat = np.ascontiguousarray([t for p in paths for t in p] or [0], np.int32)
        lens = np.ascontiguousarray([len(p) for p in paths], np.int32)
        self._chk(lib.smore_train_metapath2vec(self.ctx, int(walk_begin), int(walk_end), int(walk_times),
                                               int(walk_steps), int(window), int(K), float(alpha0), ptr(flat),
                                               ptr(lens), len(paths), int(seed), ptr(order), _lib.MODE[mode]),
                  "train_metapath2vec")

    def train_node2vec(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, p, q, seed, order,
                       mode="hogwild"):
        """(*Node2Vec).Train (Go, internal/models/node2vec/node2vec.go:178-258) over walks
        [walk_begin, walk_end); needs set_semantics("go")."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_train_node2vec(self.ctx, int(walk_begin), int(walk_end), int(walk_times),
                                           int(walk_steps), int(window), int(K), float(alpha0), float(p), float(q),
                                           int(seed), ptr(order), _lib.MODE[mode]), "train_node2vec")

    def train_walklets(self, walk_begin, walk_end, walk_times, walk_steps, window_min, window_max, K, alpha0, seed,
                       mode="hogwild"):
        """Walklets::Train (src/model/Walklets.cpp:24-63) over walks [walk_begin, walk_end)."""
        self._chk(lib.smore_train_walklets(self.ctx, int(walk_begin), int(walk_end), int(walk_times),
                                           int(walk_steps), int(window_min), int(window_max), int(K), float(alpha0),
                                           int(seed), _lib.MODE[mode]), "train_walklets")

    def train_app(self, unit_begin, unit_end, walk_times, sample_times, jump, K, alpha0, seed, order,
                  mode="hogwild"):
        """APP::Train (src/model/APP.cpp:59-120) over units [unit_begin, unit_end) of
        walk_times * V * sample_times; order = walk start vertices (walk_times * V)."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_train_app(self.ctx, int(unit_begin), int(unit_end), int(walk_times), int(sample_times),
                                      float(jump), int(K), float(alpha0), int(seed), ptr(order), _lib.MODE[mode]),
                  "train_app")

    def train_hpe(self, begin, count, total, walk_steps, K, reg, alpha0, seed, mode="hogwild"):
        """HPE::Train (src/model/HPE.cpp:94-150) over samples [begin, begin + count) of total."""
        self._chk(lib.smore_train_hpe(self.ctx, int(begin), int(count), int(total), int(walk_steps), int(K),
                                      float(reg), float(alpha0), int(seed), _lib.MODE[mode]), "train_hpe")

    def set_semantics(self, semantics):
        """"cpp" (src/proNet.cpp rules, default) or "go" (pkg/pronet rules)."""
        self._chk(lib.smore_set_semantics(self.ctx, _lib.SEM[semantics]), "set_semantics")
        self.semantics = semantics

    def set_write_combine(self, rows, flush_rounds=0):
        """Hybrid scatter: LDS write-combining of the `rows` hottest context rows,
        drained every `flush_rounds` rounds (0: automatic)."""
        self._chk(lib.smore_set_write_combine(self.ctx, int(rows), int(flush_rounds)), "set_write_combine")

    def write_combine_info(self):
        """(combined rows, drain interval) of the last hybrid launch."""
        r, f = C.c_int(), C.c_int()
        self._chk(lib.smore_write_combine_info(self.ctx, C.byref(r), C.byref(f)), "write_combine_info")
        return r.value, f.value

    def set_hot_threshold(self, tau):
        self._chk(lib.smore_set_hot_threshold(self.ctx, float(tau)), "set_hot_threshold")

    def hot_rows(self):
        w, c = C.c_int64(), C.c_int64()
        self._chk(lib.smore_hot_rows(self.ctx, C.byref(w), C.byref(c)), "hot_rows")
        return w.value, c.value

    def hot_row_ids(self, model, K, which, n):
        """The n hub rows of table `which` (0 W, 1 C) by expected touches per
        sample, highest first (int32)."""
        ids = np.zeros(max(1, n), np.int32)
        self._chk(lib.smore_hot_row_ids(self.ctx, _lib.MODEL[model], int(K), int(which), int(n),
                                        ids.ctypes.data_as(C.c_void_p)), "hot_row_ids")
        return ids[:n]

    def row_rates(self, model, K, which):
        """Expected touches per sample of every row of table `which` (0 W, 1 C)
        under `model` with K negatives (float64, V)."""
        r = np.zeros(self.MAX_vid, np.float64)
        self._chk(lib.smore_row_rates(self.ctx, _lib.MODEL[model], int(K), int(which), len(r),
                                      r.ctypes.data_as(C.c_void_p)), "row_rates")
        return r

    def source_parts(self, nparts):
        """Bounds (nparts + 1, int64) of the contiguous equal-source-mass vertex parts."""
        b = np.zeros(int(nparts) + 1, np.int64)
        self._chk(lib.smore_source_parts(self.ctx, int(nparts), b.ctypes.data_as(C.c_void_p)), "source_parts")
        return b

    def set_source_partition(self, nparts, part):
        """Draw sources from part `part` of `nparts` only (1 = the global law)."""
        self._chk(lib.smore_set_source_partition(self.ctx, int(nparts), int(part)), "set_source_partition")

    def walk_parts(self, nparts):
        """Bounds (nparts + 1, int64) of contiguous vertex parts of equal W-touch
        mass under the last row census (smore_walk_parts)."""
        b = np.zeros(int(nparts) + 1, np.int64)
        self._chk(lib.smore_walk_parts(self.ctx, int(nparts), b.ctypes.data_as(C.c_void_p)), "walk_parts")
        return b

    def set_walk_owner(self, lo, hi=-1):
        """Walk models train only the pairs whose center is in [lo, hi)
        (smore_set_walk_owner; hi < 0: every pair)."""
        self._chk(lib.smore_set_walk_owner(self.ctx, int(lo), int(hi)), "set_walk_owner")

    def synchronize(self):
        self._chk(lib.smore_synchronize(self.ctx), "synchronize")

    def skipped(self):
        s = C.c_uint64()
        self._chk(lib.smore_skipped(self.ctx, C.byref(s)), "skipped")
        return s.value

    def last_kernel_ms(self):
        return float(lib.smore_last_kernel_ms(self.ctx))

    def last_mode(self):
        """The scatter the last training call ran ("hybrid", "hogwild" = plain
        stores, ...; None before any): C++ BPR asked for "hybrid" above the
        small-graph cap runs the plain-store kernel."""
        m = int(lib.smore_last_mode(self.ctx))
        return {v: k for k, v in _lib.MODE.items()}.get(m)

    def delta_begin(self, T, S, D, R, n):
        """Replica exchange pass D = T - S; R = D; S = T (device pointers, n floats)."""
        self._chk(lib.smore_delta_begin(self.ctx, T, S, D, R, int(n)), "delta_begin")

    def delta_end(self, T, S, D, R, scale, n):
        """Replica exchange pass X = scale*R - D; T += X; S += X."""
        self._chk(lib.smore_delta_end(self.ctx, T, S, D, R, float(scale), int(n)), "delta_end")

    def delta_cycle(self, T, S, D, R, scale, n):
        """delta_end then delta_begin in one pass."""
        self._chk(lib.smore_delta_cycle(self.ctx, T, S, D, R, float(scale), int(n)), "delta_cycle")

    def delta_end_rows(self, T, S, D, R, scale, rows, stride):
        """delta_end with row i's scale scale[i] (device pointer, rows floats)."""
        self._chk(lib.smore_delta_end_rows(self.ctx, T, S, D, R, scale, int(rows), int(stride)), "delta_end_rows")

    def delta_cycle_rows(self, T, S, D, R, scale, rows, stride):
        """delta_cycle with row i's scale scale[i]."""
        self._chk(lib.smore_delta_cycle_rows(self.ctx, T, S, D, R, scale, int(rows), int(stride)),
                  "delta_cycle_rows")

    # ---------------------------------------------------------------- replica exchange (RCCL, in the library)
    def comm_init(self, nranks, rank, uid):
        """Join an RCCL communicator (uid: bytes of comm_unique_id() from rank 0)."""
        buf = (C.c_ubyte * COMM_ID_BYTES).from_buffer_copy(bytes(uid))
        self._chk(lib.smore_comm_init(self.ctx, int(nranks), int(rank), buf), "comm_init")

    def exchange_reset(self):
        """S = T: the replicas start from identical tables."""
        self._chk(lib.smore_exchange_reset(self.ctx), "exchange_reset")

    def exchange_set_adaptive(self, model, K, updates, c0=64.0):
        """Row scales of the adaptive rule for `updates` samples per rank per exchange."""
        self._chk(lib.smore_exchange_set_adaptive(self.ctx, _lib.MODEL[model], int(K), float(updates), float(c0)),
                  "exchange_set_adaptive")

    def exchange_begin(self, mean=False):
        """After a step: fold the in-flight exchange in, snapshot this rank's
        delta and start its all-reduce (overlaps the next step).  mean: a rule
        name ("sum", "mean", "adaptive") or the old boolean."""
        self._chk(lib.smore_exchange_begin(self.ctx, _lib.sync_rule(mean)), "exchange_begin")

    def exchange_end(self):
        self._chk(lib.smore_exchange_end(self.ctx), "exchange_end")

    def last_phase_ms(self):
        """(exposed draw ms, update ms, update launches) of the last LINE/MF
        edge call, or None."""
        import ctypes
        d, u, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        if lib.smore_last_phase_ms(self.ctx, ctypes.byref(d), ctypes.byref(u), ctypes.byref(n)) != 0:
            return None
        return float(d.value), float(u.value), int(n.value)

    def copy_bandwidth(self, nbytes=4 << 30, reps=5):
        """Streaming device-to-device copy rate of this GPU in GB/s (read +
        written bytes; the library's float4 copy kernel, membw.hip)."""
        import ctypes
        g = ctypes.c_double()
        self._chk(lib.smore_copy_bandwidth(self.ctx, int(nbytes), int(reps), ctypes.byref(g)), "copy_bandwidth")
        return float(g.value)

    def load_pretrain(self, which, path):
        """proNet::LoadPreTrain (src/proNet.cpp:238-286)."""
        self._chk(lib.smore_load_pretrain(self.ctx, which, path.encode()), "load_pretrain")

    def save_weights(self, which, path, fmt=0):
        self._chk(lib.smore_save_weights(self.ctx, which, path.encode(), int(fmt)), "save_weights")


COMM_ID_BYTES = 128


def comm_unique_id():
    """An RCCL unique id (bytes) for ProNet.comm_init on every rank."""
    buf = (C.c_ubyte * COMM_ID_BYTES)()
    if lib.smore_comm_unique_id(buf) != _lib.OK:
        raise _lib.SmoreError("comm_unique_id failed (RCCL unavailable?)")
    return bytes(buf)


class Group:
    """One process driving N GPUs (smore_group_*): replica 0 (`primary`, a
    ProNet view) loads, initialises and saves; broadcast_tables() copies its
    tables to every replica; training calls split the global range over the
    replicas and return with every replica holding every update.  `mean` of
    the training calls is the exchange rule: "adaptive" (default), "sum",
    "mean" (or the old boolean), smore_hip.h SMORE_SYNC_*."""

    def __init__(self, devices):
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        self.g = C.c_void_p()
        rc = lib.smore_group_create(devs, len(devices), C.byref(self.g))
        if rc != _lib.OK:
            raise _lib.SmoreError("smore_group_create(%s) failed with status %d" % (list(devices), rc))
        self.replicas = [ProNet(devices[r], _ctx=lib.smore_group_ctx(self.g, r)) for r in range(len(devices))]
        self.primary = self.replicas[0]

    def close(self):
        if self.g:
            for r in self.replicas:
                r.ctx = C.c_void_p()
            lib.smore_group_destroy(self.g)
            self.g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != _lib.OK:
            raise _lib.SmoreError("%s failed (status %d): %s" % (what, rc, lib.smore_group_last_error(self.g).decode()))

    def __len__(self):
        return int(lib.smore_group_size(self.g))

    def LoadEdgeList(self, filename, undirect, vertex_method="out_degrees", negative_method="degrees"):
        self._chk(lib.smore_group_load_edgelist(self.g, filename.encode(), int(bool(undirect)),
                                                _lib.VM[vertex_method], _lib.NM[negative_method]), "LoadEdgeList")

    def set_graph_edges(self, V, src, dst, w, vertex_method="out_degrees", negative_method="degrees"):
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        # w None: unit weights (np.ascontiguousarray(None) would be one NaN)
        w = np.ones(len(src)) if w is None else np.ascontiguousarray(w, np.float64)
        if len(dst) != len(src) or len(w) != len(src):
            raise ValueError("set_graph_edges: src, dst and w need one entry per edge slot")
        self._chk(lib.smore_group_set_graph_edges(self.g, int(V), len(src), ptr(src), ptr(dst), ptr(w),
                                                  _lib.VM[vertex_method], _lib.NM[negative_method]),
                  "set_graph_edges")

    def set_adaptive(self, c0=-1.0):
        """smore_group_set_adaptive: c0 of the adaptive exchange rule (-1: the default)."""
        self._chk(lib.smore_group_set_adaptive(self.g, float(c0)), "set_adaptive")

    def set_partition(self, on=True):
        """smore_group_set_partition: LINE-2 W rows partitioned by source (default on)."""
        self._chk(lib.smore_group_set_partition(self.g, int(bool(on))), "set_partition")

    def set_walk_partition(self, on=True):
        """smore_group_set_walk_partition: walk-model W rows partitioned by walk
        center (default off)."""
        self._chk(lib.smore_group_set_walk_partition(self.g, int(bool(on))), "set_walk_partition")

    def set_schedule(self, schedule):
        """smore_group_set_schedule: "blocks" (the 2-D block schedule: no row
        replicated while it trains, C blocks rotating; LINE-2, DeepWalk and
        Walklets on the C++ rules) or "replicas" (replicated tables, deltas
        exchanged)."""
        self._chk(lib.smore_group_set_schedule(self.g, _lib.SCHED[schedule]), "set_schedule")

    def set_hot_exchange(self, rows=-1, launches=8):
        """smore_group_set_hot_exchange: hub rows per table synced after every
        one of `launches` launches per exchange round (-1 automatic, 0 off)."""
        self._chk(lib.smore_group_set_hot_exchange(self.g, int(rows), int(launches)), "set_hot_exchange")

    def set_semantics(self, semantics):
        self._chk(lib.smore_group_set_semantics(self.g, _lib.SEM[semantics]), "set_semantics")

    def set_alias(self, which, prob, alias):
        prob = np.ascontiguousarray(prob, np.float64)
        alias = np.ascontiguousarray(alias, np.int64)
        self._chk(lib.smore_group_set_alias(self.g, which, ptr(prob), ptr(alias), len(prob)), "set_alias")

    def set_node_types(self, node_type, ntypes):
        node_type = np.ascontiguousarray(node_type, np.int32)
        self._chk(lib.smore_group_set_node_types(self.g, ptr(node_type), int(ntypes)), "set_node_types")

    def set_temporal_edges(self, src, dst, ts):
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        ts = np.ascontiguousarray(ts, np.float64)
        self._chk(lib.smore_group_set_temporal_edges(self.g, len(src), ptr(src), ptr(dst), ptr(ts)),
                  "set_temporal_edges")

    def train_metapath2vec(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, paths, seed, order,
                           mode="atomic", per=0, mean="adaptive"):
        """(*Metapath2Vec).Train (Go, internal/models/metapath2vec/metapath2vec.go:106-200) over the replicas."""
        order = np.ascontiguousarray(order, np.int64)
        flat = np.ascontiguousarray([t for p in paths for t in p] or [0], np.int32)
        lens = np.ascontiguousarray([len(p) for p in paths], np.int32)
        self._chk(lib.smore_group_train_metapath2vec(self.g, int(walk_begin), int(walk_end), int(walk_times),
                                                     int(walk_steps), int(window), int(K), float(alpha0), ptr(flat),
                                                     ptr(lens), len(paths), int(seed), ptr(order), _lib.MODE[mode],
                                                     int(per), _lib.sync_rule(mean)), "train_metapath2vec")

    def train_ctdne(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, time_window, seed, order,
                    mode="atomic", per=0, mean="adaptive"):
        """(*CTDNE).Train (Go, internal/models/ctdne/ctdne.go:80-200) over the replicas."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_group_train_ctdne(self.g, int(walk_begin), int(walk_end), int(walk_times),
                                              int(walk_steps), int(window), int(K), float(alpha0),
                                              float(time_window), int(seed), ptr(order), _lib.MODE[mode], int(per),
                                              _lib.sync_rule(mean)), "train_ctdne")

    def alloc_tables(self, dim, ntables):
        self._chk(lib.smore_group_alloc_tables(self.g, int(dim), int(ntables)), "alloc_tables")
        for r in self.replicas:
            r.dim = dim

    def broadcast_tables(self):
        self._chk(lib.smore_group_broadcast_tables(self.g), "broadcast_tables")

    def train_edges(self, model, begin, count, total, K, alpha0, reg=0.0, seed=1, mode="hybrid", per=0, mean="adaptive"):
        self._chk(lib.smore_group_train_edges(self.g, _lib.MODEL[model], int(begin), int(count), int(total), int(K),
                                              float(alpha0), float(reg), int(seed), _lib.MODE[mode], int(per),
                                              _lib.sync_rule(mean)), "train_edges")

    def train_deepwalk(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, seed, order,
                       mode="hybrid", per=0, mean="adaptive"):
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_group_train_deepwalk(self.g, int(walk_begin), int(walk_end), int(walk_times),
                                                 int(walk_steps), int(window), int(K), float(alpha0), int(seed),
                                                 ptr(order), _lib.MODE[mode], int(per), _lib.sync_rule(mean)),
                  "train_deepwalk")

    def train_node2vec(self, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, p, q, seed, order,
                       mode="atomic", per=0, mean="adaptive"):
        """(*Node2Vec).Train (Go, internal/models/node2vec/node2vec.go:178-258) over the replicas."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_group_train_node2vec(self.g, int(walk_begin), int(walk_end), int(walk_times),
                                                 int(walk_steps), int(window), int(K), float(alpha0), float(p),
                                                 float(q), int(seed), ptr(order), _lib.MODE[mode], int(per),
                                                 _lib.sync_rule(mean)), "train_node2vec")

    def train_walklets(self, walk_begin, walk_end, walk_times, walk_steps, window_min, window_max, K, alpha0, seed,
                       mode="hybrid", per=0, mean="adaptive"):
        """Walklets::Train (src/model/Walklets.cpp:24-63) over the replicas."""
        self._chk(lib.smore_group_train_walklets(self.g, int(walk_begin), int(walk_end), int(walk_times),
                                                 int(walk_steps), int(window_min), int(window_max), int(K),
                                                 float(alpha0), int(seed), _lib.MODE[mode], int(per), _lib.sync_rule(mean)),
                  "train_walklets")

    def train_app(self, unit_begin, unit_end, walk_times, sample_times, jump, K, alpha0, seed, order,
                  mode="hybrid", per=0, mean="adaptive"):
        """APP::Train (src/model/APP.cpp:59-120) over the replicas."""
        order = np.ascontiguousarray(order, np.int64)
        self._chk(lib.smore_group_train_app(self.g, int(unit_begin), int(unit_end), int(walk_times),
                                            int(sample_times), float(jump), int(K), float(alpha0), int(seed),
                                            ptr(order), _lib.MODE[mode], int(per), _lib.sync_rule(mean)), "train_app")

    def train_hpe(self, begin, count, total, walk_steps, K, reg, alpha0, seed, mode="hybrid", per=0, mean="adaptive"):
        """HPE::Train (src/model/HPE.cpp:94-150) over the replicas."""
        self._chk(lib.smore_group_train_hpe(self.g, int(begin), int(count), int(total), int(walk_steps), int(K),
                                            float(reg), float(alpha0), int(seed), _lib.MODE[mode], int(per),
                                            _lib.sync_rule(mean)), "train_hpe")


def deepwalk_order(V, walk_times, skip):
    """Walk start order of DeepWalk::Train (src/model/DeepWalk.cpp:122-131)."""
    out = np.zeros(int(V) * int(walk_times), np.int64)
    rc = lib.smore_deepwalk_order(int(V), int(walk_times), int(skip), ptr(out))
    if rc != _lib.OK:
        raise _lib.SmoreError("deepwalk_order failed")
    return out
