"""Model drivers mirroring the reference's Go models
(internal/models/{line,bpr,deepwalk}): New / LoadEdgeList / Init / Train /
SaveWeights with the Go argument meaning and the Go rules (the context runs in
Go semantics):

  * LINE   internal/models/line/line.go:73-151: total = sample_times * MaxLine,
           order 1 -> updateFirstOrder on W, order 2 -> UpdatePair on W, C;
  * BPR    internal/models/bpr/bpr.go:61-136: total = sample_times * MaxLine,
           UpdateBPRPair(W users, C items, lambda), one negative per sample;
  * DeepWalk internal/models/deepwalk/deepwalk.go:61-142: walk_times * MaxVid
           walks, dead-end stop, fixed window, UpdatePair per skip-gram pair;
  * Node2Vec internal/models/node2vec/node2vec.go:43-258: DeepWalk's loop over
           the biased second-order walk (p return, q in-out);
  * Metapath2Vec internal/models/metapath2vec/metapath2vec.go:30-200 over a
           pkg/hetero graph: meta-path-typed walks, uniform negatives;
  * CTDNE  internal/models/ctdne/ctdne.go:29-200 over a pkg/temporal graph:
           time-respecting walks, activity^0.75 negatives.

Differences from the Go code, documented in DESIGN.md: draws come from the
seeded Philox spec (not time-seeded math/rand); the learning rate of a sample
follows its global index (Go's shared counter skips dead-end samples); tables
are fp32; Init uses the on-device uniform (u - 0.5) / dim generator.
"""
from . import _lib
import numpy as np

from . import _lib as _l
from .models import CHUNK, MONITOR, _progress
from .pronet import ProNet, deepwalk_order


def _alpha(done, alpha0, total):
    return max(alpha0 * (1.0 - (done // MONITOR * MONITOR) / total), alpha0 * 1e-4)


class _GoModel:
    def __init__(self, device=0, mode="atomic", seed=1):
        self.pnet = ProNet(device)
        self.mode, self.seed = mode, seed
        self.dim = 0
        self.undirected = False

    @classmethod
    def New(cls, device=0, mode="atomic", seed=1):
        return cls(device, mode, seed)

    def LoadEdgeList(self, filename, undirected):
        """pkg/pronet/pronet.go:112-166 (same records as the C++ loader)."""
        self.pnet.LoadEdgeList(filename, undirected)
        self.pnet.set_semantics("go")
        self.undirected = bool(undirected)

    @property
    def MaxLine(self):
        # Go counts input records; an undirected record adds two edge slots
        E = self.pnet.MAX_line
        return E // 2 if self.undirected else E

    def _alloc(self, dim, ntab):
        print("Model Setting:\n\tdimension:\t\t%d" % dim)
        self.dim = dim
        self.pnet.alloc_tables(dim, ntab)
        for t in range(ntab):
            self.pnet.init_table_uniform(t, self.seed + t)

    def _run_edges(self, model, total, K, alpha, lam):
        done = 0
        while done < total:
            n = min(CHUNK, total - done)
            self.pnet.train_edges(model, done, n, total, K, alpha, lam, self.seed, self.mode)
            done += n
            _progress(_alpha(done, alpha, total), done / total)
        _progress(_alpha(total, alpha, total), 1.0, "\n")

    def SaveWeights(self, filename):
        print("Save Model:")
        self.pnet.save_weights(_lib.W, filename, 1)
        print("\tSave to <%s>" % filename)

    @property
    def w_vertex(self):
        return self.pnet.get_table(_lib.W)


class LINE(_GoModel):
    First, Second = 1, 2

    def Init(self, dim, order=2):
        self.order = 1 if order == 1 else 2
        self._alloc(dim, 1 if self.order == 1 else 2)

    def Train(self, sample_times, negative_samples, alpha, workers=1):
        print("Model:\n\t[LINE]\nLearning Parameters:")
        print("\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n\talpha:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (sample_times, negative_samples, alpha, workers))
        print("Start Training:")
        self._run_edges("line1" if self.order == 1 else "line2", int(sample_times) * self.MaxLine,
                        negative_samples, alpha, 0.0)

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)


class BPR(_GoModel):
    def Init(self, dim):
        self._alloc(dim, 2)

    def Train(self, sample_times, alpha, lam, workers=1):
        print("Model:\n\t[BPR]\nLearning Parameters:")
        print("\tsample_times:\t\t%d\n\talpha:\t\t\t%.6f\n\tlambda:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (sample_times, alpha, lam, workers))
        print("Start Training:")
        self._run_edges("bpr", int(sample_times) * self.MaxLine, 1, alpha, lam)


class DeepWalk(_GoModel):
    def Init(self, dim):
        self._alloc(dim, 2)

    def Train(self, walk_times, walk_steps, window_size, negative_samples, alpha, workers=1):
        print("Model:\n\t[DeepWalk]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_size:\t\t%d\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_size, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, 0)
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * window_size + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_deepwalk(done, done + n, walk_times, walk_steps, window_size, negative_samples,
                                     alpha, self.seed, order, self.mode)
            done += n
            _progress(_alpha(done, alpha, total), done / total)
        print()

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)


class Node2Vec(DeepWalk):
    """internal/models/node2vec/node2vec.go: Init(dim, p, q), Train as DeepWalk's
    over biasedRandomWalk (on the GPU: smore_train_node2vec)."""

    def Init(self, dim, p=1.0, q=1.0):
        if not (p > 0 and q > 0):
            raise ValueError("node2vec: p and q must be > 0")
        self.p, self.q = float(p), float(q)
        self._alloc(dim, 2)
        print("\tp (return param):\t%.2f\n\tq (in-out param):\t%.2f" % (self.p, self.q))

    def Train(self, walk_times, walk_steps, window_size, negative_samples, alpha, workers=1):
        print("Model:\n\t[Node2Vec]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_size:\t\t%d\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_size, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, 0)
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * window_size + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_node2vec(done, done + n, walk_times, walk_steps, window_size, negative_samples,
                                     alpha, self.p, self.q, self.seed, order, self.mode)
            done += n
            _progress(_alpha(done, alpha, total), done / total)
        print()


def load_hetero(filename, undirected):
    """pkg/hetero (*HeteroGraph).LoadEdgeList (hetero_graph.go:60-160): lines
    "src srcType dst dstType edgeType [weight]" (fewer than 5 fields skipped,
    an unparsable weight is 1), node ids and type ids in first-appearance
    order (a node keeps its first type), edges appended per source in input
    order, the reverse edge right after when undirected.  Host-side input
    parsing; a Go caller keeps its own loader and passes the same arrays."""
    ids, names, ntype, tids, tkeys = {}, [], [], {}, []
    src, dst, w = [], [], []

    def node(name, typ):
        if name in ids:
            return ids[name]
        ids[name] = len(names)
        names.append(name)
        if typ not in tids:
            tids[typ] = len(tkeys)
            tkeys.append(typ)
        ntype.append(tids[typ])
        return ids[name]

    with open(filename) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 5:
                continue
            x = 1.0
            if len(parts) >= 6:
                try:
                    x = float(parts[5])
                except ValueError:
                    x = 1.0
            a, b = node(parts[0], parts[1]), node(parts[2], parts[3])
            src.append(a), dst.append(b), w.append(x)
            if undirected:
                src.append(b), dst.append(a), w.append(x)
    return names, np.array(ntype, np.int32), tkeys, np.array(src, np.int32), np.array(dst, np.int32), \
        np.array(w, np.float64)


class Metapath2Vec(_GoModel):
    """internal/models/metapath2vec/metapath2vec.go: LoadEdgeList (pkg/hetero),
    AddMetaPath, Init, Train (on the GPU: smore_train_metapath2vec),
    SaveEmbeddings.  NegativeAT = BuildAliasMethod(ones, 0.75) (:140-145): every
    normalised entry is exactly 1.0, so the table is {prob 1, alias i}."""

    def LoadEdgeList(self, filename, undirected):
        names, self.ntype, self.type_keys, s, d, w = load_hetero(filename, undirected)
        self.names = names
        self.pnet.set_graph_edges(len(names), s, d, w)
        self.pnet.set_semantics("go")
        self.pnet.set_node_types(self.ntype, len(self.type_keys))
        V = len(names)
        self.pnet.set_alias(_l.AT_NEGATIVE, np.ones(V), np.arange(V, dtype=np.int64))
        self.meta_paths = []
        self.undirected = bool(undirected)

    def AddMetaPath(self, meta_path):
        types = meta_path.split()
        if len(types) < 2:
            raise ValueError("meta-path must have at least 2 types, got: %s" % meta_path)
        for t in types:
            if t not in self.type_keys:
                raise ValueError("invalid meta-path: unknown node type in meta-path: %s" % t)
        self.meta_paths.append([self.type_keys.index(t) for t in types])
        print("Added meta-path: %s" % meta_path)

    def Init(self, dim):
        self._alloc(dim, 2)

    def Train(self, walk_times, walk_steps, window_size, negative_samples, alpha, workers=1):
        if not self.meta_paths:
            print("Error: No meta-paths defined. Use AddMetaPath() before training.")
            return
        print("Model:\n\t[Metapath2Vec - Heterogeneous Graph Embedding]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_size:\t\t%d\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_size, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, 0)
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * window_size + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_metapath2vec(done, done + n, walk_times, walk_steps, window_size, negative_samples,
                                         alpha, self.meta_paths, self.seed, order, self.mode)
            done += n
            _progress(_alpha(done, alpha, total), done / total)
        print()

    def SaveEmbeddings(self, filename):
        """metapath2vec.go:218-245: "V dim" header, rows "name[type] %.6f ..."."""
        print("Save Model:")
        W = self.pnet.get_table(_lib.W)
        with open(filename, "w") as f:
            f.write("%d %d\n" % (len(self.names), self.dim))
            for i, name in enumerate(self.names):
                f.write("%s[%s]%s\n" % (name, self.type_keys[self.ntype[i]], "".join(" %.6f" % x for x in W[i])))
        print("\tSave to <%s>" % filename)

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)


def load_temporal(filename):
    """pkg/temporal (*TemporalGraph).LoadEdgeList (temporal_graph.go:60-130):
    lines "src dst timestamp" (fewer than 3 fields or an unparsable timestamp:
    skipped), ids in first-appearance order, directed edges."""
    ids, names, src, dst, ts = {}, [], [], [], []

    def node(name):
        if name not in ids:
            ids[name] = len(names)
            names.append(name)
        return ids[name]

    with open(filename) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 3:
                continue
            try:
                t = float(parts[2])
            except ValueError:
                continue
            a, b = node(parts[0]), node(parts[1])
            src.append(a), dst.append(b), ts.append(t)
    return names, np.array(src, np.int32), np.array(dst, np.int32), np.array(ts, np.float64)


class CTDNE(_GoModel):
    """internal/models/ctdne/ctdne.go: LoadEdgeList (pkg/temporal), Init(dim,
    timeWindow), Train (on the GPU: smore_train_ctdne), SaveWeights.  The
    negative table BuildAliasMethod(activity, 0.75) (:119-131) is the Go
    negative table of the temporal edges with unit weights (in + out counts;
    every loaded vertex has an edge)."""

    def LoadEdgeList(self, filename):
        self.names, s, d, ts = load_temporal(filename)
        self.pnet.set_graph_edges(len(self.names), s, d, np.ones(len(s)))
        self.pnet.set_semantics("go")
        self.pnet.set_temporal_edges(s, d, ts)
        self.span = (float(ts.max()) - float(ts.min())) if len(ts) else 0.0
        self.undirected = False

    def Init(self, dim, time_window=0.0):
        self.time_window = time_window if time_window > 0 else self.span * 0.1
        self._alloc(dim, 2)
        print("\ttime window:\t\t%.2f" % self.time_window)

    def Train(self, walk_times, walk_steps, window_size, negative_samples, alpha, workers=1):
        print("Model:\n\t[CTDNE - Continuous-Time Dynamic Network Embeddings]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_size:\t\t%d\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%.6f\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_size, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, 0)
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * window_size + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_ctdne(done, done + n, walk_times, walk_steps, window_size, negative_samples, alpha,
                                  self.time_window, self.seed, order, self.mode)
            done += n
            _progress(_alpha(done, alpha, total), done / total)
        print()

    def SaveEmbeddings(self, filename):
        """ctdne.go:212-238: "V dim" header, rows "name %.6f ..."."""
        print("Save Model:")
        W = self.pnet.get_table(_lib.W)
        with open(filename, "w") as f:
            f.write("%d %d\n" % (len(self.names), self.dim))
            for i, name in enumerate(self.names):
                f.write("%s%s\n" % (name, "".join(" %.6f" % x for x in W[i])))
        print("\tSave to <%s>" % filename)

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)
