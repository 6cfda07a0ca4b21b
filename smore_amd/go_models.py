"""Model drivers mirroring the reference's Go models
(internal/models/{line,bpr,deepwalk}): New / LoadEdgeList / Init / Train /
SaveWeights with the Go argument meaning and the Go rules (the context runs in
Go semantics):

  * LINE   internal/models/line/line.go:73-151: total = sample_times * MaxLine,
           order 1 -> updateFirstOrder on W, order 2 -> UpdatePair on W, C;
  * BPR    internal/models/bpr/bpr.go:61-136: total = sample_times * MaxLine,
           UpdateBPRPair(W users, C items, lambda), one negative per sample;
  * DeepWalk internal/models/deepwalk/deepwalk.go:61-142: walk_times * MaxVid
           walks, dead-end stop, fixed window, UpdatePair per skip-gram pair.

Differences from the Go code, documented in DESIGN.md: draws come from the
seeded Philox spec (not time-seeded math/rand); the learning rate of a sample
follows its global index (Go's shared counter skips dead-end samples); tables
are fp32; Init uses the on-device uniform (u - 0.5) / dim generator.
"""
from . import _lib
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
