"""Model drivers mirroring the reference's C++ model classes
(src/model/{LINE,MF,BPR,DeepWalk,Walklets,APP,HPE}.h): LoadEdgeList / Init / Train / SaveWeights
with the same argument meaning, banners and learning-rate schedule.  The hot
loop is one HIP launch per chunk through the C ABI.

Differences from the reference, all deliberate and documented in DESIGN.md:
  * draws come from the seeded Philox spec (`seed`), not random_device;
  * `workers` is accepted for signature parity; the GPU runs one Hogwild
    stream of samples whose learning rate follows the 1-worker schedule
    (scatter "hybrid" by default: atomic adds for hot rows);
  * embeddings are fp32.
"""
import sys

from . import _lib
from .pronet import ProNet, deepwalk_order

MONITOR = 10000
CHUNK = 1 << 26   # samples per launch between progress lines


def _progress(alpha, frac, end="\r"):
    sys.stdout.write("\tAlpha: %.6f\tProgress: %.3f %%%s" % (alpha, frac * 100, end))
    sys.stdout.flush()


def _alpha_at(c, alpha0, total):
    u = c // MONITOR
    if u == 0:
        return alpha0
    return max(alpha0 * (1.0 - ((u - 1) * MONITOR) / total), alpha0 * 0.0001)


class _EdgeModel:
    model = None
    count_base = 0

    def __init__(self, device=0, mode="hybrid", seed=1):
        self.pnet = ProNet(device)
        self.mode = mode
        self.seed = seed
        self.dim = 0

    def LoadEdgeList(self, filename, undirect):
        self.pnet.LoadEdgeList(filename, undirect)

    def SaveWeights(self, model_name, fmt=0):
        print("Save Model:")
        self.pnet.save_weights(_lib.W, model_name, fmt)
        print("\tSave to <%s>" % model_name)

    def _run(self, total, n_samples, K, alpha, reg):
        done = 0
        while done < n_samples:
            n = min(CHUNK, n_samples - done)
            self.pnet.train_edges(self.model, done, n, total, K, alpha, reg, self.seed, self.mode)
            done += n
            _progress(_alpha_at(done + self.count_base, alpha, total), done / total)
        _progress(_alpha_at(n_samples + self.count_base, alpha, total), 1.0, "\n")

    @property
    def w_vertex(self):
        return self.pnet.get_table(_lib.W)


class LINE(_EdgeModel):
    """LINE (src/model/LINE.{h,cpp}); order 2 uses W,C, order 1 shares W."""
    count_base = 1   # src/model/LINE.cpp:166 count starts at 1

    def Init(self, dimension, order=2):
        print("Model Setting:")
        print("\tdimension:\t\t%d" % dimension)
        self.dim = dimension
        self.order = 1 if order == 1 else 2
        self.model = "line1" if self.order == 1 else "line2"
        self.pnet.alloc_tables(dimension, 1 if self.order == 1 else 2)
        self.pnet.init_table_glibc(_lib.W, 0)          # src/model/LINE.cpp:83
        if self.order == 2:
            self.pnet.zero_table(_lib.CTX)            # src/model/LINE.cpp:92

    def Train(self, sample_times, negative_samples, alpha, workers=1):
        print("Model:\n\t[LINE]\nLearning Parameters:")
        print("\torder:\t\t\t%d%s" % (self.order, "st" if self.order == 1 else "nd"))
        print("\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d"
              % (sample_times, negative_samples, alpha, workers))
        print("Start Training:")
        total = int(sample_times) * 1000000
        # one worker runs counts 1 .. total-1 (src/model/LINE.cpp:166-170)
        self._run(total, total - 1, negative_samples, alpha, 0.0)

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)


class MF(_EdgeModel):
    """MF (src/model/MF.{h,cpp}): UpdateFactorizedPair on one table."""
    model = "mf"

    def __init__(self, device=0, mode="hybrid", seed=1):
        super().__init__(device, mode, seed)
        self.pnet.SetNegativeMethod("no_degrees")   # src/model/MF.cpp:4-7

    def Init(self, dim):
        print("Model Setting:\n\tdimension:\t\t%d" % dim)
        self.dim = dim
        self.pnet.alloc_tables(dim, 1)
        self.pnet.init_table_glibc(_lib.W, 0)

    def Train(self, sample_times, negative_samples, alpha, reg, workers=1):
        print("Model:\n\t[MF]\nLearning Parameters:")
        print("\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tregularization:\t\t%g"
              "\n\tworkers:\t\t%d" % (sample_times, negative_samples, alpha, reg, workers))
        print("Start Training:")
        total = int(sample_times) * 1000000
        self._run(total, total, negative_samples, alpha, reg)


class BPR(_EdgeModel):
    """BPR (src/model/BPR.{h,cpp}): UpdateBPRPair, 5 rounds, one table."""
    model = "bpr"

    def __init__(self, device=0, mode="hybrid", seed=1):
        super().__init__(device, mode, seed)
        self.pnet.SetNegativeMethod("no_degrees")   # src/model/BPR.cpp:4-7

    def Init(self, dim):
        print("Model Setting:\n\tdimension:\t\t%d" % dim)
        self.dim = dim
        self.pnet.alloc_tables(dim, 1)
        self.pnet.init_table_glibc(_lib.W, 0)

    def Train(self, sample_times, negative_samples, alpha, reg, workers=1):
        # `negative_samples` and `reg` are ignored by the reference BPR rule
        # (src/proNet.cpp:1406-1455 hard-codes 5 rounds and 0.0025/0.025)
        print("Model:\n\t[BPR]\nLearning Parameters:")
        print("\tsample_times:\t\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d" % (sample_times, alpha, workers))
        print("Start Training:")
        total = int(sample_times) * 1000000
        self._run(total, total, 5, alpha, 0.0)


class DeepWalk(_EdgeModel):
    """DeepWalk (src/model/DeepWalk.{h,cpp}): random walks + skip-gram pairs."""

    def Init(self, dim):
        print("Model Setting:\n\tdimension:\t\t%d" % dim)
        self.dim = dim
        V = self.pnet.MAX_vid
        self.pnet.alloc_tables(dim, 2)
        self.pnet.init_table_glibc(_lib.W, 0)
        self.pnet.init_table_glibc(_lib.CTX, V * dim)   # src/model/DeepWalk.cpp:50-55
        self._rand_used = 2 * V * dim

    def Train(self, walk_times, walk_steps, window_size, negative_samples, alpha, workers=1):
        print("Model:\n\t[DeepWalk]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_size:\t\t%d\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%g\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_size, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, self._rand_used)
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * window_size + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_deepwalk(done, done + n, walk_times, walk_steps, window_size, negative_samples,
                                     alpha, self.seed, order, self.mode)
            done += n
            _progress(max(alpha * (1 - (done // MONITOR * MONITOR) / total), alpha * 1e-4), done / total)
        print()

    @property
    def w_context(self):
        return self.pnet.get_table(_lib.CTX)


class Walklets(DeepWalk):
    """Walklets (src/model/Walklets.{h,cpp}; a DeepWalk subclass there too):
    walks from every vertex in id order, pairs at distances
    [window_min, window_max] (ScaleSkipGrams, src/proNet.cpp:928-987)."""

    def Train(self, walk_times, walk_steps, window_min, window_max, negative_samples, alpha, workers=1):
        print("Model:\n\t[Walklets]\nParameters:")
        print("\twalk_times:\t\t%d\n\twalk_steps:\t\t%d\n\twindow_min:\t\t%d\n\twindow_max:\t\t%d"
              "\n\tnegative_samples:\t%d\n\talpha:\t\t\t%g\n\tworkers:\t\t%d"
              % (walk_times, walk_steps, window_min, window_max, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        total = walk_times * V
        step = max(1, CHUNK // (walk_steps * 2 * (window_max - window_min + 1) + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_walklets(done, done + n, walk_times, walk_steps, window_min, window_max,
                                     negative_samples, alpha, self.seed, self.mode)
            done += n
            _progress(max(alpha * (1 - (done // MONITOR * MONITOR) / total), alpha * 1e-4), done / total)
        print("\tProgress:\t\t100.00 %")


class APP(DeepWalk):
    """APP (src/model/APP.{h,cpp}): per start vertex, sample_times jumping
    random walks (JumpingRandomWalk, src/proNet.cpp:685-701), UpdatePair of
    (start, walk end) each; both tables random-initialised, starts shuffled
    with glibc rand() as DeepWalk's."""

    def Train(self, walk_times, sample_times, jump, negative_samples, alpha, workers=1):
        print("Model:\n\t[APP]\nLearning Parameters:")
        print("\twalk_times:\t\t%d\n\tsample_times:\t\t%d\n\tjumping factor:\t\t%g\n\tnegative_samples:\t%d"
              "\n\talpha:\t\t\t%g\n\tworkers:\t\t%d"
              % (walk_times, sample_times, jump, negative_samples, alpha, workers))
        print("Start Training:")
        V = self.pnet.MAX_vid
        order = deepwalk_order(V, walk_times, self._rand_used)
        total = walk_times * V
        units = total * sample_times
        step = max(sample_times, CHUNK // sample_times * sample_times)
        done = 0
        while done < units:
            n = min(step, units - done)
            self.pnet.train_app(done, done + n, walk_times, sample_times, jump, negative_samples, alpha, self.seed,
                                order, self.mode)
            done += n
            w = done // sample_times
            _progress(max(alpha * (1 - (w // MONITOR * MONITOR) / total), alpha * 1e-4), w / total)
        print()


class HPE(LINE):
    """HPE (src/model/HPE.{h,cpp}; a LINE subclass there too): per sample
    v1 = SourceSample, v2 = TargetSample(v1), UpdateCommunity(v1, v2) over
    walk_steps steps (regularised sigmoid rule) then UpdatePair(v2, v1)."""

    def Init(self, dim):
        print("Model Setting:\n\tdimension:\t\t%d" % dim)
        self.dim = dim
        self.order = 2
        V = self.pnet.MAX_vid
        self.pnet.alloc_tables(dim, 2)
        self.pnet.init_table_glibc(_lib.W, 0)           # src/model/HPE.cpp:38-45
        self.pnet.init_table_glibc(_lib.CTX, V * dim)   # src/model/HPE.cpp:47-52

    def Train(self, sample_times, walk_steps, negative_samples, reg, alpha, workers=1):
        print("Model:\n\t[HPE]\nLearning Parameters:")
        print("\tsample_times:\t\t%d\n\tnegative_samples:\t%d\n\twalk_steps:\t\t%d\n\tregularization:\t\t%g"
              "\n\talpha:\t\t\t%g\n\tworkers:\t\t%d"
              % (sample_times, negative_samples, walk_steps, reg, alpha, workers))
        print("Start Training:")
        total = int(sample_times) * 1000000
        step = max(1, CHUNK // (walk_steps + 1))
        done = 0
        while done < total:
            n = min(step, total - done)
            self.pnet.train_hpe(done, n, total, walk_steps, negative_samples, reg, alpha, self.seed, self.mode)
            done += n
            _progress(_alpha_at(done, alpha, total), done / total)
        _progress(_alpha_at(total, alpha, total), 1.0, "\n")
