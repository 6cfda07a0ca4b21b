"""A second, independent restatement of the Go reference (pkg/pronet,
internal/models) written line by line in pure Python (fp64), used to pin the C
oracle's Go-semantics functions: there is no Go toolchain in this image, so
the Go path has no executable oracle.  Small cases only.

Draws use the build's RNG spec (Philox words from the oracle library, itself
pinned by Random123 known answers): Intn(n) -> floor(k*n/2^32),
Float64() -> k*2^-32.
"""
import math

from oracle import oracle as orc

MAX_SIGMOID, TABLE = 8.0, 1000
SIG = [1.0 / (1.0 + math.exp(-(i * 2.0 * MAX_SIGMOID / TABLE - MAX_SIGMOID))) for i in range(TABLE + 1)]


def fast_sigmoid(x):                       # pkg/pronet/pronet.go:98-109
    if x < -MAX_SIGMOID:
        return 0.0
    if x > MAX_SIGMOID:
        return 1.0
    idx = int((x + MAX_SIGMOID) * float(TABLE) / MAX_SIGMOID / 2.0)
    return SIG[min(idx, TABLE)]


def build_alias(dist, power):              # pkg/pronet/alias.go:10-90
    n = len(dist)
    prob, alias = [0.0] * n, [0] * n
    norm = [math.pow(x, power) if x > 0 else 0.0 for x in dist]
    s = 0.0
    for x in norm:
        s += x
    if s == 0:
        return [1.0] * n, list(range(n))
    norm = [x * float(n) / s for x in norm]
    small = [i for i in range(n) if norm[i] < 1.0]
    large = [i for i in range(n) if norm[i] >= 1.0]
    while small and large:
        l, g = small.pop(), large.pop()
        prob[l], alias[l] = norm[l], g
        norm[g] = norm[g] + norm[l] - 1.0
        (small if norm[g] < 1.0 else large).append(g)
    while large:
        g = large.pop()
        prob[g], alias[g] = 1.0, g
    while small:
        l = small.pop()
        prob[l], alias[l] = 1.0, l
    return prob, alias


class Rng:
    """Sequential draws of one unit (sample or walk) under the RNG spec."""

    def __init__(self, seed, stream, unit, n):
        self.w = list(orc.words(seed, stream, unit, n))
        self.i = 0

    def word(self):
        k = int(self.w[self.i])
        self.i += 1
        return k

    def intn(self, n):
        return (self.word() * n) >> 32

    def float64(self):
        return self.word() * 2.0 ** -32


class ProNet:
    def __init__(self, names, src, dst, w):
        self.V = len(names)
        self.graph = {v: [] for v in range(self.V)}
        self.weights = {v: [] for v in range(self.V)}
        for a, b, x in zip(src, dst, w):
            self.graph[int(a)].append(int(b))
            self.weights[int(a)].append(float(x))
        out_d, in_d = [0.0] * self.V, [0.0] * self.V
        for v in range(self.V):                     # buildGraph, pronet.go:202-213
            for i, n in enumerate(self.graph[v]):
                out_d[v] += self.weights[v][i]
                in_d[n] += self.weights[v][i]
        self.vertex_at = build_alias(out_d, 1.0)
        self.negative_at = build_alias([in_d[v] + out_d[v] for v in range(self.V)], 0.75)

    @staticmethod
    def alias_sample(at, rng):                      # alias.go:93-106
        prob, alias = at
        i = rng.intn(len(prob))
        r = rng.float64()
        return i if r < prob[i] else alias[i]

    def source(self, rng):
        return self.alias_sample(self.vertex_at, rng)

    def negative(self, rng):
        return self.alias_sample(self.negative_at, rng)

    def target(self, vid, rng):                     # pronet.go:257-284
        nb = self.graph[vid]
        if not nb:
            return -1
        total = 0.0
        for x in self.weights[vid]:
            total += x
        r = rng.float64() * total
        cum = 0.0
        for i, x in enumerate(self.weights[vid]):
            cum += x
            if r <= cum:
                return nb[i]
        return nb[-1]

    # ---- updates
    def sgd(self, ve, ce, label, alpha, vg, cg):  # optimizer.go:61-84
        score = 0.0
        for d in range(len(ve)):
            score += ve[d] * ce[d]
        grad = alpha * (label - fast_sigmoid(score))
        for d in range(len(ve)):
            vg[d] += grad * ce[d]
            cg[d] += grad * ve[d]

    def update_pair(self, W, C, v, c, K, alpha, rng):   # optimizer.go:21-58
        dim = len(W[v])
        vg, cg = [0.0] * dim, [0.0] * dim
        self.sgd(W[v], C[c], 1.0, alpha, vg, cg)
        for _ in range(K):
            n = self.negative(rng)
            if n == c:
                continue
            ng = [0.0] * dim
            self.sgd(W[v], C[n], 0.0, alpha, vg, ng)
            for d in range(dim):
                C[n][d] += ng[d]
        for d in range(dim):
            W[v][d] += vg[d]
            C[c][d] += cg[d]

    def first_order(self, W, s, t, K, alpha, rng):      # internal/models/line/line.go:153-200
        dim = len(W[s])
        score = 0.0
        for d in range(dim):
            score += W[s][d] * W[t][d]
        grad = alpha * (1.0 - fast_sigmoid(score))
        vg = [grad * W[t][d] for d in range(dim)]
        cg = [grad * W[s][d] for d in range(dim)]
        for _ in range(K):
            n = self.negative(rng)
            if n == t or n == s:
                continue
            sc = 0.0
            for d in range(dim):
                sc += W[s][d] * W[n][d]
            gr = alpha * (0.0 - fast_sigmoid(sc))
            for d in range(dim):
                vg[d] += gr * W[n][d]
                W[n][d] += gr * W[s][d]
        for d in range(dim):
            W[s][d] += vg[d]
            W[t][d] += cg[d]

    def bpr(self, W, C, u, i, j, alpha, lam):          # optimizer.go:87-117
        dim = len(W[u])
        pos = neg = 0.0
        for d in range(dim):
            pos += W[u][d] * C[i][d]
            neg += W[u][d] * C[j][d]
        gc = alpha * fast_sigmoid(neg - pos)
        for d in range(dim):
            vgr = gc * (C[i][d] - C[j][d])
            pg = gc * W[u][d]
            ngr = -gc * W[u][d]
            W[u][d] += vgr - lam * alpha * W[u][d]
            C[i][d] += pg - lam * alpha * C[i][d]
            C[j][d] += ngr - lam * alpha * C[j][d]


def alpha_at(count, alpha0, total):              # line.go:133-142 (count before this sample)
    u = count // 10000
    if u == 0:
        return alpha0
    return max(alpha0 * (1.0 - float(u * 10000) / float(total)), alpha0 * 0.0001)


def train(pn, model, W, C, K, alpha0, lam, total, begin, end, seed):
    for s in range(begin, end):
        nk = 1 if model == "bpr" else K
        rng = Rng(seed, 0, s, 3 + 2 * nk)
        v = pn.source(rng)
        c = pn.target(v, rng)
        if c < 0:
            continue
        a = alpha_at(s, alpha0, total)
        if model == "line2":
            pn.update_pair(W, C, v, c, K, a, rng)
        elif model == "line1":
            pn.first_order(W, v, c, K, a, rng)
        else:
            j = pn.negative(rng)
            pn.bpr(W, C, v, c, j, a, lam)


def deepwalk(pn, W, C, walk_times, steps, window, K, alpha0, seed, order):
    total = walk_times * pn.V
    for wk in range(total):
        rng = Rng(seed, 1, wk, 4096)
        walk = [int(order[wk])]
        cur = walk[0]
        for _ in range(steps):                   # pronet.go:292-307
            nxt = pn.target(cur, rng)
            if nxt == -1:
                break
            walk.append(nxt)
            cur = nxt
        a = alpha_at(wk, alpha0, total)
        for i in range(len(walk)):               # pronet.go:310-333
            for j in range(max(0, i - window), min(len(walk), i + window + 1)):
                if i != j:
                    pn.update_pair(W, C, walk[i], walk[j], K, a, rng)


def node2vec_walk(pn, start, steps, p, q, rng):
    """biasedRandomWalk / biasedTargetSample / areNeighbors
    (internal/models/node2vec/node2vec.go:82-175), literally."""
    walk = [start]
    if steps == 0:
        return walk
    first = pn.target(start, rng)
    if first == -1:
        return walk
    walk.append(first)
    for _ in range(1, steps):
        cur, prev = walk[-1], walk[-2]
        nb = pn.graph[cur]
        if not nb:
            break
        bw, total = [], 0.0
        for i, n in enumerate(nb):
            if n == prev:
                bias = 1.0 / p
            elif n in pn.graph[prev]:
                bias = 1.0
            else:
                bias = 1.0 / q
            bw.append(pn.weights[cur][i] * bias)
            total += bw[-1]
        if total == 0:
            walk.append(nb[rng.intn(len(nb))])
            continue
        r = rng.float64() * total
        cum, nxt = 0.0, nb[-1]
        for i, x in enumerate(bw):
            cum += x
            if r <= cum:
                nxt = nb[i]
                break
        walk.append(nxt)
    return walk


def metapath_walk(graph, ntype, start, meta_path, steps, rng):
    """MetaPathWalk + SampleNeighborByType (pkg/hetero/hetero_graph.go:206-256),
    literally: graph[v] = Edges[v] in push order, ntype[v] = the node's type."""
    if len(meta_path) < 2:
        return [start]
    walk, cur, idx = [start], start, 0
    while len(walk) < steps + 1:
        if ntype[cur] != meta_path[idx % len(meta_path)]:
            break
        nt = meta_path[(idx + 1) % len(meta_path)]
        indices = [i for i, n in enumerate(graph[cur]) if ntype[n] == nt]
        if not indices:
            break
        nxt = graph[cur][indices[rng.intn(len(indices))]]
        walk.append(nxt)
        cur = nxt
        idx += 1
    return walk


def ctdne_walk(out_edges, tmin, tmax, max_time, window, start, steps, rng):
    """CTDNE's start time (internal/models/ctdne/ctdne.go:159-170) and
    TemporalRandomWalk / GetTemporalNeighbors / SampleTemporalNeighbor
    (pkg/temporal/temporal_graph.go:181-252), literally; out_edges[v] = list of
    (to, ts) sorted by ts."""
    lo, hi = tmin[start], tmax[start]
    if lo == 0 and hi == 0:
        return [start]
    rng_ = hi - lo
    if rng_ == 0:
        rng_ = window
    now = lo + rng.float64() * rng_
    walk, cur = [start], start
    while len(walk) < steps + 1:
        end = min(now + window, max_time)
        nb = []
        for to, t in out_edges[cur]:
            if now <= t <= end:
                nb.append(to)
            if t > end:
                break
        if not nb:
            break
        idx = rng.intn(len(nb))
        walk.append(nb[idx])
        now = out_edges[cur][idx][1]
        cur = nb[idx]
    return walk
