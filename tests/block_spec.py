"""The 2-D block schedule's draw tables restated in numpy over the oracle's
graph (test infrastructure: the checker of smore_amd/csrc/blocks.cpp and
train_blocks.hip, never the product).

A context that is part r of N (smore_block_setup) holds:
  * W part bounds: contiguous ids of equal source mass (the midpoint rule of
    capi.cpp source_bounds) under the source law SourceSample draws
    (src/proNet.cpp:647-657);
  * 2N C block bounds: the same rule over NegativeSample's law (:623-633);
  * per C block k, the negative law restricted to the block, as a Go-rule
    alias table (power 1) over the block's vertices;
  * per C block k, the "atoms" of part r: for each source v of the part (id
    order) and CSR slot i (push order) the TargetSample outcomes (v,
    target_i) with mass p(v) prob_i / deg(v) and (v, alias_i) with mass
    p(v) (1 - prob_i) / deg(v) (:671-683), those whose context is in block k,
    in that order, with a Go-rule alias table over their masses.
A draw of sample s in cell (r, k): Philox words 0 (p), 1 (atom index) of
unit s, stream 0; negative j from block 1 + j/2 (index, then p) -- the
slots of the one-context draw kernel.
"""
import numpy as np

from oracle import oracle as orc


def alias_law(prob, alias, scale, self_ids=None):
    """Marginal of an alias table (capi alias_marginal): loop order kept, so
    the float sums are the product's."""
    n = len(prob)
    p = [0.0] * (int(max(self_ids)) + 1 if self_ids is not None else n)
    for i in range(n):
        s = int(self_ids[i]) if self_ids is not None else i
        p[s] += scale * float(prob[i])
        if alias[i] >= 0 and prob[i] < 1.0:
            p[int(alias[i])] += scale * (1.0 - float(prob[i]))
    return p


def part_bounds(p, n):
    V = len(p)
    total = 0.0
    for x in p:
        total += x
    b = [V] * (n + 1)
    b[0] = 0
    cum, nxt = 0.0, 1
    for v in range(V):
        if nxt >= n:
            break
        mid = (cum + 0.5 * p[v]) / total
        owner = min(n - 1, int(np.floor(mid * n)))
        while nxt <= owner and nxt < n:
            b[nxt] = v
            nxt += 1
        cum += p[v]
    return b


class BlockSpec:
    def __init__(self, g, nparts, part):
        self.g, self.n, self.r, self.nb = g, nparts, part, 2 * nparts
        V = g.V
        self.ps = alias_law(g.vprob, g.valias, 1.0 / V)
        self.pn = alias_law(g.nprob, g.nalias, 1.0 / V)
        self.wb = part_bounds(self.ps, nparts)
        self.cb = part_bounds(self.pn, self.nb)
        # negative tables per block (absolute ids)
        self.nthr = np.zeros(V, np.uint32)
        self.nal = np.zeros(V, np.int32)
        for k in range(self.nb):
            lo, hi = self.cb[k], self.cb[k + 1]
            prob, alias = orc.alias_go(np.array(self.pn[lo:hi]), 1.0)
            thr, al = orc.alias_encode(prob, alias + lo, np.arange(lo, hi, dtype=np.int32))
            self.nthr[lo:hi], self.nal[lo:hi] = thr, al
        # atoms of this part per block
        atoms = [[] for _ in range(self.nb)]
        off, tgt = g.offsets, g.targets
        for v in range(self.wb[part], self.wb[part + 1]):
            o, br = int(off[v]), int(off[v + 1] - off[v])
            if br == 0 or self.ps[v] <= 0:
                continue
            s = self.ps[v] / br
            for i in range(br):
                pr = float(g.cprob[o + i])
                for x, w in ((int(tgt[o + i]), s * pr),
                             (int(g.calias[o + i]), s * (1.0 - pr) if g.calias[o + i] >= 0 and pr < 1.0 else 0.0)):
                    if w > 0:
                        atoms[self.block_of(x)].append((v, x, w))
        self.atoms = atoms
        self.tabs = []
        tot = sum(w for a in atoms for _, _, w in a)
        self.mass = []
        for a in atoms:
            m = 0.0
            for _, _, w in a:
                m += w
            self.mass.append(m)
            if not a:
                self.tabs.append(None)
                continue
            prob, alias = orc.alias_go(np.array([w for _, _, w in a]), 1.0)
            self.tabs.append(orc.alias_encode(prob, alias))
        self.mass = [m / tot for m in self.mass]

    def block_of(self, x):
        return int(np.searchsorted(self.cb, x, side="right")) - 1

    def draw(self, k, seed, begin, count, K):
        """count x (2 + K) {v, c, n1..nK} of samples [begin, begin + count) in cell (r, k)."""
        out = np.zeros((count, 2 + K), np.int32)
        a = self.atoms[k]
        thr, al = self.tabs[k]
        lo, n = self.cb[k], self.cb[k + 1] - self.cb[k]
        for t in range(count):
            w = orc.words(seed, 0, begin + t, 4 + 2 * K)
            i = (int(w[1]) * len(a)) >> 32
            j = i if int(w[0]) < int(thr[i]) else int(al[i])
            out[t, 0], out[t, 1] = a[j][0], a[j][1]
            for q in range(K):
                ni = lo + ((int(w[4 + 2 * q]) * n) >> 32)
                out[t, 2 + q] = ni if int(w[5 + 2 * q]) < int(self.nthr[ni]) else int(self.nal[ni]) & 0x3FFFFFFF
        return out


def part_masses(path, nparts, undirected=1):
    """Every part's share of the source law (smore_block_part_mass) and the W
    part bounds, for the graph in `path`."""
    g = orc.Graph.from_file(path, undirected)
    ps = alias_law(g.vprob, g.valias, 1.0 / g.V)
    wb = part_bounds(ps, nparts)
    m = [sum(ps[wb[p]:wb[p + 1]]) for p in range(nparts)]
    tot = sum(m)
    return [x / tot for x in m], wb
