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


def prob_thr(p):
    """blocks.cpp prob_thr: a probability as a Philox-word threshold."""
    t = np.ceil(np.ldexp(p, 32))
    return 0 if not t > 0 else 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def hub_count(V, nb, hubs=-1, c_slots=None):
    """blocks.cpp hub_count: -1 automatic (none at 2 parts, else 4096, at most V / 8nb)."""
    c_slots = min(65536, V) if c_slots is None else c_slots
    h = (0 if nb <= 4 else min(4096, V // (8 * nb))) if hubs < 0 else hubs
    return max(0, min(h, c_slots, V // 2))


class BlockSpec:
    """One part's block tables (blocks.cpp smore_block_setup, LINE-2), with the
    hub C rows: the H rows of the largest pc + K pn (ties to the lower id) are
    slots V + j, drawn in every block -- contexts through the part's hub atoms
    (a cell takes one iff Philox word 2 < its hub threshold), negatives through
    each block's alias over its non-hub rows and the slots (1/nb of each hub's
    mass)."""

    def __init__(self, g, nparts, part, K=5, hubs=-1):
        self.g, self.n, self.r, self.nb = g, nparts, part, 2 * nparts
        V = g.V
        nb = self.nb
        self.V = V
        self.ps = alias_law(g.vprob, g.valias, 1.0 / V)
        self.pn = alias_law(g.nprob, g.nalias, 1.0 / V)
        # the context law (host_graph.cpp draw_probabilities, loop order kept)
        pc = [0.0] * V
        off, tgt = g.offsets, g.targets
        for v in range(V):
            o, br = int(off[v]), int(off[v + 1] - off[v])
            if br == 0 or self.ps[v] == 0:
                continue
            sc = self.ps[v] / br
            for i in range(br):
                pr = float(g.cprob[o + i])
                pc[int(tgt[o + i])] += sc * pr
                if g.calias[o + i] >= 0 and pr < 1.0:
                    pc[int(g.calias[o + i])] += sc * (1.0 - pr)
        self.pc = pc
        H = hub_count(V, nb, hubs)
        q = [pc[x] + float(K) * self.pn[x] for x in range(V)]
        self.hubs = sorted(range(V), key=lambda x: (-q[x], x))[:H]
        self.H = H
        hub_of = {x: j for j, x in enumerate(self.hubs)}
        self.hub_of = hub_of
        pnH = sum(self.pn[x] for x in self.hubs) if H else 0.0
        self.wb = part_bounds(self.ps, nparts)
        pcut = [0.0 if x in hub_of else self.pn[x] for x in range(V)]
        self.cb = part_bounds(pcut, nb)
        # negative tables per block: rows in place, hub slots at [k H, (k+1) H)
        self.nthr = np.zeros(V, np.uint32)
        self.nal = np.zeros(V, np.int32)
        self.hthr = np.zeros(nb * H, np.uint32)
        self.hal = np.zeros(nb * H, np.int32)
        nraw = []
        for k in range(nb):
            lo, hi = self.cb[k], self.cb[k + 1]
            n = hi - lo
            wt = [0.0 if lo + i in hub_of else self.pn[lo + i] for i in range(n)]
            wt += [self.pn[x] / nb for x in self.hubs]
            ids = np.array([lo + i for i in range(n)] + [V + j for j in range(H)], np.int32)
            prob, alias = orc.alias_go(np.array(wt), 1.0)
            thr, al = orc.alias_encode(prob, ids[alias], ids)
            self.nthr[lo:hi], self.nal[lo:hi] = thr[:n], al[:n]
            self.hthr[k * H:(k + 1) * H], self.hal[k * H:(k + 1) * H] = thr[n:], al[n:]
            r = 0.0
            for i in range(n):
                if lo + i not in hub_of:
                    r += self.pn[lo + i]
            nraw.append(r + pnH / nb)
        self.nmass = [x / sum(nraw) for x in nraw]
        # atoms of this part per block, and its hub atoms (slot ids)
        atoms = [[] for _ in range(nb)]
        hub_atoms = []
        for v in range(self.wb[part], self.wb[part + 1]):
            o, br = int(off[v]), int(off[v + 1] - off[v])
            if br == 0 or self.ps[v] <= 0:
                continue
            sv = self.ps[v] / br
            for i in range(br):
                pr = float(g.cprob[o + i])
                for x, w in ((int(tgt[o + i]), sv * pr),
                             (int(g.calias[o + i]), sv * (1.0 - pr) if g.calias[o + i] >= 0 and pr < 1.0 else 0.0)):
                    if w > 0:
                        if x in hub_of:
                            hub_atoms.append((v, V + hub_of[x], w))
                        else:
                            atoms[self.block_of(x)].append((v, x, w))
        self.atoms, self.hub_atoms = atoms, hub_atoms
        raw = []
        for a in atoms:
            m = 0.0
            for _, _, w in a:
                m += w
            raw.append(m)
        mH = 0.0
        for _, _, w in hub_atoms:
            mH += w
        self.tabs = []
        for a in atoms:
            if not a:
                self.tabs.append(None)
                continue
            prob, alias = orc.alias_go(np.array([w for _, _, w in a]), 1.0)
            self.tabs.append(orc.alias_encode(prob, alias))
        self.hub_tab = None
        if hub_atoms:
            prob, alias = orc.alias_go(np.array([w for _, _, w in hub_atoms]), 1.0)
            self.hub_tab = orc.alias_encode(prob, alias)
        cell = [raw[k] + mH / nb for k in range(nb)]
        self.hub_thr = [prob_thr((mH / nb) / cell[k]) if cell[k] > 0 and hub_atoms else 0 for k in range(nb)]
        tot = 0.0
        for x in cell:
            tot += x
        self.mass = [x / tot for x in cell]
        # the cells' negative-step weights (blocks.cpp cell_args: pn(b) / m(r, b), fp32)
        self.neg_w = [float(np.float32(self.nmass[k] / self.mass[k])) if self.mass[k] > 0 else 1.0
                      for k in range(nb)]

    def block_of(self, x):
        return int(np.searchsorted(self.cb, x, side="right")) - 1

    def draw(self, k, seed, begin, count, K):
        """count x (2 + K) {v, c, n1..nK} of samples [begin, begin + count) in cell (r, k)."""
        out = np.zeros((count, 2 + K), np.int32)
        a = self.atoms[k]
        lo, n = self.cb[k], self.cb[k + 1] - self.cb[k]
        H = self.H
        for t in range(count):
            w = orc.words(seed, 0, begin + t, 4 + 2 * K)
            hub = len(self.hub_atoms) > 0 and (len(a) == 0 or int(w[2]) < self.hub_thr[k])
            lst, (thr, al) = (self.hub_atoms, self.hub_tab) if hub else (a, self.tabs[k])
            i = (int(w[1]) * len(lst)) >> 32
            j = i if int(w[0]) < int(thr[i]) else int(al[i])
            out[t, 0], out[t, 1] = lst[j][0], lst[j][1]
            for q in range(K):
                ni = (int(w[4 + 2 * q]) * (n + H)) >> 32
                kp = int(w[5 + 2 * q])
                if ni < n:
                    e = lo + ni
                    out[t, 2 + q] = e if kp < int(self.nthr[e]) else int(self.nal[e]) & 0x3FFFFFFF
                else:
                    e = k * H + (ni - n)
                    out[t, 2 + q] = (self.V + ni - n) if kp < int(self.hthr[e]) else int(self.hal[e]) & 0x3FFFFFFF
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


def cell_masses(g, nparts):
    """Vectorised (large graphs): the W part bounds, the C block bounds, every
    cell's sample mass m[r, b] (the atoms' mass of part r whose context is in
    block b; sum 1 over all cells) and NegativeSample's block masses pn_b (sum
    1), plus the negative law pn itself.  Float sums in numpy order (not the
    product's loop order): for marginal checks, not bit-exactness."""
    V = g.V
    prob_v, alias_v = np.asarray(g.vprob, np.float64), np.asarray(g.valias, np.int64)
    prob_n, alias_n = np.asarray(g.nprob, np.float64), np.asarray(g.nalias, np.int64)

    def law(prob, alias):
        p = prob / V
        m = (alias >= 0) & (prob < 1.0)
        np.add.at(p, alias[m], (1.0 - prob[m]) / V)
        return p
    ps, pn = law(prob_v, alias_v), law(prob_n, alias_n)
    nb = 2 * nparts
    wb = np.asarray(part_bounds(list(ps), nparts), np.int64)
    cb = np.asarray(part_bounds(list(pn), nb), np.int64)
    off = np.asarray(g.offsets, np.int64)
    deg = np.diff(off)
    src = np.repeat(np.arange(V, dtype=np.int64), deg)
    tgt = np.asarray(g.targets, np.int64)
    cprob = np.asarray(g.cprob, np.float64)
    calias = np.asarray(g.calias, np.int64)
    s = np.where(deg[src] > 0, ps[src] / np.maximum(deg[src], 1), 0.0)
    part = np.searchsorted(wb, src, side="right") - 1
    m = np.zeros(nparts * nb)
    w1 = s * cprob
    np.add.at(m, part * nb + np.searchsorted(cb, tgt, side="right") - 1, w1)
    ok = (calias >= 0) & (cprob < 1.0)
    w2 = s[ok] * (1.0 - cprob[ok])
    np.add.at(m, part[ok] * nb + np.searchsorted(cb, calias[ok], side="right") - 1, w2)
    m = m.reshape(nparts, nb) / m.sum()
    pnb = np.array([pn[cb[k]:cb[k + 1]].sum() for k in range(nb)])
    return wb, cb, m, pnb / pnb.sum(), pn / pn.sum()


def negative_marginal(cb, m, pnb, pn, weights):
    """Expected negative updates per row per sample over an epoch of the block
    schedule: part r gets its share sum_b m[r, b] of the samples, cell (r, b)
    a share m[r, b] with K negatives from block b's restricted law, each step
    weighted by weights[r, b] (all ones: no correction; pnb / (m[r] / sum m[r])
    is blocks.cpp's weight).  Returns per-row marginals over all parts (sum 1
    for the exact law) and per part."""
    nparts, nb = m.shape
    blk = np.zeros(len(pn), np.int64)
    for k in range(nb):
        blk[cb[k]:cb[k + 1]] = k
    cond = pn / pnb[blk]                         # law within the row's block
    per_part = []
    tot = np.zeros(len(pn))
    for r in range(nparts):
        share = m[r] / m[r].sum()                # cell shares of part r's samples
        f = (share * weights[r])[blk] * cond
        per_part.append(f)
        tot += m[r].sum() * f
    return tot, per_part


def skewed_graph_lines(n=400, heavy=200):
    """A directed test graph whose source mass cannot be cut into equal parts:
    a ring of light edges plus, every 50th vertex, a hub with 39 heavy
    out-edges -- each hub holds a few % of the source mass, so the midpoint
    rule's parts differ by ~13 % at 2 / 4 / 8 parts, none empty."""
    lines = []
    for i in range(1, n):
        lines.append("v%d v%d 1" % (i, 1 + i % (n - 1)))
        if i % 50 == 0:
            lines += ["v%d v%d %d" % (i, 1 + (i + j) % (n - 1), heavy) for j in range(1, 40)]
    return "\n".join(lines) + "\n"
