// blocks.cpp -- the 2-D block schedule of the multi-GPU path (SURVEY.md 8e's
// conflict-free fallback), one context's side: its draw tables,
// its cell launches and, for the walk models, its bucketed round records.
//
// The reference trains one shared table pair with Hogwild threads
// (src/model/LINE.cpp:160-191, src/model/DeepWalk.cpp:128-155).  Replicated
// tables over N GPUs need an exchange that either loses samples' worth
// (averaging) or overshoots (summing stale deltas).  Here no
// row is ever replicated while it trains: GPU r owns the W rows of part r
// (equal source mass), the C table is cut into nb = 2N blocks (equal negative
// mass), and sub-round s trains cell (r, b = (2r + s) mod nb) on every GPU at
// once -- disjoint W rows, disjoint C rows.  After a sub-round GPU r passes
// block b to GPU r - 1, which trains it two sub-rounds later, so the transfer
// has a whole sub-round to overlap (exchange.cpp group_rotate, dist.py
// BlockSync).  The samples of a cell follow the one-GPU law restricted to the
// cell (train_blocks.hip); a call's samples are spread over the cells in
// proportion to their mass, so an epoch (nb sub-rounds) draws the one-GPU
// law of (source, context).  What changes is the order (cell by cell) and the
// negatives: drawn in the context's block (the law restricted to the block;
// blocks have equal negative mass), while a cell's sample count follows the
// block's CONTEXT mass -- so each cell weights its negative steps by the
// block's negative share over its sample share (cell_args, neg_law_on), and
// an epoch's expected negative updates per row are NegativeSample's.
#include <cmath>
#include <numeric>
#include <thread>

#include "ctx.h"

using namespace smore_host;

namespace {

constexpr uint64_t WALK_ROUND_MAX = (uint64_t)1 << 20;   // walks per prepared block round

int check_ctx(smore_ctx* c) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->device < 0) return fail(c, SMORE_ESTATE, "host-only context");
    return SMORE_OK;
}

BlockArgs block_args(const smore_ctx* c) {
    BlockArgs b{};
    b.atoms = c->blk.d_atoms;
    b.ntab = c->blk.d_ntab;
    b.nb = c->blk.nb;
    for (int k = 0; k <= c->blk.nb; ++k) b.cb[k] = (int32_t)c->blk.cb[k];
    b.hub_ntab = c->blk.d_hub_ntab;
    b.hub_off = c->blk.hub_off;
    b.nhub = (uint32_t)c->blk.nhub;
    b.H = (int32_t)c->blk.H;
    b.V = (int32_t)c->g->V;
    b.hub_of = c->blk.d_hub_of;
    return b;
}

// a probability as a Philox-word threshold (word < thr with probability p)
uint32_t prob_thr(double p) {
    const double t = std::ceil(std::ldexp(p, 32));
    return !(t > 0) ? 0u : t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// the resident sample groups of this context's update launches (the hot
// tags' M): the same grid the training calls use
int64_t resident_groups(smore_ctx* c, bool walk, int K, int mode) {
    EdgeArgs a{};
    a.g = dev_graph(c);
    a.dpad = c->dpad;
    a.K = K;
    a.model = SMORE_LINE2;
    a.mode = mode;
    a.count = (uint64_t)1 << 30;
    a.alpha_rec = walk ? 1 : 0;
    a.sh_rows = mode == SMORE_HYBRID ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;
    return (int64_t)launch_grid(c, a) * (256 / lanes_of(c->dpad));
}

// per-block write-combined rows: the hottest hot C rows of each block under
// its cell's C-row law (pcb, flags hcb; entry i of block k is row cb[k] + i,
// or hub slot V + i - rows past the block's rows), with the edge rule's
// staleness bound and a two-tier drain (capi build_hot_maps)
// Walk cells add their part's hottest W rows (key v | SH_WKEY, rate ps(v) N
// per record: wcand): the pair kernel keeps a run's W row in registers and
// flushed it atomically at the run's end, so C5's hub centre -- ~1 record
// runs, 16 % of its part's records at 8 parts -- queued every group's flush
// on one 512-B row (its part's cells 1.4x slower than the others'); combined,
// the block adds its groups' deltas in LDS and drains them on the row's
// interval (SMORE_WALK_WCOMB=1; off by default)
void block_sh_sets(smore_ctx* c, bool walk, bool on, int64_t Mg, const std::vector<std::vector<double>>& pcb,
                   const std::vector<std::vector<uint8_t>>& hcb, std::vector<int2>& hash, std::vector<int32_t>& ids,
                   const std::vector<std::pair<double, int32_t>>& wcand) {
    const int64_t V = c->g->V;
    auto& B = c->blk;
    const int cap = on ? std::max(0, std::min(c->sh_max, sh_rows_max(c->dpad))) : 0;
    B.sh_cap = std::max(cap, 1);
    B.sh_n.assign((size_t)B.nb, 0);
    B.sh_wn.assign((size_t)B.nb, 0);
    B.sh_lvl.assign((size_t)B.nb, std::array<int, 8>{});
    hash.assign((size_t)B.nb * SH_HASH, make_int2(-1, -1));
    ids.assign((size_t)B.nb * B.sh_cap, -1);
    const int flush_cap = c->sh_flush > 0 ? c->sh_flush : sh_flush_max(walk);
    B.sh_flush = flush_cap;
    if (cap == 0) return;
    const double M = (double)Mg, stale = sh_stale_max(walk);
    const bool two_tier = c->sh_flush <= 0;
    for (int k = 0; k < B.nb; ++k) {
        // A cell concentrates its samples on 1/nb of the C rows, so a hub row
        // takes about nb times its one-GPU share of a launch's updates (C4,
        // 8 GPUs: the top row ~18 % of a cell's C touches).  Each combined row
        // gets its own drain interval from its rate (power-of-two levels:
        // every slot every flush_cap rounds, each faster level's prefix at
        // its own interval), so the hubs stay within the staleness bound
        // without draining every other row as often.
        std::vector<std::pair<double, int32_t>> r;
        const int64_t rows = B.cb[k + 1] - B.cb[k];
        for (size_t i = 0; i < pcb[k].size(); ++i) {
            if (!hcb[k][i]) continue;
            const double p = pcb[k][i];
            const double f = two_tier ? (double)sh_slot_interval(M * p, flush_cap, walk) : (double)flush_cap;
            const int64_t id = (int64_t)i < rows ? B.cb[k] + (int64_t)i : V + ((int64_t)i - rows);
            if (M * p * f <= stale) r.push_back({p, (int32_t)id});
        }
        for (const auto& x : wcand) {
            const double f = two_tier ? (double)sh_slot_interval(M * x.first, flush_cap, walk) : (double)flush_cap;
            if (M * x.first * f <= stale) r.push_back(x);
        }
        const int64_t n = std::min<int64_t>(cap, (int64_t)r.size());
        std::partial_sort(r.begin(), r.begin() + n, r.end(), [](const auto& x, const auto& y) {
            return x.first > y.first || (x.first == y.first && x.second < y.second);
        });
        int2* h = hash.data() + (size_t)k * SH_HASH;
        for (int64_t i = 0; i < n; ++i) {
            B.sh_wn[k] += (r[i].second & SH_WKEY) ? 1 : 0;
            ids[(size_t)k * B.sh_cap + i] = r[i].second;
            uint32_t p = sh_hash_of(r[i].second);
            while (h[p & (SH_HASH - 1)].x >= 0) ++p;
            h[p & (SH_HASH - 1)] = make_int2(r[i].second, (int)i);
        }
        B.sh_n[k] = (int)n;
        if (two_tier && n > 0) {
            int lv[8];
            sh_slot_levels(Mg, flush_cap, walk, r.data(), n, lv);
            std::copy(lv, lv + 8, B.sh_lvl[k].begin());
        }
        if (getenv("SMORE_SH_DEBUG")) {
            const auto& l = B.sh_lvl[k];
            fprintf(stderr, "[sh] block %d/%d M %lld rows %lld of %zu flush %d lvl %d %d %d %d %d %d %d %d top", k, B.nb,
                    (long long)Mg, (long long)n, r.size(), flush_cap, l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]);
            for (int64_t i = 0; i < std::min<int64_t>(n, 4); ++i) fprintf(stderr, " %d:%.3g", r[i].second, M * r[i].first);
            fprintf(stderr, "\n");
        }
    }
}

// NegativeSample's law over an epoch (SMORE_NEG_LAW=0: off).  A cell (r, b)
// draws its K negatives from block b's restricted law, but the cells of part r
// get its samples in proportion to their CONTEXT mass m(r, b), while
// NegativeSample (src/proNet.cpp:623-633) would put a share pn(b) (~1/nb:
// blocks are cut to equal negative mass) of them in block b.  Scaling the
// cell's negative steps by pn(b) / m(r, b) makes part r's expected negative
// updates per row exactly the one-GPU ones (tests/test_blocks_cpu.py computes
// the epoch marginal).  LINE-2 cells take m(r, b) from the atoms' mass; walk
// cells from the round's record counts, on the device (neg_scale_of).
bool wcomb_on() {
    const char* e = getenv("SMORE_WALK_WCOMB");
    return e && atoi(e) != 0;
}

bool neg_law_on() {
    const char* e = getenv("SMORE_NEG_LAW");
    return !e || atoi(e) != 0;
}

// hub C rows of a block setup (smore_block_set_hubs / $SMORE_HUBS; -1:
// automatic), at most the C table's slot rows and half the vertices
// Automatic: none at 2 parts (a cell's rows are only 4 times hotter than
// one GPU's, and the hub copies' exchange costs more than it saves: C4 at
// 2^34 samples 1.057 vs 1.008 times one GPU's held-out loss), else 4096 --
// C4 at 8 parts: the five hub cells (10-14 ms against 7.7) disappear.
constexpr int64_t HUB_AUTO = 4096;
// The walk models the same (C5 DeepWalk at 8 parts: the capped hub cells
// and the 29 % rotation stall disappear, 1.34 -> 2.32x predicted) with their
// own exchange rule (c0 64, hub_c0: 1.026 times one GPU's held-out loss; c0
// 2048: 1.11).
int64_t hub_count(const smore_ctx* c, int64_t V, int nb, bool walk) {
    (void)walk;
    int64_t h = c->blk_hubs;
    if (const char* e = getenv("SMORE_HUBS")) h = atoll(e);
    if (h < 0) h = nb <= 4 ? 0 : std::min<int64_t>(HUB_AUTO, V / (8 * (int64_t)nb));
    return std::max<int64_t>(0, std::min(std::min(h, c->c_slots), V / 2));
}

// the update-kernel arguments shared by a context's cell launches
EdgeArgs cell_args(smore_ctx* c, int k, bool walk) {
    const auto& B = c->blk;
    EdgeArgs a{};
    a.g = dev_graph(c);
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = c->d_table[1];
    a.skipped = c->d_skipped;
    a.dpad = c->dpad;
    a.K = B.K;
    a.model = SMORE_LINE2;
    a.mode = B.mode;
    a.alpha_rec = walk ? 1 : 0;
    a.work = c->d_work;
    const bool on = B.mode == SMORE_HYBRID && B.sh_n[k] > 0;
    a.sh_rows = on ? B.sh_n[k] : 0;
    a.sh_hash = B.d_sh_hash + (size_t)k * SH_HASH;
    a.sh_ids = B.d_sh_ids + (size_t)k * B.sh_cap;
    a.sh_flush = std::max(1, B.sh_flush);
    a.sh_flush_w = 0;
    std::copy(B.sh_lvl[k].begin(), B.sh_lvl[k].end(), a.sh_lvl);
    // walk cells: cold W rows stored, not added (SMORE_WALK_WPLAIN=1; off:
    // measured no faster at C5, 8 parts -- 30.4 vs 31.6 ms per part's epoch)
    if (walk) {
        const char* e = getenv("SMORE_WALK_WPLAIN");
        a.w_plain = e && atoi(e) != 0;
        const char* x = getenv("SMORE_WALK_EDGE");   // walk cells through the edge kernel (study)
        a.rec_edge = x && atoi(x) != 0;
        a.w_comb = on && (size_t)k < B.sh_wn.size() && B.sh_wn[k] > 0;
    }
    if (neg_law_on() && (size_t)k < B.nmass.size()) {
        if (walk) {
            a.neg_scale = (float)B.nmass[k];
            a.neg_lo = B.d_off;
            a.neg_hi = B.d_off + (size_t)B.nb * B.walks;
        } else if ((size_t)k < B.mass.size() && B.mass[k] > 0) {
            a.neg_scale = (float)(B.nmass[k] / B.mass[k]);
        }
    }
    return a;
}

// A cell's launch: the context's grid, capped so that its hottest row takes
// at most SMORE_CELL_RATE concurrent updates per round (M p_max).  A cell
// concentrates its samples on 1/N of the W rows and 1/2N of the C rows, so
// its hub rows are up to 2N times as contended as at one GPU, where M p_max
// is ~130-260 (C5 DeepWalk, C2 LINE-2); Hogwild on a row with ~2000 updates in
// flight (C5 DeepWalk, 8 GPUs) diverges whether the row is atomic or
// write-combined.
int cell_grid(smore_ctx* c, const EdgeArgs& a, int k) {
    int grid = launch_grid(c, a);
    const auto& B = c->blk;
    if (a.mode == SMORE_SERIAL || (size_t)k >= B.pmax_c.size()) return grid;
    // LINE-2 cells: the one-GPU launch's Hogwild concurrency cap (capi
    // edge_grid: at most V / 16 resident sample groups) applied to the rows a
    // cell updates -- its block's C rows and the hub slots -- so a small
    // graph's cells (C2 at 8 GPUs: 62k rows per block) keep the one-GPU ratio
    // of in-flight updates per row instead of 16 times it
    if (a.alpha_rec == 0 && !getenv("SMORE_CELL_NOCAP")) {
        const int64_t rows = B.cb[k + 1] - B.cb[k] + B.H;
        const int gpb = 256 / lanes_of(c->dpad);
        const int64_t cap = std::max<int64_t>(8, (rows / 16 + gpb - 1) / gpb);
        if (cap < grid) grid = (int)cap;
    }
    double cap = cell_rate_default(a.alpha_rec == 1);
    if (const char* e = getenv("SMORE_CELL_RATE")) cap = atof(e);
    // which side's hub sets the cap: both (default), SMORE_CELL_SIDE=c or w
    const char* side = getenv("SMORE_CELL_SIDE");
    const double pmax = side && side[0] == 'c' ? B.pmax_c[k]
                        : side && side[0] == 'w' ? B.pmax_w[k] : std::max(B.pmax_w[k], B.pmax_c[k]);
    if (cap <= 0 || pmax <= 0) return grid;
    const int gpb = 256 / lanes_of(c->dpad);
    const double groups = cap / pmax;
    const int g = std::max(8, (int)(groups / gpb) / 8 * 8);   // whole rounds of the 8 XCDs
    return std::min(grid, g);
}

int grow_events(smore_ctx* c, std::vector<hipEvent_t>& v, size_t n) {
    while (v.size() < n) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        v.push_back(e);
    }
    return SMORE_OK;
}

}  // namespace

namespace smore_host {
// the exchange of the hub slots after every sub-round, one late (the rule of
// replica_sync.hip): slot j's summed delta is scaled by
// s + (1 - s) / N with s = min(1, c0 / k_j), k_j = its expected updates per
// exchange over all parts -- the sum for slots updated a few times per
// sub-round, towards the mean for the hubs that take hundreds of thousands
// (each part's copy reaches the same local equilibrium; summing N of them
// would overshoot)
void hub_scales(const smore_ctx::Blocks& B, double samples, double c0, float* out) {
    const double N = (double)B.n;
    for (int64_t j = 0; j < B.H; ++j) {
        const double k = B.hub_rate[j] * samples * N;
        const double s = k > 0 ? std::min(1.0, c0 / k) : 1.0;
        out[j] = (float)(s + (1.0 - s) / N);
    }
}

// launches per cell: with hub slots, 4 -- the slots are exchanged
// after each, so their copies are at most a quarter cell apart (C4, 8 parts:
// 1.042 times one GPU's held-out loss against 1.079 with one launch per
// cell, at 6.27 against 6.55 predicted); without, 1.  SMORE_CELL_LAUNCHES
// overrides (1..64).
int cell_launches(const smore_ctx::Blocks& B) {
    int k = B.H > 0 ? 4 : 1;
    if (const char* e = getenv("SMORE_CELL_LAUNCHES")) k = atoi(e);
    return std::max(1, std::min(64, k));
}

// largest remainder of n * mass[k] (ties to the lower index)
void largest_remainder(uint64_t n, const double* mass, int parts, uint64_t* counts) {
    std::vector<std::pair<double, int>> rem;
    uint64_t used = 0;
    for (int k = 0; k < parts; ++k) {
        const double x = (double)n * mass[k];
        counts[k] = (uint64_t)std::floor(x);
        used += counts[k];
        rem.push_back({x - std::floor(x), k});
    }
    std::stable_sort(rem.begin(), rem.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t i = 0; used < n && i < rem.size(); ++i, ++used) counts[rem[i].second]++;
    for (int k = 0; used < n; k = (k + 1) % parts, ++used) counts[k]++;   // rounding slack (never in practice)
}

int block_walks_gen(smore_ctx* c, int rule, uint64_t walk_begin, uint64_t walk_end, uint64_t gen_lo, uint64_t gen_hi,
                    int walk_times, int walk_steps, int window, int window_min, int K, double alpha0, uint64_t seed,
                    const int64_t* order, uint64_t order_base, int mode) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_CENSUS) return fail(c, SMORE_ESTATE, "no walk block setup (smore_block_setup)");
    if (K != B.K || mode != B.mode) return fail(c, SMORE_EINVAL, "K / mode differ from smore_block_setup's");
    if (rule != 0 && rule != 1) return fail(c, SMORE_EINVAL, "block rounds: DeepWalk (0) or Walklets (1)");
    if ((rule == 0 && !order) || walk_times <= 0 || walk_steps < 0 || window <= 0)
        return fail(c, SMORE_EINVAL, "bad walk arguments");
    if (rule == 1 && (window_min < 0 || window_min > window)) return fail(c, SMORE_EINVAL, "Walklets: bad window");
    const uint64_t total = (uint64_t)walk_times * (uint64_t)c->g->V;
    if (walk_end > total) walk_end = total;
    B.walks = 0;
    if (walk_begin >= walk_end) return SMORE_OK;
    const uint64_t nw = walk_end - walk_begin;
    if (nw > WALK_ROUND_MAX) return fail(c, SMORE_EINVAL, "a block round holds at most 2^20 walks");
    if (order) {
        if (walk_begin < order_base) return fail(c, SMORE_EINVAL, "walk order slice does not cover the range");
        order -= order_base;
        for (uint64_t i = walk_begin; i < walk_end; ++i)
            if (order[i] < 0 || order[i] >= c->g->V) return fail(c, SMORE_EINVAL, "walk start out of range");
    }
    if ((rc = set_device(c))) return rc;
    // the walk ids' tags: the scaled hot maps (a no-op when current)
    if (mode == SMORE_HYBRID) {
        const int64_t M = resident_groups(c, true, K, mode);
        if ((rc = hot_maps(c, SMORE_LINE2, K, M, true, (double)B.n, (double)B.nb))) return rc;
    }
    if (order) {
        if (c->order_cap < nw) {
            dfree(c->d_order);
            c->order_cap = 0;
            HIPCHK(c, hipMalloc((void**)&c->d_order, nw * sizeof(int64_t)));
            c->order_cap = nw;
        }
        HIPCHK(c, hipMemcpyAsync(c->d_order, order + walk_begin, nw * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    }
    const int RW = rec_width(kmax_of(K));
    const uint64_t pb = std::max<uint64_t>(1, pair_bound(walk_steps, window, rule, window_min));
    const size_t need = nw * (size_t)(walk_steps + 1);
    if (c->walk_buf_n < need) {
        dfree(c->d_walks);
        c->walk_buf_n = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_walks, need * sizeof(int32_t)));
        c->walk_buf_n = need;
    }
    if (c->walk_lens_n < nw) {
        dfree(c->d_lens);
        c->walk_lens_n = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_lens, nw * sizeof(int32_t)));
        c->walk_lens_n = nw;
    }
    const size_t ncount = (size_t)B.nb * nw + 1;
    if (B.count_cap < ncount) {
        dfree(B.d_count);
        dfree(B.d_off);
        B.count_cap = 0;
        HIPCHK(c, hipMalloc((void**)&B.d_count, ncount * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc((void**)&B.d_off, ncount * sizeof(uint64_t)));
        B.count_cap = ncount;
    }
    if (c->rec_cap < nw * pb * RW) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, nw * pb * RW * sizeof(int32_t)));
        c->rec_cap = nw * pb * RW;
    }
    WalkArgs w;
    w.order = order ? c->d_order : nullptr;
    w.order_base = walk_begin;
    w.walks = c->d_walks;
    w.lens = c->d_lens;
    w.walk_begin = walk_begin;
    w.nwalks = nw;
    w.total_walks = total;
    w.steps = walk_steps;
    w.window = window;
    w.rule = rule;
    w.window_min = window_min;
    w.inv_p = w.inv_q = 1.0;
    w.wts = nullptr;
    w.nbr_sorted = nullptr;
    w.ntype = nullptr;
    w.ttargets = nullptr;
    w.toff = nullptr;
    w.paths = nullptr;
    w.path_off = nullptr;
    w.ntypes = w.npaths = 0;
    w.slot_extra = 0;
    w.own_lo = (int32_t)B.wb[B.r];
    w.own_hi = (int32_t)B.wb[B.r + 1];
    B.wargs = w;
    B.wseed = seed;
    B.walpha0 = alpha0;
    B.wpairs = pb;
    B.walks = nw;
    B.rec_bound = nw * pb;
    if (gen_lo < walk_begin || gen_hi > walk_end || gen_lo > gen_hi)
        return fail(c, SMORE_EINVAL, "walk generation range outside the round");
    if (gen_hi > gen_lo) {   // this context's share of the round's walks
        WalkArgs wg = w;
        const uint64_t o = gen_lo - walk_begin;
        wg.walk_begin = gen_lo;
        wg.nwalks = gen_hi - gen_lo;
        wg.walks = w.walks + o * (uint64_t)(walk_steps + 1);
        wg.lens = w.lens + o;
        HIPCHK(c, launch_walk_gen(dev_graph(c), wg, seed, c->stream));
    }
    return SMORE_OK;
}

int block_walks_emit(smore_ctx* c) {
    auto& B = c->blk;
    if (!B.walks) return SMORE_OK;
    const WalkArgs& w = B.wargs;
    const size_t ncount = (size_t)B.nb * B.walks + 1;
    const BlockArgs ba = block_args(c);
    HIPCHK(c, hipMemsetAsync(B.d_count + (ncount - 1), 0, sizeof(uint32_t), c->stream));
    HIPCHK(c, launch_block_pair_count(w, ba, B.wseed, B.d_count, c->stream));
    HIPCHK(c, scan_pair_counts(B.d_count, B.d_off, ncount, &c->d_scan_tmp, &c->scan_tmp_bytes, c->stream));
    HIPCHK(c, launch_block_pair_emit(w, ba, B.wseed, B.K, B.walpha0, B.d_off, c->d_rec, c->stream));
    return SMORE_OK;
}


void blocks_release(smore_ctx* c) {
    auto& B = c->blk;
    dfree(B.d_atoms);
    dfree(B.d_ntab);
    dfree(B.d_sh_hash);
    dfree(B.d_sh_ids);
    dfree(B.d_count);
    dfree(B.d_off);
    dfree(B.d_hub_ntab);
    dfree(B.d_hub_ids);
    dfree(B.d_hub_of);
    for (float*& p : B.d_hub_ex) dfree(p);
    dfree(B.d_hub_scale);
    B = smore_ctx::Blocks{};
}
}  // namespace smore_host

extern "C" {

int smore_block_setup(smore_ctx* c, int model, int nparts, int part, int K, int mode) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if (model != SMORE_LINE2 && model != SMORE_CENSUS)
        return fail(c, SMORE_EINVAL, "block schedule: LINE-2 (SMORE_LINE2) or the C++ walk models (SMORE_CENSUS)");
    if (nparts < 1 || 2 * nparts > BLOCK_MAX || part < 0 || part >= nparts)
        return fail(c, SMORE_EINVAL, "block schedule: 1 <= nparts <= 16, 0 <= part < nparts");
    if (K < 0 || K > (model == SMORE_LINE2 ? 20 : 10) || mode < 0 || mode > 3)
        return fail(c, SMORE_EINVAL, "block schedule: bad K / mode");
    if (c->semantics != SMORE_SEM_CPP) return fail(c, SMORE_EINVAL, "block schedule: C++ rules only");
    if (c->ntables < 2) return fail(c, SMORE_ESTATE, "block schedule: W and C tables needed");
    if ((rc = set_device(c))) return rc;
    const bool walk = model == SMORE_CENSUS;
    if (nparts == 1) {
        blocks_release(c);
        return SMORE_OK;
    }
    const HostGraph& g = *c->g;
    const int64_t V = g.V;
    const int nb = 2 * nparts;
    if (V < nb) return fail(c, SMORE_EINVAL, "block schedule: fewer vertices than blocks");
    const int64_t H = hub_count(c, V, nb, walk);
    char key[288];
    snprintf(key, sizeof key, "%d/%d/%d/%d/%d/%lld/%lld/%d/%d/%d/%.9g/%lld/%s", model, nparts, part, K, mode,
             (long long)V, (long long)g.E, c->dpad, c->sh_max, c->sh_flush, c->hot_tau, (long long)H,
             getenv("SMORE_SH_STALE") ? getenv("SMORE_SH_STALE") : "");
    if (c->blk.key == key) return SMORE_OK;
    blocks_release(c);
    auto& B = c->blk;
    B.n = nparts;
    B.r = part;
    B.nb = nb;
    B.model = model;
    B.K = K;
    B.mode = mode;
    std::vector<double> ps, pn, pc;
    draw_probabilities(g, ps, pn, pc);
    // hub C rows: the H rows with the most expected touches per sample (as
    // a positive context plus K times as a negative); slot j is row V + j
    std::vector<int32_t> hub_of;
    double pnH = 0.0;
    if (H > 0) {
        std::vector<int32_t> idx((size_t)V);
        std::iota(idx.begin(), idx.end(), 0);
        auto q = [&](int32_t x) { return pc[x] + (double)K * pn[x]; };
        std::partial_sort(idx.begin(), idx.begin() + H, idx.end(), [&](int32_t a, int32_t b) {
            return q(a) > q(b) || (q(a) == q(b) && a < b);
        });
        hub_of.assign((size_t)V, -1);
        B.hubs.assign(idx.begin(), idx.begin() + H);
        B.hub_rate.resize((size_t)H);
        for (int64_t j = 0; j < H; ++j) {
            hub_of[B.hubs[j]] = (int32_t)j;
            B.hub_rate[j] = q(B.hubs[j]);
            pnH += pn[B.hubs[j]];
        }
        B.H = H;
    }
    part_bounds(ps, nparts, B.wb);
    {   // C blocks of equal NON-hub negative mass (the hubs are in every block)
        std::vector<double> pcut = pn;
        for (int32_t x : B.hubs) pcut[x] = 0.0;
        part_bounds(pcut, nb, B.cb);
    }
    for (int p = 0; p < nparts; ++p)
        if (B.wb[p + 1] <= B.wb[p]) return fail(c, SMORE_EINVAL, "block schedule: an empty W part");
    for (int k = 0; k < nb; ++k)
        if (B.cb[k + 1] <= B.cb[k]) return fail(c, SMORE_EINVAL, "block schedule: an empty C block");
    auto is_hub = [&](int64_t x) { return H > 0 && hub_of[x] >= 0; };
    // NegativeSample's share of each block: its non-hub rows, plus 1/nb of
    // every hub's (cell_args' negative weight)
    std::vector<double> nraw((size_t)nb, 0.0);
    {
        B.nmass.assign((size_t)nb, 0.0);
        double tot = 0.0;
        for (int k = 0; k < nb; ++k) {
            for (int64_t x = B.cb[k]; x < B.cb[k + 1]; ++x)
                if (!is_hub(x)) nraw[k] += pn[x];
            nraw[k] += pnH / nb;
            tot += nraw[k];
        }
        for (int k = 0; k < nb; ++k) B.nmass[k] = tot > 0 ? nraw[k] / tot : 1.0 / nb;
    }
    // each part's share of the source law: a round's samples are split over
    // the replicas by it (part_bounds only makes the parts roughly equal; a
    // hub above 1/N of the mass puts a part far off)
    {
        B.part_mass.assign((size_t)nparts, 0.0);
        double tot = 0.0;
        for (int p = 0; p < nparts; ++p) {
            for (int64_t v = B.wb[p]; v < B.wb[p + 1]; ++v) B.part_mass[p] += ps[v];
            tot += B.part_mass[p];
        }
        for (double& m : B.part_mass) m = tot > 0 ? m / tot : 1.0 / nparts;
    }
    // Hot tags (hybrid scatter) and the write-combined sets.  LINE-2: exact
    // per cell from its atoms -- W row v: its atoms' share of the cell's mass;
    // C row x: its atoms' share plus K times its share of the block's negative
    // law -- so a row is atomic iff M * p > tau in the launch that trains it
    // (a scaled global law misses the sources whose contexts crowd one block:
    // up to nb times hotter in that cell).  Walks: the scaled global law
    // (capi build_hot_maps), whose tags the walk ids carry.
    const bool hyb = mode == SMORE_HYBRID;
    int64_t M = 0;
    double tau = 0.0;
    bool small = false;
    if (hyb) {
        M = resident_groups(c, walk, K, mode);
        small = c->hot_tau < 0 && 16.0 * (double)M >= (double)V;
        // LINE-2 cells at 3-4 parts of a large graph: tau 0.6 (their rows are
        // 6-8x hotter than one GPU's, not 16x: C4 at 4 parts 1.037-1.040x one
        // GPU's held-out loss at 3.60x predicted, against 1.034x at 3.39x with
        // 0.3; at 8 parts 0.6 costs 1.054x; C2 -- 1M vertices, 125k rows per
        // block at 4 parts -- 1.048x, so graphs under 4M vertices keep 0.3;
        // DESIGN.md 10.6)
        const bool t06 = !walk && nparts >= 3 && nparts <= 4 && V >= ((int64_t)1 << 22);
        const double tcell = t06 ? 0.6 : hot_tau_cell_default(walk);
        tau = c->hot_tau >= 0 ? c->hot_tau : small ? 0.0 : tcell;
        if (walk && (rc = hot_maps(c, SMORE_LINE2, K, M, true, (double)nparts, (double)nb))) return rc;
    }
    const int T = (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), (unsigned)nb);
    auto par_blocks = [&](auto&& f) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (int k = t; k < nb; k += T) f(k);
            });
        for (auto& x : th) x.join();
    };
    // LINE-2 atoms of this part: the TargetSample outcomes of its sources,
    // bucketed by the context's block -- bucket nb: the hub contexts (as
    // slot ids), shared by every block's cell
    const int NBK = nb + (H > 0 ? 1 : 0);
    B.mass.assign((size_t)nb, 0.0);
    B.hub_p.assign((size_t)nb, 0.0);
    B.atom_off.assign((size_t)NBK + 1, 0);
    std::vector<int32_t> av, ac;
    std::vector<double> aw;
    std::vector<double> hubw;   // LINE-2: per hub slot, the part's atom mass of that context
    double mH = 0.0;
    const int64_t wlo = B.wb[part], whi = B.wb[part + 1];
    if (!walk) {
        auto bucket_of = [&](int64_t x) {
            if (is_hub(x)) return nb;
            return (int)(std::upper_bound(B.cb.begin(), B.cb.end(), x) - B.cb.begin()) - 1;
        };
        auto id_of = [&](int64_t x) { return is_hub(x) ? (int32_t)(V + hub_of[x]) : (int32_t)x; };
        // vertices [vb, ve) of the part, in order
        auto each_atom = [&](int64_t vb, int64_t ve, auto&& f) {
            for (int64_t v = vb; v < ve; ++v) {
                const int64_t off = g.offsets[v], br = g.offsets[v + 1] - off;
                if (br == 0 || ps[v] <= 0) continue;
                const double s = ps[v] / (double)br;
                for (int64_t i = 0; i < br; ++i) {
                    const double pr = g.cprob[off + i];
                    f(v, (int64_t)g.targets[off + i], s * pr);
                    if (g.calias[off + i] >= 0 && pr < 1.0) f(v, g.calias[off + i], s * (1.0 - pr));
                }
            }
        };
        // two passes over vertex slices on every host thread (count per
        // (slice, bucket), then fill); the slices' order keeps each bucket's
        // atoms in vertex order, as one pass would
        const int TS = (int)std::max(1u, std::min(std::thread::hardware_concurrency(), 64u));
        std::vector<int64_t> vs((size_t)TS + 1);
        {   // slices of equal edge count
            const int64_t e0 = g.offsets[wlo], e1 = g.offsets[whi];
            for (int t = 0; t <= TS; ++t) {
                const int64_t e = e0 + (e1 - e0) * t / TS;
                vs[t] = t == 0 ? wlo : t == TS ? whi
                                 : std::lower_bound(g.offsets.begin() + wlo, g.offsets.begin() + whi, e) -
                                       g.offsets.begin();
            }
        }
        auto par_slices = [&](auto&& f) {
            std::vector<std::thread> th;
            for (int t = 0; t < TS; ++t) th.emplace_back([&, t] { f(t); });
            for (auto& x : th) x.join();
        };
        std::vector<uint64_t> cnt((size_t)TS * NBK, 0);
        par_slices([&](int t) {
            uint64_t* ct = cnt.data() + (size_t)t * NBK;
            each_atom(vs[t], vs[t + 1], [&](int64_t, int64_t x, double w) {
                if (w > 0) ct[bucket_of(x)]++;
            });
        });
        std::vector<uint64_t> start((size_t)TS * NBK);
        for (int k = 0; k < NBK; ++k) {
            uint64_t acc = B.atom_off[k];
            for (int t = 0; t < TS; ++t) {
                start[(size_t)t * NBK + k] = acc;
                acc += cnt[(size_t)t * NBK + k];
            }
            B.atom_off[k + 1] = acc;
        }
        const uint64_t A = B.atom_off[NBK];
        if (A == 0) return fail(c, SMORE_EINVAL, "block schedule: a part without edges");
        av.resize(A);
        ac.resize(A);
        aw.resize(A);
        par_slices([&](int t) {
            uint64_t* pos = start.data() + (size_t)t * NBK;
            each_atom(vs[t], vs[t + 1], [&](int64_t v, int64_t x, double w) {
                if (w <= 0) return;
                const uint64_t p = pos[bucket_of(x)]++;
                av[p] = (int32_t)v;
                ac[p] = id_of(x);
                aw[p] = w;
            });
        });
        std::vector<double> m((size_t)NBK, 0.0);
        for (int k = 0; k < NBK; ++k)
            for (uint64_t p = B.atom_off[k]; p < B.atom_off[k + 1]; ++p) m[k] += aw[p];
        if (H > 0) {
            mH = m[nb];
            B.hub_off = B.atom_off[nb];
            B.nhub = B.atom_off[nb + 1] - B.atom_off[nb];
            hubw.assign((size_t)H, 0.0);
            for (uint64_t p = B.hub_off; p < B.hub_off + B.nhub; ++p) hubw[ac[p] - V] += aw[p];
        }
        // a cell's mass: its block's atoms plus 1/nb of the part's hub atoms
        double tot = 0.0;
        for (int k = 0; k < nb; ++k) {
            B.mass[k] = m[k] + mH / nb;
            B.hub_p[k] = B.mass[k] > 0 ? (mH / nb) / B.mass[k] : 0.0;
            tot += B.mass[k];
        }
        for (double& x : B.mass) x /= tot;
    }
    // per block: the C-row law of its cell (over [cb[k], cb[k+1]) then the H
    // hub slots) and the flags of its C rows and (LINE-2) of this part's W rows
    std::vector<std::vector<double>> pcb((size_t)nb);
    std::vector<std::vector<uint8_t>> hcb((size_t)nb), hwb((size_t)nb);
    // the hottest row of each cell (its launch's concurrency cap, cell_grid):
    // walks the scaled global law, LINE-2 the cell's exact one
    B.pmax_w.assign((size_t)nb, 0.0);
    B.pmax_c.assign((size_t)nb, 0.0);
    double wmax = 0.0;
    for (int64_t v = wlo; v < whi; ++v) wmax = std::max(wmax, ps[v] * nparts);
    {
        par_blocks([&](int k) {
            const int64_t lo = B.cb[k], n = B.cb[k + 1] - lo;
            auto& pcx = pcb[k];
            pcx.assign((size_t)(n + H), 0.0);
            hcb[k].assign((size_t)(n + H), 0);
            if (walk) {   // capi build_hot_maps' scaled law (hot_pc); the hub slots at their global rate
                double mx = 0.0;
                for (int64_t i = 0; i < n; ++i) {
                    pcx[i] = is_hub(lo + i) ? 0.0 : (pc[lo + i] + K * pn[lo + i]) * nb;
                    hcb[k][i] = hyb && !is_hub(lo + i) ? c->hot_c[lo + i] : 0;
                    mx = std::max(mx, pcx[i]);
                }
                for (int64_t j = 0; j < H; ++j) {
                    pcx[n + j] = B.hub_rate[j];
                    hcb[k][n + j] = hyb && (double)M * B.hub_rate[j] > tau;
                    mx = std::max(mx, pcx[n + j]);
                }
                B.pmax_w[k] = wmax;
                B.pmax_c[k] = mx;
                return;
            }
            std::vector<double> pw((size_t)(whi - wlo), 0.0);
            double mraw = 0.0;   // the cell's raw atom mass (its block's, plus 1/nb of the hub atoms')
            for (uint64_t p = B.atom_off[k]; p < B.atom_off[k + 1]; ++p) {
                pw[av[p] - wlo] += aw[p];
                pcx[ac[p] - lo] += aw[p];
                mraw += aw[p];
            }
            for (uint64_t p = B.hub_off; p < B.hub_off + B.nhub; ++p) pw[av[p] - wlo] += aw[p] / nb;
            for (int64_t j = 0; j < H; ++j) pcx[n + j] = hubw[j] / nb;
            mraw += mH / nb;
            hwb[k].assign(pw.size(), 0);
            double mw = 0.0, mc = 0.0;
            for (size_t i = 0; i < pw.size(); ++i) {
                hwb[k][i] = mraw > 0 && (double)M * pw[i] / mraw > tau;
                if (mraw > 0) mw = std::max(mw, pw[i] / mraw);
            }
            const double pnb = nraw[k];
            for (int64_t i = 0; i < n + H; ++i) {
                const double pneg = i < n ? (is_hub(lo + i) ? 0.0 : pn[lo + i]) : pn[B.hubs[i - n]] / nb;
                pcx[i] = (mraw > 0 ? pcx[i] / mraw : 0.0) + (pnb > 0 ? K * pneg / pnb : 0.0);
                hcb[k][i] = (double)M * pcx[i] > tau;
                mc = std::max(mc, pcx[i]);
            }
            B.pmax_w[k] = mw;
            B.pmax_c[k] = mc;
        });
    }
    // one tag per hub slot and per W row of the shared hub atoms (a row's
    // tag must not depend on the cell that draws it): hot in any cell
    std::vector<uint8_t> hubhot((size_t)H, 0), hwh;
    if (H > 0 && hyb && walk) {
        const int64_t n0 = B.cb[1] - B.cb[0];
        for (int64_t j = 0; j < H; ++j) hubhot[j] = hcb[0][n0 + j];
    } else if (H > 0 && hyb) {
        hwh.assign((size_t)(whi - wlo), 0);
        for (int k = 0; k < nb; ++k) {
            const int64_t n = B.cb[k + 1] - B.cb[k];
            for (int64_t j = 0; j < H; ++j) hubhot[j] |= hcb[k][n + j];
            for (size_t i = 0; i < hwh.size(); ++i) hwh[i] |= hwb[k][i];
        }
        for (int k = 0; k < nb; ++k) {
            const int64_t n = B.cb[k + 1] - B.cb[k];
            for (int64_t j = 0; j < H; ++j) hcb[k][n + j] = hubhot[j];
        }
    }
    auto hc = [&](int k, int64_t x) -> uint32_t {
        if (!hyb) return 0u;
        if (x >= V) return hubhot[x - V];
        return hcb[k][x - B.cb[k]];
    };
    auto hw = [&](int k, int64_t v) -> uint32_t { return hyb && !walk ? hwb[k][v - wlo] : 0u; };
    // negative tables: block k's law over its non-hub rows and 1/nb of every
    // hub's (Go alias rule, power 1: any exact encoding of the law), ids
    // absolute (hub slots V + j); entries of the rows in place, of the slots
    // at [k * H, (k + 1) * H)
    {
        hvec<AliasEntry> nt((size_t)V);
        std::vector<AliasEntry> hnt((size_t)nb * (size_t)H);
        par_blocks([&](int k) {
            const int64_t lo = B.cb[k], n = B.cb[k + 1] - lo, nn = n + H;
            std::vector<double> wt((size_t)nn), prob((size_t)nn);
            std::vector<int64_t> alias((size_t)nn);
            std::vector<int32_t> self((size_t)nn);
            auto id = [&](int64_t i) { return (int32_t)(i < n ? lo + i : V + (i - n)); };
            for (int64_t i = 0; i < nn; ++i) {
                wt[i] = i < n ? (is_hub(lo + i) ? 0.0 : pn[lo + i]) : pn[B.hubs[i - n]] / nb;
                self[i] = id(i);
            }
            alias_go(wt.data(), nn, 1.0, prob.data(), alias.data());
            for (int64_t i = 0; i < nn; ++i) alias[i] = id(alias[i]);
            std::vector<AliasEntry> e((size_t)nn);
            alias_encode(prob.data(), alias.data(), nn, self.data(), e.data());
            for (int64_t i = 0; i < nn; ++i) {
                const uint32_t al = (uint32_t)e[i].alias;
                e[i].alias = (int32_t)(al | (hc(k, al) << 30) | (hc(k, self[i]) << 31));
                if (i < n) nt[lo + i] = e[i];
                else hnt[(size_t)k * H + (i - n)] = e[i];
            }
        });
        if ((rc = upload(c, B.d_ntab, reinterpret_cast<const uint2*>(nt.data()), (size_t)V, true))) return rc;
        if (H > 0) {
            if ((rc = upload(c, B.d_hub_ntab, reinterpret_cast<const uint2*>(hnt.data()), hnt.size()))) return rc;
            if ((rc = upload(c, B.d_hub_ids, B.hubs.data(), B.hubs.size()))) return rc;
            if (walk) {   // the pair kernels' hub lookup: slot j | hot tag << 30
                std::vector<int32_t> ho((size_t)V, -1);
                for (int64_t j = 0; j < H; ++j) ho[B.hubs[j]] = (int32_t)(j | ((int64_t)hubhot[j] << 30));
                if ((rc = upload(c, B.d_hub_of, ho.data(), ho.size()))) return rc;
            }
        }
    }
    // LINE-2: one alias table per block over its atoms and one over the part's
    // hub atoms, tagged per cell (the hub atoms with their any-cell tags)
    if (!walk) {
        hvec<uint4> at((size_t)B.atom_off[NBK] * 2);
        auto table = [&](int k, uint64_t a0, uint64_t n, bool hubs) {
            if (n == 0) return;
            std::vector<double> prob(n);
            std::vector<int64_t> alias(n);
            std::vector<AliasEntry> e(n);
            alias_go(aw.data() + a0, (int64_t)n, 1.0, prob.data(), alias.data());
            alias_encode(prob.data(), alias.data(), (int64_t)n, nullptr, e.data());
            auto tw = [&](int32_t v) -> uint32_t { return hubs ? (hyb ? hwh[v - wlo] : 0u) : hw(k, v); };
            for (uint64_t i = 0; i < n; ++i) {
                const uint64_t s = a0 + i, a = a0 + (uint64_t)e[i].alias;
                at[2 * s] = make_uint4(e[i].thresh, (uint32_t)av[s] | (tw(av[s]) << 30),
                                       (uint32_t)ac[s] | (hc(k, ac[s]) << 30), 0u);
                at[2 * s + 1] = make_uint4((uint32_t)av[a] | (tw(av[a]) << 30),
                                           (uint32_t)ac[a] | (hc(k, ac[a]) << 30), 0u, 0u);
            }
        };
        par_blocks([&](int k) { table(k, B.atom_off[k], B.atom_off[k + 1] - B.atom_off[k], false); });
        if (H > 0) table(0, B.hub_off, B.nhub, true);
        if ((rc = upload(c, B.d_atoms, at.data(), at.size(), true))) return rc;
    }
    c->hot_M = M;
    std::vector<int2> hash;
    std::vector<int32_t> ids;
    std::vector<std::pair<double, int32_t>> wcand;   // walk cells: the part's hot W rows (block_sh_sets)
    if (walk && hyb && wcomb_on()) {
        // a W row's rate counts each record's 1 + K gradient terms against the
        // pair budget (SMORE_WALK_WCOMB_X overrides the factor)
        const char* xe = getenv("SMORE_WALK_WCOMB_X");
        const double wx = xe ? atof(xe) : (double)(1 + K);
        for (int64_t v = wlo; v < whi; ++v) {
            const double p = ps[v] * nparts * wx;
            if ((double)M * p > tau) wcand.push_back({p, (int32_t)(v | SH_WKEY)});
        }
    }
    block_sh_sets(c, walk, hyb && !small, M, pcb, hcb, hash, ids, wcand);
    if (getenv("SMORE_SH_DEBUG"))
        for (int k = 0; k < nb; ++k)
            fprintf(stderr, "[cell] part %d/%d block %d M %lld M*pmax_w %.4g M*pmax_c %.4g hubs %lld hub_p %.4g\n", part,
                    nparts, k, (long long)M, M * B.pmax_w[k], M * B.pmax_c[k], (long long)H, B.hub_p[k]);
    if ((rc = upload(c, B.d_sh_hash, hash.data(), hash.size()))) return rc;
    if ((rc = upload(c, B.d_sh_ids, ids.data(), ids.size()))) return rc;
    B.key = key;
    return SMORE_OK;
}

int smore_block_set_hubs(smore_ctx* c, int64_t hubs) {
    if (!c || hubs < -1) return SMORE_EINVAL;
    c->blk_hubs = hubs;
    return SMORE_OK;
}

int smore_block_hubs(const smore_ctx* c, int64_t* H, int64_t* first_slot, int32_t* rows, double* rates) {
    if (!c) return SMORE_EINVAL;
    if (!c->blk.nb) return SMORE_ESTATE;
    const auto& B = c->blk;
    if (H) *H = B.H;
    if (first_slot) *first_slot = c->g->V;
    if (rows) std::copy(B.hubs.begin(), B.hubs.end(), rows);
    if (rates) std::copy(B.hub_rate.begin(), B.hub_rate.end(), rates);
    return SMORE_OK;
}

int smore_block_hubs_load(smore_ctx* c) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if (!c->blk.nb) return fail(c, SMORE_ESTATE, "no block setup");
    if (!c->blk.H) return SMORE_OK;
    if ((rc = set_device(c))) return rc;
    float* C = c->d_table[1];
    HIPCHK(c, launch_rows_gather(C, c->blk.d_hub_ids, (uint64_t)c->blk.H, c->dpad, C + (size_t)c->g->V * c->dpad,
                                 c->stream));
    return SMORE_OK;
}

int smore_block_hubs_store(smore_ctx* c) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if (!c->blk.nb) return fail(c, SMORE_ESTATE, "no block setup");
    if (!c->blk.H) return SMORE_OK;
    if ((rc = set_device(c))) return rc;
    float* C = c->d_table[1];
    HIPCHK(c, launch_rows_scatter(C, c->blk.d_hub_ids, (uint64_t)c->blk.H, c->dpad, C + (size_t)c->g->V * c->dpad,
                                  c->stream));
    return SMORE_OK;
}

int smore_block_cell_launches(const smore_ctx* c) {
    if (!c || !c->blk.nb) return 1;
    return cell_launches(c->blk);
}

int smore_block_hub_scales(const smore_ctx* c, double samples, double c0, float* scales) {
    if (!c || !scales || !(samples > 0.0) || !(c0 > 0.0)) return SMORE_EINVAL;
    if (!c->blk.nb) return SMORE_ESTATE;
    hub_scales(c->blk, samples, c0, scales);
    return SMORE_OK;
}

int smore_block_info(const smore_ctx* c, int* nparts, int* part, int* nblocks) {
    if (!c) return SMORE_EINVAL;
    if (nparts) *nparts = c->blk.nb ? c->blk.n : 1;
    if (part) *part = c->blk.nb ? c->blk.r : 0;
    if (nblocks) *nblocks = c->blk.nb;
    return SMORE_OK;
}

int smore_block_bounds(const smore_ctx* c, int64_t* wb, int64_t* cb) {
    if (!c) return SMORE_EINVAL;
    if (!c->blk.nb) return SMORE_ESTATE;
    if (wb) std::copy(c->blk.wb.begin(), c->blk.wb.end(), wb);
    if (cb) std::copy(c->blk.cb.begin(), c->blk.cb.end(), cb);
    return SMORE_OK;
}

int smore_block_mass(const smore_ctx* c, double* mass) {
    if (!c || !mass) return SMORE_EINVAL;
    if (!c->blk.nb || c->blk.model != SMORE_LINE2) return SMORE_ESTATE;
    std::copy(c->blk.mass.begin(), c->blk.mass.end(), mass);
    return SMORE_OK;
}

int smore_block_part_mass(const smore_ctx* c, double* mass) {
    if (!c || !mass) return SMORE_EINVAL;
    if (!c->blk.nb || c->blk.model != SMORE_LINE2) return SMORE_ESTATE;
    std::copy(c->blk.part_mass.begin(), c->blk.part_mass.end(), mass);
    return SMORE_OK;
}

int smore_block_neg_scale(const smore_ctx* c, int block, double* w) {
    if (!c || !w) return SMORE_EINVAL;
    if (!c->blk.nb || c->blk.model != SMORE_LINE2) return SMORE_ESTATE;
    if (block < 0 || block >= c->blk.nb) return SMORE_EINVAL;
    const EdgeArgs a = cell_args(const_cast<smore_ctx*>(c), block, false);
    *w = a.neg_scale > 0.0f ? (double)a.neg_scale : 1.0;
    return SMORE_OK;
}

int smore_block_counts(const smore_ctx* c, uint64_t samples, uint64_t* counts) {
    if (!c || !counts) return SMORE_EINVAL;
    if (!c->blk.nb || c->blk.model != SMORE_LINE2) return SMORE_ESTATE;
    largest_remainder(samples, c->blk.mass.data(), c->blk.nb, counts);
    return SMORE_OK;
}

int smore_block_train_edges_async(smore_ctx* c, int block, uint64_t begin, uint64_t count, uint64_t total, int K,
                                  double alpha0, uint64_t seed, int mode) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_LINE2) return fail(c, SMORE_ESTATE, "no LINE-2 block setup (smore_block_setup)");
    if (block < 0 || block >= B.nb) return fail(c, SMORE_EINVAL, "block out of range");
    if (K != B.K || mode != B.mode) return fail(c, SMORE_EINVAL, "K / mode differ from smore_block_setup's");
    if (total == 0) return fail(c, SMORE_EINVAL, "total == 0");
    if (count == 0) return SMORE_OK;
    if ((rc = set_device(c))) return rc;
    const uint64_t na = B.atom_off[block + 1] - B.atom_off[block];
    if (na == 0 && B.nhub == 0) return fail(c, SMORE_EINVAL, "block without atoms (mass 0) asked for samples");
    EdgeArgs a = cell_args(c, block, false);
    if (const char* e = getenv("SMORE_EDGE_CHUNK")) a.pair_slice = (uint32_t)std::max(0, atoi(e));
    a.total = total;
    a.seed = seed;
    a.alpha0 = alpha0;
    a.count = count;
    const int grid = cell_grid(c, a, block);
    BlockArgs ba = block_args(c);
    ba.atom_off = B.atom_off[block];
    ba.natoms = (uint32_t)na;
    ba.hub_thr = B.nhub ? prob_thr(B.hub_p[block]) : 0u;
    const int RW = rec_width(kmax_of(K));
    const uint64_t chunk_max = mode == SMORE_SERIAL ? ((uint64_t)1 << 30) / (uint64_t)RW : (uint64_t)1 << 27;
    const uint64_t chunk = std::min<uint64_t>(count, chunk_max);
    const int nch = (int)((count + chunk - 1) / chunk);
    if (c->rec_cap < chunk * RW) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * RW * sizeof(int32_t)));
        c->rec_cap = chunk * RW;
    }
    if ((rc = grow_events(c, c->phase_ev, 2 * (size_t)nch + 1))) return rc;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream));
    for (int k = 0; k < nch; ++k) {
        const uint64_t b = (uint64_t)k * chunk, n = std::min<uint64_t>(chunk, count - b);
        if (k) HIPCHK(c, hipEventRecord(c->phase_ev[2 * k], c->stream));
        HIPCHK(c, launch_block_draw(ba, block, seed, begin + b, n, K, c->d_rec, c->stream));
        HIPCHK(c, hipEventRecord(c->phase_ev[2 * k + 1], c->stream));
        EdgeArgs ak = a;
        ak.begin = begin + b;
        ak.count = n;
        ak.rec = c->d_rec;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        HIPCHK(c, launch_edge_train(ak, grid, c->stream));
        HIPCHK(c, hipEventRecord(c->phase_ev[2 * k + 2], c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = nch;
    return SMORE_OK;
}

int smore_block_sample_edges(smore_ctx* c, int block, uint64_t seed, uint64_t begin, uint64_t count, int K,
                             int32_t* out) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if (!out) return SMORE_EINVAL;
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_LINE2) return fail(c, SMORE_ESTATE, "no LINE-2 block setup (smore_block_setup)");
    if (block < 0 || block >= B.nb || K < 0 || K > 20) return fail(c, SMORE_EINVAL, "bad block / K");
    if (count == 0) return SMORE_OK;
    if ((rc = set_device(c))) return rc;
    BlockArgs ba = block_args(c);
    ba.atom_off = B.atom_off[block];
    ba.natoms = (uint32_t)(B.atom_off[block + 1] - B.atom_off[block]);
    ba.hub_thr = B.nhub ? prob_thr(B.hub_p[block]) : 0u;
    if (ba.natoms == 0 && B.nhub == 0) return fail(c, SMORE_EINVAL, "block without atoms");
    const int RW = rec_width(kmax_of(K));
    int32_t* d = nullptr;
    HIPCHK(c, hipMalloc((void**)&d, count * RW * sizeof(int32_t)));
    hipError_t e = launch_block_draw(ba, block, seed, begin, count, K, d, c->stream);
    std::vector<int32_t> h(count * RW);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, SMORE_EHIP, std::string("block sample: ") + hipGetErrorString(e));
    for (uint64_t t = 0; t < count; ++t)
        for (int j = 0; j < 2 + K; ++j) out[t * (2 + K) + j] = h[t * RW + j] & ID_MASK;
    return SMORE_OK;
}

int smore_block_walks_generate(smore_ctx* c, int rule, uint64_t walk_begin, uint64_t walk_end, uint64_t gen_lo,
                               uint64_t gen_hi, int walk_times, int walk_steps, int window, int window_min, int K,
                               double alpha0, uint64_t seed, const int64_t* order, uint64_t order_base, int mode) {
    return block_walks_gen(c, rule, walk_begin, walk_end, gen_lo, gen_hi, walk_times, walk_steps, window, window_min,
                           K, alpha0, seed, order, order_base, mode);
}

int smore_block_walks_emit(smore_ctx* c) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if ((rc = set_device(c))) return rc;
    return block_walks_emit(c);
}

int smore_block_walks_buffer(smore_ctx* c, void** walks, void** lens, int64_t* stride) {
    if (!c) return SMORE_EINVAL;
    if (walks) *walks = c->d_walks;
    if (lens) *lens = c->d_lens;
    if (stride) *stride = (int64_t)c->blk.wargs.steps + 1;
    return SMORE_OK;
}

int smore_block_prepare_walks(smore_ctx* c, int rule, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                              int walk_steps, int window, int window_min, int K, double alpha0, uint64_t seed,
                              const int64_t* order, uint64_t order_base, int mode) {
    int rc = block_walks_gen(c, rule, walk_begin, walk_end, walk_begin, walk_end, walk_times, walk_steps, window,
                             window_min, K, alpha0, seed, order, order_base, mode);
    if (rc) return rc;
    return block_walks_emit(c);
}

int smore_block_train_walks_async(smore_ctx* c, int block) { return smore_block_train_walks_part_async(c, block, 0, 1); }

int smore_block_train_walks_part_async(smore_ctx* c, int block, int part, int parts) {
    int rc;
    if ((rc = check_ctx(c))) return rc;
    if (parts < 1 || part < 0 || part >= parts) return fail(c, SMORE_EINVAL, "bad bucket part");
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_CENSUS) return fail(c, SMORE_ESTATE, "no walk block setup (smore_block_setup)");
    if (block < 0 || block >= B.nb) return fail(c, SMORE_EINVAL, "block out of range");
    if (!B.walks) return SMORE_OK;   // an empty round
    if ((rc = set_device(c))) return rc;
    EdgeArgs a = cell_args(c, block, true);
    a.total = 1;
    a.rec = c->d_rec;
    a.count = B.rec_bound;   // the grid's bound; the launch reads its range on the device
    a.rec_base = B.d_off + (size_t)block * B.walks;
    a.count_dev = B.d_off + (size_t)(block + 1) * B.walks;
    a.part_q = (uint32_t)part;
    a.part_n = (uint32_t)parts;
    const int grid = B.mode == SMORE_SERIAL ? 1 : cell_grid(c, a, block);
    HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
    HIPCHK(c, launch_edge_train(a, grid, c->stream));
    return SMORE_OK;
}

int smore_block_walk_records(smore_ctx* c, int block, uint64_t* n) {
    if (!c || !n) return SMORE_EINVAL;
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_CENSUS || block < 0 || block >= B.nb) return SMORE_EINVAL;
    *n = 0;
    if (!B.walks) return SMORE_OK;
    uint64_t lo = 0, hi = 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(&lo, B.d_off + (size_t)block * B.walks, sizeof lo, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(&hi, B.d_off + (size_t)(block + 1) * B.walks, sizeof hi, hipMemcpyDeviceToHost));
    *n = hi - lo;
    return SMORE_OK;
}

int smore_block_walk_records_copy(smore_ctx* c, int block, int32_t* out, uint64_t cap, uint64_t* n, int* width) {
    if (!c || !n || !width) return SMORE_EINVAL;
    auto& B = c->blk;
    if (!B.nb || B.model != SMORE_CENSUS || block < 0 || block >= B.nb) return SMORE_EINVAL;
    const int RW = rec_width(kmax_of(B.K));
    *width = RW;
    *n = 0;
    if (!B.walks) return SMORE_OK;
    uint64_t lo = 0, hi = 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(&lo, B.d_off + (size_t)block * B.walks, sizeof lo, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(&hi, B.d_off + (size_t)(block + 1) * B.walks, sizeof hi, hipMemcpyDeviceToHost));
    *n = hi - lo;
    if (!out) return SMORE_OK;
    if (cap < hi - lo) return fail(c, SMORE_EINVAL, "walk records: buffer too small");
    if (hi > lo)
        HIPCHK(c, hipMemcpy(out, static_cast<const int32_t*>(c->d_rec) + lo * RW, (hi - lo) * RW * sizeof(int32_t),
                            hipMemcpyDeviceToHost));
    return SMORE_OK;
}

}  // extern "C"
