// train_kernels.h -- launch interface of the gfx950 hot-path kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"

namespace smore {

struct EdgeArgs {
    DevGraph g;
    const float* sig;              // 1001-entry fastSigmoid table
    float* W;                      // [V][dpad]
    float* C;                      // [V][dpad] (== W for shared-table models)
    unsigned long long* skipped;   // samples whose source had no out-edge
    const double* tcum;            // Go semantics: per-vertex prefix sums of edge weights
    // hybrid write-combining of the super-hot context rows (edge kernel only):
    // open-addressing hash {id, slot} (SH_HASH entries, id -1 = empty), the
    // slot -> id list, sh_rows slots (0 = off), a block flush every sh_flush rounds
    const int2* sh_hash;
    const int32_t* sh_ids;
    int sh_rows, sh_flush;
    int sh_flush_w;                // W-key slots (SMORE_SH_WROWS) drained every sh_flush_w rounds too (0: off)
    // per-slot drain intervals: every slot drains every sh_flush rounds (a
    // power of two); slot i also every 2^j rounds when i < sh_lvl[j] (the slot
    // list is sorted by rate, so the slots due at a round are a prefix;
    // all-zero sh_lvl: one interval for all)
    int sh_lvl[8];
    // edge kernels: the pre-drawn sample records of samples [begin, begin+count)
    // (draw_kernel), rec_width(KMAX) int32 each
    const int32_t* rec;
    const uint64_t* count_dev;     // non-null: the record count is read here (device-side pair totals)
    const uint64_t* rec_base;      // non-null: the launch's records are [*rec_base, *count_dev) (block buckets)
    unsigned long long* work;      // Hogwild edge kernels: chunk counter, zeroed per launch
    int alpha_rec;                 // learning rate in record word 2 + KMAX: 1 walk pairs (pair kernels),
                                   // 2 independent samples (the edge kernel: the hot/cold split)
    uint32_t pair_slice;           // pair kernels: records per group slice (0: CH_ROUNDS)
    // negative-gradient weight (2-D block schedule): a cell
    // draws its negatives from its C block's restricted law, but gets samples
    // in proportion to the block's CONTEXT mass; weighting the negatives'
    // step by NegativeSample's block mass over the cell's share restores the
    // epoch's negative law.  neg_scale <= 0: 1 (off).  neg_lo / neg_hi
    // non-null (walk cells): neg_scale is the block's negative share and the
    // weight is computed on the device from the round's record counts,
    // neg_scale * (*neg_hi - *neg_lo) / records.
    float neg_scale;
    const uint64_t* neg_lo;
    const uint64_t* neg_hi;
    // pair kernel, hybrid: a run's W row is STORED when it is not hot-tagged
    // (the edge rule), instead of adding its delta atomically (walk cells of
    // the block schedule: their runs are ~1 record long)
    int w_plain;
    // a block bucket's launch in parts: records [lo, hi) of the bucket's
    // range with lo = n part_q / part_n (part_n <= 1: the whole bucket)
    uint32_t part_q, part_n;
    // walk records through the (row-prefetching) edge kernel instead of the
    // pair kernel (block walk cells: their W runs are ~1 record long)
    int rec_edge;
    int w_comb;          // pair kernel (walk cells): the runs' W rows looked up in the write-combined set
    uint64_t begin, count, total, seed;
    double alpha0;
    float reg;
    int dpad, K, model, mode;
};

// DeepWalk: a chunk of walks [walk_begin, walk_begin + nwalks)
struct WalkArgs {
    const int64_t* order;          // walk start vertices of walks [order_base, ...) (a slice of the full order)
    uint64_t order_base;
    int32_t* walks;                // nwalks x (steps + 1); C++ walks hold id | hc << 30 | hw << 31
    int32_t* lens;                 // nwalks
    uint64_t walk_begin, nwalks, total_walks;
    int steps, window;
    int rule;                      // pair rule: 0 DeepWalk SkipGrams (random shrink), 1 Walklets ScaleSkipGrams
    int window_min;                // Walklets: pairs at distance [window_min, window] (clamped as the reference)
    // node2vec (Go, rule 2): 1/p, 1/q, raw CSR edge weights and a per-vertex
    // sorted copy of the CSR targets (areNeighbors by binary search)
    double inv_p, inv_q;
    const double* wts;
    const int32_t* nbr_sorted;
    // metapath2vec (Go, rule 3): node types, every vertex's CSR targets grouped
    // by type (push order kept) with offsets toff[v * (ntypes + 1) + t], the
    // meta-paths (type ids, path p = paths[path_off[p] .. path_off[p + 1]))
    const int32_t* ntype;
    const int32_t* ttargets;
    const int64_t* toff;
    const int32_t* paths;
    const int32_t* path_off;
    int ntypes, npaths;
    int slot_extra;                // draws before the step draws (metapath2vec: the path choice)
    // walk partition (smore_set_walk_owner): only pairs whose center (W row)
    // walk[i] is in [own_lo, own_hi) become records; every pair still takes
    // its draws, so the records are the one-context records restricted
    int32_t own_lo = 0, own_hi = 0x7FFFFFFF;
};

// APP: units [unit_begin, unit_begin + n) of walk_times * V * sample_times; unit
// u = w * sample_times + s jumps from order[w - order_base] (APP::Train)
struct AppArgs {
    const int64_t* order;
    uint64_t order_base, unit_begin, n, total_walks;
    int sample_times;
    double jump;
};

// lanes per sample group: G = min(64, pow2ceil(dpad / 4)); lane l owns the
// row's 16-B chunks l, l+G, ... in M = regs_of(dpad) registers
// (device_common.h elem_off; DESIGN.md "Arithmetic spec")
int lanes_of(int dpad);
inline int regs_of(int dpad) {
    const int G = lanes_of(dpad);
    return 4 * ((dpad / 4 + G - 1) / G);
}
// int32 words per pre-drawn edge-sample record {v, c, n_1..n_K, pad}: the
// smallest power of two >= 2 + KMAX, at least 4 (whole 16-B words)
constexpr int rec_width(int kmax) {
    int r = 4;
    while (r < 2 + kmax) r <<= 1;
    return r;
}
constexpr uint64_t CH_ROUNDS = 128;   // rounds per dynamically handed-out chunk
inline int kmax_of(int K) { return K <= 5 ? 5 : K <= 10 ? 10 : 20; }
hipError_t launch_delta_begin(const float* T, float* S, float* D, float* R, uint64_t n, int cus, hipStream_t st);
hipError_t launch_delta_end(float* T, float* S, const float* D, const float* R, float scale, uint64_t n, int cus,
                            hipStream_t st);
hipError_t launch_delta_cycle(float* T, float* S, float* D, float* R, float scale, uint64_t n, int cus,
                              hipStream_t st);
hipError_t launch_pair_count(const WalkArgs& w, uint64_t seed, uint32_t* count, hipStream_t st);
// upper bound on the skip-gram pairs of one walk of `steps` steps: DeepWalk
// (window shrink >= 1) or Walklets (two clamped ranges of window - window_min + 1)
inline uint64_t pair_bound(int steps, int window, int rule = 0, int window_min = 0) {
    const uint64_t L = (uint64_t)steps + 1;
    if (rule == 1) return L * 2 * (uint64_t)std::max(1, window - window_min + 1);
    const uint64_t r = std::min<uint64_t>(2 * (uint64_t)window, L - 1);
    return L * r;
}
hipError_t scan_pair_counts(const uint32_t* count, uint64_t* off, uint64_t n, void** temp, size_t* temp_bytes,
                            hipStream_t st);
hipError_t launch_pair_emit(const DevGraph& g, const WalkArgs& w, uint64_t seed, int K, double alpha0,
                            const uint64_t* off, int32_t* rec, hipStream_t st);
hipError_t launch_pack(const DevGraph& g, uint64_t E, uint4* vt32, uint4* ct16, hipStream_t st);
// draw_split_kernel (train_draw.hip): the draws with the rate in the record,
// hot records from the front, the others from the back; counts[0] / [1] the
// hot / cold records (zeroed by the caller)
hipError_t launch_draw_split(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K, double alpha0,
                             uint64_t total, int base, int32_t* rec, unsigned long long* skipped,
                             unsigned long long* counts, hipStream_t st);
hipError_t launch_draw(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K, int32_t* rec,
                       unsigned long long* skipped, hipStream_t st);
constexpr int SH_HASH = 256;   // entries of the super-hot row hash (power of two, > the rows)
constexpr int32_t SH_WKEY = 1 << 30;   // write-combine key bit: a W row of a two-table model
// dynamic LDS of the hybrid edge kernel: hash, slot ids, pending deltas
// write-combined rows that fit the LDS budget: SMORE_SH_LDS floats of pending
// deltas (default 8192: 32 KB, three 256-thread blocks per CU with the hash,
// ids and sigmoid table), below the hash's size.  160 rows at d=64 (40 KB,
// hash 512) measured slower at one GPU (84.1 vs 83.6 ms per 2^27, C4) and in
// the block schedule's cells (C4, 8 GPUs: 5.44 vs 5.76 x predicted)
inline int sh_rows_max(int dpad) {
    static const int lds = [] {
        const char* e = getenv("SMORE_SH_LDS");
        const int v = e ? atoi(e) : 8192;
        return v > 0 ? v : 8192;
    }();
    const int r = lds / (dpad > 0 ? dpad : 1);
    return r < SH_HASH - 1 ? r : SH_HASH - 1;
}

inline size_t sh_lds_bytes(int sh_rows, int dpad) {
    return sh_rows > 0 ? SH_HASH * 8 + (size_t)sh_rows * 4 + (size_t)sh_rows * dpad * 4 : 0;
}
inline uint32_t sh_hash_of(int32_t id) { return ((uint32_t)id * 2654435761u) >> 24; }
// Go edge models on records: go_draw_kernel (train_go.hip; unit_w: every edge
// weight is 1) then go_rec_kernel (go_rec.h; train_go_rec_<mode>.hip)
hipError_t launch_go_draw(const DevGraph& g, const double* tcum, int unit_w, uint64_t seed, uint64_t begin,
                          uint64_t count, int K, int32_t* rec, unsigned long long* skipped, hipStream_t st);
#define SMORE_DECL_GO_REC(name)                                                  \
    hipError_t launch_go_rec_##name(const EdgeArgs& a, int grid, hipStream_t st); \
    const void* go_rec_symbol_##name(const EdgeArgs& a);
SMORE_DECL_GO_REC(s) SMORE_DECL_GO_REC(a) SMORE_DECL_GO_REC(h)
#undef SMORE_DECL_GO_REC
hipError_t launch_go_walk(const EdgeArgs& a, const WalkArgs& w, int grid, hipStream_t st);
hipError_t launch_go_sample(const DevGraph& g, const double* tcum, uint64_t seed, uint64_t begin, uint64_t count,
                            int K, int32_t* out, hipStream_t st);
hipError_t launch_walk_gen(const DevGraph& g, const WalkArgs& w, uint64_t seed, hipStream_t st);
// HPE: samples [begin, begin + n) of total (HPE::Train), walk_steps community
// steps each
struct HpeArgs {
    uint64_t begin, n, total;
    int walk_steps;
};
hipError_t launch_hpe_records(const DevGraph& g, const HpeArgs& p, uint64_t seed, int K, double alpha0, int32_t* rec,
                              unsigned long long* skipped, hipStream_t st);
hipError_t launch_app_records(const DevGraph& g, const AppArgs& p, uint64_t seed, int K, double alpha0, int32_t* rec,
                              hipStream_t st);
constexpr int APP_MAX_STEPS = 1 << 24;   // jumping-walk bound (oracle APP_MAX_STEPS)
// caller-supplied pairs (smore_train_pairs): pairs per RNG unit (oracle ORC_PAIR_BLOCK)
constexpr uint64_t PAIR_BLOCK = (uint64_t)1 << 20;
hipError_t launch_caller_pairs(const DevGraph& g, const int32_t* pv, const int32_t* pc, uint64_t n, uint64_t first,
                               int K, float alpha, uint64_t seed, uint64_t unit0, int go, int tagged, int32_t* rec,
                               hipStream_t st);
// row census (smore_census_begin): per record +1 at W[word 0] and at C[word 1]
// and C[each negative >= 0]; records whose word 1 is negative (HPE's skipped
// samples and finished walks) count nothing.  count_dev: the count on the device
hipError_t launch_row_census(const int32_t* rec, uint64_t n, const uint64_t* count_dev, int RW, int K,
                             unsigned long long* cw, unsigned long long* cc, int cus, hipStream_t st);
// edge kernel instantiations, one per (scatter mode s/a/h, KMAX) (train_edge_*.hip)
#define SMORE_DECL_EDGE(name)                                                   \
    hipError_t launch_edge_##name(const EdgeArgs& a, int grid, hipStream_t st); \
    const void* edge_symbol_##name(const EdgeArgs& a);
SMORE_DECL_EDGE(s5) SMORE_DECL_EDGE(s10) SMORE_DECL_EDGE(s20)
SMORE_DECL_EDGE(a5) SMORE_DECL_EDGE(a10) SMORE_DECL_EDGE(a20)
SMORE_DECL_EDGE(h5) SMORE_DECL_EDGE(h10) SMORE_DECL_EDGE(h20)
// DeepWalk pair-kernel instantiations (train_pair_*.hip; K <= 10)
#define SMORE_DECL_PAIR(name)                                                   \
    hipError_t launch_pair_##name(const EdgeArgs& a, int grid, hipStream_t st); \
    const void* pair_symbol_##name(const EdgeArgs& a);
SMORE_DECL_PAIR(s5) SMORE_DECL_PAIR(s10) SMORE_DECL_PAIR(a5) SMORE_DECL_PAIR(a10)
SMORE_DECL_PAIR(h5) SMORE_DECL_PAIR(h10)
#undef SMORE_DECL_PAIR
#undef SMORE_DECL_EDGE
// launch_edge_train / edge_kernel_symbol route DeepWalk pair records
// (alpha_rec) in the Hogwild modes to pair_train_kernel
hipError_t launch_edge_train(const EdgeArgs& a, int grid, hipStream_t st);
const void* edge_kernel_symbol(const EdgeArgs& a);
hipError_t launch_sample(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K,
                         int bpr, int32_t* out, hipStream_t st);
// 2-D block schedule (train_blocks.hip, blocks.cpp): C blocks <= BLOCK_MAX (N <= 16 W parts)
constexpr int BLOCK_MAX = 32;
struct BlockArgs {
    const uint4* atoms;       // LINE-2: this part's atoms, 2 uint4 each {thr, v, c, 0}, {v', c', 0, 0} (tagged ids)
    uint64_t atom_off;        // first atom of the launch's block
    uint32_t natoms;          // atoms of the launch's block
    const uint2* ntab;        // V entries: block k's negative alias over its vertices [cb[k], cb[k+1])
    int nb;                   // C blocks
    int32_t cb[BLOCK_MAX + 1];
    // hub C rows (blocks.cpp): slots V .. V + H - 1, drawn in every block.  A
    // block's negative alias runs over its rows then the H slots (entries
    // hub_ntab[k * H + j]); a LINE-2 sample takes a hub atom of the part
    // (atoms [hub_off, hub_off + nhub)) iff Philox word 2 < hub_thr.
    const uint2* hub_ntab;
    uint64_t hub_off;
    uint32_t nhub, hub_thr;
    int32_t H, V;
    // walk cells: per vertex -1, or its hub slot j | hot tag << 30; a pair
    // whose context is a hub goes to block (walk + center position) mod nb
    // (a center's hub pairs stay together) as slot id V + j
    const int32_t* hub_of;
};
hipError_t launch_block_draw(const BlockArgs& b, int blk, uint64_t seed, uint64_t begin, uint64_t count, int K,
                             int32_t* rec, hipStream_t st);
// rows idx[0 .. n) of T to out (gather) / from in (scatter), dpad floats each
hipError_t launch_rows_gather(const float* T, const int32_t* idx, uint64_t n, int dpad, float* out, hipStream_t st);
hipError_t launch_rows_scatter(float* T, const int32_t* idx, uint64_t n, int dpad, const float* in, hipStream_t st);
hipError_t launch_block_pair_count(const WalkArgs& w, const BlockArgs& b, uint64_t seed, uint32_t* count,
                                   hipStream_t st);
hipError_t launch_block_pair_emit(const WalkArgs& w, const BlockArgs& b, uint64_t seed, int K, double alpha0,
                                  const uint64_t* off, int32_t* rec, hipStream_t st);
// rows `ids` of T [*][dpad] from (to_table 1) / to (0) buf [n][dim] (membw.hip)
hipError_t launch_rows_io(float* T, const int32_t* ids, uint64_t n, int dpad, int dim, float* buf, int to_table,
                          hipStream_t st);
hipError_t launch_rows_put_sel(float* T, const int32_t* ids, const int32_t* pos, uint64_t m, int dpad, int dim,
                               const float* buf, hipStream_t st);
// streaming copy of n16 16-B words (membw.hip); variant 1 = non-temporal
hipError_t launch_copy(const void* src, void* dst, uint64_t n16, int blocks, int variant, hipStream_t st);
hipError_t launch_init_uniform(float* T, int64_t rows, int dim, int dpad, uint64_t seed,
                               hipStream_t st);

}  // namespace smore
