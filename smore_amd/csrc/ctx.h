// ctx.h -- the library context (one GPU's graph, tables and buffers) and the
// host-side helpers shared by the C ABI translation units (capi.cpp,
// exchange.cpp).  Internal: not part of the installed interface.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/smore_hip.h"
#include "host_graph.h"
#include "train_kernels.h"

using namespace smore;

struct smore_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    hipStream_t draw_stream = nullptr;   // draw kernels overlapping the previous chunk's update
    std::vector<hipEvent_t> sync_ev;     // draw-done / update-done hand-offs between the two streams
    std::string err;
    std::shared_ptr<HostGraph> g = std::make_shared<HostGraph>();   // shared by the replicas of a group
    bool has_graph = false;
    // device graph
    int64_t* d_offsets = nullptr;
    int32_t* d_targets = nullptr;
    AliasEntry* d_vtab = nullptr;
    AliasEntry* d_ntab = nullptr;
    AliasEntry* d_ctab = nullptr;
    float* d_sig = nullptr;
    unsigned long long* d_skipped = nullptr;
    unsigned long long* d_work = nullptr;   // chunk counter of the Hogwild edge kernels
    // tables
    float* d_table[2] = {nullptr, nullptr};
    int dim = 0, dpad = 0, ntables = 0;
    // hybrid scatter: hot-row bitmaps (1 bit per row), keyed by what built them
    double hot_tau = -1.0;               // < 0: the per-path default (HOT_TAU_EDGE / HOT_TAU_WALK)
    std::string hot_key;
    int64_t hot_rows[2] = {0, 0};
    // DeepWalk buffers
    int64_t* d_order = nullptr;         // the walk starts of the current call (a slice of the order)
    size_t order_cap = 0;
    int32_t* d_walks = nullptr;
    int32_t* d_lens = nullptr;
    size_t walk_buf_n = 0;              // int32 capacity of d_walks
    size_t walk_lens_n = 0;             // walk capacity of d_lens
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    int last_mode = -1;                 // scatter (SMORE_* mode) the last timed training call ran
    // smore_train_pairs_rows_mt: the combining queue of concurrent callers
    // (capi.cpp PairCombiner; created on first use)
    std::shared_ptr<struct PairCombiner> pair_comb;
    int64_t blk_hubs = -1;              // hub C rows of the block schedule (smore_block_set_hubs; -1 automatic)
    int64_t c_slots = 0;                // rows after V in the C table (the block schedule's hub slots)
    int cus = 0;
    int64_t last_loaded = 0;
    // edge-list loader: binary cache directory ("" = off) and the last load's figures
    std::string cache_dir;
    LoadStats load_stats;
    double load_seconds = 0.0;
    // semantics: SMORE_SEM_CPP (default) or SMORE_SEM_GO
    int semantics = 0;
    double* d_tcum = nullptr;
    int go_unit_w = 0;             // Go semantics: every edge weight is 1 (O(1) CDF target draws)
    // node2vec (Go): raw CSR weights and per-vertex sorted CSR targets, built on first use
    double* d_wts = nullptr;
    int32_t* d_nbr_sorted = nullptr;
    // metapath2vec (Go): node types and the per-type neighbour index (smore_set_node_types)
    int32_t* d_ntype = nullptr;
    int32_t* d_ttargets = nullptr;
    int64_t* d_toff = nullptr;
    int ntypes = 0;
    int32_t* d_paths = nullptr;
    int32_t* d_path_off = nullptr;
    std::vector<int32_t> path_host;     // the uploaded meta-paths (lens then types): re-upload only on change
    // CTDNE (Go): time-sorted out-edges and active time ranges (smore_set_temporal_edges)
    int64_t* d_t_off = nullptr;
    int32_t* d_t_tgt = nullptr;
    double* d_t_ts = nullptr;
    double* d_t_min = nullptr;
    double* d_t_max = nullptr;
    double t_min_time = 0.0, t_max_time = 0.0;
    bool has_temporal = false;
    // hybrid write-combining: super-hot context rows (hash + slot ids)
    int2* d_sh_hash = nullptr;
    int32_t* d_sh_ids = nullptr;
    int sh_rows = 0;
    int sh_max = 128, sh_flush = 0;      // flush 0: automatic drain interval (capi build_hot_maps)
    int sh_flush_eff = 32;               // the interval of the last hybrid launch
    int sh_flush_w_eff = 0;              // its W-key slots' own interval (0: none)
    int sh_lvl_eff[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // its per-slot drain levels (EdgeArgs::sh_lvl)
    // pre-drawn edge-sample records (train_draw.hip) and per-phase timing
    int32_t* d_rec = nullptr;
    unsigned long long* d_split = nullptr;   // hot / cold record counts of the split draw (2 per chunk buffer)
    // DeepWalk pair records: per-walk pair counts, their exclusive scan, scan scratch
    uint32_t* d_pcount = nullptr;
    uint64_t* d_poff = nullptr;
    size_t pair_walks = 0;
    void* d_scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    // packed draw tables (train_draw.hip), rebuilt when the graph tables change
    uint4* d_vt32 = nullptr;
    uint4* d_ct16 = nullptr;
    bool packed_ok = false;
    size_t rec_cap = 0;                 // int32 words
    std::vector<hipEvent_t> phase_ev;   // {before draw 0, after draw 0, after update 0, after draw 1, ...}
    int phase_n = 0;                    // chunks of the last edge launch
    // replica exchange over RCCL (exchange.cpp): snapshot S, own delta D and
    // the all-reduced deltas R per table, a communicator and its stream
    void* comm = nullptr;               // ncclComm_t (a same-device group: the group, no RCCL)
    bool own_comm = false;              // created by smore_comm_init (destroyed with the context)
    bool local_comm = false;            // replica of a same-device group (exchange.cpp local collectives)
    int nranks = 1, rank = 0;
    hipStream_t comm_stream = nullptr;
    hipEvent_t ex_ready = nullptr, ex_done = nullptr;
    float* ex_buf[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};   // [table][S, D, R]
    size_t ex_n = 0;                    // floats per exchanged table
    int ex_tables = 0;
    bool ex_pending = false;            // an all-reduce is in flight
    bool coll_queued = false;           // own communicator: collectives queued since the last watched sync
    int ex_mode = 0;                    // SMORE_SYNC_* of the in-flight exchange
    int ex_t0 = 0;                      // first exchanged table (1: W partitioned by source, C only)
    // adaptive exchange: per-row scales of the summed deltas per table and
    // the (model, K, updates, c0, N) they were made for
    float* ex_scale[2] = {nullptr, nullptr};
    std::string ex_scale_key;
    // hub-row exchange between launches (hot_exchange.h): row ids and the
    // packed own-delta / all-reduced buffers per table
    int32_t* hot_idx[2] = {nullptr, nullptr};
    float* hot_buf[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};   // [table][P, R]
    int64_t hot_n = 0;
    std::string hot_ex_key;
    // source partition (smore_set_source_partition): this context draws its
    // sources from part part_i of part_n -- contiguous vertex ranges of equal
    // source mass -- through part_vtab, the restricted vertex table on the
    // device; the host graph keeps the global one (shared by the replicas)
    int part_n = 1, part_i = 0;
    hvec<AliasEntry> part_vtab;
    std::vector<int64_t> part_bounds;   // part_n + 1 bounds of the current partition
    // row census (smore_census_begin / _end): while `census` is set the record
    // paths count the rows each record would update (d_census: W, C; V
    // counters each) instead of training; census_rate = counts per unit
    // walk partition (smore_set_walk_owner): W rows [own_lo, own_hi) owned;
    // the walk models emit only pairs of owned centers.  own_hi < 0: all
    int64_t own_lo = 0, own_hi = -1;
    bool census = false;
    unsigned long long* d_census[2] = {nullptr, nullptr};
    std::vector<double> census_rate[2];
    bool census_ok = false;
    uint64_t census_gen = 0;            // bumped by every smore_census_end (the adaptive scales' key)
    std::string census_key;             // what the group driver censused (exchange.cpp)
    // caller-supplied pairs (smore_train_pairs): a chunk of (v, c) on the device
    int32_t* d_pairs = nullptr;
    size_t pairs_cap = 0;               // pairs
    // row transfers (smore_set_rows / smore_get_rows): ids and dense rows
    int32_t* d_io_ids[2] = {nullptr, nullptr};   // [W, C] of smore_train_pairs_rows
    float* d_io_rows[2] = {nullptr, nullptr};
    size_t io_cap[2] = {0, 0};          // rows
    // the last hybrid hot maps' host side (capi build_hot_maps): row flags and
    // the C-row touch law they were made from, for the block tables' own tags
    std::vector<uint8_t> hot_c, hot_w;
    std::vector<double> hot_pc;
    int64_t hot_M = 0;
    bool hot_small = false;
    // 2-D block schedule (blocks.cpp): this context is part r of
    // N W parts; the C table is cut into nb = 2N blocks; a launch trains one
    // (part r, block b) cell from the cell's own draw tables
    struct Blocks {
        int n = 1, r = 0, nb = 0;       // nb 0: off
        int model = -1, K = 0, mode = -1;
        std::vector<int64_t> wb, cb;    // W part bounds (n + 1), C block bounds (nb + 1)
        std::vector<double> mass;       // LINE-2: this part's sample mass per C block (sums to 1)
        std::vector<double> part_mass;  // every part's share of the global source law (n, sums to 1)
        std::vector<double> nmass;      // NegativeSample's share of each C block (nb, sums to 1)
        std::vector<uint64_t> atom_off; // LINE-2: first atom of each block (nb + 1; + 1: the hub atoms' end)
        // hub C rows (smore_block_set_hubs): the H hottest C
        // rows are taken out of the blocks and trained in every cell on every
        // part, each part on its own copy in the C table's slot rows V .. V + H
        // (never inside a rotating block), the copies kept equal by a small
        // exchange after every sub-round
        int64_t H = 0;
        std::vector<int32_t> hubs;      // hub j's C row
        std::vector<double> hub_rate;   // hub j's expected C-row touches per sample (context + K negative law)
        uint64_t hub_off = 0, nhub = 0; // LINE-2: this part's hub atoms, atoms [hub_off, hub_off + nhub)
        std::vector<double> hub_p;      // LINE-2: per block, a cell sample's probability of being a hub atom
        uint2* d_hub_ntab = nullptr;    // nb x H: block k's negative alias entries of the hub slots
        int32_t* d_hub_ids = nullptr;   // H: the hubs' C rows (slot gather / scatter)
        int32_t* d_hub_of = nullptr;    // walks: V entries, -1 or the vertex's slot | hot tag << 30
        float* d_hub_ex[3] = {nullptr, nullptr, nullptr};   // group exchange over the slots: S, D, R
        float* d_hub_scale = nullptr;   // group exchange: per-slot scales (adaptive rule)
        std::string hub_scale_key;
        bool hub_pending = false;       // group exchange: an all-reduce of R is in flight
        uint4* d_atoms = nullptr;       // LINE-2: 2 uint4 per atom {thr, v, c, 0}, {v', c', 0, 0}
        uint2* d_ntab = nullptr;        // V entries: block b's negative alias at [cb[b], cb[b+1])
        int2* d_sh_hash = nullptr;      // nb x SH_HASH: per-block write-combined rows
        int32_t* d_sh_ids = nullptr;    // nb x sh_cap
        int sh_cap = 0;
        std::vector<int> sh_n;
        std::vector<int> sh_wn;                   // per block: W-row slots (walk cells: EdgeArgs::w_comb)
        std::vector<std::array<int, 8>> sh_lvl;   // per block: EdgeArgs::sh_lvl
        int sh_flush = 32;              // every slot's drain interval
        std::vector<double> pmax_w, pmax_c;   // per block: the cell's largest per-sample W / C row probability
        std::string key;
        // walk records of the current round, bucketed by C block: per (block,
        // walk) counts and their exclusive scan (nb * walks + 1)
        uint32_t* d_count = nullptr;
        uint64_t* d_off = nullptr;
        size_t count_cap = 0;
        uint64_t walks = 0;             // walks of the prepared round (0: none)
        uint64_t rec_bound = 0;         // records the prepared round may hold
        // the round being prepared (block_walks_gen -> block_walks_emit):
        // its walk arguments over all the round's walks, and the pair draws'
        WalkArgs wargs{};
        uint64_t wseed = 0;
        double walpha0 = 0.0;
        uint64_t wpairs = 0;            // pair bound per walk
    } blk;
};

// exchange.cpp: frees the exchange buffers and the communicator
void smore_exchange_release(smore_ctx* c);

namespace smore_host {

// rows after V in a two-table model's C table: the block schedule's hub slots
constexpr int64_t HUB_SLOTS_MAX = 65536;

// blocks.cpp: frees the block tables (a new graph, smore_destroy)
void blocks_release(smore_ctx* c);
// blocks.cpp: a walk round in two steps -- the walks [gen_lo, gen_hi) of the
// round [walk_begin, walk_end) generated into this context's round buffer
// (the rest may come from the other parts: walk-partitioned generation), then
// every walk's owned pairs bucketed into records (smore_block_prepare_walks =
// both over the whole round)
int block_walks_gen(smore_ctx* c, int rule, uint64_t walk_begin, uint64_t walk_end, uint64_t gen_lo, uint64_t gen_hi,
                    int walk_times, int walk_steps, int window, int window_min, int K, double alpha0, uint64_t seed,
                    const int64_t* order, uint64_t order_base, int mode);
int block_walks_emit(smore_ctx* c);
// blocks.cpp: launches per cell (the hub slots are exchanged after each)
int cell_launches(const smore_ctx::Blocks& B);
// blocks.cpp: the hub slots' exchange scales for `samples` per part per exchange
void hub_scales(const smore_ctx::Blocks& B, double samples, double c0, float* out);
// blocks.cpp: counts[k] = n * mass[k] by largest remainder (ties to the lower k)
void largest_remainder(uint64_t n, const double* mass, int parts, uint64_t* counts);
// exchange.cpp: the stream's completion under the RCCL failure watch (a
// context with its own communicator; SMORE_OK otherwise)
int comm_sync(smore_ctx* c);

inline int fail(smore_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(c, expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((c), SMORE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
inline void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

// the draw kernel's random-read tables (packed vertex / context tables, the
// negative alias table): default device memory; SMORE_DRAW_MEM=uncached
// allocates them uncached (memory-side reads sized to the access instead of
// 128-B L2 lines; an experiment knob)
inline hipError_t draw_malloc(void** p, size_t n) {
    static const bool unc = [] {
        const char* e = getenv("SMORE_DRAW_MEM");
        return e && !strcmp(e, "uncached");
    }();
    return unc ? hipExtMallocWithFlags(p, n, hipDeviceMallocUncached) : hipMalloc(p, n);
}

template <class T>
int upload(smore_ctx* c, T*& d, const T* h, size_t n, bool draw_table = false) {
    dfree(d);
    if (n == 0) n = 1;
    HIPCHK(c, draw_table ? draw_malloc((void**)&d, n * sizeof(T)) : hipMalloc((void**)&d, n * sizeof(T)));
    if (h) HIPCHK(c, hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
    return SMORE_OK;
}

inline int set_device(smore_ctx* c) {
    if (c->device < 0) return fail(c, SMORE_ESTATE, "host-only context (device < 0) has no GPU state");
    HIPCHK(c, hipSetDevice(c->device));
    return SMORE_OK;
}

inline int upload_graph(smore_ctx* c) {
    int rc;
    dfree(c->d_wts);
    dfree(c->d_nbr_sorted);
    dfree(c->d_ntype);
    dfree(c->d_ttargets);
    dfree(c->d_toff);
    c->ntypes = 0;
    dfree(c->d_t_off);
    dfree(c->d_t_tgt);
    dfree(c->d_t_ts);
    dfree(c->d_t_min);
    dfree(c->d_t_max);
    c->has_temporal = false;
    // everything keyed by the previous graph: hub-row ids of the exchange,
    // the adaptive scales, the census rates
    c->hot_ex_key.clear();
    c->ex_scale_key.clear();
    c->own_lo = 0;
    c->own_hi = -1;
    c->census = false;
    c->census_ok = false;
    c->census_key.clear();
    c->census_rate[0].clear();
    c->census_rate[1].clear();
    dfree(c->d_census[0]);
    dfree(c->d_census[1]);
    blocks_release(c);
    if (c->device < 0) {
        c->has_graph = true;
        return SMORE_OK;
    }
    if ((rc = set_device(c))) return rc;
    HostGraph& g = *c->g;
    c->packed_ok = false;
    c->part_n = 1;          // a new graph: the global source law
    c->part_i = 0;
    c->part_vtab.clear();
    c->part_bounds.clear();
    dfree(c->d_vt32);
    dfree(c->d_ct16);
    if ((rc = upload(c, c->d_offsets, g.offsets.data(), g.offsets.size()))) return rc;
    if ((rc = upload(c, c->d_targets, g.targets.data(), g.targets.size()))) return rc;
    if ((rc = upload(c, c->d_vtab, g.vtab.data(), g.vtab.size()))) return rc;
    if ((rc = upload(c, c->d_ntab, g.ntab.data(), g.ntab.size(), true))) return rc;
    if ((rc = upload(c, c->d_ctab, g.ctab.data(), g.ctab.size()))) return rc;
    // fastSigmoid table, 1001 entries (src/proNet.cpp:52-60; the reference
    // sizes it 1000 and writes 1001 -- the build keeps all 1001)
    std::vector<float> sig(1001);
    for (int i = 0; i != 1000 + 1; i++) {
        double x = i * 2.0 * 8.0 / 1000 - 8.0;
        sig[i] = (float)(1.0 / (1.0 + std::exp(-x)));
    }
    if ((rc = upload(c, c->d_sig, sig.data(), sig.size()))) return rc;
    c->has_graph = true;
    return SMORE_OK;
}

inline DevGraph dev_graph(const smore_ctx* c) {
    DevGraph d;
    d.offsets = c->d_offsets;
    d.targets = c->d_targets;
    d.vtab = reinterpret_cast<const uint2*>(c->d_vtab);
    d.ntab = reinterpret_cast<const uint2*>(c->d_ntab);
    d.ctab = reinterpret_cast<const uint2*>(c->d_ctab);
    d.vt32 = c->packed_ok ? c->d_vt32 : nullptr;
    d.ct16 = c->packed_ok ? c->d_ct16 : nullptr;
    d.V = (uint32_t)c->g->V;
    return d;
}

// capi.cpp helpers shared with blocks.cpp
void part_bounds(const std::vector<double>& ps, int n, std::vector<int64_t>& bound);
int hot_maps(smore_ctx* c, int model, int K, int64_t M, bool walk, double w_scale, double c_scale);
int launch_grid(smore_ctx* c, const EdgeArgs& a);
int sh_flush_max(bool walk);
int sh_slot_interval(double Mp, int cap, bool walk);
void sh_slot_levels(int64_t M, int cap, bool walk, const std::pair<double, int32_t>* r, int64_t n, int (&lvl)[8]);
double hot_tau_default(bool walk);
double hot_tau_cell_default(bool walk);
double cell_rate_default(bool walk);
double sh_stale_max(bool walk);
inline float* table_ptr(smore_ctx* c, int which) {
    if (which < 0 || which > 1) return nullptr;
    return c->d_table[which];
}

}  // namespace smore_host
