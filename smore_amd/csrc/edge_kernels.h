// edge_kernels.h -- the fused sampled-SGD kernels for gfx950 (templates).
//
// One "sample group" of G lanes owns one edge sample at a time.  Lane l of
// the group owns the row's 16-B chunks l, l+G, ... (M elements in M/4 chunks,
// device_common.h elem_off), so every row load / store of a wave instruction
// is a dwordx4 per lane covering 16G contiguous bytes of each row it touches
// (d=64: G=16, four whole 256-B rows per wave instruction; d=128: G=32, two
// whole 512-B rows).
//
// Per sample:
//   [edge models: the draws come pre-drawn from train_draw.hip, one 32-B
//    record per sample, prefetched one round ahead; BPR / DeepWalk draw here:
//    Philox words (each lane computes one 4-word block, broadcast by shuffle)
//    -> alias draws: source, target, K negatives]
//   -> gather of the K+2 rows into registers
//   -> K+1 sequential Opt_SigmoidSGD / Opt_SGD steps (fmaf chain + pairwise
//      lane tree; fastSigmoid table in LDS)
//   -> scatter: float atomic add of each row's delta (MODE 1), or plain
//      stores of the new rows (MODE 0: lock-free read-modify-write).
// Rows stay in registers for the whole sample; a row id repeated inside one
// sample is resolved in registers, so the in-place semantics of
// src/proNet.cpp:1312-1330 / 1784-1809 hold exactly.
#pragma once
#include "train_kernels.h"

namespace smore {

enum { MODE_STORE = 0, MODE_ATOMIC = 1, MODE_HYBRID = 3 };


// minimum waves per SIMD the register allocator must allow, per scatter mode
// (0 = compiler default); overridable at build time for tuning.
#ifndef SMORE_WAVES_STORE
#define SMORE_WAVES_STORE 0
#endif
#ifndef SMORE_WAVES_ATOMIC
#define SMORE_WAVES_ATOMIC 0
#endif
#ifndef SMORE_WAVES_HYBRID
#define SMORE_WAVES_HYBRID 3
#endif
#ifndef SMORE_WAVES_BPR
#define SMORE_WAVES_BPR 0
#endif
constexpr int waves_of(int mode, int shared = 0) {
    return shared == 2 ? SMORE_WAVES_BPR   // BPR: 7 rows and their originals
                       : mode == MODE_STORE ? SMORE_WAVES_STORE : mode == MODE_ATOMIC ? SMORE_WAVES_ATOMIC : SMORE_WAVES_HYBRID;
}

// hybrid scatter: a row is added atomically iff its id tag says hot
template <int MODE>
__device__ __forceinline__ bool scatter_atomic(int32_t tagged) {
    if constexpr (MODE == MODE_ATOMIC) return true;
    else if constexpr (MODE == MODE_HYBRID) return tagged >= 0 && tag_hot(tagged);
    else return false;
}

// Block-local write-combining of the super-hot context rows (hybrid scatter):
// their deltas accumulate in LDS and a block adds them to HBM every sh_flush
// rounds (one 256-B atomic wave-instruction per row) instead of every sample
// adding to the same few HBM lines.  The block reads such a row as HBM value +
// its own pending delta.
struct ShState {
    const int2* hash;      // LDS, SH_HASH entries {id, slot}
    float* pend;           // LDS, [n][dpad]
    int n;
};

__device__ __forceinline__ int sh_lookup(const int2* h, int32_t id) {
    uint32_t p = ((uint32_t)id * 2654435761u) >> 24;
    for (int i = 0; i < SH_HASH; ++i) {
        const int2 e = h[(p + (uint32_t)i) & (SH_HASH - 1)];
        if (e.x == id) return e.y;
        if (e.x < 0) return -1;
    }
    return -1;
}

// The 4+2K (or 14 for BPR) words of a sample: lane l of the group computes
// Philox block (l % NBLK) of unit s; word j is broadcast from lane j/4.
template <int G, int NSLOT>
struct SampleWords {
    static constexpr int NBLK = (NSLOT + 3) / 4;
    uint32_t w[NSLOT];
    __device__ __forceinline__ void draw(uint64_t seed, uint32_t stream, uint64_t unit, int lane) {
        if constexpr (G >= NBLK) {
            const uint4 b = philox_block(seed, stream, unit, (uint32_t)(lane % NBLK));
#pragma unroll
            for (int j = 0; j < NSLOT; ++j) w[j] = __shfl(comp(b, j & 3), j >> 2, G);
        } else {
#pragma unroll
            for (int k = 0; k < NBLK; ++k) {
                const uint4 b = philox_block(seed, stream, unit, (uint32_t)k);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (4 * k + c < NSLOT) w[4 * k + c] = comp(b, c);
            }
        }
    }
};

// NW consecutive words of one unit starting at an arbitrary slot0 (the
// DeepWalk draw sequence): lane l computes block slot0/4 + l % NB, word j is
// broadcast from the lane holding slot0 + j.
template <int G, int NW>
struct SlotWords {
    static constexpr int NB = (NW + 3) / 4 + 1;
    uint32_t w[NW];
    __device__ __forceinline__ void draw(uint64_t seed, uint32_t stream, uint64_t unit, uint32_t slot0,
                                         int lane) {
        const uint32_t b0 = slot0 >> 2, off = slot0 & 3;
        if constexpr (G >= NB) {
            const uint4 b = philox_block(seed, stream, unit, b0 + (uint32_t)(lane % NB));
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const uint32_t x = off + (uint32_t)j;
                w[j] = __shfl(comp(b, (int)(x & 3)), (int)(x >> 2), G);
            }
        } else {
            uint4 b[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) b[k] = philox_block(seed, stream, unit, b0 + (uint32_t)k);
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const uint32_t x = off + (uint32_t)j;
                uint32_t r = 0;
#pragma unroll
                for (int k = 0; k < NB; ++k)
                    if ((x >> 2) == (uint32_t)k) r = comp(b[k], (int)(x & 3));
                w[j] = r;
            }
        }
    }
};

// ------------------------------------------------------------------ update core
// One UpdatePair / UpdateFactorizedPair on rows W_v and the K+1 context refs
// id[0] (positive) and id[1..K] (negatives), done by the G lanes of a group.
// Ids are untagged; hotw / hot[k] select the atomic scatter (MODE_HYBRID).
//
// Scatter bookkeeping without a copy of the original rows: after reference k
// is processed its new value is propagated to the LATER references with the
// same id (the in-place semantics), then rows[k] is turned into this step's
// delta if the row is scattered by atomic add (every occurrence adds its own
// delta), or kept as the value if it is stored (only the last occurrence of an
// id stores, and it holds the final value).  A reference to W_v's own row in
// a shared table is never scattered itself: W_v's scatter carries it.
template <int G, int M, int KMAX>
__device__ __forceinline__ void gather_rows(const EdgeArgs& a, int lane, const bool (&ev)[M], int32_t v,
                                            const int32_t (&id)[KMAX + 1], bool shared, float (&wv)[M],
                                            float (&rows)[KMAX + 1][M]) {
    const int dpad = a.dpad;
    const float* const Tc = shared ? a.W : a.C;
    ld_row<G, M>(wv, a.W + (int64_t)(v < 0 ? 0 : v) * dpad, lane, ev, v >= 0);
#pragma unroll
    for (int k = 0; k <= KMAX; ++k)
        ld_row<G, M>(rows[k], Tc + (int64_t)(id[k] < 0 ? 0 : id[k]) * dpad, lane, ev, id[k] >= 0);
}

// the K+1 context rows only (W_v held by the caller)
template <int G, int M, int KMAX>
__device__ __forceinline__ void gather_ctx_rows(const EdgeArgs& a, int lane, const bool (&ev)[M],
                                                const int32_t (&id)[KMAX + 1], float (&rows)[KMAX + 1][M]) {
#pragma unroll
    for (int k = 0; k <= KMAX; ++k)
        ld_row<G, M>(rows[k], a.C + (int64_t)(id[k] < 0 ? 0 : id[k]) * a.dpad, lane, ev, id[k] >= 0);
}

// sgd_update on rows already gathered by gather_rows (wv, rows are consumed).
// SHARED: -1 = runtime (a.model), 0 = two tables (LINE-2), 1 = one table.
// WOUT false (two tables only): W_v is not scattered; wv returns its new value
// (the caller keeps it in registers over a run of samples with the same v).
// REG (two tables only): reg_rt selects Opt_SigmoidRegSGD (src/proNet.cpp:
// 1332-1351, HPE's UpdateCommunity) instead of Opt_SigmoidSGD at run time:
// g = label - sig(f); e = fmaf(alpha, g*c - reg*w, e); c = fmaf(alpha, g*w - reg*c, c).
// nsc: the negatives' step weight (EdgeArgs::neg_scale; 1 everywhere but the
// block schedule's cells): negative k uses alpha * nsc, which is alpha bit for
// bit when nsc == 1.
template <int G, int M, int KMAX, int MODE, int SHARED = -1, bool WOUT = true, bool REG = false>
__device__ __forceinline__ void sgd_update_rows(const EdgeArgs& a, const float* s_sig, int lane,
                                                const bool (&ev)[M], int32_t v, const int32_t (&id)[KMAX + 1],
                                                bool hotw, const bool (&hot)[KMAX + 1], float alpha, bool shared_rt,
                                                bool mf_rt, const ShState& sh, float (&wv)[M],
                                                float (&rows)[KMAX + 1][M], bool reg_rt = false, float nsc = 1.0f) {
    constexpr bool DELTA = MODE == MODE_ATOMIC || MODE == MODE_HYBRID;
    const bool shared = SHARED < 0 ? shared_rt : SHARED == 1;
    const bool mf = SHARED == 0 ? false : mf_rt;
    const bool regr = (REG && SHARED == 0) ? reg_rt : false;
    const int dpad = a.dpad;
    float* const Tw = a.W;
    float* const Tc = shared ? a.W : a.C;
    const int32_t vs = shared ? v : -2;   // id of W_v inside the context table

    // super-hot rows: add this block's pending deltas
    int slot[KMAX + 1];
    int slotw = -1;
#pragma unroll
    for (int k = 0; k <= KMAX; ++k) slot[k] = -1;
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) {
#pragma unroll
            for (int k = 0; k <= KMAX; ++k) {
                if (id[k] >= 0 && hot[k]) slot[k] = sh_lookup(sh.hash, id[k]);
                if (slot[k] >= 0) {
                    const float* pp = sh.pend + slot[k] * dpad;
#pragma unroll
                    for (int m = 0; m < M; ++m)
                        if (ev[m]) rows[k][m] += pp[elem_off<G>(lane, m)];
                }
            }
            if (hotw) {
                // W rows of two-table models are combined too (key v | SH_WKEY)
                slotw = sh_lookup(sh.hash, shared ? v : (v | SH_WKEY));
                if (slotw >= 0) {
                    const float* pp = sh.pend + slotw * dpad;
#pragma unroll
                    for (int m = 0; m < M; ++m)
                        if (ev[m]) wv[m] += pp[elem_off<G>(lane, m)];
                }
            }
        }
    }
    // canonicalise repeated ids onto their first occurrence
#pragma unroll
    for (int k = 1; k <= KMAX; ++k)
#pragma unroll
        for (int k2 = 0; k2 < k; ++k2)
            if (id[k2] == id[k]) {
#pragma unroll
                for (int m = 0; m < M; ++m) rows[k][m] = rows[k2][m];
            }
#pragma unroll
    for (int k = 0; k <= KMAX; ++k)
        if (id[k] == vs) {
#pragma unroll
            for (int m = 0; m < M; ++m) rows[k][m] = wv[m];
        }
    float wv0[(DELTA && SHARED != 0) ? M : 1];
    if constexpr (DELTA && SHARED != 0) {
#pragma unroll
        for (int m = 0; m < M; ++m) wv0[m] = wv[m];
    }
    float e[M];
#pragma unroll
    for (int m = 0; m < M; ++m) e[m] = 0.0f;

    // ---- K+1 sequential Opt_SigmoidSGD / Opt_SGD steps
#pragma unroll
    for (int k = 0; k <= KMAX; ++k) {
        if (id[k] >= 0) {
            float p = 0.0f;
#pragma unroll
            for (int m = 0; m < M; ++m) p = __builtin_fmaf(wv[m], rows[k][m], p);
            const float f = group_sum<G>(p);
            float nk[M];
            if (mf) {
                const float gg = (k == 0 ? 1.0f : -1.0f) - f;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const float ce = rows[k][m], we = wv[m];
                    const float t1 = gg * ce - a.reg * we;
                    const float t2 = gg * we - a.reg * ce;
                    e[m] = __builtin_fmaf(alpha, t1, e[m]);
                    nk[m] = __builtin_fmaf(alpha, t2, ce);
                }
            } else if (regr) {
                const float gg = (k == 0 ? 1.0f : 0.0f) - fast_sigmoid(f, s_sig);
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const float ce = rows[k][m], we = wv[m];
                    const float t1 = gg * ce - a.reg * we;
                    const float t2 = gg * we - a.reg * ce;
                    e[m] = __builtin_fmaf(alpha, t1, e[m]);
                    nk[m] = __builtin_fmaf(alpha, t2, ce);
                }
            } else {
                const float gg = ((k == 0 ? 1.0f : 0.0f) - fast_sigmoid(f, s_sig)) * (k == 0 ? alpha : alpha * nsc);
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const float ce = rows[k][m];
                    e[m] = __builtin_fmaf(gg, ce, e[m]);
                    nk[m] = __builtin_fmaf(gg, wv[m], ce);
                }
            }
            // in-place semantics: later references to this row see it
#pragma unroll
            for (int k2 = k + 1; k2 <= KMAX; ++k2)
                if (id[k2] == id[k]) {
#pragma unroll
                    for (int m = 0; m < M; ++m) rows[k2][m] = nk[m];
                }
            if (id[k] == vs) {
#pragma unroll
                for (int m = 0; m < M; ++m) wv[m] = nk[m];
            }
#pragma unroll
            for (int m = 0; m < M; ++m) rows[k][m] = (DELTA && hot[k]) ? nk[m] - rows[k][m] : nk[m];
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) wv[m] = wv[m] + e[m];

    // ---- scatter
    static_assert(WOUT || SHARED == 0, "W_v stays in registers only with two tables");
    if constexpr (WOUT) {
        float* wq = Tw + (int64_t)v * dpad;
        if (DELTA && hotw) {
            float d[M];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                d[m] = e[m];
                if constexpr (SHARED != 0)
                    if (shared) d[m] = wv[m] - wv0[m];
            }
            if (MODE == MODE_HYBRID && slotw >= 0) {
#pragma unroll
                for (int m = 0; m < M; ++m)
                    if (ev[m]) atomicAdd(sh.pend + slotw * dpad + elem_off<G>(lane, m), d[m]);
            } else {
                atomic_row<G, M>(wq, d, lane, dpad);
            }
        } else {
            st_row<G, M>(wq, wv, lane, ev);
        }
    }
#pragma unroll
    for (int k = 0; k <= KMAX; ++k) {
        if (id[k] < 0 || id[k] == vs) continue;
        if (DELTA && hot[k]) {
            if (MODE == MODE_HYBRID && slot[k] >= 0) {
                float* pq = sh.pend + slot[k] * dpad;
#pragma unroll
                for (int m = 0; m < M; ++m)
                    if (ev[m]) atomicAdd(pq + elem_off<G>(lane, m), rows[k][m]);
            } else {
                atomic_row<G, M>(Tc + (int64_t)id[k] * dpad, rows[k], lane, dpad);
            }
        } else {
            bool last = true;
#pragma unroll
            for (int k2 = k + 1; k2 <= KMAX; ++k2) last = last && (id[k2] != id[k]);
            if (last) st_row<G, M>(Tc + (int64_t)id[k] * dpad, rows[k], lane, ev);
        }
    }
}

// gather + update (callers without row prefetch)
template <int G, int M, int KMAX, int MODE>
__device__ __forceinline__ void sgd_update(const EdgeArgs& a, const float* s_sig, int lane, const bool (&ev)[M],
                                           int32_t v, const int32_t (&id)[KMAX + 1], bool hotw,
                                           const bool (&hot)[KMAX + 1], float alpha, bool shared, bool mf,
                                           const ShState& sh) {
    float wv[M], rows[KMAX + 1][M];
    gather_rows<G, M, KMAX>(a, lane, ev, v, id, shared, wv, rows);
    sgd_update_rows<G, M, KMAX, MODE>(a, s_sig, lane, ev, v, id, hotw, hot, alpha, shared, mf, sh, wv, rows);
}

// ------------------------------------------------------------------ BPR update
// UpdateBPRPair (src/proNet.cpp:1406-1455), one shared table, 5 rounds, on
// rows gathered by gather_rows: wv = W[u], rows[0] = W[i], rows[1+n] = W[j_n].
// Hybrid: rows in the block's write-combined set (sh, the hottest hot rows)
// are read as HBM value + this block's pending delta and add their delta in
// LDS; the block drains them every sh_flush rounds (sh_drain).
template <int G, int M, int KMAX, int MODE>
__device__ __forceinline__ void bpr_update_rows(const EdgeArgs& a, const float* s_sig, int lane,
                                                const bool (&ev)[M], int32_t u, const int32_t (&idc)[KMAX + 1],
                                                bool hotu, const bool (&hotc)[KMAX + 1], float alpha,
                                                float (&wv)[M], float (&rows)[KMAX + 1][M], const ShState& sh) {
    static_assert(KMAX == 5, "BPR: 5 rounds");
    constexpr int NS = 7;
    const int dpad = a.dpad;
    float* const T = a.W;
    int32_t id[NS];
    bool hot[NS];
    float row[NS][M];
    id[0] = u;
    hot[0] = hotu;
#pragma unroll
    for (int m = 0; m < M; ++m) row[0][m] = wv[m];
#pragma unroll
    for (int k = 0; k <= KMAX; ++k) {
        id[1 + k] = idc[k];
        hot[1 + k] = hotc[k];
#pragma unroll
        for (int m = 0; m < M; ++m) row[1 + k][m] = rows[k][m];
    }
    int slot[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) slot[k] = -1;
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) {
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                if (hot[k]) slot[k] = sh_lookup(sh.hash, id[k]);
                if (slot[k] >= 0) {
                    const float* pp = sh.pend + slot[k] * dpad;
#pragma unroll
                    for (int m = 0; m < M; ++m)
                        if (ev[m]) row[k][m] += pp[elem_off<G>(lane, m)];
                }
            }
        }
    }
#pragma unroll
    for (int k = 1; k < NS; ++k)
#pragma unroll
        for (int k2 = 0; k2 < k; ++k2)
            if (id[k2] == id[k]) {
#pragma unroll
                for (int m = 0; m < M; ++m) row[k][m] = row[k2][m];
            }
    constexpr bool DELTA = MODE == MODE_ATOMIC || MODE == MODE_HYBRID;
    float orig[DELTA ? NS : 1][M];
    if constexpr (DELTA) {
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
            for (int m = 0; m < M; ++m) orig[k][m] = row[k][m];
    }
    const float r1 = alpha * 0.0025f, r2 = alpha * 0.025f;
    float ve[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ve[m] = 0.0f;

#define SMORE_PROPAGATE(K_)                                                              \
_Pragma("unroll") for (int k2 = 0; k2 < NS; ++k2) if (k2 != (K_) && id[k2] == id[(K_)]) { \
    _Pragma("unroll") for (int m = 0; m < M; ++m) row[k2][m] = row[(K_)][m];                \
}

#pragma unroll
    for (int n = 0; n < 5; ++n) {
        const int J = 2 + n;
        float x[M], ce[M];
        float p = 0.0f;
#pragma unroll
        for (int m = 0; m < M; ++m) {
            x[m] = row[1][m] - row[J][m];
            p = __builtin_fmaf(row[0][m], x[m], p);
        }
        const float f = group_sum<G>(p);
        const float gg = fast_sigmoid(-f, s_sig) * alpha;
#pragma unroll
        for (int m = 0; m < M; ++m) {
            ve[m] = __builtin_fmaf(gg, x[m], ve[m]);
            ce[m] = gg * row[0][m];
        }
#pragma unroll
        for (int m = 0; m < M; ++m) row[1][m] = __builtin_fmaf(-r1, row[1][m], row[1][m]);
        SMORE_PROPAGATE(1)
#pragma unroll
        for (int m = 0; m < M; ++m) row[J][m] = __builtin_fmaf(-r1, row[J][m], row[J][m]);
        SMORE_PROPAGATE(J)
#pragma unroll
        for (int m = 0; m < M; ++m) row[1][m] = row[1][m] + ce[m];
        SMORE_PROPAGATE(1)
#pragma unroll
        for (int m = 0; m < M; ++m) row[J][m] = row[J][m] - ce[m];
        SMORE_PROPAGATE(J)
    }
#pragma unroll
    for (int m = 0; m < M; ++m) row[0][m] = __builtin_fmaf(-r2, row[0][m], row[0][m]) + ve[m];
    SMORE_PROPAGATE(0)
#undef SMORE_PROPAGATE

#pragma unroll
    for (int k = 0; k < NS; ++k) {
        bool last = true;
#pragma unroll
        for (int k2 = k + 1; k2 < NS; ++k2) last = last && (id[k2] != id[k]);
        if (last) {
            float* q = T + (int64_t)id[k] * dpad;
            bool atom = false;
            if constexpr (DELTA) atom = hot[k];
            if (atom) {
                float dd[M];
#pragma unroll
                for (int m = 0; m < M; ++m) dd[m] = row[k][m] - orig[DELTA ? k : 0][m];
                int sk = -1;
#pragma unroll
                for (int k2 = 0; k2 < NS; ++k2)
                    if (id[k2] == id[k] && slot[k2] >= 0) sk = slot[k2];
                if (MODE == MODE_HYBRID && sk >= 0) {
                    float* pq = sh.pend + sk * dpad;
#pragma unroll
                    for (int m = 0; m < M; ++m)
                        if (ev[m]) atomicAdd(pq + elem_off<G>(lane, m), dd[m]);
                } else {
                    atomic_row<G, M>(q, dd, lane, dpad);
                }
            } else {
                st_row<G, M>(q, row[k], lane, ev);
            }
        }
    }
}

// ------------------------------------------------------------------ block setup
// fastSigmoid table into LDS and, for the hybrid scatter, the write-combining
// state (hash, slot ids, zeroed pending deltas) in the dynamic LDS; ends with
// a workgroup barrier.
template <int MODE>
__device__ __forceinline__ ShState block_setup(const EdgeArgs& a, float* s_sig, float* s_dyn, int32_t*& sh_ids) {
    for (int i = threadIdx.x; i < 1001; i += blockDim.x) s_sig[i] = a.sig[i];
    ShState sh{nullptr, nullptr, 0};
    sh_ids = nullptr;
    if constexpr (MODE == MODE_HYBRID) {
        if (a.sh_rows > 0) {
            int2* h = reinterpret_cast<int2*>(s_dyn);
            sh_ids = reinterpret_cast<int32_t*>(h + SH_HASH);
            float* pend = reinterpret_cast<float*>(sh_ids + a.sh_rows);
            for (int i = threadIdx.x; i < SH_HASH; i += blockDim.x) h[i] = a.sh_hash[i];
            for (int i = threadIdx.x; i < a.sh_rows; i += blockDim.x) sh_ids[i] = a.sh_ids[i];
            for (int i = threadIdx.x; i < a.sh_rows * a.dpad; i += blockDim.x) pend[i] = 0.0f;
            sh = ShState{h, pend, a.sh_rows};
        }
    }
    __syncthreads();
    return sh;
}

// Adds pending write-combined deltas to HBM (one row per wave-instruction).
// Wave w of the block drains its share of the pending rows with an LDS
// exchange (read-and-zero in one atomic), so there is no workgroup barrier:
// an LDS add racing with the drain lands either in this drain or in the
// wave's next one, never lost.  A slot's key is a Tc row id, or (two-table
// models) a Tw row id | SH_WKEY.
__device__ __forceinline__ void sh_drain_n(const ShState& sh, const int32_t* sh_ids, float* Tw, float* Tc, int dpad,
                                           int slots) {
    const int nwaves = blockDim.x / 64, wave = threadIdx.x / 64;
    const int n = slots * dpad;
    const int per = (n + nwaves - 1) / nwaves;
    const int lo = wave * per, hi = n < lo + per ? n : lo + per;
    for (int i = lo + (threadIdx.x & 63); i < hi; i += 64) {
        const float x = atomicExch(&sh.pend[i], 0.0f);
        if (x != 0.0f) {
            const int s = i / dpad, e = i - s * dpad;
            const int32_t key = sh_ids[s];
            float* const T = (key & SH_WKEY) ? Tw : Tc;
            unsafeAtomicAdd(T + (int64_t)(key & ~SH_WKEY) * dpad + e, x);
        }
    }
}

__device__ __forceinline__ void sh_drain(const ShState& sh, const int32_t* sh_ids, float* Tw, float* Tc, int dpad) {
    sh_drain_n(sh, sh_ids, Tw, Tc, dpad, sh.n);
}

// the drain schedule of a hybrid launch, called once per round: every slot
// every sh_flush rounds, and at round t the slots whose own interval 2^j
// divides t -- a prefix of sh_lvl[j] slots (sorted by rate) -- in between
__device__ __forceinline__ void sh_tick(const EdgeArgs& a, const ShState& sh, const int32_t* sh_ids, float* Tw,
                                        float* Tc, uint32_t& round) {
    if (sh.n <= 0) return;
    if (++round == (uint32_t)a.sh_flush) {
        sh_drain(sh, sh_ids, Tw, Tc, a.dpad);
        round = 0;
        return;
    }
    int ns = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((round & ((1u << j) - 1u)) == 0u) ns = a.sh_lvl[j];
    if (ns > 0) sh_drain_n(sh, sh_ids, Tw, Tc, a.dpad, ns < sh.n ? ns : sh.n);
}

// sh_drain of the W-key slots only (the combined hub W rows of a two-table
// model, drained on their own shorter interval: EdgeArgs::sh_flush_w)
__device__ __forceinline__ void sh_drain_w(const ShState& sh, const int32_t* sh_ids, float* Tw, int dpad) {
    const int nwaves = blockDim.x / 64, wave = threadIdx.x / 64;
    const int n = sh.n * dpad;
    const int per = (n + nwaves - 1) / nwaves;
    const int lo = wave * per, hi = n < lo + per ? n : lo + per;
    for (int i = lo + (threadIdx.x & 63); i < hi; i += 64) {
        const int s = i / dpad;
        const int32_t key = sh_ids[s];
        if (!(key & SH_WKEY)) continue;
        const float x = atomicExch(&sh.pend[i], 0.0f);
        if (x != 0.0f) unsafeAtomicAdd(Tw + (int64_t)(key & ~SH_WKEY) * dpad + (i - s * dpad), x);
    }
}

// the launch's negative-gradient weight (EdgeArgs::neg_scale / neg_lo / neg_hi)
__device__ __forceinline__ float neg_scale_of(const EdgeArgs& a, uint64_t count) {
    if (a.neg_lo && a.neg_hi) {
        const uint64_t tot = *a.neg_hi - *a.neg_lo;
        return count > 0 && tot > 0 && a.neg_scale > 0.0f
                   ? (float)((double)a.neg_scale * (double)tot / (double)count) : 1.0f;
    }
    return a.neg_scale > 0.0f ? a.neg_scale : 1.0f;
}

// ------------------------------------------------------------------ edge kernel
// LINE-2 (W,C; SHARED 0), LINE-1 / MF (W,W; SHARED 1, Opt_SGD for MF at run
// time) and BPR (W,W; SHARED 2, UpdateBPRPair); the scatter MODE is
// compile-time.
template <int G, int M, int KMAX, int MODE, int SHARED>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(waves_of(MODE, SHARED))))
edge_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    extern __shared__ float s_dyn[];   // hybrid: int2 hash[SH_HASH], int ids[n], float pend[n][dpad]
    int32_t* sh_ids = nullptr;
    const ShState sh = block_setup<MODE>(a, s_sig, s_dyn, sh_ids);

    const int lane = threadIdx.x & (G - 1);
    // records of this launch: [0, count) of a.rec, or a block bucket [*rec_base, *count_dev)
    uint64_t rb = a.rec_base ? *a.rec_base : 0;
    uint64_t count = (a.count_dev ? *a.count_dev : a.count) - rb;
    const float nsc = neg_scale_of(a, count);            // the whole bucket's weight
    if (a.part_n > 1) {                                  // one part of the bucket
        const uint64_t lo = count * a.part_q / a.part_n, hi = count * (a.part_q + 1) / a.part_n;
        rb += lo;
        count = hi - lo;
    }
    const int32_t* const recs = a.rec + rb * (uint64_t)rec_width(KMAX);
    const uint64_t gpb = blockDim.x / G;                 // groups per block
    uint64_t r0 = (uint64_t)blockIdx.x * gpb;            // block-uniform round base
    const uint64_t gib = threadIdx.x / G;
    if (a.mode == 2) {               // serial: one group, samples in order
        if (blockIdx.x != 0 || gib != 0) return;
    }
    const bool shared = SHARED >= 1;  // LINE-1 / MF / BPR: one table (host dispatches on a.model)
    const bool mf = SHARED == 1 && a.model == 2;
    bool ev[M];                      // register m's element exists
    row_valid<G, M>(ev, lane, a.dpad);
    const uint64_t base = (mf || SHARED == 2) ? 0 : 1;   // LINE counts from 1, MF and BPR from 0
    float* const Tc = a.C;

    // pending super-hot deltas -> HBM (sh_drain)
    auto drain = [&]() { sh_drain(sh, sh_ids, a.W, Tc, a.dpad); };
    auto flush = [&]() {   // end of the kernel: every wave is done adding
        __syncthreads();
        drain();
    };

    uint32_t round = 0;
    // the update rule on gathered rows
    auto update_rows = [&](int32_t v, const int32_t (&id)[KMAX + 1], bool hotw, const bool (&hot)[KMAX + 1],
                           float alpha, float (&wv)[M], float (&rows)[KMAX + 1][M], bool reg) {
        if constexpr (SHARED == 2) {
            if constexpr (KMAX == 5) bpr_update_rows<G, M, KMAX, MODE>(a, s_sig, lane, ev, v, id, hotw, hot, alpha, wv, rows, sh);
        } else {
            sgd_update_rows<G, M, KMAX, MODE, SHARED, true, true>(a, s_sig, lane, ev, v, id, hotw, hot, alpha, shared,
                                                                  mf, sh, wv, rows, reg, nsc);
        }
    };
    // the update of one sample, ids tagged as drawn (c < 0: source without out-edges)
    auto process = [&](float alpha, int32_t tv, int32_t c, const int32_t (&negs)[KMAX]) {
        const int32_t v = untag(tv);
        int32_t id[KMAX + 1];
        bool hot[KMAX + 1];
        id[0] = c;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) id[j + 1] = (j < a.K) ? negs[j] : -1;
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            hot[k] = scatter_atomic<MODE>(id[k]);
            id[k] = id[k] < 0 ? -1 : untag(id[k]);
        }
        float wv[M], rows[KMAX + 1][M];
        gather_rows<G, M, KMAX>(a, lane, ev, v, id, shared, wv, rows);
        // word 0 bit 31: HPE community record (Opt_SigmoidRegSGD)
        update_rows(v, id, scatter_atomic<MODE>(tv), hot, alpha, wv, rows, tv < 0);
    };
    auto maybe_flush = [&]() {
        if constexpr (MODE == MODE_HYBRID) {
            if (a.sh_flush_w > 0) {   // W-key slots on their own interval (SMORE_SH_WROWS)
                if (sh.n > 0 && ++round == (uint32_t)a.sh_flush) {
                    drain();
                    round = 0;
                } else if (sh.n > 0 && round % (uint32_t)a.sh_flush_w == 0) {
                    sh_drain_w(sh, sh_ids, a.W, a.dpad);
                }
            } else {
                sh_tick(a, sh, sh_ids, a.W, Tc, round);
            }
        }
    };

    // learning rate of record t: from the global sample index (LINE / MF / BPR),
    // or carried in the record's word 2 + KMAX (DeepWalk pairs, per walk)
    auto rec_alpha = [&](uint64_t t, const i32x4* r) -> float {
        if (a.alpha_rec) return __int_as_float(r[(2 + KMAX) / 4][(2 + KMAX) % 4]);
        return alpha_at(a.begin + t + base, a.alpha0, a.total);
    };
    if (a.mode == 2) {
        // serial: records in order, gather after the previous sample's scatter
        constexpr int RW = rec_width(KMAX);
        for (; r0 < count; ++r0) {
            const i32x4* p = reinterpret_cast<const i32x4*>(recs + r0 * RW);
            i32x4 r[RW / 4];
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) r[q] = p[q];
            if (r[0][1] >= 0) {   // c < 0: counted by the draw kernel
                int32_t negs[KMAX];
#pragma unroll
                for (int j = 0; j < KMAX; ++j) negs[j] = r[(j + 2) / 4][(j + 2) % 4];
                process(rec_alpha(r0, r), r[0][0], r[0][1], negs);
            }
        }
    } else {
        // Hogwild modes: pre-drawn records (train_draw.hip), and the rows of
        // the group's next sample are gathered BEFORE this sample's scatter:
        // vector-memory ops retire in issue order (one vmcnt for loads, stores
        // and atomics), so a gather issued after a scatter would wait for the
        // scatter's acknowledgements too.  The next sample may thus read a row
        // this sample is about to write -- the staleness every other resident
        // group already has (Hogwild); the serial mode above keeps strict order.
        constexpr int RW = rec_width(KMAX);
        // a decoded sample keeps its TAGGED words (v, c, negatives; -1 = none)
        // across the pipeline; ids and hot flags are split off where used,
        // which keeps two samples' state in fewer registers
        struct Ids {
            int32_t w[KMAX + 2];
            bool live;
            float alpha;
            __device__ __forceinline__ int32_t v() const { return live ? untag(w[0]) : -1; }
            __device__ __forceinline__ void ids(int32_t (&id)[KMAX + 1]) const {
#pragma unroll
                for (int k = 0; k <= KMAX; ++k) id[k] = (!live || w[k + 1] < 0) ? -1 : untag(w[k + 1]);
            }
            __device__ __forceinline__ void hots(bool (&hot)[KMAX + 1]) const {
#pragma unroll
                for (int k = 0; k <= KMAX; ++k) hot[k] = scatter_atomic<MODE>(w[k + 1]);
            }
        };
        auto decode = [&](uint64_t t, uint64_t lim, const i32x4 (&r)[RW / 4], Ids& x) {
            x.live = t < lim && r[0][1] >= 0;   // c < 0: counted by the draw kernel
            x.alpha = rec_alpha(t, r);
            x.w[0] = r[0][0];
#pragma unroll
            for (int k = 0; k <= KMAX; ++k)
                x.w[k + 1] = (k == 0) ? r[0][1] : (k - 1 < a.K ? r[(k + 1) / 4][(k + 1) % 4] : -1);
        };
        auto load_rec = [&](uint64_t t, uint64_t lim, i32x4 (&r)[RW / 4]) {
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) r[q] = i32x4{-1, -1, -1, -1};
            if (t < lim) {
                const i32x4* p = reinterpret_cast<const i32x4*>(recs + t * RW);
#pragma unroll
                for (int q = 0; q < RW / 4; ++q) r[q] = __builtin_nontemporal_load(p + q);
            }
        };
        i32x4 rr[RW / 4];
        Ids xa, xb;
        float wva[M], rowsa[KMAX + 1][M], wvb[M], rowsb[KMAX + 1][M];
        // Work is handed out in chunks of CH_ROUNDS rounds (CH_ROUNDS * gpb
        // consecutive samples per block) from a per-launch counter: a block
        // that starts late (a collective's kernel holding CU slots, uneven
        // XCD clocks) takes fewer chunks instead of stretching the launch by
        // a whole fixed share.  Within a chunk the block's groups take samples
        // c0 + gib, c0 + gib + gpb, ... with the row prefetch above.
        // Chunks shrink for a short launch (a cell of the 2-D block schedule:
        // ~8M samples over ~768 blocks is ~5 chunks of CH_ROUNDS per block,
        // so the last chunks leave most blocks idle): about 16 chunks per
        // block, at least 8 rounds each, at most CH_ROUNDS (a one-GPU launch
        // of 2^27 samples keeps CH_ROUNDS).
        __shared__ uint64_t s_next;
        uint64_t ch_rounds = count / ((uint64_t)gridDim.x * gpb * 16u);
        ch_rounds = ch_rounds < 8 ? 8 : ch_rounds > CH_ROUNDS ? CH_ROUNDS : ch_rounds;
        if (a.pair_slice && !a.alpha_rec) ch_rounds = a.pair_slice;   // fixed (SMORE_EDGE_CHUNK, experiments)
        const uint64_t span = ch_rounds * gpb;
        auto grab = [&]() -> uint64_t {
            __syncthreads();   // every wave has read the previous s_next
            if (threadIdx.x == 0) s_next = atomicAdd(a.work, 1ull) * span;
            __syncthreads();
            return s_next;
        };
        for (uint64_t c0 = grab(); c0 < count; c0 = grab()) {
            const uint64_t lim = c0 + span < count ? c0 + span : count;
            if constexpr (SHARED == 2) {
                // BPR: no row prefetch -- gathering the next sample's 7 rows
                // before this sample's scatter was measured no faster at C3
                // (639 vs 637 M samples/s, 2 waves/SIMD either way, 221 vs 184
                // VGPRs); the next record is still loaded one round ahead
                uint64_t t = c0 + gib;
                load_rec(t, lim, rr);
                for (uint64_t r = c0; r < lim; r += gpb) {
                    t = r + gib;
                    decode(t, lim, rr, xa);
                    load_rec(t + gpb, lim, rr);
                    if (xa.live) {
                        int32_t id[KMAX + 1];
                        bool hot[KMAX + 1];
                        xa.ids(id);
                        xa.hots(hot);
                        gather_rows<G, M, KMAX>(a, lane, ev, xa.v(), id, shared, wva, rowsa);
                        if constexpr (KMAX == 5)
                            bpr_update_rows<G, M, KMAX, MODE>(a, s_sig, lane, ev, xa.v(), id,
                                                              scatter_atomic<MODE>(xa.w[0]), hot, xa.alpha, wva, rowsa,
                                                              sh);
                    }
                    maybe_flush();
                }
                continue;
            }
            uint64_t t = c0 + gib;
            load_rec(t, lim, rr);
            decode(t, lim, rr, xa);
            {
                int32_t id[KMAX + 1];
                xa.ids(id);
                gather_rows<G, M, KMAX>(a, lane, ev, xa.v(), id, shared, wva, rowsa);
            }
            load_rec(t + gpb, lim, rr);
            for (uint64_t r = c0; r < lim; r += gpb) {
                t = r + gib;
                decode(t + gpb, lim, rr, xb);
                load_rec(t + 2 * gpb, lim, rr);
                {
                    int32_t id[KMAX + 1];
                    xb.ids(id);
                    gather_rows<G, M, KMAX>(a, lane, ev, xb.v(), id, shared, wvb, rowsb);
                }
                if (xa.live) {
                    if constexpr (SHARED != 2) {
                        int32_t id[KMAX + 1];
                        bool hot[KMAX + 1];
                        xa.ids(id);
                        xa.hots(hot);
                        sgd_update_rows<G, M, KMAX, MODE, SHARED>(a, s_sig, lane, ev, xa.v(), id,
                                                                 scatter_atomic<MODE>(xa.w[0]), hot, xa.alpha, shared,
                                                                 mf, sh, wva, rowsa, false, nsc);
                    }
                }
                xa = xb;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    wva[m] = wvb[m];
#pragma unroll
                    for (int k = 0; k <= KMAX; ++k) rowsa[k][m] = rowsb[k][m];
                }
                maybe_flush();
            }
        }
    }
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) flush();
    }
}

// ------------------------------------------------------------------ pair kernel
// DeepWalk skip-gram pair records (train_pairs.hip: {walk[i], walk[j], K
// negatives, .., alpha bits at word 2 + KMAX}, walk-major in the reference's
// pair order) in the Hogwild modes; the serial mode runs them through
// edge_train_kernel.  A walk's pairs are consecutive and share rows (walk[i]
// is the W row of up to 2*window pairs in a row), so they are not spread over
// concurrent groups: each group takes a contiguous slice of CH_ROUNDS records
// and runs it in order (gather after the previous scatter), keeps W_v in
// registers while v repeats and adds W_v's accumulated delta atomically when v
// changes -- no W update is lost, and W moves once per run instead of once per
// pair.  Context rows scatter as the MODE says (the tables are uncached
// device memory, so a plain store is seen by every XCD: capi alloc_tables).
template <int G, int M, int KMAX, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(waves_of(MODE))))
pair_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    extern __shared__ float s_dyn[];
    int32_t* sh_ids = nullptr;
    const ShState sh = block_setup<MODE>(a, s_sig, s_dyn, sh_ids);
    const int lane = threadIdx.x & (G - 1);
    constexpr int RW = rec_width(KMAX);
    uint64_t rb = a.rec_base ? *a.rec_base : 0;   // a block bucket: [*rec_base, *count_dev)
    uint64_t count = (a.count_dev ? *a.count_dev : a.count) - rb;
    const float nsc = neg_scale_of(a, count);      // the whole bucket's weight
    if (a.part_n > 1) {                            // one part of the bucket
        const uint64_t lo = count * a.part_q / a.part_n, hi = count * (a.part_q + 1) / a.part_n;
        rb += lo;
        count = hi - lo;
    }
    const int32_t* const recs = a.rec + rb * (uint64_t)RW;
    const uint64_t gpb = blockDim.x / G, gib = threadIdx.x / G;
    bool ev[M];
    row_valid<G, M>(ev, lane, a.dpad);
    uint32_t round = 0;
    __shared__ uint64_t s_next;
    // records per group slice: CH_ROUNDS, or for a launch with fewer than
    // CH_ROUNDS records per resident group (a cell of the 2-D block schedule:
    // ~360k records at 8 GPUs) an even share, so every group works -- at
    // CH_ROUNDS a 360k-record cell ran on 352 of 768 blocks, 128 records deep
    uint64_t sl = a.pair_slice ? (uint64_t)a.pair_slice : CH_ROUNDS;
    if (!a.pair_slice) {
        const uint64_t groups = (uint64_t)gridDim.x * gpb;
        if (count < groups * CH_ROUNDS) sl = count > groups ? (count + groups - 1) / groups : 1;
    }
    const uint64_t span = sl * gpb;
    for (;;) {
        __syncthreads();   // every wave has read the previous s_next
        if (threadIdx.x == 0) s_next = atomicAdd(a.work, 1ull) * span;
        __syncthreads();
        const uint64_t c0 = s_next;
        if (c0 >= count) break;
        const uint64_t lim = c0 + span < count ? c0 + span : count;
        const uint64_t s0 = c0 + gib * sl;
        const uint64_t s1 = s0 + sl < lim ? s0 + sl : lim;
        int32_t cv = -1;
        int slotw = -1;    // the run's W row's write-combined slot (EdgeArgs::w_comb)
        bool cvh = true;   // the run's W row is hot-tagged (or the flush is atomic anyway)
        float wv[M], wv0[M], rows[KMAX + 1][M];
#pragma unroll
        for (int m = 0; m < M; ++m) wv[m] = wv0[m] = 0.0f;
        i32x4 r[RW / 4];
        auto load_rec = [&](uint64_t t) {
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) r[q] = i32x4{-1, -1, -1, -1};
            if (t < s1) {
                const i32x4* p = reinterpret_cast<const i32x4*>(recs + t * RW);
#pragma unroll
                for (int q = 0; q < RW / 4; ++q) r[q] = __builtin_nontemporal_load(p + q);
            }
        };
        auto flush_w = [&]() {
            if (cv < 0) return;
            if constexpr (MODE == MODE_HYBRID) {
                if (slotw >= 0) {   // a combined W row: the run's delta into the block's pending row
                    float* pp = sh.pend + slotw * a.dpad;
#pragma unroll
                    for (int m = 0; m < M; ++m)
                        if (ev[m]) atomicAdd(pp + elem_off<G>(lane, m), wv[m] - wv0[m]);
                    return;
                }
            }
            if (MODE == MODE_HYBRID && !cvh) {   // a cold W row: plain store (EdgeArgs::w_plain)
                st_row<G, M>(a.W + (int64_t)cv * a.dpad, wv, lane, ev);
                return;
            }
            float d[M];
#pragma unroll
            for (int m = 0; m < M; ++m) d[m] = wv[m] - wv0[m];
            atomic_row<G, M>(a.W + (int64_t)cv * a.dpad, d, lane, a.dpad);
        };
        load_rec(s0);
        for (uint64_t t = s0; t < s1; ++t) {
            // decode this record, then load the next one behind it
            const int32_t tv = r[0][0], c = r[0][1];
            const float alpha = __int_as_float(r[(2 + KMAX) / 4][(2 + KMAX) % 4]);
            int32_t id[KMAX + 1];
            bool hot[KMAX + 1];
#pragma unroll
            for (int k = 0; k <= KMAX; ++k) {
                const int32_t w = (k == 0) ? c : (k - 1 < a.K ? r[(k + 1) / 4][(k + 1) % 4] : -1);
                hot[k] = scatter_atomic<MODE>(w);
                id[k] = w < 0 ? -1 : untag(w);
            }
            load_rec(t + 1);
            if (c < 0) continue;
            const int32_t v = untag(tv);
            if (v != cv) {
                flush_w();
                cv = v;
                cvh = !a.w_plain || scatter_atomic<MODE>(tv);
                ld_row<G, M>(wv, a.W + (int64_t)cv * a.dpad, lane, ev);
                if constexpr (MODE == MODE_HYBRID) {
                    slotw = a.w_comb && sh.n > 0 ? sh_lookup(sh.hash, cv | SH_WKEY) : -1;
                    if (slotw >= 0) {   // HBM value + the block's pending delta
                        const float* pp = sh.pend + slotw * a.dpad;
#pragma unroll
                        for (int m = 0; m < M; ++m)
                            if (ev[m]) wv[m] += pp[elem_off<G>(lane, m)];
                    }
                }
#pragma unroll
                for (int m = 0; m < M; ++m) wv0[m] = wv[m];
            }
            gather_ctx_rows<G, M, KMAX>(a, lane, ev, id, rows);
            // word 0 bit 31: HPE community record (Opt_SigmoidRegSGD)
            sgd_update_rows<G, M, KMAX, MODE, 0, false, true>(a, s_sig, lane, ev, v, id, false, hot, alpha, false,
                                                              false, sh, wv, rows, tv < 0, nsc);
            if constexpr (MODE == MODE_HYBRID) sh_tick(a, sh, sh_ids, a.W, a.C, round);
        }
        flush_w();
    }
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) {
            __syncthreads();
            sh_drain(sh, sh_ids, a.W, a.C, a.dpad);
        }
    }
}

// ---------------------------------------------------------------- dispatch
// (G, M) pairs for dpad in [4, 512]: G = min(64, pow2ceil(dpad / 4)) lanes,
// M = 4 * ceil(dpad / 4 / G) registers (train_kernels.h lanes_of / regs_of;
// oracle orc_lane_width).
#define SMORE_FOR_EACH_GM(X) \
    X(1, 4) X(2, 4) X(4, 4) X(8, 4) X(16, 4) X(32, 4) X(64, 4) X(64, 8)

}  // namespace smore
