// edge_kernels.h -- the fused sampled-SGD kernels for gfx950 (templates).
//
// One "sample group" of G lanes owns one edge sample at a time.  Lane l of
// the group owns the row elements l, l+G, l+2G, ... (M of them), so every
// row load / store / atomic of a wave instruction covers a contiguous
// 4G-byte segment of each row it touches (d=64: G=16, four 64-B segments per
// wave instruction; d=128: G=32, two 128-B segments).
//
// Per sample:
//   Philox draws (each lane computes one 4-word block, broadcast by shuffle)
//   -> alias draws: source, target (CSR + per-vertex context table), K
//      negatives (all independent 8-B / 4-B loads)
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

enum { MODE_STORE = 0, MODE_ATOMIC = 1 };

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

// ------------------------------------------------------------------ edge kernel
// LINE-2 (W,C), LINE-1 (W,W), MF (W,W, Opt_SGD): the model is a wave-uniform
// runtime switch; the scatter MODE is compile-time.
template <int G, int M, int KMAX, int MODE>
__global__ void __launch_bounds__(256) edge_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    for (int i = threadIdx.x; i < 1001; i += blockDim.x) s_sig[i] = a.sig[i];
    __syncthreads();

    constexpr int NSLOT = 4 + 2 * KMAX;
    const int lane = threadIdx.x & (G - 1);
    uint64_t group = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;
    if (a.mode == 2) {               // serial: one group, samples in order
        if (group != 0) return;
        ngroups = 1;
    }
    const bool shared = a.model != 0;
    const bool mf = a.model == 2;
    const int dpad = a.dpad;
    bool ev[M];                      // element lane + G*m exists
#pragma unroll
    for (int m = 0; m < M; ++m) ev[m] = lane + G * m < dpad;
    float* const Tw = a.W;
    float* const Tc = shared ? a.W : a.C;
    const uint64_t base = mf ? 0 : 1;   // LINE counts from 1, MF from 0

    for (uint64_t t = group; t < a.count; t += ngroups) {
        const uint64_t s = a.begin + t;
        SampleWords<G, NSLOT> wd;
        wd.draw(a.seed, 0, s, lane);

        const int32_t v = source_sample(a.g, wd.w[0], wd.w[1]);
        const int32_t c = target_sample(a.g, v, wd.w[2], wd.w[3]);
        if (c < 0) {
            if (lane == 0) atomicAdd(a.skipped, 1ull);
            continue;
        }
        int32_t id[KMAX + 1];
        id[0] = c;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            id[j + 1] = (j < a.K) ? negative_sample(a.g, wd.w[4 + 2 * j], wd.w[5 + 2 * j]) : -1;
        const int32_t vs = shared ? v : -2;   // id of W_v inside the context table

        // ---- gather
        float wv[M], rows[KMAX + 1][M];
        {
            const float* wp = Tw + (int64_t)v * dpad + lane;
#pragma unroll
            for (int m = 0; m < M; ++m) wv[m] = ev[m] ? wp[m * G] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            const float* cp = Tc + (int64_t)(id[k] < 0 ? 0 : id[k]) * dpad + lane;
#pragma unroll
            for (int m = 0; m < M; ++m) rows[k][m] = (ev[m] && id[k] >= 0) ? cp[m * G] : 0.0f;
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
        float orig[MODE == MODE_ATOMIC ? KMAX + 1 : 1][M], wv0[M];
        if constexpr (MODE == MODE_ATOMIC) {
#pragma unroll
            for (int m = 0; m < M; ++m) {
                wv0[m] = wv[m];
#pragma unroll
                for (int k = 0; k <= KMAX; ++k) orig[k][m] = rows[k][m];
            }
        }

        const float alpha = alpha_at(s + base, a.alpha0, a.total);
        float e[M];
#pragma unroll
        for (int m = 0; m < M; ++m) e[m] = 0.0f;

        // ---- K+1 sequential Opt_SigmoidSGD / Opt_SGD steps
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            if (k <= a.K) {
                float p = 0.0f;
#pragma unroll
                for (int m = 0; m < M; ++m) p = __builtin_fmaf(wv[m], rows[k][m], p);
                const float f = group_sum<G>(p);
                if (mf) {
                    const float gg = (k == 0 ? 1.0f : -1.0f) - f;
#pragma unroll
                    for (int m = 0; m < M; ++m) {
                        const float ce = rows[k][m], we = wv[m];
                        const float t1 = gg * ce - a.reg * we;
                        const float t2 = gg * we - a.reg * ce;
                        e[m] = __builtin_fmaf(alpha, t1, e[m]);
                        rows[k][m] = __builtin_fmaf(alpha, t2, ce);
                    }
                } else {
                    const float gg = ((k == 0 ? 1.0f : 0.0f) - fast_sigmoid(f, s_sig)) * alpha;
#pragma unroll
                    for (int m = 0; m < M; ++m) {
                        const float ce = rows[k][m];
                        e[m] = __builtin_fmaf(gg, ce, e[m]);
                        rows[k][m] = __builtin_fmaf(gg, wv[m], ce);
                    }
                }
                // in-place semantics: every other reference to this row sees it
#pragma unroll
                for (int k2 = 0; k2 <= KMAX; ++k2)
                    if (k2 != k && id[k2] == id[k]) {
#pragma unroll
                        for (int m = 0; m < M; ++m) rows[k2][m] = rows[k][m];
                    }
                if (id[k] == vs) {
#pragma unroll
                    for (int m = 0; m < M; ++m) wv[m] = rows[k][m];
                }
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m) wv[m] = wv[m] + e[m];

        // ---- scatter
        {
            float* wq = Tw + (int64_t)v * dpad + lane;
#pragma unroll
            for (int m = 0; m < M; ++m) {
                if (!ev[m]) continue;
                if constexpr (MODE == MODE_ATOMIC) unsafeAtomicAdd(wq + m * G, shared ? wv[m] - wv0[m] : e[m]);
                else wq[m * G] = wv[m];
            }
        }
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            bool last = id[k] >= 0 && id[k] != vs;
#pragma unroll
            for (int k2 = k + 1; k2 <= KMAX; ++k2) last = last && (id[k2] != id[k]);
            if (last) {
                float* cq = Tc + (int64_t)id[k] * dpad + lane;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    if (!ev[m]) continue;
                    if constexpr (MODE == MODE_ATOMIC) unsafeAtomicAdd(cq + m * G, rows[k][m] - orig[k][m]);
                    else cq[m * G] = rows[k][m];
                }
            }
        }
    }
}

// ------------------------------------------------------------------ BPR kernel
// UpdateBPRPair (src/proNet.cpp:1406-1455), one shared table, 5 rounds.
// Slots: 0 = u, 1 = i, 2+n = j_n.
template <int G, int M, int MODE>
__global__ void __launch_bounds__(256) bpr_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    for (int i = threadIdx.x; i < 1001; i += blockDim.x) s_sig[i] = a.sig[i];
    __syncthreads();

    constexpr int NS = 7;
    const int lane = threadIdx.x & (G - 1);
    uint64_t group = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;
    if (a.mode == 2) {
        if (group != 0) return;
        ngroups = 1;
    }
    const int dpad = a.dpad;
    bool ev[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ev[m] = lane + G * m < dpad;
    float* const T = a.W;

    for (uint64_t t = group; t < a.count; t += ngroups) {
        const uint64_t s = a.begin + t;
        SampleWords<G, 14> wd;
        wd.draw(a.seed, 0, s, lane);
        int32_t id[NS];
        id[0] = source_sample(a.g, wd.w[0], wd.w[1]);
        id[1] = target_sample(a.g, id[0], wd.w[2], wd.w[3]);
        if (id[1] < 0) {
            if (lane == 0) atomicAdd(a.skipped, 1ull);
            continue;
        }
#pragma unroll
        for (int n = 0; n < 5; ++n) id[2 + n] = negative_sample(a.g, wd.w[4 + 2 * n], wd.w[5 + 2 * n]);

        float row[NS][M];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const float* p = T + (int64_t)id[k] * dpad + lane;
#pragma unroll
            for (int m = 0; m < M; ++m) row[k][m] = ev[m] ? p[m * G] : 0.0f;
        }
#pragma unroll
        for (int k = 1; k < NS; ++k)
#pragma unroll
            for (int k2 = 0; k2 < k; ++k2)
                if (id[k2] == id[k]) {
#pragma unroll
                    for (int m = 0; m < M; ++m) row[k][m] = row[k2][m];
                }
        float orig[MODE == MODE_ATOMIC ? NS : 1][M];
        if constexpr (MODE == MODE_ATOMIC) {
#pragma unroll
            for (int k = 0; k < NS; ++k)
#pragma unroll
                for (int m = 0; m < M; ++m) orig[k][m] = row[k][m];
        }
        const float alpha = alpha_at(s, a.alpha0, a.total);
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
                float* q = T + (int64_t)id[k] * dpad + lane;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    if (!ev[m]) continue;
                    if constexpr (MODE == MODE_ATOMIC) unsafeAtomicAdd(q + m * G, row[k][m] - orig[k][m]);
                    else q[m * G] = row[k][m];
                }
            }
        }
    }
}

// ---------------------------------------------------------------- dispatch
// (G, M) pairs for dpad in [4, 512]: G = min(64, pow2ceil(dpad/4)),
// M = ceil(dpad / G).
#define SMORE_FOR_EACH_GM(X) \
    X(1, 4) X(2, 4) X(4, 3) X(4, 4) X(8, 3) X(8, 4) X(16, 3) X(16, 4) X(32, 3) X(32, 4) \
    X(64, 3) X(64, 4) X(64, 5) X(64, 6) X(64, 7) X(64, 8)

}  // namespace smore
