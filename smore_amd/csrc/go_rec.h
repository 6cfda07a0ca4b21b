// go_rec.h -- the Go-rule edge updates on pre-drawn records: the fast path of
// Go LINE (order 2 and 1), BPR and HPE.
//
// Records come from go_draw_kernel (train_go.hip: Go's index-first alias draws
// and CDF target draw), one per sample, tagged like the C++ records, so the
// update runs on edge_train_kernel's machinery: chunked work from a per-launch
// counter, the next sample's rows gathered before this sample's scatter, and
// the hybrid scatter (hot rows by atomic add, the hottest context rows
// write-combined per workgroup in LDS).  The arithmetic is the Go rule of
// pkg/pronet/optimizer.go as train_go.hip's serial kernels state it (fp32,
// no fused multiply-adds in the updates; the oracle's orc_go_*_f32):
//   model 0  UpdatePair (optimizer.go:21-58): negatives equal to the positive
//            skipped (not redrawn), negatives updated immediately, the
//            positive context's and W_v's gradients applied at the end;
//   model 1  updateFirstOrder (internal/models/line/line.go:153-200) on W;
//   model 3  UpdateBPRPair (optimizer.go:87-117): W users, C items, lambda.
#pragma once
#include "edge_kernels.h"

namespace smore {

// pending write-combined deltas of the super-hot rows onto gathered rows
template <int G, int M, int KMAX, int MODE>
__device__ __forceinline__ void go_sh_pending(const ShState& sh, int dpad, int lane, const bool (&ev)[M],
                                              const int32_t (&id)[KMAX + 1], const bool (&hot)[KMAX + 1],
                                              int (&slot)[KMAX + 1], float (&rows)[KMAX + 1][M]) {
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
        }
    }
}

// one row's update: value `val` (plain store) or per-occurrence delta `d`
// (atomic add, or the LDS pending sum of a write-combined row)
template <int G, int M, int MODE>
__device__ __forceinline__ void go_put(float* row, const ShState& sh, int slot, int dpad, int lane,
                                       const bool (&ev)[M], bool hot, const float (&val)[M], const float (&d)[M]) {
    constexpr bool DELTA = MODE == MODE_ATOMIC || MODE == MODE_HYBRID;
    if (DELTA && hot) {
        if (MODE == MODE_HYBRID && slot >= 0) {
#pragma unroll
            for (int m = 0; m < M; ++m)
                if (ev[m]) atomicAdd(sh.pend + slot * dpad + elem_off<G>(lane, m), d[m]);
        } else {
            atomic_row<G, M>(row, d, lane, dpad);
        }
    } else {
        st_row<G, M>(row, val, lane, ev);
    }
}

template <int G, int M>
__device__ __forceinline__ float go_dot(const float (&a)[M], const float (&b)[M]) {
    float p = 0.0f;
#pragma unroll
    for (int m = 0; m < M; ++m) p = __builtin_fmaf(a[m], b[m], p);
    return group_sum<G>(p);
}

// The Go rules on gathered rows: wv = W[v]; rows[0] = the positive's row
// (C[c], or W[t] for LINE-1, or C[i] for BPR); rows[1 + j] = negative j's row
// (ids of skipped negatives are -1).  Ids untagged; hot flags from the tags.
template <int G, int M, int KMAX, int MODE>
__device__ __forceinline__ void go_update_rows(const EdgeArgs& a, const float* s_sig, int lane, const bool (&ev)[M],
                                               int model, int32_t v, const int32_t (&id)[KMAX + 1], bool hotw,
                                               const bool (&hot)[KMAX + 1], float alpha, const ShState& sh,
                                               float (&wv)[M], float (&rows)[KMAX + 1][M]) {
    constexpr bool DELTA = MODE == MODE_ATOMIC || MODE == MODE_HYBRID;
    const int dpad = a.dpad;
    const bool one = model == 1;                  // LINE-1: every row is a W row
    float* const Tc = one ? a.W : a.C;
    int slot[KMAX + 1];
    go_sh_pending<G, M, KMAX, MODE>(sh, dpad, lane, ev, id, hot, slot, rows);
    int slotw = -1;
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0 && hotw) {
            slotw = sh_lookup(sh.hash, one ? v : (v | SH_WKEY));
            if (slotw >= 0) {
#pragma unroll
                for (int m = 0; m < M; ++m)
                    if (ev[m]) wv[m] += sh.pend[slotw * dpad + elem_off<G>(lane, m)];
            }
        }
    }
    if (model == 3) {
        // UpdateBPRPair: u = v, i = id[0], j = id[1]
        const int32_t i = id[0], j = id[1];
        if (i == j) {
#pragma unroll
            for (int m = 0; m < M; ++m) rows[1][m] = rows[0][m];
        }
        const float pos = go_dot<G, M>(wv, rows[0]), neg = go_dot<G, M>(wv, rows[1]);
        const float gc = alpha * fast_sigmoid(neg - pos, s_sig);
        const float la = a.reg * alpha;
        float nu[M], ni[M], nj[M], du[M], di[M], dj[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const float ci = rows[0][m], cj = rows[1][m], wu = wv[m];
            const float vgr = gc * (ci - cj);
            const float pg = gc * wu;
            const float ngr = -gc * wu;
            nu[m] = wu + (vgr - la * wu);
            ni[m] = ci + (pg - la * ci);
            const float base = i == j ? ni[m] : cj;
            nj[m] = base + (ngr - la * base);
            du[m] = nu[m] - wu;
            di[m] = ni[m] - ci;
            dj[m] = nj[m] - base;
        }
        go_put<G, M, MODE>(a.W + (int64_t)v * dpad, sh, slotw, dpad, lane, ev, hotw, nu, du);
        if (i == j) {
            float dd[M];
#pragma unroll
            for (int m = 0; m < M; ++m) dd[m] = nj[m] - rows[0][m];
            go_put<G, M, MODE>(a.C + (int64_t)i * dpad, sh, slot[0], dpad, lane, ev, hot[0], nj, dd);
        } else {
            go_put<G, M, MODE>(a.C + (int64_t)i * dpad, sh, slot[0], dpad, lane, ev, hot[0], ni, di);
            go_put<G, M, MODE>(a.C + (int64_t)j * dpad, sh, slot[1], dpad, lane, ev, hot[1], nj, dj);
        }
        return;
    }
    // repeated negatives start from their first occurrence
#pragma unroll
    for (int k = 2; k <= KMAX; ++k)
#pragma unroll
        for (int k2 = 1; k2 < k; ++k2)
            if (id[k2] >= 0 && id[k2] == id[k]) {
#pragma unroll
                for (int m = 0; m < M; ++m) rows[k][m] = rows[k2][m];
            }
    float vg[M], cg[M];
    {
        const float grad = alpha * (1.0f - fast_sigmoid(go_dot<G, M>(wv, rows[0]), s_sig));
#pragma unroll
        for (int m = 0; m < M; ++m) {
            vg[m] = grad * rows[0][m];
            cg[m] = grad * wv[m];
        }
    }
#pragma unroll
    for (int k = 1; k <= KMAX; ++k) {
        if (id[k] < 0) continue;
        const float gr = alpha * (0.0f - fast_sigmoid(go_dot<G, M>(wv, rows[k]), s_sig));
        float nk[M], dk[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            dk[m] = gr * wv[m];
            vg[m] = vg[m] + gr * rows[k][m];
            nk[m] = rows[k][m] + dk[m];
        }
        bool last = true;
#pragma unroll
        for (int k2 = k + 1; k2 <= KMAX; ++k2)
            if (id[k2] == id[k]) {
                last = false;
#pragma unroll
                for (int m = 0; m < M; ++m) rows[k2][m] = nk[m];
            }
        if ((DELTA && hot[k]) || last)
            go_put<G, M, MODE>(Tc + (int64_t)id[k] * dpad, sh, slot[k], dpad, lane, ev, hot[k], nk, dk);
    }
    // the positive's row and W_v last
    float nw[M];
#pragma unroll
    for (int m = 0; m < M; ++m) nw[m] = wv[m] + vg[m];
    if (one && id[0] == v) {
        // updateFirstOrder with s == t: one row, both gradients
        float nt[M], d2[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            nt[m] = nw[m] + cg[m];
            d2[m] = vg[m] + cg[m];
        }
        go_put<G, M, MODE>(a.W + (int64_t)v * dpad, sh, slotw, dpad, lane, ev, hotw, nt, d2);
        return;
    }
    float nc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) nc[m] = rows[0][m] + cg[m];
    if (one) {
        go_put<G, M, MODE>(a.W + (int64_t)v * dpad, sh, slotw, dpad, lane, ev, hotw, nw, vg);
        go_put<G, M, MODE>(a.W + (int64_t)id[0] * dpad, sh, slot[0], dpad, lane, ev, hot[0], nc, cg);
    } else {
        go_put<G, M, MODE>(a.C + (int64_t)id[0] * dpad, sh, slot[0], dpad, lane, ev, hot[0], nc, cg);
        go_put<G, M, MODE>(a.W + (int64_t)v * dpad, sh, slotw, dpad, lane, ev, hotw, nw, vg);
    }
}

// Go records (go_draw_kernel) -> Go updates.  a.model: 0 LINE-2, 1 LINE-1,
// 3 BPR (K = 1); a.mode 2 = serial (one group, records in order).
template <int G, int M, int KMAX, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(waves_of(MODE))))
go_rec_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    extern __shared__ float s_dyn[];
    int32_t* sh_ids = nullptr;
    const ShState sh = block_setup<MODE>(a, s_sig, s_dyn, sh_ids);
    const int lane = threadIdx.x & (G - 1);
    const uint64_t count = a.count;
    const uint64_t gpb = blockDim.x / G, gib = threadIdx.x / G;
    bool ev[M];
    row_valid<G, M>(ev, lane, a.dpad);
    constexpr int RW = rec_width(KMAX);
    const int model = a.model;
    const bool one = model == 1;
    float* const Tc = one ? a.W : a.C;
    uint32_t round = 0;

    // record t -> (tagged v, ids, hot flags); skipped negatives -> -1
    struct Rec {
        int32_t w[KMAX + 2];
        bool live;
        __device__ __forceinline__ int32_t v() const { return live ? untag(w[0]) : -1; }
        __device__ __forceinline__ void ids(int model_, int32_t (&id)[KMAX + 1]) const {
            const int32_t v0 = untag(w[0]), c0 = untag(w[1]);
#pragma unroll
            for (int k = 0; k <= KMAX; ++k) {
                int32_t x = (!live || w[k + 1] < 0) ? -1 : untag(w[k + 1]);
                if (k > 0 && model_ != 3 && (x == c0 || (model_ == 1 && x == v0))) x = -1;
                id[k] = x;
            }
        }
        __device__ __forceinline__ void hots(bool (&hot)[KMAX + 1]) const {
#pragma unroll
            for (int k = 0; k <= KMAX; ++k) hot[k] = scatter_atomic<MODE>(w[k + 1]);
        }
    };
    auto load = [&](uint64_t t, uint64_t lim, Rec& x) {
        x.live = false;
#pragma unroll
        for (int k = 0; k < KMAX + 2; ++k) x.w[k] = -1;
        if (t < lim) {
            const i32x4* p = reinterpret_cast<const i32x4*>(a.rec + t * RW);
            i32x4 r[RW / 4];
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) r[q] = __builtin_nontemporal_load(p + q);
#pragma unroll
            for (int k = 0; k < KMAX + 2; ++k) x.w[k] = (k < 2 + a.K) ? r[k / 4][k % 4] : -1;
            x.live = x.w[1] >= 0;        // c < 0: counted by the draw kernel
        }
    };
    auto alpha_of = [&](uint64_t t) { return alpha_walk(a.begin + t, a.alpha0, a.total); };
    auto gather = [&](const Rec& x, float (&wv)[M], float (&rows)[KMAX + 1][M]) {
        int32_t id[KMAX + 1];
        x.ids(model, id);
        gather_rows<G, M, KMAX>(a, lane, ev, x.v(), id, one, wv, rows);
    };
    auto update = [&](const Rec& x, float alpha, float (&wv)[M], float (&rows)[KMAX + 1][M]) {
        int32_t id[KMAX + 1];
        bool hot[KMAX + 1];
        x.ids(model, id);
        x.hots(hot);
        go_update_rows<G, M, KMAX, MODE>(a, s_sig, lane, ev, model, x.v(), id, scatter_atomic<MODE>(x.w[0]), hot,
                                         alpha, sh, wv, rows);
    };
    auto maybe_flush = [&]() {
        if constexpr (MODE == MODE_HYBRID) {
            if (sh.n > 0 && ++round == (uint32_t)a.sh_flush) {
                sh_drain(sh, sh_ids, a.W, Tc, a.dpad);
                round = 0;
            } else if (sh.n > 0 && a.sh_flush_w > 0 && round % (uint32_t)a.sh_flush_w == 0) {
                sh_drain_w(sh, sh_ids, a.W, a.dpad);
            }
        }
    };
    float wva[M], rowsa[KMAX + 1][M], wvb[M], rowsb[KMAX + 1][M];
    if (a.mode == 2) {
        // serial: one group, records in order, each gathered after the
        // previous sample's scatter (the Go loop's order)
        if (blockIdx.x != 0 || gib != 0) return;
        for (uint64_t t = 0; t < count; ++t) {
            Rec x;
            load(t, count, x);
            if (!x.live) continue;
            gather(x, wva, rowsa);
            update(x, alpha_of(t), wva, rowsa);
        }
        return;
    }
    __shared__ uint64_t s_next;
    const uint64_t span = CH_ROUNDS * gpb;
    auto grab = [&]() -> uint64_t {
        __syncthreads();
        if (threadIdx.x == 0) s_next = atomicAdd(a.work, 1ull) * span;
        __syncthreads();
        return s_next;
    };
    for (uint64_t c0 = grab(); c0 < count; c0 = grab()) {
        const uint64_t lim = c0 + span < count ? c0 + span : count;
        uint64_t t = c0 + gib;
        Rec xa, xb;
        load(t, lim, xa);
        gather(xa, wva, rowsa);
        for (uint64_t r = c0; r < lim; r += gpb) {
            t = r + gib;
            load(t + gpb, lim, xb);
            gather(xb, wvb, rowsb);
            if (xa.live) update(xa, alpha_of(t), wva, rowsa);
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
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) {
            __syncthreads();
            sh_drain(sh, sh_ids, a.W, Tc, a.dpad);
        }
    }
}

// ------------------------------------------------------------------ Go walk pairs
// Go SkipGrams pair records (train_go.hip go_pair_emit_kernel: {walk[i],
// walk[j], negatives, .., alpha bits at word 2 + KMAX}, walk-major) -> Go
// UpdatePair (optimizer.go:21-58) per pair, for Go DeepWalk, node2vec,
// metapath2vec and CTDNE.  A walk position's pairs are consecutive and share
// W_v, which only they change (contexts and negatives are C rows): each group
// takes a contiguous slice of CH_ROUNDS records and keeps W_v in registers
// while v repeats, the Go loop's per-pair W_v += vg included, and puts the row
// back when v changes -- stored in the serial mode (the sequential value),
// otherwise the run's summed gradient added atomically (no W update lost).
// Context rows: atomic adds of each update's delta (MODE_ATOMIC), plain
// stores (MODE_STORE), or by the records' hot tags (MODE_HYBRID: bit 30 of a
// context / negative id, set by go_pair_emit_kernel from the C hot map; the
// hottest are write-combined in LDS as in edge_train_kernel).  The next
// record is loaded while this one updates.
// Serial (a.mode 2): one group, all records in order.
template <int G, int M, int KMAX, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(waves_of(MODE))))
go_pair_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    extern __shared__ float s_dyn[];   // hybrid: the write-combined hottest context rows
    int32_t* sh_ids = nullptr;
    const ShState sh = block_setup<MODE>(a, s_sig, s_dyn, sh_ids);
    constexpr bool DELTA = MODE == MODE_ATOMIC || MODE == MODE_HYBRID;
    const int lane = threadIdx.x & (G - 1);
    const uint64_t count = a.count_dev ? *a.count_dev : a.count;
    const uint64_t gpb = blockDim.x / G, gib = threadIdx.x / G;
    bool ev[M];
    row_valid<G, M>(ev, lane, a.dpad);
    constexpr int RW = rec_width(KMAX);
    const int dpad = a.dpad;
    const bool serial = a.mode == 2;
    uint32_t round = 0;
    auto slice = [&](uint64_t s0, uint64_t s1) {
        int32_t cv = -1;
        float wv[M], wsum[M];
        auto flush = [&]() {
            if (cv < 0) return;
            if (serial) st_row<G, M>(a.W + (int64_t)cv * dpad, wv, lane, ev);
            else atomic_row<G, M>(a.W + (int64_t)cv * dpad, wsum, lane, dpad);
        };
        i32x4 r[RW / 4];
        auto load_rec = [&](uint64_t t) {
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) r[q] = i32x4{-1, -1, -1, -1};
            if (t < s1) {
                const i32x4* p = reinterpret_cast<const i32x4*>(a.rec + t * RW);
#pragma unroll
                for (int q = 0; q < RW / 4; ++q) r[q] = __builtin_nontemporal_load(p + q);
            }
        };
        load_rec(s0);
        for (uint64_t t = s0; t < s1; ++t) {
            // decode this record, then load the next one behind it
            const int32_t v = r[0][0], c_t = r[0][1];
            const float alpha = __int_as_float(r[(2 + KMAX) / 4][(2 + KMAX) % 4]);
            const int32_t c = c_t < 0 ? -1 : untag(c_t);
            // the context's row and the negatives' (a negative equal to the
            // context is skipped, not redrawn; repeats start from the first)
            int32_t id[KMAX + 1];
            bool hot[KMAX + 1];
            id[0] = c;
            hot[0] = MODE == MODE_ATOMIC || (MODE == MODE_HYBRID && c_t >= 0 && tag_hot(c_t));
#pragma unroll
            for (int k = 1; k <= KMAX; ++k) {
                const int32_t x = k - 1 < a.K ? r[(k + 1) / 4][(k + 1) % 4] : -1;
                id[k] = (x < 0 || untag(x) == c) ? -1 : untag(x);
                hot[k] = MODE == MODE_ATOMIC || (MODE == MODE_HYBRID && x >= 0 && tag_hot(x));
            }
            load_rec(t + 1);
            if (c < 0) continue;
            if (v != cv) {
                flush();
                cv = v;
                ld_row<G, M>(wv, a.W + (int64_t)v * dpad, lane, ev);
#pragma unroll
                for (int m = 0; m < M; ++m) wsum[m] = 0.0f;
            }
            float rows[KMAX + 1][M];
#pragma unroll
            for (int k = 0; k <= KMAX; ++k)
                ld_row<G, M>(rows[k], a.C + (int64_t)(id[k] < 0 ? 0 : id[k]) * dpad, lane, ev, id[k] >= 0);
            int slot[KMAX + 1];
            go_sh_pending<G, M, KMAX, MODE>(sh, dpad, lane, ev, id, hot, slot, rows);
#pragma unroll
            for (int k = 2; k <= KMAX; ++k)
#pragma unroll
                for (int k2 = 1; k2 < k; ++k2)
                    if (id[k2] >= 0 && id[k2] == id[k]) {
#pragma unroll
                        for (int m = 0; m < M; ++m) rows[k][m] = rows[k2][m];
                    }
            float vg[M], cg[M];
            {
                const float grad = alpha * (1.0f - fast_sigmoid(go_dot<G, M>(wv, rows[0]), s_sig));
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    vg[m] = grad * rows[0][m];
                    cg[m] = grad * wv[m];
                }
            }
#pragma unroll
            for (int k = 1; k <= KMAX; ++k) {
                if (id[k] < 0) continue;
                const float gr = alpha * (0.0f - fast_sigmoid(go_dot<G, M>(wv, rows[k]), s_sig));
                float nk[M], dk[M];
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    dk[m] = gr * wv[m];
                    vg[m] = vg[m] + gr * rows[k][m];
                    nk[m] = rows[k][m] + dk[m];
                }
                bool last = true;
#pragma unroll
                for (int k2 = k + 1; k2 <= KMAX; ++k2)
                    if (id[k2] == id[k]) {
                        last = false;
#pragma unroll
                        for (int m = 0; m < M; ++m) rows[k2][m] = nk[m];
                    }
                if ((DELTA && hot[k]) || last)
                    go_put<G, M, MODE>(a.C + (int64_t)id[k] * dpad, sh, slot[k], dpad, lane, ev, hot[k], nk, dk);
            }
            {
                float nc[M];
#pragma unroll
                for (int m = 0; m < M; ++m) nc[m] = rows[0][m] + cg[m];
                go_put<G, M, MODE>(a.C + (int64_t)c * dpad, sh, slot[0], dpad, lane, ev, hot[0], nc, cg);
            }
#pragma unroll
            for (int m = 0; m < M; ++m) {
                wv[m] = wv[m] + vg[m];
                wsum[m] = wsum[m] + vg[m];
            }
            if constexpr (MODE == MODE_HYBRID) {
                if (sh.n > 0 && ++round == (uint32_t)a.sh_flush) {
                    sh_drain(sh, sh_ids, a.W, a.C, dpad);
                    round = 0;
                }
            }
        }
        flush();
    };
    if (serial) {
        if (blockIdx.x == 0 && gib == 0) slice(0, count);
        return;
    }
    __shared__ uint64_t s_next;
    const uint64_t sl = a.pair_slice ? (uint64_t)a.pair_slice : CH_ROUNDS;   // records per group slice
    const uint64_t span = sl * gpb;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) s_next = atomicAdd(a.work, 1ull) * span;
        __syncthreads();
        const uint64_t c0 = s_next;
        if (c0 >= count) break;
        const uint64_t lim = c0 + span < count ? c0 + span : count;
        const uint64_t s0 = c0 + gib * sl;
        slice(s0 < lim ? s0 : lim, s0 + sl < lim ? s0 + sl : lim);
    }
    if constexpr (MODE == MODE_HYBRID) {
        if (sh.n > 0) {
            __syncthreads();
            sh_drain(sh, sh_ids, a.W, a.C, dpad);
        }
    }
}

template <int KMAX, int MODE>
struct GoPairInst {
    static hipError_t launch(const EdgeArgs& a, int grid, hipStream_t st) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m)                                                                          \
    if (G == g && M == m) {                                                              \
        hipLaunchKernelGGL((go_pair_kernel<g, m, KMAX, MODE>), dim3(grid), dim3(256),              \
                           sh_lds_bytes(MODE == MODE_HYBRID ? a.sh_rows : 0, a.dpad), st, a);    \
        return hipGetLastError();                                                        \
    }
        SMORE_FOR_EACH_GM(X)
#undef X
        return hipErrorInvalidValue;
    }
    static const void* symbol(const EdgeArgs& a) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m) \
    if (G == g && M == m) return (const void*)go_pair_kernel<g, m, KMAX, MODE>;
        SMORE_FOR_EACH_GM(X)
#undef X
        return nullptr;
    }
};

template <int KMAX, int MODE>
struct GoRecInst {
    static hipError_t launch(const EdgeArgs& a, int grid, hipStream_t st) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
        const size_t lds = MODE == MODE_HYBRID ? sh_lds_bytes(a.sh_rows, a.dpad) : 0;
#define X(g, m)                                                                                  \
    if (G == g && M == m) {                                                                      \
        hipLaunchKernelGGL((go_rec_kernel<g, m, KMAX, MODE>), dim3(grid), dim3(256), lds, st, a); \
        return hipGetLastError();                                                                \
    }
        SMORE_FOR_EACH_GM(X)
#undef X
        return hipErrorInvalidValue;
    }
    static const void* symbol(const EdgeArgs& a) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m) \
    if (G == g && M == m) return (const void*)go_rec_kernel<g, m, KMAX, MODE>;
        SMORE_FOR_EACH_GM(X)
#undef X
        return nullptr;
    }
};

}  // namespace smore

// defines launch_go_rec_<name>(a, grid, st) and go_rec_symbol_<name>(a)
#define SMORE_GO_REC_INST(name, MODE)                                                           \
    namespace smore {                                                                           \
    hipError_t launch_go_rec_##name(const EdgeArgs& a, int grid, hipStream_t st) {              \
        return a.K <= 5 ? GoRecInst<5, MODE>::launch(a, grid, st) : GoRecInst<10, MODE>::launch(a, grid, st); \
    }                                                                                           \
    const void* go_rec_symbol_##name(const EdgeArgs& a) {                                       \
        return a.K <= 5 ? GoRecInst<5, MODE>::symbol(a) : GoRecInst<10, MODE>::symbol(a);        \
    }                                                                                           \
    }

// defines launch_go_pair_<name>(a, grid, st) and go_pair_symbol_<name>(a)
#define SMORE_GO_PAIR_INST(name, MODE)                                                          \
    namespace smore {                                                                           \
    hipError_t launch_go_pair_##name(const EdgeArgs& a, int grid, hipStream_t st) {             \
        return a.K <= 5 ? GoPairInst<5, MODE>::launch(a, grid, st) : GoPairInst<10, MODE>::launch(a, grid, st); \
    }                                                                                           \
    const void* go_pair_symbol_##name(const EdgeArgs& a) {                                      \
        return a.K <= 5 ? GoPairInst<5, MODE>::symbol(a) : GoPairInst<10, MODE>::symbol(a);      \
    }                                                                                           \
    }
