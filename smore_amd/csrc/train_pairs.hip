// train_pairs.hip -- DeepWalk / Walklets skip-gram pairs as sample records for
// the update kernel (edge_kernels.h: pair_train_kernel in the Hogwild modes,
// edge_train_kernel's serial mode), and APP's jumping-walk pairs.
//
// DeepWalk::Train's per-walk body after RandomWalk (src/model/DeepWalk.cpp:
// 133-139): SkipGrams with the random window shrink (src/proNet.cpp:769-809)
// and UpdatePairs -> UpdatePair per pair (src/proNet.cpp:2741-2753).  Per walk
// (one thread): the window draws (slots 2(L-1) + i, stream 1), then for each
// pair in the reference's order its K negatives (2K consecutive slots from
// 2(L-1) + L: index, then p), as the oracle restates them.  Two passes:
// count the pairs of each walk, exclusive-scan the counts, emit the records
//     {walk[i], walk[j], n_1 .. n_K, .., alpha bits at word 2 + KMAX}
// walk-major in pair order, so a serial update over them is the reference's
// order.  alpha is DeepWalk's per-walk rate (src/model/DeepWalk.cpp:141-147).
// Walklets (rule 1, src/model/Walklets.cpp:46-48): walks start at vid in
// order, pairs of ScaleSkipGrams (src/proNet.cpp:928-987), which draws
// nothing: the negatives start right after the walk's 2(L-1) draws.
#include <cstring>
#include <rocprim/device/device_scan.hpp>

#include "train_kernels.h"

namespace smore {

struct WalkWords {   // consecutive Philox words of one unit (walk models: stream 1)
    uint64_t seed, unit;
    uint32_t blk = 0xFFFFFFFFu;
    uint4 b;
    uint32_t stream = 1;
    __device__ uint32_t operator()(uint32_t slot) {
        if ((slot >> 2) != blk) {
            blk = slot >> 2;
            b = philox_block(seed, stream, unit, blk);
        }
        return comp(b, (int)(slot & 3));
    }
};

// Walklets' two ranges around position i (ScaleSkipGrams src/proNet.cpp:928-987,
// clamped exactly as written: a clamped range may hold i itself, which is skipped)
struct ScaleRanges {
    int l0, r0, l1, r1;
    __device__ ScaleRanges(int i, int L, int wmin, int wmax) {
        l0 = i - wmax < 0 ? 0 : i - wmax;
        r0 = i - wmin < 0 ? 0 : i - wmin;
        l1 = i + wmin >= L ? L - 1 : i + wmin;
        r1 = i + wmax >= L ? L - 1 : i + wmax;
    }
    __device__ static uint32_t span(int l, int r, int i) {
        return r < l ? 0u : (uint32_t)(r - l + 1) - ((i >= l && i <= r) ? 1u : 0u);
    }
};

// the walk partition's filter: is walk position i's center (W row) owned?
__device__ __forceinline__ bool center_owned(const WalkArgs& w, const int32_t* walk, int i) {
    const int32_t v = walk[i] & ID_MASK;
    return v >= w.own_lo && v < w.own_hi;
}

__global__ void __launch_bounds__(256) pair_count_kernel(WalkArgs w, uint64_t seed, uint32_t* count) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const int L = w.lens[t];
    const bool all = w.own_lo <= 0 && w.own_hi == 0x7FFFFFFF;
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    uint32_t n = 0;
    if (w.rule == 1) {
        for (int i = 0; i < L; ++i) {
            if (!all && !center_owned(w, walk, i)) continue;
            const ScaleRanges q(i, L, w.window_min, w.window);
            n += ScaleRanges::span(q.l0, q.r0, i) + ScaleRanges::span(q.l1, q.r1, i);
        }
    } else {
        WalkWords wd{seed, w.walk_begin + t};
        const uint32_t win_base = 2u * (uint32_t)(L - 1);
        for (int i = 0; i < L; ++i) {
            const int r = (int)draw_index(wd(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
            const int left = i - r < 0 ? 0 : i - r, right = i + r >= L ? L - 1 : i + r;
            if (all || center_owned(w, walk, i)) n += (uint32_t)(right - left);   // [left, right] minus i itself
        }
    }
    count[t] = n;
}

template <int KMAX>
__global__ void __launch_bounds__(256) pair_emit_kernel(DevGraph g, WalkArgs w, uint64_t seed, int K, double alpha0,
                                                        const uint64_t* off, int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const int L = w.lens[t];
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    const uint64_t unit = w.walk_begin + t;
    const float alpha = alpha_walk(unit, alpha0, w.total_walks);
    WalkWords win{seed, unit}, neg{seed, unit};
    const uint32_t win_base = 2u * (uint32_t)(L - 1);
    // negatives follow the walk's draws (and DeepWalk's L window draws)
    uint32_t slot = win_base + (w.rule == 1 ? 0u : (uint32_t)L);
    int32_t* out = rec + off[t] * RW;
    for (int i = 0; i < L; ++i) {
        // DeepWalk: one range [i-r, i+r], r = shrunk window; Walklets: two ranges
        int ranges[2][2];
        int nr = 1;
        if (w.rule == 1) {
            const ScaleRanges q(i, L, w.window_min, w.window);
            ranges[0][0] = q.l0; ranges[0][1] = q.r0; ranges[1][0] = q.l1; ranges[1][1] = q.r1;
            nr = 2;
        } else {
            const int r = (int)draw_index(win(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
            ranges[0][0] = i - r < 0 ? 0 : i - r;
            ranges[0][1] = i + r >= L ? L - 1 : i + r;
        }
        const int32_t vi = walk[i];
        const bool own = center_owned(w, walk, i);
        for (int q = 0; q < nr; ++q)
        for (int j = ranges[q][0]; j <= ranges[q][1]; ++j) {
            if (j == i) continue;
            if (!own) {                     // another part's pair: its draws only
                slot += 2u * (uint32_t)K;
                continue;
            }
            int32_t x[RW];
            // W row walk[i] with its W tag, C row walk[j] with its C tag
            x[0] = (vi & ID_MASK) | (int32_t)((((uint32_t)vi >> 31) & 1u) << 30);
            x[1] = walk[j] & (ID_MASK | (1 << 30));
#pragma unroll
            for (int n = 0; n < RW - 2; ++n) x[2 + n] = -1;
#pragma unroll
            for (int n = 0; n < KMAX; ++n) {
                if (n < K) {
                    const uint32_t ki = neg(slot + 2u * (uint32_t)n), kp = neg(slot + 2u * (uint32_t)n + 1u);
                    const uint32_t ni = draw_index(ki, g.V);
                    x[2 + n] = alias_pick(ni, g.ntab[ni], kp);
                }
            }
            x[2 + KMAX] = __float_as_int(alpha);
            slot += 2u * (uint32_t)K;
            i32x4* o = reinterpret_cast<i32x4*>(out);
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) {
                const i32x4 v = {x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
                __builtin_nontemporal_store(v, o + q);
            }
            out += RW;
        }
    }
}

hipError_t launch_pair_count(const WalkArgs& w, uint64_t seed, uint32_t* count, hipStream_t st) {
    const int block = 256;
    hipLaunchKernelGGL(pair_count_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st, w,
                       seed, count);
    return hipGetLastError();
}

// exclusive scan of the per-walk counts into 64-bit offsets; temp is grown on demand
hipError_t scan_pair_counts(const uint32_t* count, uint64_t* off, uint64_t n, void** temp, size_t* temp_bytes,
                            hipStream_t st) {
    size_t need = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, need, count, off, (uint64_t)0, (size_t)n,
                                           rocprim::plus<uint64_t>(), st);
    if (e != hipSuccess) return e;
    if (need > *temp_bytes) {
        if (*temp) (void)hipFree(*temp);
        *temp = nullptr;
        *temp_bytes = 0;
        if ((e = hipMalloc(temp, need)) != hipSuccess) return e;
        *temp_bytes = need;
    }
    size_t have = *temp_bytes;
    return rocprim::exclusive_scan(*temp, have, count, off, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), st);
}

hipError_t launch_pair_emit(const DevGraph& g, const WalkArgs& w, uint64_t seed, int K, double alpha0,
                            const uint64_t* off, int32_t* rec, hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((w.nwalks + block - 1) / block));
    switch (kmax_of(K)) {
        case 5: hipLaunchKernelGGL(pair_emit_kernel<5>, grid, dim3(block), 0, st, g, w, seed, K, alpha0, off, rec); break;
        case 10: hipLaunchKernelGGL(pair_emit_kernel<10>, grid, dim3(block), 0, st, g, w, seed, K, alpha0, off, rec); break;
        default: hipLaunchKernelGGL(pair_emit_kernel<20>, grid, dim3(block), 0, st, g, w, seed, K, alpha0, off, rec); break;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- APP
// APP::Train's sample (src/model/APP.cpp:93-99): JumpingRandomWalk from the
// start vertex (src/proNet.cpp:685-701: while the vertex has out-edges,
// TargetSample -- p, then index -- then stop when random_gen(0,1) < jump),
// then UpdatePair(start, walk.back()) with K negatives (index, then p).  One
// thread per unit u = w * sample_times + s, all draws from stream 1, unit u,
// consecutive slots (the oracle's orc_train_app).  One record per unit, so a
// serial update over the records is the reference's order; consecutive
// records share the start's W row (pair_train_kernel keeps it in registers).
template <int KMAX>
__global__ void __launch_bounds__(256) app_record_kernel(DevGraph g, AppArgs p, uint64_t seed, int K, double alpha0,
                                                         int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.n) return;
    const uint64_t u = p.unit_begin + t, w = u / (uint64_t)p.sample_times;
    const int32_t start = (int32_t)p.order[w - p.order_base];
    WalkWords wd{seed, u};
    uint32_t slot = 0;
    int32_t next = start;
    for (int s = 0; s < APP_MAX_STEPS; ++s) {
        if (g.offsets[next + 1] - g.offsets[next] == 0) break;
        const uint32_t kp = wd(slot), ki = wd(slot + 1);
        next = untag(target_sample(g, next, kp, ki));
        const double jmp = (double)wd(slot + 2) * 0x1p-32;   // random_gen(0, 1)
        slot += 3;
        if (jmp < p.jump) break;
    }
    int32_t x[RW];
    // W row start with its W tag, C row next with its C tag
    x[0] = start | (int32_t)((g.vtab[start].y >> 31) << 30);
    x[1] = next | (int32_t)((g.ntab[next].y >> 31) << 30);
#pragma unroll
    for (int n = 0; n < RW - 2; ++n) x[2 + n] = -1;
#pragma unroll
    for (int n = 0; n < KMAX; ++n) {
        if (n < K) {
            const uint32_t ki = wd(slot + 2u * (uint32_t)n), kp = wd(slot + 2u * (uint32_t)n + 1u);
            const uint32_t ni = draw_index(ki, g.V);
            x[2 + n] = alias_pick(ni, g.ntab[ni], kp);
        }
    }
    x[2 + KMAX] = __float_as_int(alpha_walk(w, alpha0, p.total_walks));
    i32x4* o = reinterpret_cast<i32x4*>(rec + t * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) {
        const i32x4 v = {x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
        __builtin_nontemporal_store(v, o + q);
    }
}

hipError_t launch_app_records(const DevGraph& g, const AppArgs& p, uint64_t seed, int K, double alpha0, int32_t* rec,
                              hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((p.n + block - 1) / block));
    if (kmax_of(K) == 5) hipLaunchKernelGGL(app_record_kernel<5>, grid, dim3(block), 0, st, g, p, seed, K, alpha0, rec);
    else hipLaunchKernelGGL(app_record_kernel<10>, grid, dim3(block), 0, st, g, p, seed, K, alpha0, rec);
    return hipGetLastError();
}

// ---------------------------------------------------------------- HPE
// HPE::Train's sample (src/model/HPE.cpp:118-131): v1 = SourceSample, v2 =
// TargetSample(v1), UpdateCommunity(v1, v2) (src/proNet.cpp:3018-3054: step j
// > 0 walks on with TargetSample of the previous context, -1 ends it; each
// step an Opt_SigmoidRegSGD of W[v1] against the context and K negatives),
// then UpdatePair(v2, v1).  One thread per sample s, draws from stream 0, unit
// s, consecutive slots (the oracle's orc_train_hpe); TargetSample on a vertex
// without out-edges draws nothing.  Emits walk_steps + 1 records per sample:
// the community steps (word 0 bit 31 set: the regularised rule; word 1 -1
// after the walk ended) and the pair record {v2, v1}.  A source without
// out-edges (v2 = -1, undefined in the reference) is skipped and counted.
template <int KMAX>
__global__ void __launch_bounds__(256) hpe_record_kernel(DevGraph g, HpeArgs p, uint64_t seed, int K, double alpha0,
                                                         int32_t* rec, unsigned long long* skipped) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.n) return;
    const uint64_t s = p.begin + t;
    WalkWords wd{seed, s};
    wd.stream = 0;
    uint32_t slot = 0;
    const int nrec = p.walk_steps + 1;
    i32x4* o = reinterpret_cast<i32x4*>(rec + t * (uint64_t)nrec * RW);
    const float alpha = alpha_at(s, alpha0, p.total);   // MF/BPR-style count from 0
    auto put = [&](int j, int32_t w0, int32_t w1, const int32_t (&negs)[KMAX]) {
        int32_t x[RW];
        x[0] = w0;
        x[1] = w1;
#pragma unroll
        for (int n = 0; n < RW - 2; ++n) x[2 + n] = -1;
#pragma unroll
        for (int n = 0; n < KMAX; ++n) x[2 + n] = negs[n];
        x[2 + KMAX] = __float_as_int(alpha);
#pragma unroll
        for (int q = 0; q < RW / 4; ++q) {
            const i32x4 v = {x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
            __builtin_nontemporal_store(v, o + (uint64_t)j * (RW / 4) + q);
        }
    };
    auto draw_negs = [&](int32_t (&negs)[KMAX]) {
#pragma unroll
        for (int n = 0; n < KMAX; ++n) {
            negs[n] = -1;
            if (n < K) {
                const uint32_t ki = wd(slot), kp = wd(slot + 1);
                slot += 2;
                const uint32_t ni = draw_index(ki, g.V);
                negs[n] = alias_pick(ni, g.ntab[ni], kp);
            }
        }
    };
    int32_t none[KMAX];
#pragma unroll
    for (int n = 0; n < KMAX; ++n) none[n] = -1;
    const uint32_t kp0 = wd(0), ki0 = wd(1);
    slot = 2;
    const int32_t v1 = untag(source_sample(g, kp0, ki0));
    int32_t ctx = -1, ctxt = -1;
    if (g.offsets[v1 + 1] - g.offsets[v1] != 0) {
        ctxt = target_sample(g, v1, wd(slot), wd(slot + 1));
        slot += 2;
        ctx = untag(ctxt);
    }
    if (ctx < 0) {   // v1 without out-edges: the whole sample is skipped
        for (int j = 0; j < nrec; ++j) put(j, -1, -1, none);
        atomicAdd(skipped, 1ull);
        return;
    }
    const int32_t v2 = ctx;
    int j = 0;
    for (; j < p.walk_steps; ++j) {
        if (j != 0) {
            if (g.offsets[ctx + 1] - g.offsets[ctx] == 0) break;
            ctxt = target_sample(g, ctx, wd(slot), wd(slot + 1));
            slot += 2;
            ctx = untag(ctxt);
        }
        int32_t negs[KMAX];
        draw_negs(negs);
        put(j, (int32_t)((uint32_t)v1 | 0x80000000u), ctxt, negs);
    }
    for (int k = j; k < p.walk_steps; ++k) put(k, (int32_t)((uint32_t)v1 | 0x80000000u), -1, none);
    int32_t negs[KMAX];
    draw_negs(negs);
    // UpdatePair(v2, v1): W row v2 (W tag), C row v1 (C tag)
    put(p.walk_steps, v2 | (int32_t)((g.vtab[v2].y >> 31) << 30), v1 | (int32_t)((g.ntab[v1].y >> 31) << 30), negs);
}

hipError_t launch_hpe_records(const DevGraph& g, const HpeArgs& p, uint64_t seed, int K, double alpha0, int32_t* rec,
                              unsigned long long* skipped, hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((p.n + block - 1) / block));
    if (kmax_of(K) == 5)
        hipLaunchKernelGGL(hpe_record_kernel<5>, grid, dim3(block), 0, st, g, p, seed, K, alpha0, rec, skipped);
    else
        hipLaunchKernelGGL(hpe_record_kernel<10>, grid, dim3(block), 0, st, g, p, seed, K, alpha0, rec, skipped);
    return hipGetLastError();
}

// ---------------------------------------------------------------- caller pairs
// proNet::UpdatePairs (src/proNet.cpp:2741-2753) / Go (*ProNet).UpdatePairs
// (pkg/pronet/optimizer.go:8-18) over caller-supplied pairs: one record per
// pair, {v | W tag, c | C tag, n_1 .. n_K, -1 .., alpha bits at 2 + KMAX}, for
// the pair kernels.  Pair i (of the call; this launch holds pairs first ..
// first + n) draws its K negatives (index, then p) from stream 3, unit
// unit0 + i / PAIR_BLOCK, slots 2K (i % PAIR_BLOCK) + 2j, +1 (the oracle's
// orc_update_pairs).  go: the Go record form (go_pair_emit_kernel: untagged W
// row, the C tag only when `tagged`).
template <int KMAX>
__global__ void __launch_bounds__(256) caller_pair_kernel(DevGraph g, const int32_t* __restrict__ pv,
                                                          const int32_t* __restrict__ pc, uint64_t n, uint64_t first,
                                                          int K, float alpha, uint64_t seed, uint64_t unit0, int go,
                                                          int tagged, int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint64_t i = first + t;
    WalkWords wd{seed, unit0 + i / PAIR_BLOCK};
    wd.stream = 3;
    const uint32_t base = 2u * (uint32_t)K * (uint32_t)(i % PAIR_BLOCK);
    const int32_t v = pv[t], c = pc[t];
    int32_t x[RW];
    if (go) {
        x[0] = v;
        x[1] = tagged ? (int32_t)(c | ((g.ntab[c].y >> 31) << 30)) : c;
    } else {
        x[0] = v | (int32_t)((g.vtab[v].y >> 31) << 30);
        x[1] = c | (int32_t)((g.ntab[c].y >> 31) << 30);
    }
#pragma unroll
    for (int q = 0; q < RW - 2; ++q) x[2 + q] = -1;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        if (q < K) {
            const uint32_t ki = wd(base + 2u * (uint32_t)q), kp = wd(base + 2u * (uint32_t)q + 1u);
            const uint32_t ni = draw_index(ki, g.V);
            const int32_t id = alias_pick(ni, g.ntab[ni], kp);
            x[2 + q] = go && !tagged ? untag(id) : id;
        }
    }
    x[2 + KMAX] = __float_as_int(alpha);
    i32x4* o = reinterpret_cast<i32x4*>(rec + t * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) {
        const i32x4 y = {x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
        __builtin_nontemporal_store(y, o + q);
    }
}

hipError_t launch_caller_pairs(const DevGraph& g, const int32_t* pv, const int32_t* pc, uint64_t n, uint64_t first,
                               int K, float alpha, uint64_t seed, uint64_t unit0, int go, int tagged, int32_t* rec,
                               hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((n + block - 1) / block));
    if (kmax_of(K) == 5)
        hipLaunchKernelGGL(caller_pair_kernel<5>, grid, dim3(block), 0, st, g, pv, pc, n, first, K, alpha, seed, unit0,
                           go, tagged, rec);
    else
        hipLaunchKernelGGL(caller_pair_kernel<10>, grid, dim3(block), 0, st, g, pv, pc, n, first, K, alpha, seed,
                           unit0, go, tagged, rec);
    return hipGetLastError();
}

}  // namespace smore
