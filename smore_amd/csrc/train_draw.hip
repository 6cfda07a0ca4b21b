// train_draw.hip -- the sampling half of the edge hot path.
//
// LINE::Train's per-sample draws (src/model/LINE.cpp:171-176 -> SourceSample
// src/proNet.cpp:647-657, TargetSample :671-683, and UpdatePair's K
// NegativeSample calls :623-633; MF::Train and LINE order 1 the same) for a
// range of global sample indices, written as one record per sample for the
// update kernel (edge_kernels.h edge_train_kernel):
//     rec[t] = {v, c, n_1 .. n_K, -1 ...}   (rec_width(KMAX) int32, tagged ids)
// c = -1 when the source has no out-edge (the reference's TargetSample -1;
// such samples are counted in *skipped and skipped by the update).
//
// Why a separate kernel: the draws are a 3-deep chain of dependent random
// 8-16 B reads (vertex alias -> CSR offsets -> context alias + target) plus K
// independent negative-alias reads.  Inside the update kernel every sample
// waited on that chain before its row gathers; here one thread per sample
// keeps thousands of chains in flight per CU (few registers), and the update
// kernel sees one streaming 32-B read per sample.  Draws are identical to the
// fused form (same Philox slots, same compares), so results are unchanged.
#include <cstdlib>

#include "train_kernels.h"

namespace smore {

// loads of the random draw-table entries (non-temporal loads were measured
// slower at C4: 21.0 vs 17.4 ms per 2^27 samples, same fetched bytes)
__device__ __forceinline__ uint2 ldr(const uint2* p) { return *p; }
__device__ __forceinline__ uint4 ldr(const uint4* p) { return *p; }

// PART: 0 = the whole record; 1 = {v, c} only; 2 = negatives only (a pass
// whose only random reads are the negative table, small enough to stay in the
// Infinity Cache while it runs)
template <int KMAX, int PART>
__global__ void __launch_bounds__(256) draw_kernel(DevGraph g, uint64_t seed, uint64_t begin, uint64_t count,
                                                   int K, int32_t* rec, unsigned long long* skipped) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    // slots 0-3: source p, source index, target p, target index
    int32_t* const r = rec + t * RW;
    if constexpr (PART == 1) {
        const uint4 b0 = philox_block(seed, 0, s, 0);
        const uint32_t vi = draw_index(b0.y, g.V);
        const int32_t tv = alias_pick(vi, g.vtab[vi], b0.x);
        const int32_t c = target_sample(g, untag(tv), b0.z, b0.w);
        __builtin_nontemporal_store(tv, r);
        __builtin_nontemporal_store(c, r + 1);
        if (c < 0) atomicAdd(skipped, 1ull);
        return;
    }
    if constexpr (PART == 2) {
#pragma unroll
        for (int j = 0; j < KMAX; j += 2) {
            if (j < K) {
                const uint4 b = philox_block(seed, 0, s, 1 + j / 2);
                const uint32_t i0 = draw_index(b.x, g.V);
                __builtin_nontemporal_store(alias_pick(i0, g.ntab[i0], b.y), r + 2 + j);
                if (j + 1 < K) {
                    const uint32_t i1 = draw_index(b.z, g.V);
                    __builtin_nontemporal_store(alias_pick(i1, g.ntab[i1], b.w), r + 3 + j);
                }
            }
        }
        return;
    }
    const uint4 b0 = philox_block(seed, 0, s, 0);
    const uint32_t vi = draw_index(b0.y, g.V);
    uint2 ve = make_uint2(0u, 0u);
    uint4 p0 = make_uint4(0u, 0u, 0u, 0u), p1 = p0;
    if (g.vt32) {
        p0 = ldr(g.vt32 + 2 * (uint64_t)vi);
        p1 = ldr(g.vt32 + 2 * (uint64_t)vi + 1);
    } else {
        ve = g.vtab[vi];
    }
    // slots 4+2j (index), 5+2j (p): block 1 + j/2, components 2(j&1), 2(j&1)+1
    uint32_t nidx[KMAX], np[KMAX];
    uint2 ne[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; j += 2) {
        if (j < K) {
            const uint4 b = philox_block(seed, 0, s, 1 + j / 2);
            nidx[j] = draw_index(b.x, g.V);
            np[j] = b.y;
            if (j + 1 < KMAX) {
                nidx[j + 1] = draw_index(b.z, g.V);
                np[j + 1] = b.w;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
        if (j < K) ne[j] = ldr(g.ntab + nidx[j]);
    int32_t tv, c;
    if (g.vt32) {
        // source draw and its CSR row from one packed entry; one context read
        const bool acc = b0.x < p0.x;
        tv = alias_pick(vi, make_uint2(p0.x, p0.y), b0.x);
        const uint32_t off = acc ? p0.z : p1.x, br = acc ? p0.w : p1.y;
        c = -1;
        if (br != 0) {
            const uint4 ce = ldr(g.ct16 + (uint64_t)off + draw_index(b0.w, br));
            c = b0.z < ce.x ? (int32_t)ce.z : (int32_t)ce.y;
        }
    } else {
        tv = alias_pick(vi, ve, b0.x);
        c = target_sample(g, untag(tv), b0.z, b0.w);
    }
    int32_t w[RW];
    w[0] = tv;
    w[1] = c;
#pragma unroll
    for (int j = 0; j < RW - 2; ++j) w[2 + j] = (j < KMAX && j < K) ? alias_pick(nidx[j], ne[j], np[j]) : -1;
    i32x4* o = reinterpret_cast<i32x4*>(rec + t * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) {
        const i32x4 x = {w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        __builtin_nontemporal_store(x, o + q);
    }
    if (c < 0) atomicAdd(skipped, 1ull);
}

// Hot/cold record split (hybrid scatter): the same draws as
// draw_kernel<KMAX, 0>, each record written with its learning rate in word
// 2 + KMAX (the rate of its global sample index, as the update kernel would
// compute it: base 1 for LINE, 0 for MF / BPR) and placed by whether any of
// its ids carries a hot tag: hot records fill rec[0 ..) in arrival order,
// the others rec[.. count) from the back (one counter add per wave each), so
// counts[0] hot records then count - counts[0] cold ones.  The cold ones touch
// no hot row and run through the plain-store update kernel (more resident
// blocks, less code), the hot ones through the hybrid kernel.
template <int KMAX>
__global__ void __launch_bounds__(256) draw_split_kernel(DevGraph g, uint64_t seed, uint64_t begin, uint64_t count,
                                                         int K, double alpha0, uint64_t total, int base, int32_t* rec,
                                                         unsigned long long* skipped, unsigned long long* counts) {
    constexpr int RW = rec_width(KMAX);
    static_assert(RW > 2 + KMAX, "a record needs a free word for the rate");
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    const uint4 b0 = philox_block(seed, 0, s, 0);
    const uint32_t vi = draw_index(b0.y, g.V);
    const uint4 p0 = ldr(g.vt32 + 2 * (uint64_t)vi), p1 = ldr(g.vt32 + 2 * (uint64_t)vi + 1);
    uint32_t nidx[KMAX], np[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; j += 2) {
        if (j < K) {
            const uint4 b = philox_block(seed, 0, s, 1 + j / 2);
            nidx[j] = draw_index(b.x, g.V);
            np[j] = b.y;
            if (j + 1 < KMAX) {
                nidx[j + 1] = draw_index(b.z, g.V);
                np[j + 1] = b.w;
            }
        }
    }
    uint2 ne[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
        if (j < K) ne[j] = ldr(g.ntab + nidx[j]);
    const bool acc = b0.x < p0.x;
    const int32_t tv = alias_pick(vi, make_uint2(p0.x, p0.y), b0.x);
    const uint32_t off = acc ? p0.z : p1.x, br = acc ? p0.w : p1.y;
    int32_t c = -1;
    if (br != 0) {
        const uint4 ce = ldr(g.ct16 + (uint64_t)off + draw_index(b0.w, br));
        c = b0.z < ce.x ? (int32_t)ce.z : (int32_t)ce.y;
    }
    int32_t w[RW];
    w[0] = tv;
    w[1] = c;
    bool hot = tag_hot(tv) || (c >= 0 && tag_hot(c));
#pragma unroll
    for (int j = 0; j < RW - 2; ++j) {
        w[2 + j] = (j < KMAX && j < K) ? alias_pick(nidx[j], ne[j], np[j]) : -1;
        if (j < KMAX && j < K) hot = hot || tag_hot(w[2 + j]);
    }
    w[2 + KMAX] = __float_as_int(alpha_at(s + (uint64_t)base, alpha0, total));
    // wave-aggregated slots: one counter add per wave and class
    const uint64_t act = __ballot(1), hm = __ballot(hot);
    const int lane = (int)__lane_id();
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int leader = __ffsll((unsigned long long)act) - 1;
    unsigned long long hb = 0, cb = 0;
    if (lane == leader) {
        const int nh = __popcll(hm), nc = __popcll(act & ~hm);
        if (nh) hb = atomicAdd(counts, (unsigned long long)nh);
        if (nc) cb = atomicAdd(counts + 1, (unsigned long long)nc);
    }
    hb = __shfl(hb, leader);
    cb = __shfl(cb, leader);
    const uint64_t idx = hot ? hb + (uint64_t)__popcll(hm & below)
                             : count - 1 - (cb + (uint64_t)__popcll(act & ~hm & below));
    i32x4* o = reinterpret_cast<i32x4*>(rec + idx * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) {
        const i32x4 x = {w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        __builtin_nontemporal_store(x, o + q);
    }
    if (c < 0) atomicAdd(skipped, 1ull);
}

hipError_t launch_draw_split(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K, double alpha0,
                             uint64_t total, int base, int32_t* rec, unsigned long long* skipped,
                             unsigned long long* counts, hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((count + block - 1) / block));
    switch (kmax_of(K)) {
        case 5:
            hipLaunchKernelGGL(draw_split_kernel<5>, grid, dim3(block), 0, st, g, seed, begin, count, K, alpha0, total,
                               base, rec, skipped, counts);
            break;
        case 10:
            hipLaunchKernelGGL(draw_split_kernel<10>, grid, dim3(block), 0, st, g, seed, begin, count, K, alpha0,
                               total, base, rec, skipped, counts);
            break;
        default:
            hipLaunchKernelGGL(draw_split_kernel<20>, grid, dim3(block), 0, st, g, seed, begin, count, K, alpha0,
                               total, base, rec, skipped, counts);
            break;
    }
    return hipGetLastError();
}

// packed draw tables from the device graph (after any re-tagging)
__global__ void pack_vertex_kernel(DevGraph g, uint4* vt32) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.V) return;
    const uint2 e = g.vtab[i];
    const int32_t al = (int32_t)(e.y & (uint32_t)ID_MASK);
    const int64_t oi = g.offsets[i], oa = g.offsets[al];
    vt32[2 * i] = make_uint4(e.x, e.y, (uint32_t)oi, (uint32_t)(g.offsets[i + 1] - oi));
    vt32[2 * i + 1] = make_uint4((uint32_t)oa, (uint32_t)(g.offsets[al + 1] - oa), 0u, 0u);
}

__global__ void pack_edge_kernel(DevGraph g, uint64_t E, uint4* ct16) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const uint2 e = g.ctab[i];
    ct16[i] = make_uint4(e.x, e.y, (uint32_t)g.targets[i], 0u);
}

hipError_t launch_pack(const DevGraph& g, uint64_t E, uint4* vt32, uint4* ct16, hipStream_t st) {
    const int block = 256;
    hipLaunchKernelGGL(pack_vertex_kernel, dim3((unsigned)((g.V + block - 1) / block)), dim3(block), 0, st, g, vt32);
    hipLaunchKernelGGL(pack_edge_kernel, dim3((unsigned)((E + block - 1) / block)), dim3(block), 0, st, g, E, ct16);
    return hipGetLastError();
}

hipError_t launch_draw(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K, int32_t* rec,
                       unsigned long long* skipped, hipStream_t st) {
    static const int block = [] {   // tuning knob: SMORE_DRAW_BLOCK (64..256 threads)
        const char* e = getenv("SMORE_DRAW_BLOCK");
        const int b = e ? atoi(e) : 256;
        return (b == 64 || b == 128 || b == 256) ? b : 256;
    }();
    const dim3 grid((unsigned)((count + block - 1) / block));
#if SMORE_DRAW_SPLIT
    // negatives first, then source/target (unused record words stay as written by
    // the previous launch; the update kernel reads only words 0 .. 1+K)
#define SMORE_DRAW(KM)                                                                                        \
    hipLaunchKernelGGL((draw_kernel<KM, 2>), grid, dim3(block), 0, st, g, seed, begin, count, K, rec, skipped); \
    hipLaunchKernelGGL((draw_kernel<KM, 1>), grid, dim3(block), 0, st, g, seed, begin, count, K, rec, skipped);
#else
#define SMORE_DRAW(KM) \
    hipLaunchKernelGGL((draw_kernel<KM, 0>), grid, dim3(block), 0, st, g, seed, begin, count, K, rec, skipped);
#endif
    switch (kmax_of(K)) {
        case 5: SMORE_DRAW(5) break;
        case 10: SMORE_DRAW(10) break;
        default: SMORE_DRAW(20) break;
    }
#undef SMORE_DRAW
    return hipGetLastError();
}

}  // namespace smore
