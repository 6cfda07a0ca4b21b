// train_pairs.hip -- DeepWalk skip-gram pairs as sample records for the update
// kernel (edge_kernels.h), so DeepWalk gets the same row prefetch, chunked
// scheduling and write-combining as LINE.
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
#include <cstring>
#include <rocprim/device/device_scan.hpp>

#include "train_kernels.h"

namespace smore {

struct WalkWords {   // consecutive Philox words of one walk unit (stream 1)
    uint64_t seed, unit;
    uint32_t blk = 0xFFFFFFFFu;
    uint4 b;
    __device__ uint32_t operator()(uint32_t slot) {
        if ((slot >> 2) != blk) {
            blk = slot >> 2;
            b = philox_block(seed, 1, unit, blk);
        }
        return comp(b, (int)(slot & 3));
    }
};

__global__ void __launch_bounds__(256) pair_count_kernel(WalkArgs w, uint64_t seed, uint32_t* count) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const int L = w.lens[t];
    WalkWords wd{seed, w.walk_begin + t};
    const uint32_t win_base = 2u * (uint32_t)(L - 1);
    uint32_t n = 0;
    for (int i = 0; i < L; ++i) {
        const int r = (int)draw_index(wd(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
        const int left = i - r < 0 ? 0 : i - r, right = i + r >= L ? L - 1 : i + r;
        n += (uint32_t)(right - left);   // [left, right] minus i itself
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
    uint32_t slot = win_base + (uint32_t)L;
    int32_t* out = rec + off[t] * RW;
    for (int i = 0; i < L; ++i) {
        const int r = (int)draw_index(win(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
        const int left = i - r < 0 ? 0 : i - r, right = i + r >= L ? L - 1 : i + r;
        const int32_t vi = walk[i];
        for (int j = left; j <= right; ++j) {
            if (j == i) continue;
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

}  // namespace smore
