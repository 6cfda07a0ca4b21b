// train_walk.hip -- DeepWalk walk generation on the GPU (RandomWalk,
// src/proNet.cpp:704-724); the skip-gram pairs become sample records
// (train_pairs.hip) for the update kernel.
#include "train_kernels.h"

namespace smore {

// One thread per walk; dependent CSR / context-alias loads per step.
// Draw slots 2s, 2s+1 of walk unit (stream 1) for step s (p, then index).
// Each walk vertex carries both hybrid tags: bit 30 = hot as a C row (the
// target / negative tag), bit 31 = hot as a W row (the vertex table's self
// bit), so a pair can tag walk[i] as its W row and walk[j] as its C row.
__device__ __forceinline__ int32_t walk_word(const DevGraph& g, int32_t v) {
    const uint32_t hw = g.vtab[v].y >> 31, hc = g.ntab[v].y >> 31;
    return (int32_t)((uint32_t)v | (hc << 30) | (hw << 31));
}

__global__ void walk_gen_kernel(DevGraph g, WalkArgs w, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const uint64_t unit = w.walk_begin + t;
    // no order: walk unit starts at unit mod V (Walklets::Train, src/model/Walklets.cpp:45)
    const int32_t start = w.order ? (int32_t)w.order[unit - w.order_base] : (int32_t)(unit % g.V);
    int32_t* out = w.walks + t * (uint64_t)(w.steps + 1);
    int L = 0;
    int32_t next = start;
    out[L++] = walk_word(g, start);
    uint4 b = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < w.steps; ++s) {
        if (g.offsets[next + 1] - g.offsets[next] == 0) {
            if (next == start) break;
            next = start;
        }
        const uint32_t s0 = 2u * (uint32_t)s;
        if ((s0 & 3) == 0) b = philox_block(seed, 1, unit, s0 >> 2);
        const uint32_t kp = comp(b, (int)(s0 & 3)), ki = comp(b, (int)((s0 + 1) & 3));
        next = untag(target_sample(g, next, kp, ki));
        out[L++] = walk_word(g, next);
    }
    w.lens[t] = L;
}

hipError_t launch_walk_gen(const DevGraph& g, const WalkArgs& w, uint64_t seed, hipStream_t st) {
    const int block = 256;
    hipLaunchKernelGGL(walk_gen_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st, g,
                       w, seed);
    return hipGetLastError();
}

}  // namespace smore
