// train_kernels.hip -- sampler / init kernels and the launch dispatch of the
// sampled-SGD update kernels (edge_kernels.h; instantiated in
// train_edge_<mode>_k<KMAX>.hip).

#include "train_kernels.h"

namespace smore {

// ------------------------------------------------------------------ sampler
__global__ void sample_kernel(DevGraph g, uint64_t seed, uint64_t begin, uint64_t count, int K,
                              int bpr, int32_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    const int nslot = bpr ? 14 : 4 + 2 * K;
    const int width = bpr ? 7 : 2 + K;
    int32_t* o = out + t * width;
    uint32_t w[4];
    uint32_t blk = 0xFFFFFFFFu;
    auto word = [&](int j) -> uint32_t {
        if ((uint32_t)(j >> 2) != blk) {
            blk = (uint32_t)(j >> 2);
            const uint4 b = philox_block(seed, 0, s, blk);
            w[0] = b.x; w[1] = b.y; w[2] = b.z; w[3] = b.w;
        }
        return w[j & 3];
    };
    (void)nslot;
    const int32_t v = untag(source_sample(g, word(0), word(1)));
    o[0] = v;
    const uint32_t tp = word(2), ti = word(3);
    const int32_t c = target_sample(g, v, tp, ti);
    o[1] = c < 0 ? -1 : untag(c);
    const int nn = bpr ? 5 : K;
    for (int j = 0; j < nn; ++j) {
        const uint32_t ki = word(4 + 2 * j), kp = word(5 + 2 * j);
        o[2 + j] = untag(negative_sample(g, ki, kp));
    }
}

// ------------------------------------------------------------------ init
__global__ void init_uniform_kernel(float* T, int64_t rows, int dim, int dpad, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * dpad) return;
    const int64_t v = i / dpad;
    const int d = (int)(i % dpad);
    float x = 0.0f;
    if (d < dim) {
        const uint4 b = philox_block(seed, 2, (uint64_t)v, (uint32_t)(d >> 2));
        const double u = ldexp((double)comp(b, d & 3), -32);
        x = (float)((u - 0.5) / dim);
    }
    T[i] = x;
}

// ------------------------------------------------------------------ dispatch
int lanes_of(int dpad) {
    int nq = (dpad + 3) / 4, G = 1;
    while (G < nq && G < 64) G <<= 1;
    return G;
}

#define SMORE_EDGE_DISPATCH(fn, ...)                                           \
    {                                                                          \
        const int k = kmax_of(a.K);                                            \
        if (a.mode == 1) return k == 5 ? fn##a5(__VA_ARGS__) : k == 10 ? fn##a10(__VA_ARGS__) : fn##a20(__VA_ARGS__); \
        if (a.mode == 3) return k == 5 ? fn##h5(__VA_ARGS__) : k == 10 ? fn##h10(__VA_ARGS__) : fn##h20(__VA_ARGS__); \
        return k == 5 ? fn##s5(__VA_ARGS__) : k == 10 ? fn##s10(__VA_ARGS__) : fn##s20(__VA_ARGS__);                \
    }

#define SMORE_PAIR_DISPATCH(fn, ...)                                           \
    {                                                                          \
        const bool k5 = kmax_of(a.K) == 5;                                     \
        if (a.mode == 1) return k5 ? fn##a5(__VA_ARGS__) : fn##a10(__VA_ARGS__); \
        if (a.mode == 3) return k5 ? fn##h5(__VA_ARGS__) : fn##h10(__VA_ARGS__); \
        return k5 ? fn##s5(__VA_ARGS__) : fn##s10(__VA_ARGS__);                \
    }

static bool pair_path(const EdgeArgs& a) { return a.alpha_rec == 1 && a.mode != 2 && a.K <= 10 && !a.rec_edge; }

hipError_t launch_edge_train(const EdgeArgs& a, int grid, hipStream_t st) {
    if (pair_path(a)) SMORE_PAIR_DISPATCH(launch_pair_, a, grid, st)
    SMORE_EDGE_DISPATCH(launch_edge_, a, grid, st)
}

const void* edge_kernel_symbol(const EdgeArgs& a) {
    if (pair_path(a)) SMORE_PAIR_DISPATCH(pair_symbol_, a)
    SMORE_EDGE_DISPATCH(edge_symbol_, a)
}
#undef SMORE_EDGE_DISPATCH
#undef SMORE_PAIR_DISPATCH

hipError_t launch_sample(const DevGraph& g, uint64_t seed, uint64_t begin, uint64_t count, int K,
                         int bpr, int32_t* out, hipStream_t st) {
    const int block = 256;
    const uint64_t grid = (count + block - 1) / block;
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)grid), dim3(block), 0, st, g, seed, begin, count, K,
                       bpr, out);
    return hipGetLastError();
}

hipError_t launch_init_uniform(float* T, int64_t rows, int dim, int dpad, uint64_t seed, hipStream_t st) {
    const int64_t n = rows * dpad;
    const int block = 256;
    hipLaunchKernelGGL(init_uniform_kernel, dim3((unsigned)((n + block - 1) / block)), dim3(block), 0, st, T,
                       rows, dim, dpad, seed);
    return hipGetLastError();
}

}  // namespace smore
