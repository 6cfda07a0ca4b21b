// probe_rows.hip -- the ceiling of the LINE-2 update's memory pattern alone:
// per sample, read and rewrite 7 random 256-B rows (W_v and 6 context rows of
// two [V][64] fp32 tables, C4's 10M rows each), no arithmetic, no draws, no
// records.  Same layout as the product (16 lanes per sample, one 16-B chunk
// per lane, dwordx4 loads/stores), the same one-sample-ahead row prefetch,
// the tables in the product's uncached device memory (capi smore_alloc_tables)
// or in default memory.  Row ids come from a hash of (sample, slot): uniform
// over V, i.e. no hot rows (the product's hot rows are cheaper, if anything).
// Answers: how many 3584-B read+write updates per second can this GPU do at
// all, against which edge_train_kernel's rate is measured.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_rows tools/probe_rows.hip
// Run:   tools/probe_rows [V=10000000] [samples=134217728]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

template <int NB>   // NB: rows per sample (1 in W, NB - 1 in C)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
rows_kernel(float* W, float* C, uint32_t V, uint64_t n, unsigned long long* work, float* sink) {
    const int lane = threadIdx.x & 15;
    const uint64_t gpb = blockDim.x / 16, gib = threadIdx.x / 16;
    __shared__ uint64_t s_next;
    constexpr uint64_t ROUNDS = 128;
    const uint64_t span = ROUNDS * gpb;
    float acc = 0.f;
    auto ids = [&](uint64_t s, uint32_t (&id)[NB]) {
#pragma unroll
        for (int k = 0; k < NB; ++k) id[k] = (uint32_t)(((uint64_t)mix(s * 8 + k) * V) >> 32);
    };
    auto row = [&](int k, uint32_t i) -> float* { return (k == 0 ? W : C) + (uint64_t)i * 64 + 4 * lane; };
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) s_next = atomicAdd(work, 1ull) * span;
        __syncthreads();
        const uint64_t c0 = s_next;
        if (c0 >= n) break;
        const uint64_t lim = c0 + span < n ? c0 + span : n;
        uint32_t ia[NB], ib[NB];
        f4 ra[NB], rb[NB];
        uint64_t t = c0 + gib;
        ids(t, ia);
#pragma unroll
        for (int k = 0; k < NB; ++k) ra[k] = t < lim ? *reinterpret_cast<const f4*>(row(k, ia[k])) : f4{0, 0, 0, 0};
        for (uint64_t r = c0; r < lim; r += gpb) {
            t = r + gib;
            const uint64_t tn = t + gpb;
            ids(tn, ib);
#pragma unroll
            for (int k = 0; k < NB; ++k)
                rb[k] = tn < lim ? *reinterpret_cast<const f4*>(row(k, ib[k])) : f4{0, 0, 0, 0};
            if (t < lim) {
#pragma unroll
                for (int k = 0; k < NB; ++k) {
                    acc += ra[k].x;
                    *reinterpret_cast<f4*>(row(k, ia[k])) = ra[k] * 0.999f;
                }
            }
#pragma unroll
            for (int k = 0; k < NB; ++k) { ra[k] = rb[k]; ia[k] = ib[k]; }
        }
    }
    if (acc == 1234.5f) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint32_t V = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
    const uint64_t n = argc > 2 ? (uint64_t)atoll(argv[2]) : (1ull << 27);
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t bytes = (size_t)V * 64 * sizeof(float);
    unsigned long long* work;
    float* sink;
    CHK(hipMalloc(&work, sizeof(unsigned long long)));
    CHK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int mem = 0; mem < 2; ++mem) {
        float *W, *C;
        const unsigned flags = mem == 0 ? hipDeviceMallocUncached : hipDeviceMallocDefault;
        CHK(hipExtMallocWithFlags((void**)&W, bytes, flags));
        CHK(hipExtMallocWithFlags((void**)&C, bytes, flags));
        CHK(hipMemset(W, 0, bytes));
        CHK(hipMemset(C, 0, bytes));
        for (int bpc : {2, 3, 4}) {
            const int grid = cus * bpc;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CHK(hipMemset(work, 0, sizeof(unsigned long long)));
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(rows_kernel<7>, dim3(grid), dim3(256), 0, 0, W, C, V, n, work, sink);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                if (rep > 0 && ms < best) best = ms;
            }
            const double rw = 2.0 * 7 * 256;   // bytes read + written per sample
            printf("{\"probe\": \"rows\", \"memory\": \"%s\", \"V\": %u, \"samples\": %llu, \"rows_per_sample\": 7, "
                   "\"blocks_per_cu\": %d, \"ms\": %.3f, \"Msamples_per_s\": %.1f, \"rw_GBs\": %.1f}\n",
                   mem == 0 ? "uncached" : "default", V, (unsigned long long)n, bpc, best, n / best / 1e3,
                   rw * n / best / 1e6);
            fflush(stdout);
        }
        CHK(hipFree(W));
        CHK(hipFree(C));
    }
    return 0;
}
