// probe_scatter.hip -- ceilings of the hot path's memory pattern on gfx950.
// Each "sample" touches 7 rows of a [V][64] fp32 table (d=64, G=16 lanes per
// sample, lane l owns elements l, l+16, l+32, l+48 -- the kernels' layout).
//   op 0: gather only            op 1: gather + plain store of each row
//   op 2: gather + atomic add     op 3: atomic add only (no gather)
//   op 4: gather + atomic add for the H hottest rows (Zipf rank < H), plain
//         store for the rest (the hybrid scatter)
// Row ids: uniform or Zipf(0.8) over V (inverse CDF on the host).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_scatter tools/probe_scatter.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

template <int OP>
__global__ void __launch_bounds__(256) probe(float* T, const int* ids, long n, float* sink) {
    const int lane = threadIdx.x & 15;
    long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const long ng = ((long)gridDim.x * blockDim.x) >> 4;
    float acc = 0.f;
    for (; g < n; g += ng) {
        const int* id = ids + g * 7;
        float r[7][4];
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const float* p = T + (long)(id[k] & 0x7fffffff) * 64 + lane;
#pragma unroll
            for (int m = 0; m < 4; ++m) r[k][m] = OP == 3 ? 1e-7f : p[m * 16];
        }
#pragma unroll
        for (int k = 0; k < 7; ++k)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc += r[k][m];
        if (OP == 0) continue;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            float* p = T + (long)(id[k] & 0x7fffffff) * 64 + lane;
            const bool hot = OP == 4 ? (id[k] < 0) : OP != 1;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                if (!hot) p[m * 16] = r[k][m] * 0.999f;
                else unsafeAtomicAdd(p + m * 16, r[k][m] * 1e-3f);
            }
        }
    }
    if (acc == 12345.f) sink[0] = acc;
}

int main(int argc, char** argv) {
    const long V = argc > 1 ? atol(argv[1]) : 1000000;
    const long n = argc > 2 ? atol(argv[2]) : 1 << 25;
    const int blocks_per_cu = argc > 3 ? atoi(argv[3]) : 8;
    const long H = argc > 4 ? atol(argv[4]) : 20000;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float *T, *sink;
    int* ids;
    CHK(hipMalloc(&T, V * 64 * sizeof(float)));
    CHK(hipMemset(T, 0, V * 64 * sizeof(float)));
    CHK(hipMalloc(&sink, 4));
    CHK(hipMalloc(&ids, n * 7 * sizeof(int)));
    std::mt19937_64 rng(1);
    std::vector<double> cdf(V);
    double acc = 0;
    for (long i = 0; i < V; ++i) { acc += 1.0 / pow((double)(i + 1), 0.8); cdf[i] = acc; }
    std::vector<int> perm(V);
    for (long i = 0; i < V; ++i) perm[i] = (int)i;
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<int> h(n * 7);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int dist = 0; dist < 2; ++dist) {
        std::uniform_real_distribution<double> U(0, 1);
        for (long i = 0; i < n * 7; ++i) {
            if (dist == 0) h[i] = (int)(rng() % V);
            else {
                long j = std::lower_bound(cdf.begin(), cdf.end(), U(rng) * acc) - cdf.begin();
                if (j >= V) j = V - 1;
                h[i] = perm[j] | (j < H ? (int)0x80000000 : 0);
            }
        }
        CHK(hipMemcpy(ids, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
        for (int op = 0; op < 5; ++op) {
            if (op == 4 && dist == 0) continue;
            const int grid = cus * blocks_per_cu;
            for (int rep = 0; rep < 3; ++rep) {
                CHK(hipEventRecord(a));
                if (op == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, T, ids, n, sink);
                if (op == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, T, ids, n, sink);
                if (op == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, T, ids, n, sink);
                if (op == 3) hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(256), 0, 0, T, ids, n, sink);
                if (op == 4) hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(256), 0, 0, T, ids, n, sink);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                if (rep == 2) {
                    const double rows = 7.0 * n;
                    printf("{\"dist\": \"%s\", \"op\": \"%s\", \"V\": %ld, \"samples\": %ld, \"ms\": %.3f, "
                           "\"Msamples_per_s\": %.1f, \"row_GBps\": %.1f, \"hot_rows\": %ld}\n",
                           dist ? "zipf0.8" : "uniform",
                           op == 0 ? "gather" : op == 1 ? "gather+store" : op == 2 ? "gather+atomic" : op == 3 ? "atomic" : "gather+hybrid",
                           V, n, ms, n / ms / 1e3, rows * 256 / ms / 1e6, op == 4 ? H : 0L);
                }
            }
        }
    }
    return 0;
}
