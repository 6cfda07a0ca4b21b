// probe_layout.hip -- what the row layout and the sample order are worth for
// the LINE-2 update's memory pattern at config c4 (d=64, K=5), before building
// them into the product.  Each sample reads and rewrites 7 rows of 256 B:
// W[v] (v ~ source law p ~ r^-0.6), C[c] (c ~ Zipf(0.8) endpoint law,
// p ~ r^-0.8) and 5 negatives C[n] (p ~ r^-0.6), two [V][64] fp32 tables.
//   layout 0: vertex ids randomly permuted (today's tables)
//   layout 1: hot-first ids (row r = popularity rank r)
//   order  0: samples in draw order        (one group per sample, strided)
//   order  1: samples sorted by source v, each group walks a contiguous run
//             of samples and keeps W[v] in registers while v repeats
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_layout tools/probe_layout.hip
// Run:   tools/probe_layout [V=10000000] [samples=16777216] [run=64]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
    } while (0)

// ids: n x 8 int {v, c, n1..n5, pad}; run: samples per group chunk (order 1)
template <int ORDER>
__global__ void __launch_bounds__(256) probe(float* W, float* C, const int* ids, long n, int run, float* sink) {
    const int lane = threadIdx.x & 15;
    const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const long ng = ((long)gridDim.x * blockDim.x) >> 4;
    float acc = 0.f;
    if (ORDER == 0) {
        for (long s = g; s < n; s += ng) {
            const int* id = ids + s * 8;
            float r[7][4];
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                const float* p = (k == 0 ? W : C) + (long)id[k] * 64 + lane;
#pragma unroll
                for (int m = 0; m < 4; ++m) r[k][m] = p[m * 16];
            }
#pragma unroll
            for (int k = 0; k < 7; ++k)
#pragma unroll
                for (int m = 0; m < 4; ++m) acc += r[k][m];
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                float* p = (k == 0 ? W : C) + (long)id[k] * 64 + lane;
#pragma unroll
                for (int m = 0; m < 4; ++m) p[m * 16] = r[k][m] * 0.999f;
            }
        }
    } else {
        for (long b = g * run; b < n; b += ng * run) {
            const long e = b + run < n ? b + run : n;
            int cur = -1;
            float wv[4] = {0, 0, 0, 0};
            for (long s = b; s < e; ++s) {
                const int* id = ids + s * 8;
                if (id[0] != cur) {
                    if (cur >= 0) {
                        float* p = W + (long)cur * 64 + lane;
#pragma unroll
                        for (int m = 0; m < 4; ++m) p[m * 16] = wv[m];
                    }
                    cur = id[0];
                    const float* p = W + (long)cur * 64 + lane;
#pragma unroll
                    for (int m = 0; m < 4; ++m) wv[m] = p[m * 16];
                }
                float r[6][4];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const float* p = C + (long)id[k + 1] * 64 + lane;
#pragma unroll
                    for (int m = 0; m < 4; ++m) r[k][m] = p[m * 16];
                }
#pragma unroll
                for (int k = 0; k < 6; ++k)
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        acc += r[k][m];
                        wv[m] *= 0.9999f;
                    }
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    float* p = C + (long)id[k + 1] * 64 + lane;
#pragma unroll
                    for (int m = 0; m < 4; ++m) p[m * 16] = r[k][m] * 0.999f;
                }
            }
            if (cur >= 0) {
                float* p = W + (long)cur * 64 + lane;
#pragma unroll
                for (int m = 0; m < 4; ++m) p[m * 16] = wv[m];
            }
        }
    }
    if (acc == 12345.f) sink[0] = acc;
}

struct Zipf {   // inverse CDF of p(r) ~ (r+1)^-s over [0, V)
    std::vector<double> cdf;
    Zipf(long V, double s) : cdf(V) {
        double a = 0;
        for (long i = 0; i < V; ++i) { a += std::pow((double)(i + 1), -s); cdf[i] = a; }
    }
    int draw(double u) const {
        long j = std::lower_bound(cdf.begin(), cdf.end(), u * cdf.back()) - cdf.begin();
        return (int)std::min<long>(j, (long)cdf.size() - 1);
    }
};

int main(int argc, char** argv) {
    const long V = argc > 1 ? atol(argv[1]) : 10000000;
    const long n = argc > 2 ? atol(argv[2]) : 1 << 24;
    const int run = argc > 3 ? atoi(argv[3]) : 64;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float *W, *C, *sink;
    int* ids;
    CHK(hipMalloc(&W, V * 64 * sizeof(float)));
    CHK(hipMalloc(&C, V * 64 * sizeof(float)));
    CHK(hipMemset(W, 0, V * 64 * sizeof(float)));
    CHK(hipMemset(C, 0, V * 64 * sizeof(float)));
    CHK(hipMalloc(&sink, 4));
    CHK(hipMalloc(&ids, n * 8 * sizeof(int)));
    Zipf z6(V, 0.6), z8(V, 0.8);
    std::mt19937_64 rng(1);
    std::uniform_real_distribution<double> U(0, 1);
    std::vector<int> rank(n * 8);   // popularity ranks
    for (long s = 0; s < n; ++s) {
        rank[s * 8 + 0] = z6.draw(U(rng));
        rank[s * 8 + 1] = z8.draw(U(rng));
        for (int k = 0; k < 5; ++k) rank[s * 8 + 2 + k] = z6.draw(U(rng));
        rank[s * 8 + 7] = 0;
    }
    std::vector<int> perm(V);
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<long> by_src(n);
    std::iota(by_src.begin(), by_src.end(), 0);
    std::stable_sort(by_src.begin(), by_src.end(), [&](long a, long b) { return rank[a * 8] < rank[b * 8]; });
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    std::vector<int> h(n * 8);
    for (int layout = 0; layout < 2; ++layout) {
        for (int order = 0; order < 2; ++order) {
            for (long s = 0; s < n; ++s) {
                const long src = order ? by_src[s] : s;
                for (int k = 0; k < 8; ++k) {
                    const int r = rank[src * 8 + k];
                    h[s * 8 + k] = layout ? r : perm[r];
                }
            }
            CHK(hipMemcpy(ids, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
            for (int bpc : {4, 8}) {
                const int grid = cus * bpc;
                float best = 1e30f;
                for (int rep = 0; rep < 3; ++rep) {
                    CHK(hipEventRecord(a));
                    if (order == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, W, C, ids, n, run, sink);
                    else hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, W, C, ids, n, run, sink);
                    CHK(hipEventRecord(b));
                    CHK(hipEventSynchronize(b));
                    float ms;
                    CHK(hipEventElapsedTime(&ms, a, b));
                    best = std::min(best, ms);
                }
                printf("{\"layout\": \"%s\", \"order\": \"%s\", \"V\": %ld, \"samples\": %ld, \"run\": %d, "
                       "\"blocks_per_cu\": %d, \"ms\": %.3f, \"Msamples_per_s\": %.1f}\n",
                       layout ? "hot-first" : "permuted", order ? "source-sorted" : "draw-order", V, n, run, bpc,
                       best, n / best / 1e3);
                fflush(stdout);
            }
        }
    }
    return 0;
}
