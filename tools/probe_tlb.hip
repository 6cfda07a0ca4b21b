// probe_tlb.hip -- does the update kernel's time level follow how the two
// 2.56-GB tables are mapped?  The C4 update pattern (tools/probe_layout.hip's
// draw-order kernel: 7 random 256-B rows read and rewritten per sample, Zipf
// ranks over permuted ids) on tables allocated in several ways, each
// allocated / timed / freed several times in one process:
//   alloc 0: hipMalloc
//   alloc 1: hipExtMallocWithFlags(hipDeviceMallocUncached)
//   alloc 2: VMM: 1-GiB-aligned VA, physical memory in 1-GiB hipMemCreate chunks
//   alloc 3: VMM with the minimum granularity chunks (2 MiB)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_tlb tools/probe_tlb.hip
// Run:   tools/probe_tlb [reps=5] [uniform ids=0|1] [kinds=3]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

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

__global__ void __launch_bounds__(256) rmw(float* W, float* C, const int* ids, long n, float* sink) {
    const int lane = threadIdx.x & 15;
    const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const long ng = ((long)gridDim.x * blockDim.x) >> 4;
    float acc = 0.f;
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
    if (acc == 12345.f) sink[0] = acc;
}

struct Vmm {
    void* va = nullptr;
    size_t size = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};

static float* vmm_alloc(size_t bytes, size_t chunk, Vmm& m) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CHK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    if (chunk < gran) chunk = gran;
    chunk = (chunk + gran - 1) / gran * gran;
    m.size = (bytes + chunk - 1) / chunk * chunk;
    CHK(hipMemAddressReserve(&m.va, m.size, (size_t)1 << 30, nullptr, 0));
    for (size_t off = 0; off < m.size; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        CHK(hipMemCreate(&h, chunk, &prop, 0));
        CHK(hipMemMap((char*)m.va + off, chunk, 0, h, 0));
        m.h.push_back(h);
    }
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CHK(hipMemSetAccess(m.va, m.size, &d, 1));
    return (float*)m.va;
}

static void vmm_free(Vmm& m) {
    CHK(hipMemUnmap(m.va, m.size));
    for (auto h : m.h) CHK(hipMemRelease(h));
    CHK(hipMemAddressFree(m.va, m.size));
    m = Vmm{};
}

struct Zipf {
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
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const bool uniform = argc > 2 && atoi(argv[2]) == 1;   // 1: uniform row ids instead of Zipf ranks
    const int kinds = argc > 3 ? atoi(argv[3]) : 3;         // allocation kinds to run (0..kinds-1)
    const long V = 10000000, n = 1 << 24;
    const size_t bytes = (size_t)V * 64 * sizeof(float);
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float* sink;
    int* ids;
    CHK(hipMalloc(&sink, 4));
    CHK(hipMalloc(&ids, n * 8 * sizeof(int)));
    {
        Zipf z6(V, uniform ? 0.0 : 0.6), z8(V, uniform ? 0.0 : 0.8);
        std::mt19937_64 rng(1);
        std::uniform_real_distribution<double> U(0, 1);
        std::vector<int> perm(V);
        std::iota(perm.begin(), perm.end(), 0);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<int> h(n * 8);
        for (long s = 0; s < n; ++s) {
            h[s * 8 + 0] = perm[z6.draw(U(rng))];
            h[s * 8 + 1] = perm[z8.draw(U(rng))];
            for (int k = 0; k < 5; ++k) h[s * 8 + 2 + k] = perm[z6.draw(U(rng))];
            h[s * 8 + 7] = 0;
        }
        CHK(hipMemcpy(ids, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const char* names[] = {"hipMalloc", "uncached", "vmm_1GiB_chunks", "vmm_min_chunks"};
    for (int kind = 0; kind < kinds; ++kind) {
        for (int r = 0; r < reps; ++r) {
            float *W = nullptr, *C = nullptr;
            Vmm mw, mc;
            if (kind == 0) { CHK(hipMalloc(&W, bytes)); CHK(hipMalloc(&C, bytes)); }
            else if (kind == 1) {
                CHK(hipExtMallocWithFlags((void**)&W, bytes, hipDeviceMallocUncached));
                CHK(hipExtMallocWithFlags((void**)&C, bytes, hipDeviceMallocUncached));
            } else {
                const size_t chunk = kind == 2 ? (size_t)1 << 30 : 0;
                W = vmm_alloc(bytes, chunk, mw);
                C = vmm_alloc(bytes, chunk, mc);
            }
            CHK(hipMemset(W, 0, bytes));
            CHK(hipMemset(C, 0, bytes));
            float best = 1e30f;
            for (int t = 0; t < 4; ++t) {
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(rmw, dim3(cus * 4), dim3(256), 0, 0, W, C, ids, n, sink);
                CHK(hipGetLastError());
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                best = std::min(best, ms);
            }
            printf("{\"ids\": \"%s\", \"alloc\": \"%s\", \"rep\": %d, \"W\": \"%p\", \"C\": \"%p\", \"ms\": %.3f, "
                   "\"Msamples_per_s\": %.1f}\n", uniform ? "uniform" : "zipf", names[kind], r, (void*)W, (void*)C, best, n / best / 1e3);
            fflush(stdout);
            if (kind <= 1) { CHK(hipFree(W)); CHK(hipFree(C)); }
            else { vmm_free(mw); vmm_free(mc); }
        }
    }
    return 0;
}
