// probe_draw.hip -- what the draw kernel's memory pattern costs under different
// memory types, before changing the product's allocations.  The LINE-2 draw
// of one sample (train_draw.hip) is: one 32-B entry of a 320-MB vertex table,
// one 16-B entry of a 6.4-GB context table, five 8-B entries of an 80-MB
// negative table (all uniformly random), and one 32-B record written.  On
// coarse-grained memory every random read fills a 128-B L2 line.
//   alloc 0: hipMalloc (coarse-grained)
//   alloc 1: hipExtMallocWithFlags(hipDeviceMallocUncached)
//   alloc 2: hipExtMallocWithFlags(hipDeviceMallocFinegrained)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_draw tools/probe_draw.hip
// Run:   tools/probe_draw [samples=134217728]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}
__device__ __forceinline__ uint32_t pick(uint64_t t, int j, uint32_t n) {
    return __umulhi(mix(t * 16 + (uint64_t)j), n);
}

// WHICH: 0 = the whole draw pattern; 1 = negatives only (5 x 8 B of the 80-MB
// table); 2 = context only (16 B of the 6.4-GB table); 3 = vertex only (32 B)
template <int WHICH, bool NT>
__global__ void __launch_bounds__(256) draw_probe(const u4* vt, uint32_t nv, const u4* ct, uint32_t nc,
                                                  const u2* nt, uint32_t nn, u4* rec, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (WHICH == 0 || WHICH == 3) {
        const u4* p = vt + 2 * (uint64_t)pick(t, 0, nv);
        const u4 a = NT ? __builtin_nontemporal_load(p) : p[0];
        const u4 b = NT ? __builtin_nontemporal_load(p + 1) : p[1];
        acc[0] = a.x ^ b.y; acc[1] = a.y ^ b.x;
    }
    if (WHICH == 0 || WHICH == 2) {
        const u4* p = ct + pick(t, 1, nc) + (acc[0] & 1);
        const u4 c = NT ? __builtin_nontemporal_load(p) : p[0];
        acc[2] = c.x ^ c.y; acc[3] = c.z;
    }
    if (WHICH == 0 || WHICH == 1) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const u2* p = nt + pick(t, 2 + j, nn);
            const u2 e = NT ? __builtin_nontemporal_load(p) : p[0];
            acc[3 + j] = e.x ^ e.y;
        }
    }
    __builtin_nontemporal_store(u4{acc[0], acc[1], acc[2], acc[3]}, rec + 2 * t);
    __builtin_nontemporal_store(u4{acc[4], acc[5], acc[6], acc[7]}, rec + 2 * t + 1);
}

static void* alloc(size_t n, int kind) {
    void* p = nullptr;
    if (kind == 0) CHK(hipMalloc(&p, n));
    else if (kind == 1) CHK(hipExtMallocWithFlags(&p, n, hipDeviceMallocUncached));
    else CHK(hipExtMallocWithFlags(&p, n, hipDeviceMallocFinegrained));
    CHK(hipMemset(p, 0x11, n));
    return p;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 27);
    const uint32_t nv = 10000000, nc = 400000000, nn = 10000000;
    u4* rec;
    CHK(hipMalloc(&rec, n * 32));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const char* names[] = {"coarse", "uncached", "finegrained"};
    const char* what[] = {"draw (32B vt + 16B ct + 5x8B nt)", "negatives 5x8B of 80MB", "context 16B of 6.4GB",
                          "vertex 32B of 320MB"};
    for (int kind = 0; kind < 3; ++kind) {
        const u4* vt = (const u4*)alloc((size_t)nv * 32, kind);
        const u4* ct = (const u4*)alloc((size_t)nc * 16, kind);
        const u2* nt = (const u2*)alloc((size_t)nn * 8, kind);
        const dim3 grid((unsigned)((n + 255) / 256));
        for (int which = 0; which < 4; ++which) {
            for (int ntf = 0; ntf < 2; ++ntf) {
                float best = 1e30f;
                for (int rep = 0; rep < 3; ++rep) {
                    CHK(hipEventRecord(a));
#define L(W, N) hipLaunchKernelGGL((draw_probe<W, N>), grid, dim3(256), 0, 0, vt, nv, ct, nc, nt, nn, rec, n)
                    if (ntf) {
                        if (which == 0) L(0, true); else if (which == 1) L(1, true); else if (which == 2) L(2, true); else L(3, true);
                    } else {
                        if (which == 0) L(0, false); else if (which == 1) L(1, false); else if (which == 2) L(2, false); else L(3, false);
                    }
#undef L
                    CHK(hipGetLastError());
                    CHK(hipEventRecord(b));
                    CHK(hipEventSynchronize(b));
                    float ms;
                    CHK(hipEventElapsedTime(&ms, a, b));
                    if (ms < best) best = ms;
                }
                printf("{\"alloc\": \"%s\", \"pattern\": \"%s\", \"nt_loads\": %d, \"samples\": %llu, \"ms\": %.3f, "
                       "\"ms_per_2^27\": %.3f}\n",
                       names[kind], what[which], ntf, (unsigned long long)n, best, best * (double)(1ull << 27) / n);
                fflush(stdout);
            }
        }
        CHK(hipFree((void*)vt));
        CHK(hipFree((void*)ct));
        CHK(hipFree((void*)nt));
    }
    return 0;
}
