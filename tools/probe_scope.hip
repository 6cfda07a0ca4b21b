// probe_scope.hip -- where do gfx950 float atomics execute?  Every wave adds
// 1.0 to all 64 floats (256 B) of a random row of an [R][64] fp32 table in
// coarse-grained memory, `iters` times; the table is summed afterwards, so a
// lost add shows.  Variants:
//   op 0: agent scope (unsafeAtomicAdd, the training kernels' form)
//   op 1: workgroup scope (__hip_atomic_fetch_add, __HIP_MEMORY_SCOPE_WORKGROUP)
//   op 2: workgroup scope into a per-XCD copy of the table (copy = the XCC_ID
//         hardware register of the issuing wave), i.e. one XCD per address
// Reports added GB/s, the fraction of adds lost, and how XCC_ID relates to
// blockIdx.x % 8 (a per-XCD shadow needs the real XCD id, not the dispatch
// order).  Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_scope tools/probe_scope.hip
//   tools/probe_scope [rows] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
    } while (0)

// s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): simm16 = (size - 1) << 11 | offset << 6 | id
__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; }

template <int OP>
__global__ void __launch_bounds__(256) probe(float* T, long R, long iters, unsigned* xcc_out) {
    const int lane = threadIdx.x & 63;
    const unsigned xcc = xcc_id();
    if (threadIdx.x == 0) xcc_out[blockIdx.x] = xcc;
    uint32_t h = (blockIdx.x * 4u + threadIdx.x / 64u) * 2654435761u + 12345u;
    float* base = T + (OP == 2 ? (long)xcc * R * 64 : 0);
    for (long i = 0; i < iters; ++i) {
        h = h * 1664525u + 1013904223u;
        float* p = base + (long)((h >> 8) % (uint32_t)R) * 64 + lane;
        if (OP == 0) unsafeAtomicAdd(p, 1.0f);
        else __hip_atomic_fetch_add(p, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

int main(int argc, char** argv) {
    const long R = argc > 1 ? atol(argv[1]) : 4096;
    const long iters = argc > 2 ? atol(argv[2]) : 2000;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 8;
    const size_t n = (size_t)16 * R * 64;   // room for 16 per-XCD copies
    float* T;
    unsigned* xo;
    CHK(hipMalloc(&T, n * sizeof(float)));
    CHK(hipMalloc(&xo, grid * sizeof(unsigned)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<float> h(n);
    std::vector<unsigned> hx(grid);
    for (int op = 0; op < 3; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipMemset(T, 0, n * sizeof(float)));
            CHK(hipEventRecord(e0));
            if (op == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(h.data(), T, n * sizeof(float), hipMemcpyDeviceToHost));
            CHK(hipMemcpy(hx.data(), xo, grid * sizeof(unsigned), hipMemcpyDeviceToHost));
            double sum = 0;
            for (size_t i = 0; i < n; ++i) sum += h[i];
            const double expect = (double)grid * 4 * iters * 64;
            int cnt[16] = {0}, same = 0;
            for (int b = 0; b < grid; ++b) {
                cnt[hx[b] & 15]++;
                same += (int)(hx[b] == (unsigned)(b % 8));
            }
            printf("{\"op\": %d, \"rows\": %ld, \"iters\": %ld, \"ms\": %.3f, \"added_GBs\": %.1f, "
                   "\"lost_frac\": %.6f, \"xcc_blocks\": [%d, %d, %d, %d, %d, %d, %d, %d], "
                   "\"xcc_eq_block_mod8\": %.4f}\n",
                   op, R, iters, ms, expect * 4 / ms / 1e6, 1.0 - sum / expect, cnt[0], cnt[1], cnt[2], cnt[3],
                   cnt[4], cnt[5], cnt[6], cnt[7], (double)same / grid);
        }
    }
    return 0;
}
