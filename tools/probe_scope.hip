// probe_scope.hip -- where do gfx950 float atomics execute?  Every wave adds
// 1.0 to all 64 floats (256 B) of a random row of an [R][64] fp32 table in
// coarse-grained memory, `iters` times; the table is summed afterwards, so a
// lost add shows.  Variants:
//   op 0: agent scope (unsafeAtomicAdd, the training kernels' form)
//   op 1: workgroup scope (__hip_atomic_fetch_add, __HIP_MEMORY_SCOPE_WORKGROUP)
//   op 2: workgroup scope into a per-XCD copy of the table (copy = the XCC_ID
//         hardware register of the issuing wave), i.e. one XCD per address
//   op 3: 32-bit INTEGER add (agent scope) into the per-XCD copy (fixed-point
//         shadow rows: do integer atomics resolve in the XCD's L2?)
//   op 4: 32-bit integer add (agent scope) into the one shared table
//   op 5: 64-bit integer add (agent scope) into the per-XCD copy (2 dwords/lane)
//   op 6: plain load + store (NOT atomic, loses adds) into the per-XCD copy: the
//         L2 read-modify-write rate for comparison
//   op 7: 32-bit integer add, WORKGROUP scope, into the per-XCD copy
//   op 8: 64-bit integer add, WORKGROUP scope, into the per-XCD copy
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
    float* base = T + ((OP == 2 || OP == 3 || OP >= 5) ? (long)xcc * R * 64 * ((OP == 5 || OP == 8) ? 2 : 1) : 0);
    for (long i = 0; i < iters; ++i) {
        h = h * 1664525u + 1013904223u;
        float* p = base + (long)((h >> 8) % (uint32_t)R) * 64 + lane;
        if (OP == 0) unsafeAtomicAdd(p, 1.0f);
        else if (OP == 1 || OP == 2) __hip_atomic_fetch_add(p, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (OP == 3 || OP == 4)
            __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(p), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (OP == 5)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(base) + (p - base), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        else if (OP == 7)
            __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(p), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (OP == 8)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(base) + (p - base), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        else { *p = *p + 1.0f; }
    }
}

int main(int argc, char** argv) {
    const long R = argc > 1 ? atol(argv[1]) : 4096;
    const long iters = argc > 2 ? atol(argv[2]) : 2000;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 8;
    const size_t n = (size_t)32 * R * 64;   // room for 16 per-XCD copies (64-bit: 2 words per element)
    float* T;
    unsigned* xo;
    CHK(hipMalloc(&T, n * sizeof(float)));
    CHK(hipMalloc(&xo, grid * sizeof(unsigned)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<float> h(n);
    std::vector<unsigned> hx(grid);
    for (int op = 0; op < 9; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipMemset(T, 0, n * sizeof(float)));
            CHK(hipEventRecord(e0));
            if (op == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 3) hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 4) hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 5) hipLaunchKernelGGL(probe<5>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 6) hipLaunchKernelGGL(probe<6>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 7) hipLaunchKernelGGL(probe<7>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            if (op == 8) hipLaunchKernelGGL(probe<8>, dim3(grid), dim3(256), 0, 0, T, R, iters, xo);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(h.data(), T, n * sizeof(float), hipMemcpyDeviceToHost));
            CHK(hipMemcpy(hx.data(), xo, grid * sizeof(unsigned), hipMemcpyDeviceToHost));
            double sum = 0;
            const uint32_t* hu = reinterpret_cast<const uint32_t*>(h.data());
            const unsigned long long* hl = reinterpret_cast<const unsigned long long*>(h.data());
            if (op == 3 || op == 4 || op == 7)
                for (size_t i = 0; i < n; ++i) sum += hu[i];
            else if (op == 5 || op == 8)
                for (size_t i = 0; i < n / 2; ++i) sum += (double)hl[i];
            else
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
                   op, R, iters, ms, expect * ((op == 5 || op == 8) ? 8 : 4) / ms / 1e6, 1.0 - sum / expect, cnt[0], cnt[1], cnt[2], cnt[3],
                   cnt[4], cnt[5], cnt[6], cnt[7], (double)same / grid);
        }
    }
    return 0;
}
