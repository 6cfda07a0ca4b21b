// membw.hip -- the box's streaming-copy bandwidth, the `measured_peak` the
// benchmark prices the path against (SURVEY.md 8d "plus the measured copy
// bandwidth on the box").  A grid-stride float4 copy: every lane moves 16 B per
// load/store (global_load_dwordx4 / global_store_dwordx4), UNROLL independent
// loads in flight per lane before the stores, one full 1-KiB segment per
// wave-instruction; a few blocks per CU over the whole chip.
#include "train_kernels.h"

namespace smore {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                   uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        f32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// one 16-B word per thread, as many blocks as words / 256 (the dispatcher
// keeps every CU full)
__global__ void __launch_bounds__(256) copy_flat_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                        uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

// variant 0: default cache policy, 1: non-temporal loads and stores (grid-
// stride, `blocks` blocks); 2: one word per thread over the whole buffer
hipError_t launch_copy(const void* src, void* dst, uint64_t n16, int blocks, int variant, hipStream_t st) {
    const f32x4* s = reinterpret_cast<const f32x4*>(src);
    f32x4* d = reinterpret_cast<f32x4*>(dst);
    if (variant == 2)
        hipLaunchKernelGGL(copy_flat_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st, s, d, n16);
    else if (variant == 1) hipLaunchKernelGGL((copy_kernel<4, true>), dim3(blocks), dim3(256), 0, st, s, d, n16);
    else hipLaunchKernelGGL((copy_kernel<4, false>), dim3(blocks), dim3(256), 0, st, s, d, n16);
    return hipGetLastError();
}

// rows `ids` of a table [*][dpad] to / from a dense host-order buffer [n][dim]
// (smore_set_rows / smore_get_rows: the Go UpdatePairs hook moves only the
// rows a batch touches); one float per thread
__global__ void __launch_bounds__(256) rows_io_kernel(float* T, const int32_t* ids, uint64_t n, int dpad, int dim,
                                                      float* buf, int to_table) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * (uint64_t)dim) return;
    const uint64_t r = i / (uint64_t)dim, e = i - r * (uint64_t)dim;
    float* t = T + (uint64_t)ids[r] * (uint64_t)dpad + e;
    if (to_table) *t = buf[i];
    else buf[i] = *t;
}

hipError_t launch_rows_io(float* T, const int32_t* ids, uint64_t n, int dpad, int dim, float* buf, int to_table,
                          hipStream_t st) {
    const uint64_t m = n * (uint64_t)dim;
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(rows_io_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, T, ids, n, dpad, dim, buf,
                       to_table);
    return hipGetLastError();
}

// rows ids[pos[j]] <- buf[pos[j]] for j < m (the combining pairs call's
// upload of the rows an earlier request in the call did not already bring)
__global__ void __launch_bounds__(256) rows_put_sel_kernel(float* T, const int32_t* ids, const int32_t* pos,
                                                           uint64_t m, int dpad, int dim, const float* buf) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m * (uint64_t)dim) return;
    const uint64_t j = i / (uint64_t)dim, e = i - j * (uint64_t)dim;
    const uint64_t r = (uint64_t)pos[j];
    T[(uint64_t)ids[r] * (uint64_t)dpad + e] = buf[r * (uint64_t)dim + e];
}

hipError_t launch_rows_put_sel(float* T, const int32_t* ids, const int32_t* pos, uint64_t m, int dpad, int dim,
                               const float* buf, hipStream_t st) {
    const uint64_t n = m * (uint64_t)dim;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rows_put_sel_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, T, ids, pos, m, dpad,
                       dim, buf);
    return hipGetLastError();
}

}  // namespace smore
