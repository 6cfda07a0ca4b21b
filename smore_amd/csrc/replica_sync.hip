// replica_sync.hip -- the two fused passes of the multi-GPU replica exchange
// (new in this build -- the reference is single-process Hogwild,
// src/model/LINE.cpp:162).  Every rank holds the whole table T; S is the
// snapshot at the previous exchange.  Per exchange:
//   begin (compute stream):  D = T - S;  R = D;  S = T
//   all-reduce R (SUM) over RCCL, asynchronously, overlapping the next
//   compute step (smore_amd/dist.py OverlapSync)
//   end (compute stream):    X = scale * R - D;  T += X;  S += X
// so every rank's samples land once on every replica (one exchange late),
// and the next begin's D is again only this rank's own updates.  Streaming,
// 16 B per lane, HBM-bound (begin moves 5 and end 6 table-sized streams).
#include "train_kernels.h"
#include "hot_exchange.h"

namespace smore {

__global__ void __launch_bounds__(256) delta_begin_kernel(const float4* __restrict__ T, float4* __restrict__ S,
                                                          float4* __restrict__ D, float4* __restrict__ R,
                                                          uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 t = T[i], s = S[i];
        const float4 d = make_float4(t.x - s.x, t.y - s.y, t.z - s.z, t.w - s.w);
        D[i] = d;
        R[i] = d;
        S[i] = t;
    }
}

__global__ void __launch_bounds__(256) delta_end_kernel(float4* __restrict__ T, float4* __restrict__ S,
                                                        const float4* __restrict__ D,
                                                        const float4* __restrict__ R, float scale, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 r = R[i], d = D[i];
        const float4 x = make_float4(scale * r.x - d.x, scale * r.y - d.y, scale * r.z - d.z, scale * r.w - d.w);
        float4 t = T[i], s = S[i];
        t.x += x.x; t.y += x.y; t.z += x.z; t.w += x.w;
        s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        T[i] = t;
        S[i] = s;
    }
}

// end of exchange k fused with begin of exchange k+1 (8 streams instead of
// 5 + 6): X = scale*R - D; T' = T + X; then D' = T' - (S + X) = T - S,
// R' = D', S' = T'
__global__ void __launch_bounds__(256) delta_cycle_kernel(float4* __restrict__ T, float4* __restrict__ S,
                                                          float4* __restrict__ D, float4* __restrict__ R, float scale,
                                                          uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 r = R[i], d = D[i], t = T[i], s = S[i];
        const float4 x = make_float4(scale * r.x - d.x, scale * r.y - d.y, scale * r.z - d.z, scale * r.w - d.w);
        const float4 tn = make_float4(t.x + x.x, t.y + x.y, t.z + x.z, t.w + x.w);
        const float4 sn = make_float4(s.x + x.x, s.y + x.y, s.z + x.z, s.w + x.w);
        const float4 dn = make_float4(tn.x - sn.x, tn.y - sn.y, tn.z - sn.z, tn.w - sn.w);
        T[i] = tn;
        D[i] = dn;
        R[i] = dn;
        S[i] = tn;
    }
}

// the adaptive exchange's end / cycle: the same arithmetic with row i / dp4's
// scale (a float4 never straddles two rows: dpad % 4 == 0)
__global__ void __launch_bounds__(256) delta_end_rows_kernel(float4* __restrict__ T, float4* __restrict__ S,
                                                             const float4* __restrict__ D,
                                                             const float4* __restrict__ R,
                                                             const float* __restrict__ scale, uint64_t n4, int dp4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float sc = scale[i / (uint64_t)dp4];
        const float4 r = R[i], d = D[i];
        const float4 x = make_float4(sc * r.x - d.x, sc * r.y - d.y, sc * r.z - d.z, sc * r.w - d.w);
        float4 t = T[i], s = S[i];
        t.x += x.x; t.y += x.y; t.z += x.z; t.w += x.w;
        s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        T[i] = t;
        S[i] = s;
    }
}

__global__ void __launch_bounds__(256) delta_cycle_rows_kernel(float4* __restrict__ T, float4* __restrict__ S,
                                                               float4* __restrict__ D, float4* __restrict__ R,
                                                               const float* __restrict__ scale, uint64_t n4,
                                                               int dp4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float sc = scale[i / (uint64_t)dp4];
        const float4 r = R[i], d = D[i], t = T[i], s = S[i];
        const float4 x = make_float4(sc * r.x - d.x, sc * r.y - d.y, sc * r.z - d.z, sc * r.w - d.w);
        const float4 tn = make_float4(t.x + x.x, t.y + x.y, t.z + x.z, t.w + x.w);
        const float4 sn = make_float4(s.x + x.x, s.y + x.y, s.z + x.z, s.w + x.w);
        const float4 dn = make_float4(tn.x - sn.x, tn.y - sn.y, tn.z - sn.z, tn.w - sn.w);
        T[i] = tn;
        D[i] = dn;
        R[i] = dn;
        S[i] = tn;
    }
}

// hub-row exchange passes (hot_exchange.h): element i of the packed buffers
// is element i % dpad of row idx[i / dpad]; 16 B per lane (dpad % 4 == 0)
__global__ void __launch_bounds__(256) hot_pack_kernel(const float4* __restrict__ T, const float4* __restrict__ S,
                                                       const int32_t* __restrict__ idx, uint64_t n4, int dp4,
                                                       float4* __restrict__ P, float4* __restrict__ R) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = (uint64_t)idx[i / dp4], j = row * dp4 + i % dp4;
        const float4 t = T[j], s = S[j];
        const float4 d = make_float4(t.x - s.x, t.y - s.y, t.z - s.z, t.w - s.w);
        P[i] = d;
        R[i] = d;
    }
}

__global__ void __launch_bounds__(256) hot_unpack_kernel(float4* __restrict__ T, float4* __restrict__ S,
                                                         const int32_t* __restrict__ idx, uint64_t n4, int dp4,
                                                         const float4* __restrict__ P, const float4* __restrict__ R) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = (uint64_t)idx[i / dp4], j = row * dp4 + i % dp4;
        const float4 r = R[i], p = P[i];
        float4 t = T[j], s = S[j];
        t.x += r.x - p.x; t.y += r.y - p.y; t.z += r.z - p.z; t.w += r.w - p.w;
        s.x += r.x; s.y += r.y; s.z += r.z; s.w += r.w;
        T[j] = t;
        S[j] = s;
    }
}

static unsigned stream_grid(uint64_t n4, int cus) {
    const uint64_t want = (n4 + 255) / 256, cap = (uint64_t)(cus > 0 ? cus : 256) * 16;
    return (unsigned)(want < cap ? (want ? want : 1) : cap);
}

// row census: the rows each record would update (smore_census_begin; the walk
// models' adaptive exchange scales).  One record per thread.
__global__ void __launch_bounds__(256) row_census_kernel(const int32_t* __restrict__ rec, uint64_t n,
                                                         const uint64_t* count_dev, int RW, int K,
                                                         unsigned long long* cw, unsigned long long* cc) {
    const uint64_t cnt = count_dev ? *count_dev : n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t* r = rec + i * (uint64_t)RW;
        const int32_t w0 = r[0], w1 = r[1];
        if (w1 < 0) continue;
        atomicAdd(cw + untag(w0), 1ull);
        atomicAdd(cc + untag(w1), 1ull);
        for (int k = 0; k < K; ++k) {
            const int32_t x = r[2 + k];
            if (x >= 0) atomicAdd(cc + untag(x), 1ull);
        }
    }
}

hipError_t launch_row_census(const int32_t* rec, uint64_t n, const uint64_t* count_dev, int RW, int K,
                             unsigned long long* cw, unsigned long long* cc, int cus, hipStream_t st) {
    hipLaunchKernelGGL(row_census_kernel, dim3(stream_grid(n, cus)), dim3(256), 0, st, rec, n, count_dev, RW, K, cw,
                       cc);
    return hipGetLastError();
}

hipError_t launch_delta_begin(const float* T, float* S, float* D, float* R, uint64_t n, int cus, hipStream_t st) {
    const uint64_t n4 = n / 4;
    hipLaunchKernelGGL(delta_begin_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(T), reinterpret_cast<float4*>(S),
                       reinterpret_cast<float4*>(D), reinterpret_cast<float4*>(R), n4);
    return hipGetLastError();
}

hipError_t launch_delta_end(float* T, float* S, const float* D, const float* R, float scale, uint64_t n, int cus,
                            hipStream_t st) {
    const uint64_t n4 = n / 4;
    hipLaunchKernelGGL(delta_end_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st, reinterpret_cast<float4*>(T),
                       reinterpret_cast<float4*>(S), reinterpret_cast<const float4*>(D),
                       reinterpret_cast<const float4*>(R), scale, n4);
    return hipGetLastError();
}

hipError_t launch_delta_cycle(float* T, float* S, float* D, float* R, float scale, uint64_t n, int cus,
                              hipStream_t st) {
    const uint64_t n4 = n / 4;
    hipLaunchKernelGGL(delta_cycle_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st, reinterpret_cast<float4*>(T),
                       reinterpret_cast<float4*>(S), reinterpret_cast<float4*>(D), reinterpret_cast<float4*>(R), scale,
                       n4);
    return hipGetLastError();
}

}  // namespace smore

namespace smore {

hipError_t launch_hot_pack(const float* T, const float* S, const int32_t* idx, uint64_t n, int dpad, float* P,
                           float* R, int cus, hipStream_t st) {
    const uint64_t n4 = n * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(hot_pack_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(T), reinterpret_cast<const float4*>(S), idx, n4, dpad / 4,
                       reinterpret_cast<float4*>(P), reinterpret_cast<float4*>(R));
    return hipGetLastError();
}

hipError_t launch_hot_unpack(float* T, float* S, const int32_t* idx, uint64_t n, int dpad, const float* P,
                             const float* R, int cus, hipStream_t st) {
    const uint64_t n4 = n * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(hot_unpack_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st, reinterpret_cast<float4*>(T),
                       reinterpret_cast<float4*>(S), idx, n4, dpad / 4, reinterpret_cast<const float4*>(P),
                       reinterpret_cast<const float4*>(R));
    return hipGetLastError();
}

// the all-reduce of a same-device group: out = sum over the replicas' buffers
// in replica order, written back to every buffer (16 B per lane)
struct LocalBufs {
    float4* p[LOCAL_MAX];
    int n;
};

__global__ void __launch_bounds__(256) local_sum_kernel(LocalBufs b, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x) {
        float4 s = b.p[0][i];
        for (int r = 1; r < b.n; ++r) s = add4(s, b.p[r][i]);
        for (int r = 0; r < b.n; ++r) b.p[r][i] = s;
    }
}

hipError_t launch_local_sum(float* const* bufs, int nrep, uint64_t n, int cus, hipStream_t st) {
    if (nrep < 1 || nrep > LOCAL_MAX || (n & 3)) return hipErrorInvalidValue;
    LocalBufs b{};
    for (int r = 0; r < nrep; ++r) b.p[r] = reinterpret_cast<float4*>(bufs[r]);
    b.n = nrep;
    const uint64_t n4 = n / 4;
    hipLaunchKernelGGL(local_sum_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st, b, n4);
    return hipGetLastError();
}

hipError_t launch_delta_end_rows(float* T, float* S, const float* D, const float* R, const float* scale,
                                 uint64_t rows, int dpad, int cus, hipStream_t st) {
    const uint64_t n4 = rows * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(delta_end_rows_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st,
                       reinterpret_cast<float4*>(T), reinterpret_cast<float4*>(S),
                       reinterpret_cast<const float4*>(D), reinterpret_cast<const float4*>(R), scale, n4, dpad / 4);
    return hipGetLastError();
}

hipError_t launch_delta_cycle_rows(float* T, float* S, float* D, float* R, const float* scale, uint64_t rows,
                                   int dpad, int cus, hipStream_t st) {
    const uint64_t n4 = rows * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(delta_cycle_rows_kernel, dim3(stream_grid(n4, cus)), dim3(256), 0, st,
                       reinterpret_cast<float4*>(T), reinterpret_cast<float4*>(S), reinterpret_cast<float4*>(D),
                       reinterpret_cast<float4*>(R), scale, n4, dpad / 4);
    return hipGetLastError();
}

}  // namespace smore
