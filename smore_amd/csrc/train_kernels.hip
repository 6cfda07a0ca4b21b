// train_kernels.hip -- the fused sampled-SGD kernels for gfx950.
//
// One "sample group" of G lanes owns one edge sample at a time (G = lanes per
// d-vector: d=64 -> 16 lanes x float4, 4 samples per wave64).  Per sample:
//   Philox draws (distributed over the group's lanes, broadcast by shuffle)
//   -> alias draws (source, target, K negatives; dependent 8-B/4-B loads)
//   -> gather of the K+2 rows (float4 per lane, each row one 256-B segment)
//   -> K+1 dot products (fmaf chain + pairwise lane tree)
//   -> fastSigmoid table in LDS -> in-register row updates
//   -> scatter: Hogwild float4 stores, or float atomic adds of the deltas.
// Rows live in registers for the whole sample; ids that repeat inside one
// sample are resolved in registers so the in-place semantics of
// src/proNet.cpp:1312-1330 / 1784-1809 hold exactly.
#include "train_kernels.h"

namespace smore {

// ------------------------------------------------------------------ words
// The 4+2K (or 14 for BPR) words of a sample: lane l of the group computes
// Philox block (l % NBLK) of unit s; word j is broadcast from lane j/4.
template <int G, int NSLOT>
struct SampleWords {
    static constexpr int NBLK = (NSLOT + 3) / 4;
    uint32_t w[NSLOT];
    __device__ __forceinline__ void draw(uint64_t seed, uint32_t stream, uint64_t unit, int lane) {
        if constexpr (G >= NBLK) {
            const uint4 b = philox_block(seed, stream, unit, (uint32_t)(lane % NBLK));
#pragma unroll
            for (int j = 0; j < NSLOT; ++j) w[j] = __shfl(comp(b, j & 3), j >> 2, G);
        } else {
#pragma unroll
            for (int k = 0; k < NBLK; ++k) {
                const uint4 b = philox_block(seed, stream, unit, (uint32_t)k);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (4 * k + c < NSLOT) w[4 * k + c] = comp(b, c);
            }
        }
    }
};

// ------------------------------------------------------------------ edge kernel
// LINE-2 (W,C), LINE-1 (W,W), MF (W,W, Opt_SGD) -- one kernel, the model is a
// wave-uniform runtime switch.
template <int G, int R, int KMAX>
__global__ void __launch_bounds__(256) edge_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    for (int i = threadIdx.x; i < 1001; i += blockDim.x) s_sig[i] = a.sig[i];
    __syncthreads();

    constexpr int NSLOT = 4 + 2 * KMAX;
    const int lane = threadIdx.x & (G - 1);
    uint64_t group = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;
    if (a.mode == 2) {               // serial: one group, samples in order
        if (group != 0) return;
        ngroups = 1;
    }
    const bool shared = a.model != 0;
    const bool mf = a.model == 2;
    const int dpad = a.dpad;
    float* const Tw = a.W;
    float* const Tc = shared ? a.W : a.C;
    const uint64_t base = mf ? 0 : 1;   // LINE counts from 1, MF from 0

    for (uint64_t t = group; t < a.count; t += ngroups) {
        const uint64_t s = a.begin + t;
        SampleWords<G, NSLOT> wd;
        wd.draw(a.seed, 0, s, lane);

        const int32_t v = source_sample(a.g, wd.w[0], wd.w[1]);
        const int32_t c = target_sample(a.g, v, wd.w[2], wd.w[3]);
        if (c < 0) {
            if (lane == 0) atomicAdd(a.skipped, 1ull);
            continue;
        }
        int32_t id[KMAX + 1];
        id[0] = c;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            id[j + 1] = (j < a.K) ? negative_sample(a.g, wd.w[4 + 2 * j], wd.w[5 + 2 * j]) : -1;
        const int32_t vs = shared ? v : -2;   // id of W_v inside the context table

        // ---- gather
        float4 wv[R], rows[KMAX + 1][R];
        const float* wp = Tw + (int64_t)v * dpad + lane * 4;
#pragma unroll
        for (int r = 0; r < R; ++r) wv[r] = ld4(wp + r * G * 4);
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            if (id[k] >= 0) {
                const float* cp = Tc + (int64_t)id[k] * dpad + lane * 4;
#pragma unroll
                for (int r = 0; r < R; ++r) rows[k][r] = ld4(cp + r * G * 4);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) rows[k][r] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        // canonicalise repeated ids onto their first occurrence
#pragma unroll
        for (int k = 1; k <= KMAX; ++k) {
#pragma unroll
            for (int k2 = 0; k2 < k; ++k2)
                if (id[k2] == id[k]) {
#pragma unroll
                    for (int r = 0; r < R; ++r) rows[k][r] = rows[k2][r];
                }
        }
#pragma unroll
        for (int k = 0; k <= KMAX; ++k)
            if (id[k] == vs) {
#pragma unroll
                for (int r = 0; r < R; ++r) rows[k][r] = wv[r];
            }
        float4 orig[KMAX + 1][R], wv0[R];
        if (a.mode == 1) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                wv0[r] = wv[r];
#pragma unroll
                for (int k = 0; k <= KMAX; ++k) orig[k][r] = rows[k][r];
            }
        }

        const float alpha = alpha_at(s + base, a.alpha0, a.total);
        float4 e[R];
#pragma unroll
        for (int r = 0; r < R; ++r) e[r] = make_float4(0.f, 0.f, 0.f, 0.f);

        // ---- K+1 sequential Opt_SigmoidSGD / Opt_SGD steps
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            if (k <= a.K) {
            float p = 0.0f;
#pragma unroll
            for (int r = 0; r < R; ++r) p = dot4(wv[r], rows[k][r], p);
            const float f = group_sum<G>(p);
            if (mf) {
                const float gg = (k == 0 ? 1.0f : -1.0f) - f;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float4 ce = rows[k][r], we = wv[r];
                    float4 t1, t2;
                    t1.x = gg * ce.x - a.reg * we.x; t2.x = gg * we.x - a.reg * ce.x;
                    t1.y = gg * ce.y - a.reg * we.y; t2.y = gg * we.y - a.reg * ce.y;
                    t1.z = gg * ce.z - a.reg * we.z; t2.z = gg * we.z - a.reg * ce.z;
                    t1.w = gg * ce.w - a.reg * we.w; t2.w = gg * we.w - a.reg * ce.w;
                    e[r] = fma4(alpha, t1, e[r]);
                    rows[k][r] = fma4(alpha, t2, ce);
                }
            } else {
                const float gg = ((k == 0 ? 1.0f : 0.0f) - fast_sigmoid(f, s_sig)) * alpha;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float4 ce = rows[k][r];
                    e[r] = fma4(gg, ce, e[r]);
                    rows[k][r] = fma4(gg, wv[r], ce);
                }
            }
            // in-place semantics: every other reference to this row sees it
#pragma unroll
            for (int k2 = 0; k2 <= KMAX; ++k2)
                if (k2 != k && id[k2] == id[k]) {
#pragma unroll
                    for (int r = 0; r < R; ++r) rows[k2][r] = rows[k][r];
                }
            if (id[k] == vs) {
#pragma unroll
                for (int r = 0; r < R; ++r) wv[r] = rows[k][r];
            }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) wv[r] = add4(wv[r], e[r]);

        // ---- scatter
        float* wq = Tw + (int64_t)v * dpad + lane * 4;
        if (a.mode == 1) {
#pragma unroll
            for (int r = 0; r < R; ++r) atomic_add4(wq + r * G * 4, shared ? sub4(wv[r], wv0[r]) : e[r]);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) st4(wq + r * G * 4, wv[r]);
        }
#pragma unroll
        for (int k = 0; k <= KMAX; ++k) {
            bool last = id[k] >= 0 && id[k] != vs;
#pragma unroll
            for (int k2 = k + 1; k2 <= KMAX; ++k2) last = last && (id[k2] != id[k]);
            if (last) {
                float* cq = Tc + (int64_t)id[k] * dpad + lane * 4;
                if (a.mode == 1) {
#pragma unroll
                    for (int r = 0; r < R; ++r) atomic_add4(cq + r * G * 4, sub4(rows[k][r], orig[k][r]));
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) st4(cq + r * G * 4, rows[k][r]);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ BPR kernel
// UpdateBPRPair (src/proNet.cpp:1406-1455), one shared table, 5 rounds.
// Slots: 0 = u, 1 = i, 2+n = j_n.
template <int G, int R>
__global__ void __launch_bounds__(256) bpr_train_kernel(EdgeArgs a) {
    __shared__ float s_sig[1001];
    for (int i = threadIdx.x; i < 1001; i += blockDim.x) s_sig[i] = a.sig[i];
    __syncthreads();

    constexpr int NS = 7;
    const int lane = threadIdx.x & (G - 1);
    uint64_t group = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;
    if (a.mode == 2) {
        if (group != 0) return;
        ngroups = 1;
    }
    const int dpad = a.dpad;
    float* const T = a.W;

    for (uint64_t t = group; t < a.count; t += ngroups) {
        const uint64_t s = a.begin + t;
        SampleWords<G, 14> wd;
        wd.draw(a.seed, 0, s, lane);
        int32_t id[NS];
        id[0] = source_sample(a.g, wd.w[0], wd.w[1]);
        id[1] = target_sample(a.g, id[0], wd.w[2], wd.w[3]);
        if (id[1] < 0) {
            if (lane == 0) atomicAdd(a.skipped, 1ull);
            continue;
        }
#pragma unroll
        for (int n = 0; n < 5; ++n) id[2 + n] = negative_sample(a.g, wd.w[4 + 2 * n], wd.w[5 + 2 * n]);

        float4 row[NS][R], orig[NS][R];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const float* p = T + (int64_t)id[k] * dpad + lane * 4;
#pragma unroll
            for (int r = 0; r < R; ++r) row[k][r] = ld4(p + r * G * 4);
        }
#pragma unroll
        for (int k = 1; k < NS; ++k)
#pragma unroll
            for (int k2 = 0; k2 < k; ++k2)
                if (id[k2] == id[k]) {
#pragma unroll
                    for (int r = 0; r < R; ++r) row[k][r] = row[k2][r];
                }
        if (a.mode == 1) {
#pragma unroll
            for (int k = 0; k < NS; ++k)
#pragma unroll
                for (int r = 0; r < R; ++r) orig[k][r] = row[k][r];
        }
        const float alpha = alpha_at(s, a.alpha0, a.total);
        const float r1 = alpha * 0.0025f, r2 = alpha * 0.025f;
        float4 ve[R];
#pragma unroll
        for (int r = 0; r < R; ++r) ve[r] = make_float4(0.f, 0.f, 0.f, 0.f);

#define SMORE_PROPAGATE(K_)                                                    \
    _Pragma("unroll") for (int k2 = 0; k2 < NS; ++k2) if (k2 != (K_) && id[k2] == id[(K_)]) { \
        _Pragma("unroll") for (int r = 0; r < R; ++r) row[k2][r] = row[(K_)][r];            \
    }

#pragma unroll
        for (int n = 0; n < 5; ++n) {
            const int J = 2 + n;
            float4 x[R], ce[R];
            float p = 0.0f;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                x[r] = sub4(row[1][r], row[J][r]);
                p = dot4(row[0][r], x[r], p);
            }
            const float f = group_sum<G>(p);
            const float gg = fast_sigmoid(-f, s_sig) * alpha;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                ve[r] = fma4(gg, x[r], ve[r]);
                ce[r] = make_float4(gg * row[0][r].x, gg * row[0][r].y, gg * row[0][r].z, gg * row[0][r].w);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) row[1][r] = fma4(-r1, row[1][r], row[1][r]);
            SMORE_PROPAGATE(1)
#pragma unroll
            for (int r = 0; r < R; ++r) row[J][r] = fma4(-r1, row[J][r], row[J][r]);
            SMORE_PROPAGATE(J)
#pragma unroll
            for (int r = 0; r < R; ++r) row[1][r] = add4(row[1][r], ce[r]);
            SMORE_PROPAGATE(1)
#pragma unroll
            for (int r = 0; r < R; ++r) row[J][r] = sub4(row[J][r], ce[r]);
            SMORE_PROPAGATE(J)
        }
#pragma unroll
        for (int r = 0; r < R; ++r) row[0][r] = add4(fma4(-r2, row[0][r], row[0][r]), ve[r]);
        SMORE_PROPAGATE(0)
#undef SMORE_PROPAGATE

#pragma unroll
        for (int k = 0; k < NS; ++k) {
            bool last = true;
#pragma unroll
            for (int k2 = k + 1; k2 < NS; ++k2) last = last && (id[k2] != id[k]);
            if (last) {
                float* q = T + (int64_t)id[k] * dpad + lane * 4;
                if (a.mode == 1) {
#pragma unroll
                    for (int r = 0; r < R; ++r) atomic_add4(q + r * G * 4, sub4(row[k][r], orig[k][r]));
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) st4(q + r * G * 4, row[k][r]);
                }
            }
        }
    }
}

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
    const int32_t v = source_sample(g, word(0), word(1));
    o[0] = v;
    const uint32_t tp = word(2), ti = word(3);
    o[1] = target_sample(g, v, tp, ti);
    const int nn = bpr ? 5 : K;
    for (int j = 0; j < nn; ++j) {
        const uint32_t ki = word(4 + 2 * j), kp = word(5 + 2 * j);
        o[2 + j] = negative_sample(g, ki, kp);
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
template <int G, int R>
static hipError_t launch_edge_gr(const EdgeArgs& a, int grid, hipStream_t st) {
    if (a.K <= 5) hipLaunchKernelGGL((edge_train_kernel<G, R, 5>), dim3(grid), dim3(256), 0, st, a);
    else if (a.K <= 10) hipLaunchKernelGGL((edge_train_kernel<G, R, 10>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((edge_train_kernel<G, R, 20>), dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

template <int G, int R>
static hipError_t launch_bpr_gr(const EdgeArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL((bpr_train_kernel<G, R>), dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

#define SMORE_DISPATCH_GR(FN, a, grid, st)                              \
    switch (lanes_of((a).dpad)) {                                       \
        case 1: return FN<1, 1>(a, grid, st);                           \
        case 2: return FN<2, 1>(a, grid, st);                           \
        case 4: return FN<4, 1>(a, grid, st);                           \
        case 8: return FN<8, 1>(a, grid, st);                           \
        case 16: return FN<16, 1>(a, grid, st);                         \
        case 32: return FN<32, 1>(a, grid, st);                         \
        default:                                                        \
            switch (((a).dpad / 4 + 63) / 64) {                         \
                case 1: return FN<64, 1>(a, grid, st);                  \
                case 2: return FN<64, 2>(a, grid, st);                  \
                case 3: return FN<64, 3>(a, grid, st);                  \
                case 4: return FN<64, 4>(a, grid, st);                  \
                default: return hipErrorInvalidValue;                   \
            }                                                           \
    }

int lanes_of(int dpad) {
    int nq = dpad / 4, G = 1;
    while (G < nq && G < 64) G <<= 1;
    return G;
}

hipError_t launch_edge_train(const EdgeArgs& a, int grid, hipStream_t st) {
    if (a.model == 3) { SMORE_DISPATCH_GR(launch_bpr_gr, a, grid, st) }
    SMORE_DISPATCH_GR(launch_edge_gr, a, grid, st)
}

const void* edge_kernel_symbol(const EdgeArgs& a) {
    // the instantiation launch_edge_train would pick (for occupancy queries)
    const int G = lanes_of(a.dpad);
    const int R = (a.dpad / 4 + 63) / 64;
#define SMORE_SYM(GG, RR)                                                         \
    if (G == GG && (GG < 64 || R == RR)) {                                        \
        if (a.model == 3) return (const void*)bpr_train_kernel<GG, RR>;           \
        if (a.K <= 5) return (const void*)edge_train_kernel<GG, RR, 5>;           \
        if (a.K <= 10) return (const void*)edge_train_kernel<GG, RR, 10>;         \
        return (const void*)edge_train_kernel<GG, RR, 20>;                        \
    }
    SMORE_SYM(1, 1) SMORE_SYM(2, 1) SMORE_SYM(4, 1) SMORE_SYM(8, 1) SMORE_SYM(16, 1)
    SMORE_SYM(32, 1) SMORE_SYM(64, 1) SMORE_SYM(64, 2) SMORE_SYM(64, 3) SMORE_SYM(64, 4)
#undef SMORE_SYM
    return nullptr;
}

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
