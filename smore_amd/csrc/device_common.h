// device_common.h -- gfx950 device helpers shared by the hot-path kernels:
// the Philox RNG spec, the alias samplers, the fastSigmoid table lookup and
// the lane-group reductions.  Arithmetic follows DESIGN.md "Arithmetic spec"
// (mirrored bit for bit by oracle/smore_oracle.c *_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smore {

// ---- RNG spec: Philox4x32-10, ctr = {lo(unit), hi(unit), slot/4, stream},
// key = {lo(seed), hi(seed)}; replaces src/random.cpp:5-13.
__device__ __forceinline__ uint4 philox_block(uint64_t seed, uint32_t stream, uint64_t unit,
                                              uint32_t blk) {
    uint32_t c0 = (uint32_t)unit, c1 = (uint32_t)(unit >> 32), c2 = blk, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t comp(const uint4& b, int c) {
    return c == 0 ? b.x : c == 1 ? b.y : c == 2 ? b.z : b.w;
}

// Encoded graph in HBM (DESIGN.md "Data layout").  Vertex ids stored in the
// device graph are TAGGED: bits 0-29 the id, bit 30 = "hot row" (the hybrid
// scatter adds to it atomically).  vtab/ntab alias words hold alias | tag(alias)
// << 30 | tag(self) << 31, ctab alias words alias | tag << 30, targets t | tag
// << 30.  Tags are all zero unless a hybrid run set them (capi build_hot_maps);
// every kernel splits them off, so stale tags never change a result.
struct DevGraph {
    const int64_t* offsets;   // V+1
    const int32_t* targets;   // E   tagged target vid
    const uint2* vtab;        // V   {accept threshold, tagged alias word}
    const uint2* ntab;        // V
    const uint2* ctab;        // E   alias already a (tagged) target vid
    // packed copies for the draw kernel (nullptr when E >= 2^32): per vertex
    // entry i two uint4 {thresh, alias word, off(i), deg(i)}, {off(a), deg(a),
    // 0, 0} (a = alias(i)) -- a source draw plus its CSR row in one 32-B read;
    // per edge slot {thresh, tagged alias vid, tagged target, 0}
    const uint4* vt32;
    const uint4* ct16;
    uint32_t V;
};

constexpr int32_t ID_MASK = 0x3FFFFFFF;
__device__ __forceinline__ int32_t untag(int32_t t) { return t & ID_MASK; }
__device__ __forceinline__ bool tag_hot(int32_t t) { return (t >> 30) & 1; }

// index draw floor(k*n/2^32) == interposed random_gen(0, n) truncated.
__device__ __forceinline__ uint32_t draw_index(uint32_t k, uint32_t n) { return __umulhi(k, n); }

// alias draw on a vtab/ntab entry -> tagged id
__device__ __forceinline__ int32_t alias_pick(uint32_t i, uint2 e, uint32_t kp) {
    return kp < e.x ? (int32_t)(i | ((e.y >> 31) << 30)) : (int32_t)(e.y & 0x7FFFFFFFu);
}

// SourceSample src/proNet.cpp:647-657 (p, then index); tagged id
__device__ __forceinline__ int32_t source_sample(const DevGraph& g, uint32_t kp, uint32_t ki) {
    const uint32_t i = draw_index(ki, g.V);
    return alias_pick(i, g.vtab[i], kp);
}

// TargetSample(vid) src/proNet.cpp:671-683 (branch 0 -> -1; p, then index);
// v untagged, result tagged
__device__ __forceinline__ int32_t target_sample(const DevGraph& g, int32_t v, uint32_t kp,
                                                 uint32_t ki) {
    const int64_t off = g.offsets[v];
    const int64_t br = g.offsets[v + 1] - off;
    if (br == 0) return -1;
    const int64_t i = off + draw_index(ki, (uint32_t)br);
    const uint2 e = g.ctab[i];
    const int32_t t = g.targets[i];
    return kp < e.x ? t : (int32_t)e.y;
}

// NegativeSample src/proNet.cpp:623-633 (index FIRST, then p); tagged id
__device__ __forceinline__ int32_t negative_sample(const DevGraph& g, uint32_t ki, uint32_t kp) {
    const uint32_t i = draw_index(ki, g.V);
    return alias_pick(i, g.ntab[i], kp);
}

// fastSigmoid src/proNet.cpp:62-71 on an fp32 dot: bucket index in fp64.
__device__ __forceinline__ float fast_sigmoid(float f, const float* tab) {
    const double x = (double)f;
    if (x < -8.0) return 0.0f;
    if (x > 8.0) return 1.0f;
    return tab[(int)((x + 8.0) * 1000 / 8.0 / 2)];
}

// learning rate of the sample run with counter value c
// (src/model/LINE.cpp:180-184, MF.cpp:95-99, BPR.cpp:95-99)
__device__ __forceinline__ float alpha_at(uint64_t c, double alpha0, uint64_t total) {
    const uint64_t u = c / 10000;
    double a = alpha0;
    if (u != 0) {
        a = alpha0 * (1.0 - (double)((u - 1) * 10000) / (double)total);
        const double amin = alpha0 * 0.0001;
        if (a < amin) a = amin;
    }
    return (float)a;
}

// DeepWalk walk w (src/model/DeepWalk.cpp:141-147)
__device__ __forceinline__ float alpha_walk(uint64_t w, double alpha0, uint64_t total) {
    const uint64_t u = w / 10000;
    double a = alpha0;
    if (u != 0) {
        a = alpha0 * (1.0 - (double)(u * 10000) / (double)total);
        const double amin = alpha0 * 0.0001;
        if (a < amin) a = amin;
    }
    return (float)a;
}

// pairwise-tree sum over the G lanes of a sample group; every lane of the
// group ends with the bit-identical total (IEEE add is commutative).
template <int G>
__device__ __forceinline__ float group_sum(float p) {
#pragma unroll
    for (int m = 1; m < G; m <<= 1) p += __shfl_xor(p, m, G);
    return p;
}

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- row layout (DESIGN.md "Arithmetic spec").  A sample's G lanes own the
// row's 16-B chunks: lane l owns chunks q = l + G*k (k = 0 .. M/4 - 1), and its
// register m holds element 4*(l + G*(m/4)) + m%4.  Every row access is one
// global_load/store_dwordx4 per chunk round: a wave instruction moves 16G
// contiguous bytes of each of the 64/G rows it touches (d = 64: four whole
// 256-B rows).  dpad is a multiple of 4, so a chunk is wholly valid or not.
template <int G>
__device__ __forceinline__ int elem_off(int lane, int m) {
    return 4 * (lane + G * (m >> 2)) + (m & 3);
}

template <int G, int M>
__device__ __forceinline__ void row_valid(bool (&ev)[M], int lane, int dpad) {
#pragma unroll
    for (int m = 0; m < M; ++m) ev[m] = lane + G * (m >> 2) < (dpad >> 2);
}

// r = row (zeros where the chunk does not exist or !use)
template <int G, int M>
__device__ __forceinline__ void ld_row(float (&r)[M], const float* row, int lane, const bool (&ev)[M],
                                       bool use = true) {
#pragma unroll
    for (int k = 0; k < M / 4; ++k) {
        f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
        if (use && ev[4 * k]) x = *reinterpret_cast<const f32x4*>(row + 4 * (lane + G * k));
#pragma unroll
        for (int i = 0; i < 4; ++i) r[4 * k + i] = x[i];
    }
}

template <int G, int M>
__device__ __forceinline__ void st_row(float* row, const float (&r)[M], int lane, const bool (&ev)[M]) {
#pragma unroll
    for (int k = 0; k < M / 4; ++k)
        if (ev[4 * k])
            *reinterpret_cast<f32x4*>(row + 4 * (lane + G * k)) = f32x4{r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]};
}

// row += d by float atomics.  A float atomic moves one dword per lane, so the
// chunks are transposed across the group first (lane shuffles): atomic
// instruction i of round k has lane l add element 4Gk + iG + l, held by lane
// iG/4 + l/4 in register 4k + l%4 -- each instruction covers 4G contiguous
// bytes of the row, not 4 dwords of every 16 B (G < 4: element by element).
template <int G, int M>
__device__ __forceinline__ void atomic_row(float* row, const float (&d)[M], int lane, int dpad) {
#ifdef SMORE_ATOMIC_STRIDED
    if constexpr (true) {
#else
    if constexpr (G < 4) {
#endif
#pragma unroll
        for (int m = 0; m < M; ++m)
            if (lane + G * (m >> 2) < (dpad >> 2)) unsafeAtomicAdd(row + elem_off<G>(lane, m), d[m]);
    } else {
#pragma unroll
        for (int k = 0; k < M / 4; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int s = i * (G / 4) + (lane >> 2);
                float t[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) t[j] = __shfl(d[4 * k + j], s, G);
                const int j = lane & 3;
                const float v = j == 0 ? t[0] : j == 1 ? t[1] : j == 2 ? t[2] : t[3];
                if (G * k + s < (dpad >> 2)) unsafeAtomicAdd(row + 4 * G * k + i * G + lane, v);
            }
    }
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, const float4& v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ void atomic_add4(float* p, const float4& d) {
    unsafeAtomicAdd(p + 0, d.x);
    unsafeAtomicAdd(p + 1, d.y);
    unsafeAtomicAdd(p + 2, d.z);
    unsafeAtomicAdd(p + 3, d.w);
}

__device__ __forceinline__ float4 sub4(const float4& a, const float4& b) {
    return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
__device__ __forceinline__ float4 add4(const float4& a, const float4& b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 fma4(float s, const float4& a, const float4& b) {
    return make_float4(__builtin_fmaf(s, a.x, b.x), __builtin_fmaf(s, a.y, b.y),
                       __builtin_fmaf(s, a.z, b.z), __builtin_fmaf(s, a.w, b.w));
}
// partial dot: fmaf chain in element order starting from p
__device__ __forceinline__ float dot4(const float4& a, const float4& b, float p) {
    p = __builtin_fmaf(a.x, b.x, p);
    p = __builtin_fmaf(a.y, b.y, p);
    p = __builtin_fmaf(a.z, b.z, p);
    p = __builtin_fmaf(a.w, b.w, p);
    return p;
}

}  // namespace smore
