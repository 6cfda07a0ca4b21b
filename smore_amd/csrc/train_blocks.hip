// train_blocks.hip -- draws and records of the 2-D block schedule (blocks.cpp,
// DESIGN.md 10; SURVEY.md 8e's conflict-free multi-GPU layout).
//
// With N GPUs, GPU r owns the W rows of part r (contiguous ids of equal source
// mass) and the C table is cut into nb = 2N blocks (contiguous ids of equal
// negative mass) that rotate around the ring.  A launch trains one cell
// (part r, block b): every sample's source is in part r and its context and
// negatives are in block b, so the N GPUs of a sub-round touch disjoint rows
// of both tables and need no reduction -- the cells' union is one shared table
// pair, as in the reference (src/model/LINE.cpp:160-191, DeepWalk.cpp:128-155).
//
// LINE-2 (block_draw_kernel): the cell's (v, c) pairs are drawn from one alias
// table over the cell's "atoms" -- per CSR slot i of a source v in part r the
// reference's TargetSample outcomes (v, target_i) with mass p(v) * prob_i / deg
// and (v, alias_i) with mass p(v) * (1 - prob_i) / deg (src/proNet.cpp:647-683)
// whose context falls in block b -- so a cell's samples follow the joint law
// of SourceSample x TargetSample restricted to the cell; the K negatives come
// from NegativeSample's law restricted to block b (:623-633).  Philox slots as
// draw_kernel: word 0 p, word 1 the atom index, negatives from block 1 + j/2.
//
// Walk models (block_pair_count / emit): every GPU runs every walk of a round
// (deterministic per walk index) and keeps the skip-gram pairs whose center is
// in its part, bucketed by the context's block; a pair's negatives come from
// its block's restricted law (same slots as pair_emit_kernel, the index drawn
// over the block).  Buckets keep walk order, so a bucket's records are the
// one-GPU records restricted to the cell, in order.  The group driver walks
// 1/N of a round per GPU and broadcasts the slices (exchange.cpp); the count
// and the emit run one wave per walk (block_pairs_wave_kernel).
#include "train_kernels.h"

#include <string>

namespace smore {

__device__ __forceinline__ int block_of(const BlockArgs& b, int32_t x) {
    int lo = 0, hi = b.nb;   // cb[lo] <= x < cb[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (x >= b.cb[mid]) lo = mid;
        else hi = mid;
    }
    return lo;
}

// a negative of block k: index over the block's rows and the H hub slots,
// alias entry of vertex cb[k] + i, or of hub slot j = i - rows (id V + j)
__device__ __forceinline__ int32_t block_negative(const BlockArgs& b, int k, uint32_t ki, uint32_t kp) {
    const int32_t lo = b.cb[k];
    const uint32_t nk = (uint32_t)(b.cb[k + 1] - lo);
    const uint32_t i = draw_index(ki, nk + (uint32_t)b.H);
    if (i < nk) return alias_pick((uint32_t)lo + i, b.ntab[(uint32_t)lo + i], kp);
    const uint32_t j = i - nk;
    return alias_pick((uint32_t)b.V + j, b.hub_ntab[(uint64_t)k * (uint32_t)b.H + j], kp);
}

template <int KMAX>
__global__ void __launch_bounds__(256) block_draw_kernel(BlockArgs b, int blk, uint64_t seed, uint64_t begin,
                                                         uint64_t count, int K, int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    const uint4 b0 = philox_block(seed, 0, s, 0);
    // a hub atom of the part (word 2 against the cell's hub share), else one
    // of the block's own atoms
    const bool hub = b.nhub > 0 && (b.natoms == 0 || b0.z < b.hub_thr);
    const uint64_t ai = hub ? b.hub_off + draw_index(b0.y, b.nhub) : b.atom_off + draw_index(b0.y, b.natoms);
    const uint4 e0 = b.atoms[2 * ai], e1 = b.atoms[2 * ai + 1];
    const bool acc = b0.x < e0.x;
    int32_t w[RW];
    w[0] = (int32_t)(acc ? e0.y : e1.x);
    w[1] = (int32_t)(acc ? e0.z : e1.y);
#pragma unroll
    for (int j = 0; j < RW - 2; ++j) w[2 + j] = -1;
#pragma unroll
    for (int j = 0; j < KMAX; j += 2) {
        if (j < K) {
            const uint4 q = philox_block(seed, 0, s, 1 + j / 2);
            w[2 + j] = block_negative(b, blk, q.x, q.y);
            if (j + 1 < KMAX && j + 1 < K) w[3 + j] = block_negative(b, blk, q.z, q.w);
        }
    }
    i32x4* o = reinterpret_cast<i32x4*>(rec + t * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) {
        const i32x4 x = {w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        __builtin_nontemporal_store(x, o + q);
    }
}

__global__ void __launch_bounds__(256) rows_gather_kernel(const float4* __restrict__ T, const int32_t* __restrict__ idx,
                                                          uint64_t n4, int dp4, float4* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = T[(uint64_t)idx[i / dp4] * dp4 + i % dp4];
}

__global__ void __launch_bounds__(256) rows_scatter_kernel(float4* __restrict__ T, const int32_t* __restrict__ idx,
                                                           uint64_t n4, int dp4, const float4* __restrict__ in) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        T[(uint64_t)idx[i / dp4] * dp4 + i % dp4] = in[i];
}

static unsigned rows_grid(uint64_t n4) {
    const uint64_t g = (n4 + 255) / 256;
    return (unsigned)(g < 4096 ? (g ? g : 1) : 4096);
}

hipError_t launch_rows_gather(const float* T, const int32_t* idx, uint64_t n, int dpad, float* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t n4 = n * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(rows_gather_kernel, dim3(rows_grid(n4)), dim3(256), 0, st, reinterpret_cast<const float4*>(T),
                       idx, n4, dpad / 4, reinterpret_cast<float4*>(out));
    return hipGetLastError();
}

hipError_t launch_rows_scatter(float* T, const int32_t* idx, uint64_t n, int dpad, const float* in, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t n4 = n * (uint64_t)(dpad / 4);
    hipLaunchKernelGGL(rows_scatter_kernel, dim3(rows_grid(n4)), dim3(256), 0, st, reinterpret_cast<float4*>(T), idx,
                       n4, dpad / 4, reinterpret_cast<const float4*>(in));
    return hipGetLastError();
}

hipError_t launch_block_draw(const BlockArgs& b, int blk, uint64_t seed, uint64_t begin, uint64_t count, int K,
                             int32_t* rec, hipStream_t st) {
    const int block = 256;
    const dim3 grid((unsigned)((count + block - 1) / block));
    switch (kmax_of(K)) {
        case 5: hipLaunchKernelGGL(block_draw_kernel<5>, grid, dim3(block), 0, st, b, blk, seed, begin, count, K, rec); break;
        case 10: hipLaunchKernelGGL(block_draw_kernel<10>, grid, dim3(block), 0, st, b, blk, seed, begin, count, K, rec); break;
        default: hipLaunchKernelGGL(block_draw_kernel<20>, grid, dim3(block), 0, st, b, blk, seed, begin, count, K, rec); break;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- walk pairs
struct WalkWordsB {   // consecutive Philox words of one walk (stream 1), as train_pairs.hip
    uint64_t seed, unit;
    uint32_t blk = 0xFFFFFFFFu;
    uint4 q;
    __device__ uint32_t operator()(uint32_t slot) {
        if ((slot >> 2) != blk) {
            blk = slot >> 2;
            q = philox_block(seed, 1, unit, blk);
        }
        return comp(q, (int)(slot & 3));
    }
};

// Walklets' ranges (ScaleSkipGrams src/proNet.cpp:928-987, as train_pairs.hip)
__device__ __forceinline__ void scale_ranges(int i, int L, int wmin, int wmax, int (&rg)[2][2]) {
    rg[0][0] = i - wmax < 0 ? 0 : i - wmax;
    rg[0][1] = i - wmin < 0 ? 0 : i - wmin;
    rg[1][0] = i + wmin >= L ? L - 1 : i + wmin;
    rg[1][1] = i + wmax >= L ? L - 1 : i + wmax;
}

// a walk pair's block and C word: the context's block and tagged id, or for
// a hub context (b.hub_of) block (walk + i) mod nb and its slot id
__device__ __forceinline__ int pair_block(const BlockArgs& b, int32_t cj, uint64_t walk, int i, int32_t& cw) {
    const int32_t x = cj & ID_MASK;
    if (b.hub_of) {
        const int32_t h = b.hub_of[x];
        if (h >= 0) {
            cw = (b.V + (h & ID_MASK)) | (h & (1 << 30));
            return (int)((walk + (uint64_t)i) % (uint64_t)b.nb);
        }
    }
    cw = cj & (ID_MASK | (1 << 30));
    return block_of(b, x);
}

// per (block, walk) pair counts of the owned centers: count[k * nwalks + t]
__global__ void __launch_bounds__(256) block_pair_count_kernel(WalkArgs w, BlockArgs b, uint64_t seed,
                                                               uint32_t* count) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    uint32_t cnt[BLOCK_MAX];
    for (int k = 0; k < b.nb; ++k) cnt[k] = 0;
    const int L = w.lens[t];
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    WalkWordsB wd{seed, w.walk_begin + t};
    const uint32_t win_base = 2u * (uint32_t)(L - 1);
    for (int i = 0; i < L; ++i) {
        int rg[2][2];
        int nr = 1;
        if (w.rule == 1) {
            scale_ranges(i, L, w.window_min, w.window, rg);
            nr = 2;
        } else {
            const int r = (int)draw_index(wd(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
            rg[0][0] = i - r < 0 ? 0 : i - r;
            rg[0][1] = i + r >= L ? L - 1 : i + r;
        }
        const int32_t v = walk[i] & ID_MASK;
        if (v < w.own_lo || v >= w.own_hi) continue;
        for (int q = 0; q < nr; ++q)
            for (int j = rg[q][0]; j <= rg[q][1]; ++j)
                if (j != i) {
                    int32_t cw;
                    cnt[pair_block(b, walk[j], w.walk_begin + t, i, cw)]++;
                }
    }
    for (int k = 0; k < b.nb; ++k) count[(uint64_t)k * w.nwalks + t] = cnt[k];
}

template <int KMAX>
__global__ void __launch_bounds__(256) block_pair_emit_kernel(WalkArgs w, BlockArgs b, uint64_t seed, int K,
                                                              double alpha0, const uint64_t* off, int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    uint64_t cur[BLOCK_MAX];
    for (int k = 0; k < b.nb; ++k) cur[k] = off[(uint64_t)k * w.nwalks + t];
    const int L = w.lens[t];
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    const uint64_t unit = w.walk_begin + t;
    const float alpha = alpha_walk(unit, alpha0, w.total_walks);
    WalkWordsB win{seed, unit}, neg{seed, unit};
    const uint32_t win_base = 2u * (uint32_t)(L - 1);
    // negatives follow the walk's draws (and DeepWalk's L window draws)
    uint32_t slot = win_base + (w.rule == 1 ? 0u : (uint32_t)L);
    for (int i = 0; i < L; ++i) {
        int rg[2][2];
        int nr = 1;
        if (w.rule == 1) {
            scale_ranges(i, L, w.window_min, w.window, rg);
            nr = 2;
        } else {
            const int r = (int)draw_index(win(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
            rg[0][0] = i - r < 0 ? 0 : i - r;
            rg[0][1] = i + r >= L ? L - 1 : i + r;
        }
        const int32_t vi = walk[i];
        const int32_t v = vi & ID_MASK;
        const bool own = v >= w.own_lo && v < w.own_hi;
        for (int q = 0; q < nr; ++q)
            for (int j = rg[q][0]; j <= rg[q][1]; ++j) {
                if (j == i) continue;
                if (!own) {   // another part's pair: its draws only
                    slot += 2u * (uint32_t)K;
                    continue;
                }
                int32_t cw;
                const int k = pair_block(b, walk[j], unit, i, cw);
                int32_t x[RW];
                // W row walk[i] with its W tag, C row walk[j] (or its hub slot) with its C tag
                x[0] = v | (int32_t)((((uint32_t)vi >> 31) & 1u) << 30);
                x[1] = cw;
#pragma unroll
                for (int n = 0; n < RW - 2; ++n) x[2 + n] = -1;
#pragma unroll
                for (int n = 0; n < KMAX; ++n)
                    if (n < K) x[2 + n] = block_negative(b, k, neg(slot + 2u * (uint32_t)n), neg(slot + 2u * (uint32_t)n + 1u));
                x[2 + KMAX] = __float_as_int(alpha);
                slot += 2u * (uint32_t)K;
                i32x4* o = reinterpret_cast<i32x4*>(rec + cur[k] * RW);
                cur[k] += 1;
#pragma unroll
                for (int qq = 0; qq < RW / 4; ++qq) {
                    const i32x4 y = {x[4 * qq], x[4 * qq + 1], x[4 * qq + 2], x[4 * qq + 3]};
                    __builtin_nontemporal_store(y, o + qq);
                }
            }
    }
}

// ---- the same count and emit with one wave per walk.  The kernels above give
// a thread a whole walk: 2^18 threads per round, each looping over ~40
// positions with its 2N block cursors in scratch (C5, 8 parts: emit 3.0 ms,
// count 0.8 ms of a 20-30 ms part epoch).  Here lane i takes position i (64
// at a time) and its pair counts are scanned across the wave: all pairs for
// the negatives' Philox words (a position's start after every earlier pair's,
// own or not), the owned ones for the records.  The records are then spread
// over the lanes (lane r: record r of the chunk, looked up in the wave's LDS
// tables), so a part's 1/N of the positions does not idle the other lanes
// through the K negative draws; a record's place in block k is the walk's
// base for k plus its rank among the lanes' block-k records (ballots).  Same
// words, same records, same order as the per-walk kernels (bit-exact).
constexpr int WALKS_PER_BLOCK = 4;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// LDS written by one lane and read by another of the same wave: the writes
// complete (s_waitcnt) and the compiler keeps the order
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// position i's context ranges (as the per-walk kernels) and its pair count
__device__ __forceinline__ uint32_t position_ranges(const WalkArgs& w, WalkWordsB& wd, uint32_t win_base, int i,
                                                    int L, int (&rg)[2][2], int& nr) {
    if (w.rule == 1) {
        scale_ranges(i, L, w.window_min, w.window, rg);
        nr = 2;
    } else {
        const int r = (int)draw_index(wd(win_base + (uint32_t)i), (uint32_t)w.window) + 1;
        rg[0][0] = i - r < 0 ? 0 : i - r;
        rg[0][1] = i + r >= L ? L - 1 : i + r;
        nr = 1;
    }
    uint32_t n = 0;
    for (int q = 0; q < nr; ++q)
        if (rg[q][1] >= rg[q][0]) n += (uint32_t)(rg[q][1] - rg[q][0] + 1) - (i >= rg[q][0] && i <= rg[q][1] ? 1u : 0u);
    return n;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t x, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

template <int KMAX, bool EMIT>
__global__ void __launch_bounds__(256) block_pairs_wave_kernel(WalkArgs w, BlockArgs b, uint64_t seed, int K,
                                                               double alpha0, const uint64_t* off, uint32_t* count,
                                                               int32_t* rec) {
    constexpr int RW = rec_width(KMAX);
    // per wave: the chunk's owned-pair prefix (e), negative-word start (s0)
    // and context ranges of each position, for the record lanes to look up
    __shared__ uint32_t s_e[WALKS_PER_BLOCK][65];
    __shared__ uint32_t s_s0[WALKS_PER_BLOCK][64];
    __shared__ int4 s_rg[WALKS_PER_BLOCK][64];
    const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const uint64_t t = (uint64_t)blockIdx.x * WALKS_PER_BLOCK + (uint64_t)wv;
    if (t >= w.nwalks) return;   // whole waves: nothing below syncs the block
    const int nb = b.nb;
    const int L = w.lens[t];
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    const uint64_t unit = w.walk_begin + t;
    const float alpha = alpha_walk(unit, alpha0, w.total_walks);
    WalkWordsB win{seed, unit}, neg{seed, unit};
    const uint32_t win_base = 2u * (uint32_t)(L - 1);
    uint32_t slot_run = win_base + (w.rule == 1 ? 0u : (uint32_t)L);   // the chunk's first negative word
    // lane k < nb: block k's next record of this walk (emit) / its pairs (count)
    uint64_t kb = (EMIT && lane < nb) ? off[(uint64_t)lane * w.nwalks + t] : 0;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;   // lanes below this one
    for (int p0 = 0; p0 < L; p0 += 64) {
        const int i = p0 + lane;
        int rg[2][2] = {{0, -1}, {0, -1}};
        int nr = 0;
        uint32_t np = 0;
        bool own = false;
        if (i < L) {
            np = position_ranges(w, win, win_base, i, L, rg, nr);
            const int32_t v = walk[i] & ID_MASK;
            own = v >= w.own_lo && v < w.own_hi;
        }
        // every pair draws 2K negative words, own or not; owned pairs become records
        const uint32_t incl = wave_incl_scan(np, lane);
        const uint32_t no = own ? np : 0u, oincl = wave_incl_scan(no, lane);
        const uint32_t T = (uint32_t)__shfl((int)oincl, 63, 64);
        s_e[wv][lane] = oincl - no;
        if (lane == 63) s_e[wv][64] = oincl;
        s_s0[wv][lane] = slot_run + 2u * (uint32_t)K * (incl - np);
        s_rg[wv][lane] = make_int4(rg[0][0], rg[0][1], nr == 2 ? rg[1][0] : 0, nr == 2 ? rg[1][1] : -1);
        slot_run += 2u * (uint32_t)K * (uint32_t)__shfl((int)incl, 63, 64);
        wave_lds_sync();
        // the chunk's T records, 64 at a time: record r is pair m of position
        // li, the last lane whose prefix is <= r
        for (uint32_t r0 = 0; r0 < T; r0 += 64) {
            const uint32_t r = r0 + (uint32_t)lane;
            const bool act = r < T;
            int k = -1, li = 0, j = 0;
            uint32_t m = 0;
            int32_t cw = 0;
            if (act) {
                int lo = 0, hi = 64;   // s_e[lo] <= r < s_e[hi]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (s_e[wv][mid] <= r) lo = mid;
                    else hi = mid;
                }
                li = lo;
                m = r - s_e[wv][li];
                const int ip = p0 + li;
                const int4 g = s_rg[wv][li];
                // the m-th context of position ip: its ranges in order, ip skipped
                uint32_t x = m;
                int a0 = g.x, a1 = g.y;
                uint32_t n0 = a1 >= a0 ? (uint32_t)(a1 - a0 + 1) - (ip >= a0 && ip <= a1 ? 1u : 0u) : 0u;
                if (x >= n0) {
                    x -= n0;
                    a0 = g.z;
                    a1 = g.w;
                }
                j = a0 + (int)x;
                if (ip >= a0 && ip <= a1 && j >= ip) ++j;
                k = pair_block(b, walk[j], unit, ip, cw);
            }
            // the record's place in block k: after every earlier record of k
            // (this walk's base for k from lane k, its rank among the lanes)
            uint32_t rank = 0;
            uint64_t base = 0;
            for (int kk = 0; kk < nb; ++kk) {
                const uint64_t mask = __ballot(k == kk);
                const uint64_t bk = shfl_u64(kb, kk);
                if (k == kk) {
                    rank = (uint32_t)__popcll(mask & lt);
                    base = bk;
                }
                if (lane == kk) kb += (uint64_t)__popcll(mask);
            }
            if (EMIT && act) {
                const int ip = p0 + li;
                const int32_t vi = walk[ip];
                const uint32_t slot = s_s0[wv][li] + 2u * (uint32_t)K * m;
                int32_t xr[RW];
                xr[0] = (vi & ID_MASK) | (int32_t)((((uint32_t)vi >> 31) & 1u) << 30);
                xr[1] = cw;
#pragma unroll
                for (int n = 0; n < RW - 2; ++n) xr[2 + n] = -1;
#pragma unroll
                for (int n = 0; n < KMAX; ++n)
                    if (n < K)
                        xr[2 + n] = block_negative(b, k, neg(slot + 2u * (uint32_t)n), neg(slot + 2u * (uint32_t)n + 1u));
                xr[2 + KMAX] = __float_as_int(alpha);
                i32x4* o = reinterpret_cast<i32x4*>(rec + (base + rank) * RW);
#pragma unroll
                for (int qq = 0; qq < RW / 4; ++qq) {
                    const i32x4 y = {xr[4 * qq], xr[4 * qq + 1], xr[4 * qq + 2], xr[4 * qq + 3]};
                    __builtin_nontemporal_store(y, o + qq);
                }
            }
        }
        wave_lds_sync();   // the next chunk rewrites the wave's tables
    }
    if (!EMIT && lane < nb) count[(uint64_t)lane * w.nwalks + t] = (uint32_t)kb;
}

// which kernels (SMORE_WALK_PAIR_KERNELS): "wave" (default) or "walk" (the
// per-walk ones); windows wider than a wave's chunk can hold take the per-walk
bool wave_pairs_ok(const WalkArgs& w, bool) {
    const char* e = getenv("SMORE_WALK_PAIR_KERNELS");
    if (e && std::string(e) == "walk") return false;
    return w.window > 0 && w.window < 1024;
}

hipError_t launch_block_pair_count(const WalkArgs& w, const BlockArgs& b, uint64_t seed, uint32_t* count,
                                   hipStream_t st) {
    const int block = 256;
    if (wave_pairs_ok(w, false)) {
        const dim3 grid((unsigned)((w.nwalks + WALKS_PER_BLOCK - 1) / WALKS_PER_BLOCK));
        hipLaunchKernelGGL((block_pairs_wave_kernel<5, false>), grid, dim3(block), 0, st, w, b, seed, 0, 0.0, nullptr,
                           count, nullptr);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(block_pair_count_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st,
                       w, b, seed, count);
    return hipGetLastError();
}

hipError_t launch_block_pair_emit(const WalkArgs& w, const BlockArgs& b, uint64_t seed, int K, double alpha0,
                                  const uint64_t* off, int32_t* rec, hipStream_t st) {
    const int block = 256;
    if (wave_pairs_ok(w, true)) {
        const dim3 grid((unsigned)((w.nwalks + WALKS_PER_BLOCK - 1) / WALKS_PER_BLOCK));
        if (kmax_of(K) == 5)
            hipLaunchKernelGGL((block_pairs_wave_kernel<5, true>), grid, dim3(block), 0, st, w, b, seed, K, alpha0, off,
                               nullptr, rec);
        else
            hipLaunchKernelGGL((block_pairs_wave_kernel<10, true>), grid, dim3(block), 0, st, w, b, seed, K, alpha0,
                               off, nullptr, rec);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((w.nwalks + block - 1) / block));
    if (kmax_of(K) == 5)
        hipLaunchKernelGGL(block_pair_emit_kernel<5>, grid, dim3(block), 0, st, w, b, seed, K, alpha0, off, rec);
    else
        hipLaunchKernelGGL(block_pair_emit_kernel<10>, grid, dim3(block), 0, st, w, b, seed, K, alpha0, off, rec);
    return hipGetLastError();
}

}  // namespace smore
