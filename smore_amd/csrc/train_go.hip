// train_go.hip -- Go-semantics kernels, the rules of
// pkg/pronet/{pronet,alias,optimizer}.go and internal/models/{line,bpr,deepwalk}:
//   * draws: aliasSample takes the index first (alias.go:99-100); TargetSample
//     is a CDF scan over the raw weights (pronet.go:257-284), done here as a
//     binary search over the same sequential fp64 prefix sums;
//   * UpdatePair (optimizer.go:21-58): negatives equal to the positive are
//     skipped (not redrawn), negatives update C_n immediately, the positive
//     context's gradient and W_v's are applied at the end;
//   * LINE order 1, BPR: on records, go_rec.h (this file draws them:
//     go_draw_kernel);
//   * DeepWalk: walks stop at a dead end, fixed window (pronet.go:292-333);
//     the walks' pairs become records (go_pair_emit_kernel) for go_rec.h
//     go_pair_kernel;
//   * node2vec: the biased second-order walk (internal/models/node2vec), then
//     the DeepWalk pairs;
//   * metapath2vec: meta-path-typed uniform walks (internal/models/metapath2vec,
//     pkg/hetero), then the DeepWalk pairs.
// fp32 arithmetic without fused multiply-adds (amd64 Go does not fuse); the
// oracle's orc_go_*_f32 is the bit-exact spec.  Same lane layout as
// edge_kernels.h.
#include "edge_kernels.h"
#include "go_walks.h"

namespace smore {

__device__ __forceinline__ int32_t go_alias(const uint2* tab, uint32_t n, uint32_t ki, uint32_t kp) {
    const uint32_t i = draw_index(ki, n);
    const uint2 e = tab[i];
    return kp < e.x ? (int32_t)i : untag((int32_t)e.y);   // ids untagged (no hybrid scatter here)
}

// Go TargetSample (untagged id).  tcum == nullptr: every edge weight is 1, so
// the CDF is e + 1 exactly and the first e with r <= e + 1 is ceil(r) - 1 (as
// go_target_tagged's unit_w path) -- no binary search over the prefix sums.
__device__ __forceinline__ int32_t go_target(const DevGraph& g, const double* tcum, int32_t v, uint32_t kr) {
    const int64_t off = g.offsets[v];
    const int64_t br = g.offsets[v + 1] - off;
    if (br == 0) return -1;
    int64_t lo;
    if (!tcum) {
        lo = (int64_t)ceil(ldexp((double)kr, -32) * (double)br) - 1;
        lo = lo < 0 ? 0 : (lo > br - 1 ? br - 1 : lo);
    } else {
        const double r = ldexp((double)kr, -32) * tcum[off + br - 1];
        int64_t hi = br - 1;
        lo = 0;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (r <= tcum[off + mid]) hi = mid;
            else lo = mid + 1;
        }
    }
    return untag(g.targets[off + lo]);
}

// Go RandomWalk: stops at a dead end; step s draws slot s (stream 1).
__global__ void go_walk_gen_kernel(DevGraph g, const double* tcum, WalkArgs w, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const uint64_t unit = w.walk_begin + t;
    int32_t* out = w.walks + t * (uint64_t)(w.steps + 1);
    int L = 0;
    int32_t cur = (int32_t)w.order[unit - w.order_base];
    out[L++] = cur;
    uint4 b = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < w.steps; ++s) {
        if (g.offsets[cur + 1] - g.offsets[cur] == 0) break;
        if ((s & 3) == 0) b = philox_block(seed, 1, unit, (uint32_t)s >> 2);
        cur = go_target(g, tcum, cur, comp(b, s & 3));
        out[L++] = cur;
    }
    w.lens[t] = L;
}

// areNeighbors(a, b) (internal/models/node2vec/node2vec.go:167-175): a linear
// scan of Graph[a] there; membership does not depend on the order, so here a
// binary search in a's sorted copy of its CSR targets.
__device__ __forceinline__ bool n2v_adjacent(const DevGraph& g, const int32_t* nbr, int32_t a, int32_t b) {
    int64_t lo = g.offsets[a], hi = g.offsets[a + 1];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t x = nbr[mid];
        if (x == b) return true;
        if (x < b) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

// node2vec biased weight of Graph[cur][i] after prev (node2vec.go:126-146)
__device__ __forceinline__ double n2v_weight(const DevGraph& g, const WalkArgs& w, int32_t prev, int64_t e) {
    const int32_t nb = untag(g.targets[e]);
    const double bias = nb == prev ? w.inv_p : (n2v_adjacent(g, w.nbr_sorted, prev, nb) ? 1.0 : w.inv_q);
    return w.wts[e] * bias;
}

// biasedRandomWalk (node2vec.go:82-110): the first step is Go's TargetSample,
// every later step biasedTargetSample (:114-164) -- total of the biased weights
// in the Go loop's order, r = Float64() * total, first i with r <= cum_i (the
// last neighbour if rounding leaves none; Intn(deg) when total == 0).  Step s
// draws slot s of stream 1 (as the Go RandomWalk); a dead end stops the walk
// before drawing.
//
// One wavefront per walk: hub vertices make a step cost O(deg) membership
// tests, so the 64 lanes compute the biased weights of 64 edges at a time and
// every lane then adds the 64 values in edge order through lane shuffles --
// the sums keep the Go loop's sequential fp64 order (bit-exact), only the
// membership tests run in parallel.  All control flow is wave-uniform.
constexpr int N2V_WAVES = 4;   // walks per 256-thread block
__global__ void __launch_bounds__(256) go_n2v_walk_gen_kernel(DevGraph g, const double* tcum, WalkArgs w,
                                                              uint64_t seed) {
    const int lane = threadIdx.x & 63;
    const uint64_t t = (uint64_t)blockIdx.x * N2V_WAVES + (threadIdx.x >> 6);
    if (t >= w.nwalks) return;   // whole waves leave together
    const uint64_t unit = w.walk_begin + t;
    int32_t* out = w.walks + t * (uint64_t)(w.steps + 1);
    int L = 0;
    int32_t prev = -1, cur = (int32_t)w.order[unit - w.order_base];
    if (lane == 0) out[L] = cur;
    ++L;
    uint4 b = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < w.steps; ++s) {
        const int64_t off = g.offsets[cur], deg = g.offsets[cur + 1] - off;
        if (deg == 0) break;
        if ((s & 3) == 0) b = philox_block(seed, 1, unit, (uint32_t)s >> 2);
        const uint32_t k = comp(b, s & 3);
        int32_t next;
        if (s == 0) {
            next = go_target(g, tcum, cur, k);
        } else {
            double total = 0.0;
            for (int64_t base = 0; base < deg; base += 64) {
                const int64_t e = base + lane;
                const double bw = e < deg ? n2v_weight(g, w, prev, off + e) : 0.0;
                const int cnt = (int)(deg - base < 64 ? deg - base : 64);
                for (int i = 0; i < cnt; ++i) total += __shfl(bw, i, 64);
            }
            int64_t pick = deg - 1;
            if (total == 0.0) {
                pick = draw_index(k, (uint32_t)deg);
            } else {
                const double r = ldexp((double)k, -32) * total;
                double cum = 0.0;
                bool found = false;
                for (int64_t base = 0; base < deg && !found; base += 64) {
                    const int64_t e = base + lane;
                    const double bw = e < deg ? n2v_weight(g, w, prev, off + e) : 0.0;
                    const int cnt = (int)(deg - base < 64 ? deg - base : 64);
                    for (int i = 0; i < cnt; ++i) {
                        cum += __shfl(bw, i, 64);
                        if (r <= cum) {
                            pick = base + i;
                            found = true;
                            break;
                        }
                    }
                }
            }
            next = untag(g.targets[off + pick]);
        }
        prev = cur;
        cur = next;
        if (lane == 0) out[L] = cur;
        ++L;
    }
    if (lane == 0) w.lens[t] = L;
}

// metapath2vec walk (internal/models/metapath2vec/metapath2vec.go:184-188,
// pkg/hetero/hetero_graph.go:206-256): slot 0 picks the meta-path
// (Intn(len(metaPaths))); while the walk is shorter than steps + 1 the
// current vertex must have the path's current type, and the next vertex is a
// uniform pick (Intn, the next slot) among its neighbours of the next type, in
// push order.  A type mismatch or no such neighbour ends the walk before
// drawing.
__global__ void go_mp_walk_gen_kernel(WalkArgs w, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const uint64_t unit = w.walk_begin + t;
    int32_t* out = w.walks + t * (uint64_t)(w.steps + 1);
    int32_t cur = (int32_t)w.order[unit - w.order_base];
    out[0] = cur;
    uint4 b = philox_block(seed, 1, unit, 0);
    const int pi = (int)draw_index(comp(b, 0), (uint32_t)w.npaths);
    const int32_t* path = w.paths + w.path_off[pi];
    const int plen = w.path_off[pi + 1] - w.path_off[pi];
    int L = 1;
    if (plen >= 2) {
        for (int idx = 0; L < w.steps + 1; ++idx) {
            if (w.ntype[cur] != path[idx % plen]) break;
            const int nt = path[(idx + 1) % plen];
            const int64_t* to = w.toff + (int64_t)cur * (w.ntypes + 1);
            const int64_t lo = to[nt], n = to[nt + 1] - lo;
            if (n == 0) break;
            const uint32_t s = (uint32_t)L;   // slot L: the step's Intn
            if ((s & 3) == 0) b = philox_block(seed, 1, unit, s >> 2);
            cur = w.ttargets[lo + draw_index(comp(b, s & 3), (uint32_t)n)];
            out[L++] = cur;
        }
    }
    w.lens[t] = L;
}

// CTDNE walk (internal/models/ctdne/ctdne.go:159-188, pkg/temporal/
// temporal_graph.go:181-252).  A start vertex without edges (active range
// {0, 0}) trains nothing and draws nothing.  Slot 0: startTime = min +
// Float64() * (max - min, or timeWindow when 0).  Each step: the out-edges of
// cur with timestamp in [t, min(t + timeWindow, MaxTime)] -- contiguous in the
// time-sorted list, found by binary search -- one picked by Intn (the next
// slot); the walk moves to its target and, as the Go code does, to the
// timestamp of the idx-th out-edge of cur overall (OutEdges[cur][idx]).
__global__ void go_ctdne_walk_gen_kernel(TemporalArgs tg, WalkArgs w, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const uint64_t unit = w.walk_begin + t;
    int32_t* out = w.walks + t * (uint64_t)(w.steps + 1);
    int32_t cur = (int32_t)w.order[unit - w.order_base];
    out[0] = cur;
    int L = 1;
    const double lo_t = tg.tmin[cur], hi_t = tg.tmax[cur];
    if (!(lo_t == 0.0 && hi_t == 0.0)) {
        uint4 b = philox_block(seed, 1, unit, 0);
        double range = hi_t - lo_t;
        if (range == 0.0) range = tg.window;
        double now = lo_t + ldexp((double)comp(b, 0), -32) * range;
        while (L < w.steps + 1) {
            double end = now + tg.window;
            if (end > tg.max_time) end = tg.max_time;
            const int64_t off = tg.off[cur], deg = tg.off[cur + 1] - off;
            int64_t a = 0, z = deg;   // first edge with ts >= now
            while (a < z) {
                const int64_t m = (a + z) >> 1;
                if (tg.ts[off + m] >= now) z = m;
                else a = m + 1;
            }
            int64_t e = a, y = deg;   // first edge with ts > end (from a)
            while (e < y) {
                const int64_t m = (e + y) >> 1;
                if (tg.ts[off + m] > end) y = m;
                else e = m + 1;
            }
            const int64_t n = e - a;
            if (n <= 0) break;
            const uint32_t s = (uint32_t)L;
            if ((s & 3) == 0) b = philox_block(seed, 1, unit, s >> 2);
            const int64_t idx = (int64_t)draw_index(comp(b, s & 3), (uint32_t)n);
            cur = tg.tgt[off + a + idx];
            now = tg.ts[off + idx];
            out[L++] = cur;
        }
    }
    w.lens[t] = L;
}

hipError_t launch_go_ctdne_walk(const TemporalArgs& tg, const WalkArgs& w, uint64_t seed, hipStream_t st) {
    const int block = 256;
    hipLaunchKernelGGL(go_ctdne_walk_gen_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st,
                       tg, w, seed);
    return hipGetLastError();
}

// Go TargetSample keeping the target's tag (hybrid scatter).  unit_w: every
// edge weight is 1, so tcum[off + e] == e + 1 exactly and the first e with
// r <= tcum[off + e] is max(0, ceil(r) - 1) -- the binary search's answer
// without its reads (r is the same fp64 product as go_target's).
__device__ __forceinline__ int32_t go_target_tagged(const DevGraph& g, const double* tcum, int32_t v, uint32_t kr,
                                                    int unit_w) {
    const int64_t off = g.offsets[v];
    const int64_t br = g.offsets[v + 1] - off;
    if (br == 0) return -1;
    int64_t lo;
    if (unit_w) {
        const double r = ldexp((double)kr, -32) * (double)br;
        lo = (int64_t)ceil(r) - 1;
        lo = lo < 0 ? 0 : (lo > br - 1 ? br - 1 : lo);
    } else {
        const double r = ldexp((double)kr, -32) * tcum[off + br - 1];
        int64_t hi = br - 1;
        lo = 0;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (r <= tcum[off + mid]) hi = mid;
            else lo = mid + 1;
        }
    }
    return g.targets[off + lo];
}

// The sampling half of the Go edge models (LINE::Train / BPR::Train / HPE
// loops of internal/models): per sample one record {v, c, n_1 .. n_K, -1 ..}
// of tagged ids for go_rec_kernel (go_rec.h), Go slot layout (stream 0: 0
// source index, 1 source p, 2 target, 3 + 2j negative index, 4 + 2j its p).
// c = -1 when the source has no out-edge (counted in *skipped).
template <int KMAX>
__global__ void __launch_bounds__(256) go_draw_kernel(DevGraph g, const double* tcum, int unit_w, uint64_t seed,
                                                      uint64_t begin, uint64_t count, int K, int32_t* rec,
                                                      unsigned long long* skipped) {
    constexpr int RW = rec_width(KMAX);
    constexpr int NW = 3 + 2 * KMAX;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    uint32_t w[(NW + 3) / 4 * 4];
#pragma unroll
    for (int b = 0; b < (NW + 3) / 4; ++b) {
        if (4 * b < 3 + 2 * K) {
            const uint4 x = philox_block(seed, 0, s, (uint32_t)b);
            w[4 * b] = x.x; w[4 * b + 1] = x.y; w[4 * b + 2] = x.z; w[4 * b + 3] = x.w;
        }
    }
    const uint32_t vi = draw_index(w[0], g.V);
    int32_t v, c;
    if (g.vt32) {
        // the source draw and its CSR row from one packed 32-B entry
        // (train_draw.hip pack_vertex_kernel), as the C++ draw kernel
        const uint4 p0 = g.vt32[2 * (uint64_t)vi], p1 = g.vt32[2 * (uint64_t)vi + 1];
        const bool acc = w[1] < p0.x;
        v = alias_pick(vi, make_uint2(p0.x, p0.y), w[1]);
        const uint64_t off = acc ? p0.z : p1.x;
        const uint32_t br = acc ? p0.w : p1.y;
        c = -1;
        if (br != 0) {
            int64_t lo;
            if (unit_w) {
                lo = (int64_t)ceil(ldexp((double)w[2], -32) * (double)br) - 1;
                lo = lo < 0 ? 0 : (lo > (int64_t)br - 1 ? (int64_t)br - 1 : lo);
            } else {
                const double r = ldexp((double)w[2], -32) * tcum[off + br - 1];
                int64_t hi = br - 1;
                lo = 0;
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (r <= tcum[off + mid]) hi = mid;
                    else lo = mid + 1;
                }
            }
            c = g.targets[off + lo];
        }
    } else {
        v = alias_pick(vi, g.vtab[vi], w[1]);
        c = go_target_tagged(g, tcum, untag(v), w[2], unit_w);
    }
    int32_t o[RW];
    o[0] = v;
    o[1] = c;
#pragma unroll
    for (int j = 0; j < RW - 2; ++j) {
        o[2 + j] = -1;
        if (j < KMAX && j < K) {
            const uint32_t ni = draw_index(w[3 + 2 * j], g.V);
            o[2 + j] = alias_pick(ni, g.ntab[ni], w[4 + 2 * j]);
        }
    }
    i32x4* out = reinterpret_cast<i32x4*>(rec + t * RW);
#pragma unroll
    for (int q = 0; q < RW / 4; ++q) __builtin_nontemporal_store(i32x4{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]}, out + q);
    if (c < 0) atomicAdd(skipped, 1ull);
}

hipError_t launch_go_draw(const DevGraph& g, const double* tcum, int unit_w, uint64_t seed, uint64_t begin,
                          uint64_t count, int K, int32_t* rec, unsigned long long* skipped, hipStream_t st) {
    const dim3 grid((unsigned)((count + 255) / 256));
    if (K <= 5)
        hipLaunchKernelGGL((go_draw_kernel<5>), grid, dim3(256), 0, st, g, tcum, unit_w, seed, begin, count, K, rec,
                           skipped);
    else
        hipLaunchKernelGGL((go_draw_kernel<10>), grid, dim3(256), 0, st, g, tcum, unit_w, seed, begin, count, K, rec,
                           skipped);
    return hipGetLastError();
}

// draws only (parity tests): {v, c, n1..nK} per sample, Go slot layout
__global__ void go_sample_kernel(DevGraph g, const double* tcum, uint64_t seed, uint64_t begin, uint64_t count, int K,
                                 int32_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const uint64_t s = begin + t;
    int32_t* o = out + t * (2 + K);
    uint4 b = philox_block(seed, 0, s, 0);
    uint32_t cur = 0;
    auto word = [&](uint32_t j) -> uint32_t {
        if ((j >> 2) != cur) { cur = j >> 2; b = philox_block(seed, 0, s, cur); }
        return comp(b, (int)(j & 3));
    };
    const uint32_t w0 = word(0), w1 = word(1);
    const int32_t v = go_alias(g.vtab, g.V, w0, w1);
    o[0] = v;
    o[1] = go_target(g, tcum, v, word(2));
    for (int j = 0; j < K; ++j) {
        const uint32_t ki = word(3 + 2 * j), kp = word(4 + 2 * j);
        o[2 + j] = go_alias(g.ntab, g.V, ki, kp);
    }
}

hipError_t launch_go_sample(const DevGraph& g, const double* tcum, uint64_t seed, uint64_t begin, uint64_t count,
                            int K, int32_t* out, hipStream_t st) {
    const int block = 256;
    hipLaunchKernelGGL(go_sample_kernel, dim3((unsigned)((count + block - 1) / block)), dim3(block), 0, st, g, tcum,
                       seed, begin, count, K, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ Go pair records
// Go SkipGrams (pkg/pronet/pronet.go:310-333: fixed window, pairs (walk[i],
// walk[j]) for j in [i - window, i + window], j != i, walk-major in i then j)
// as records {walk[i], walk[j], n_1 .. n_K, -1 .., alpha bits at 2 + KMAX}
// for go_pair_kernel (go_rec.h); pair p of a walk draws its K negatives from
// slots L - 1 + slot_extra + 2K p .. (index, then p), stream 1 (the walk's
// own steps take slots 0 .. L - 2, the start pick slot_extra of them).  The count of a walk depends on its length only.
__device__ __forceinline__ uint32_t go_pair_count(int L, int window) {
    uint32_t n = 0;
    for (int i = 0; i < L; ++i) {
        const int lo = i - window < 0 ? 0 : i - window;
        const int hi = i + window + 1 > L ? L : i + window + 1;
        n += (uint32_t)(hi - lo - 1);
    }
    return n;
}

__global__ void __launch_bounds__(256) go_pair_count_kernel(WalkArgs w, uint32_t* count) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const int L = w.lens[t];
    if (w.own_lo <= 0 && w.own_hi == 0x7FFFFFFF) {
        count[t] = go_pair_count(L, w.window);
        return;
    }
    // the walk partition (smore_set_walk_owner): pairs of owned centers only
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    uint32_t n = 0;
    for (int i = 0; i < L; ++i) {
        if (walk[i] < w.own_lo || walk[i] >= w.own_hi) continue;
        const int lo = i - w.window < 0 ? 0 : i - w.window;
        const int hi = i + w.window + 1 > L ? L : i + w.window + 1;
        n += (uint32_t)(hi - lo - 1);
    }
    count[t] = n;
}

template <int KMAX>
__global__ void __launch_bounds__(256) go_pair_emit_kernel(DevGraph g, WalkArgs w, uint64_t seed, int K,
                                                           double alpha0, const uint64_t* off, int32_t* rec,
                                                           int tagged) {
    constexpr int RW = rec_width(KMAX);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.nwalks) return;
    const int L = w.lens[t];
    const int32_t* walk = w.walks + t * (uint64_t)(w.steps + 1);
    const uint64_t unit = w.walk_begin + t;
    const float alpha = alpha_walk(unit, alpha0, w.total_walks);
    uint32_t slot = (uint32_t)(L - 1 + w.slot_extra);
    uint32_t blk = 0xFFFFFFFFu;
    uint4 b = make_uint4(0u, 0u, 0u, 0u);
    auto word = [&](uint32_t j) -> uint32_t {
        if ((j >> 2) != blk) {
            blk = j >> 2;
            b = philox_block(seed, 1, unit, blk);
        }
        return comp(b, (int)(j & 3));
    };
    int32_t* out = rec + off[t] * RW;
    for (int i = 0; i < L; ++i) {
        const int lo = i - w.window < 0 ? 0 : i - w.window;
        const int hi = i + w.window + 1 > L ? L : i + w.window + 1;
        const bool own = walk[i] >= w.own_lo && walk[i] < w.own_hi;
        for (int j = lo; j < hi; ++j) {
            if (j == i) continue;
            if (!own) {                     // another part's pair: its draws only
                slot += 2u * (uint32_t)K;
                continue;
            }
            int32_t x[RW];
            x[0] = walk[i];
            // hybrid: the context's C hot bit is bit 31 of its own negative
            // alias word (build_hot_maps), the negatives' come with the draw
            x[1] = tagged ? (int32_t)(walk[j] | ((g.ntab[walk[j]].y >> 31) << 30)) : walk[j];
#pragma unroll
            for (int n = 0; n < RW - 2; ++n) x[2 + n] = -1;
#pragma unroll
            for (int n = 0; n < KMAX; ++n)
                if (n < K) {
                    const uint32_t ki = word(slot + 2u * n), kp = word(slot + 2u * n + 1u);
                    x[2 + n] = tagged ? alias_pick(draw_index(ki, g.V), g.ntab[draw_index(ki, g.V)], kp)
                                      : go_alias(g.ntab, g.V, ki, kp);
                }
            slot += 2u * (uint32_t)K;
            x[2 + KMAX] = __float_as_int(alpha);
            i32x4* o = reinterpret_cast<i32x4*>(out);
#pragma unroll
            for (int q = 0; q < RW / 4; ++q) o[q] = i32x4{x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
            out += RW;
        }
    }
}

hipError_t launch_go_pair_count(const WalkArgs& w, uint32_t* count, hipStream_t st) {
    hipLaunchKernelGGL(go_pair_count_kernel, dim3((unsigned)((w.nwalks + 255) / 256)), dim3(256), 0, st, w, count);
    return hipGetLastError();
}

hipError_t launch_go_pair_emit(const DevGraph& g, const WalkArgs& w, uint64_t seed, int K, double alpha0,
                               const uint64_t* off, int32_t* rec, int tagged, hipStream_t st) {
    const dim3 grid((unsigned)((w.nwalks + 255) / 256));
    if (K <= 5)
        hipLaunchKernelGGL((go_pair_emit_kernel<5>), grid, dim3(256), 0, st, g, w, seed, K, alpha0, off, rec, tagged);
    else
        hipLaunchKernelGGL((go_pair_emit_kernel<10>), grid, dim3(256), 0, st, g, w, seed, K, alpha0, off, rec, tagged);
    return hipGetLastError();
}

// the Go walk generators (DeepWalk, node2vec, metapath2vec): walks into
// w.walks / w.lens; the pairs follow as records
hipError_t launch_go_walk(const EdgeArgs& a, const WalkArgs& w, int grid, hipStream_t st) {
    (void)grid;
    const int block = 256;
    if (w.rule == 3)
        hipLaunchKernelGGL(go_mp_walk_gen_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st,
                           w, a.seed);
    else if (w.rule == 2)
        hipLaunchKernelGGL(go_n2v_walk_gen_kernel, dim3((unsigned)((w.nwalks + N2V_WAVES - 1) / N2V_WAVES)), dim3(256),
                           0, st, a.g, a.tcum, w, a.seed);
    else
        hipLaunchKernelGGL(go_walk_gen_kernel, dim3((unsigned)((w.nwalks + block - 1) / block)), dim3(block), 0, st,
                           a.g, a.tcum, w, a.seed);
    return hipGetLastError();
}

}  // namespace smore
