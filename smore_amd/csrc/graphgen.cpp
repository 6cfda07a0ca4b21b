// graphgen.cpp -- seeded synthetic power-law edge lists for the benchmark
// configurations (both endpoints ~ Zipf(s) over V, vertex ids
// randomly permuted, weight 1.0).  Not part of the reference; it produces the
// bench inputs at C4 size (200M lines) in seconds instead of minutes.
//
// Draws use the build's Philox spec on streams of their own:
//   permutation  stream 17, unit i (Fisher-Yates from V-1 down to 1),
//   line l       stream 16, unit l: words 0,1 -> rank of v1; 2,3 -> rank of v2,
// each rank an alias draw over w_r = (r+1)^-s.  Output is independent of the
// thread count.
#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "host_graph.h"
#include "../../include/smore_hip.h"

namespace {

void philox(uint64_t seed, uint32_t stream, uint64_t unit, uint32_t block, uint32_t out[4]) {
    uint32_t c0 = (uint32_t)unit, c1 = (uint32_t)(unit >> 32), c2 = block, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Zipf {
    std::vector<uint32_t> thresh;
    std::vector<uint32_t> alias;
    int64_t n;
    Zipf(int64_t V, double s) : thresh((size_t)V), alias((size_t)V), n(V) {
        std::vector<double> q((size_t)V);
        double sum = 0;
        for (int64_t r = 0; r < V; ++r) sum += (q[r] = std::pow((double)(r + 1), -s));
        std::vector<int64_t> small, large;
        for (int64_t r = 0; r < V; ++r) {
            q[r] *= (double)V / sum;
            (q[r] < 1.0 ? small : large).push_back(r);
        }
        std::vector<double> prob((size_t)V, 1.0);
        for (int64_t r = 0; r < V; ++r) alias[r] = (uint32_t)r;
        while (!small.empty() && !large.empty()) {
            const int64_t l = small.back(), g = large.back();
            small.pop_back();
            large.pop_back();
            prob[l] = q[l];
            alias[l] = (uint32_t)g;
            q[g] = q[g] + q[l] - 1.0;
            (q[g] < 1.0 ? small : large).push_back(g);
        }
        for (int64_t r = 0; r < V; ++r)
            thresh[r] = prob[r] >= 1.0 ? 0xFFFFFFFFu : (uint32_t)std::ceil(prob[r] * 4294967296.0);
    }
    uint32_t draw(uint32_t ki, uint32_t kp) const {
        const uint32_t i = (uint32_t)(((uint64_t)ki * (uint64_t)n) >> 32);
        return kp < thresh[i] || thresh[i] == 0xFFFFFFFFu ? i : alias[i];
    }
};

template <class F>
void threads(int64_t n, F fn) {
    const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                               (n + (1 << 16) - 1) >> 16}));
    std::vector<std::thread> th;
    const int64_t chunk = (n + nt - 1) / nt;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back(fn, b, e);
    }
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" int smore_gen_powerlaw(int64_t V, int64_t lines, int undirected, double s, uint64_t seed, int32_t* src,
                                  int32_t* dst) {
    if (V <= 0 || V >= ((int64_t)1 << 31) || lines < 0 || !src || !dst || !(s >= 0)) return SMORE_EINVAL;
    std::vector<int32_t> perm((size_t)V);
    for (int64_t i = 0; i < V; ++i) perm[i] = (int32_t)i;
    for (int64_t i = V - 1; i > 0; --i) {
        uint32_t w[4];
        philox(seed, 17, (uint64_t)i, 0, w);
        const int64_t j = (int64_t)(((uint64_t)w[0] * (uint64_t)(i + 1)) >> 32);
        std::swap(perm[i], perm[j]);
    }
    const Zipf z(V, s);
    threads(lines, [&](int64_t b, int64_t e) {
        for (int64_t l = b; l < e; ++l) {
            uint32_t w[4];
            philox(seed, 16, (uint64_t)l, 0, w);
            const int32_t a = perm[z.draw(w[0], w[1])], c = perm[z.draw(w[2], w[3])];
            if (undirected) {
                src[2 * l] = a; dst[2 * l] = c;
                src[2 * l + 1] = c; dst[2 * l + 1] = a;
            } else {
                src[l] = a; dst[l] = c;
            }
        }
    });
    return SMORE_OK;
}
