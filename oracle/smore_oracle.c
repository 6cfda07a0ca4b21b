#include <float.h>
/*
 * smore_oracle.c -- CPU restatement of SMORe's sampled negative-sampling SGD hot
 * path (proNet alias samplers + Opt_SigmoidSGD / Opt_SGD / Opt_BPRSGD updates).
 *
 * TEST INFRASTRUCTURE ONLY (see smore_oracle.h).  Not shipped, not measured
 * except as bench.py's cpu_baseline ("port").
 *
 * Reference citations are to RainBoltz/smore (C++ proNet-core, src/...).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  No fast-math:
 * the fp64 paths must reproduce the reference's sequential operation order.
 */
#include "smore_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ========================================================================== */
/* RNG spec.  Philox4x32-10 (Salmon et al., SC'11; Random123 constants).       */
/* word(seed, stream, unit, slot) = philox(ctr = {lo(unit), hi(unit),          */
/*   slot/4, stream}, key = {lo(seed), hi(seed)})[slot % 4].                   */
/* It replaces src/random.cpp:5-13 (thread_local mt19937 seeded by            */
/* random_device), which is non-reproducible by construction.                 */
/* ========================================================================== */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t orc_word(uint64_t seed, uint32_t stream, uint64_t unit, uint32_t slot) {
    uint32_t ctr[4] = {(uint32_t)unit, (uint32_t)(unit >> 32), slot >> 2, stream};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    orc_philox4x32_10(ctr, key, o);
    return o[slot & 3];
}

void orc_words(uint64_t seed, uint32_t stream, uint64_t unit, uint32_t nslots, uint32_t* out) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (uint32_t b = 0; b * 4 < nslots; ++b) {
        uint32_t ctr[4] = {(uint32_t)unit, (uint32_t)(unit >> 32), b, stream};
        uint32_t o[4];
        orc_philox4x32_10(ctr, key, o);
        for (uint32_t j = 0; j < 4 && b * 4 + j < nslots; ++j) out[b * 4 + j] = o[j];
    }
}

/* index draw: floor(k * n / 2^32) -- the value the interposed random_gen(0, n)
 * returns and the reference truncates to long (src/proNet.cpp:638,650,676). */
static inline uint32_t draw_index(uint32_t k, uint64_t n) {
    return (uint32_t)(((uint64_t)k * n) >> 32);
}
/* uniform draw u = k * 2^-32, exact in fp64 (random_gen(0,1)). */
static inline double draw_unit(uint32_t k) { return ldexp((double)k, -32); }

/* ========================================================================== */
/* glibc rand(): TYPE_3 additive feedback generator, srand(1) default state.   */
/* The reference initialises embeddings with rand() (src/model/LINE.cpp:83,    */
/* src/model/BPR.cpp:49, src/model/MF.cpp:50, src/model/DeepWalk.cpp:47,54)    */
/* and shuffles DeepWalk starts with it (src/model/DeepWalk.cpp:124-131).      */
/* ========================================================================== */
void orc_glibc_srand(orc_glibc_rand* st, uint32_t seed) {
    int32_t r[344];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        /* Schrage: 16807 * r mod (2^31 - 1), as glibc srandom_r */
        int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int32_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = word;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 34; i < 344; ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    for (int i = 0; i < 34; ++i) st->tbl[i] = (uint32_t)r[310 + i];
    st->fptr = 0;
}

int32_t orc_glibc_rand_next(orc_glibc_rand* st) {
    /* ring of the last 34 outputs: x[n] = x[n-31] + x[n-3] */
    int n = st->fptr;                      /* position to write (mod 34) */
    uint32_t v = st->tbl[(n + 34 - 31) % 34] + st->tbl[(n + 34 - 3) % 34];
    st->tbl[n] = v;
    st->fptr = (n + 1) % 34;
    return (int32_t)(v >> 1);
}

void orc_glibc_rand_fill(uint32_t seed, int32_t* out, int64_t n) {
    orc_glibc_rand st;
    orc_glibc_srand(&st, seed);
    for (int64_t i = 0; i < n; ++i) out[i] = orc_glibc_rand_next(&st);
}

/* ========================================================================== */
/* Alias method.                                                               */
/* ========================================================================== */

/* C++ rule, src/proNet.cpp:544-620: q_i = d_i^0.75 * n / sum (the `power`
 * argument is ignored, :558,564); LIFO small/large stacks (:570-603);
 * leftovers get prob 1.0 and keep alias -1 (:605-617). */
void orc_alias_cpp(const double* dist, int64_t n, double* prob, int64_t* alias) {
    double sum = 0.0;
    for (int64_t i = 0; i < n; ++i) sum += pow(dist[i], 0.75);
    double norm = (double)n / sum;
    double* q = (double*)malloc(sizeof(double) * (n ? n : 1));
    int64_t* small = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
    int64_t* large = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
    int64_t ns = 0, nl = 0;
    for (int64_t i = 0; i < n; ++i) {
        q[i] = pow(dist[i], 0.75) * norm;
        alias[i] = -1;
        prob[i] = 0.0;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (q[i] < 1) small[ns++] = i; else large[nl++] = i;
    }
    while (ns && nl) {
        int64_t s = small[--ns];
        int64_t l = large[--nl];
        alias[s] = l;
        prob[s] = q[s];
        q[l] = q[l] + q[s] - 1;
        if (q[l] < 1) small[ns++] = l; else large[nl++] = l;
    }
    while (nl) prob[large[--nl]] = 1.0;
    while (ns) prob[small[--ns]] = 1.0;
    free(q); free(small); free(large);
}

/* Go rule, pkg/pronet/alias.go:10-90: q_i = d_i^power (0 for d_i <= 0),
 * sum == 0 -> uniform; leftovers alias = self. */
void orc_alias_go(const double* dist, int64_t n, double power, double* prob, int64_t* alias) {
    double* q = (double*)malloc(sizeof(double) * (n ? n : 1));
    int64_t* small = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
    int64_t* large = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
    int64_t ns = 0, nl = 0;
    double sum = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        q[i] = dist[i] > 0 ? pow(dist[i], power) : 0.0;
        sum += q[i];
        prob[i] = 0.0; alias[i] = 0;
    }
    if (sum == 0) {
        for (int64_t i = 0; i < n; ++i) { prob[i] = 1.0; alias[i] = i; }
        free(q); free(small); free(large);
        return;
    }
    for (int64_t i = 0; i < n; ++i) q[i] = q[i] * (double)n / sum;
    for (int64_t i = 0; i < n; ++i) { if (q[i] < 1.0) small[ns++] = i; else large[nl++] = i; }
    while (ns && nl) {
        int64_t l = small[--ns];
        int64_t g = large[--nl];
        prob[l] = q[l]; alias[l] = g;
        q[g] = q[g] + q[l] - 1.0;
        if (q[g] < 1.0) small[ns++] = g; else large[nl++] = g;
    }
    while (nl) { int64_t g = large[--nl]; prob[g] = 1.0; alias[g] = g; }
    while (ns) { int64_t l = small[--ns]; prob[l] = 1.0; alias[l] = l; }
    free(q); free(small); free(large);
}

/* Encode {prob, alias} as {accept threshold, alias id}: u < prob with
 * u = k * 2^-32  <=>  k < ceil(prob * 2^32).  T >= 2^32 (always accept) is
 * stored as {0xFFFFFFFF, self} so the draw never needs a 33-bit compare.
 * self_ids == NULL: self = entry index; else self = self_ids[i] (context
 * table: the entry's target vid).  alias -1 (C++ leftovers, prob 1) -> self. */
void orc_alias_encode(const double* prob, const int64_t* alias, int64_t n,
                      const int32_t* self_ids, uint32_t* thresh, int32_t* alias_out) {
    for (int64_t i = 0; i < n; ++i) {
        int32_t self = self_ids ? self_ids[i] : (int32_t)i;
        double t = ceil(ldexp(prob[i], 32));
        if (!(t >= 0)) t = 0;                      /* NaN guard: never accept */
        if (t >= 4294967296.0) {
            thresh[i] = 0xFFFFFFFFu;
            alias_out[i] = self;
        } else {
            thresh[i] = (uint32_t)t;
            alias_out[i] = alias[i] < 0 ? self : (int32_t)alias[i];
        }
    }
}

/* ========================================================================== */
/* Graph build, src/proNet.cpp:410-542 (BuildAliasMethod).                    */
/* Input: directed edge slots in the reference's push order (per input line:   */
/* v1->v2, then v2->v1 if undirected, src/proNet.cpp:208-215).                 */
/* CSR: vertex[v].offset/branch with targets in push order (:417-446).         */
/* ========================================================================== */
int orc_build_graph(int64_t V, int64_t E, const int32_t* src, const int32_t* dst,
                    const double* w, int vertex_method, int negative_method,
                    int64_t* offsets, int32_t* targets, double* out_deg, double* in_deg,
                    double* vprob, int64_t* valias, double* nprob, int64_t* nalias,
                    double* cprob, int64_t* calias) {
    int64_t* cnt = (int64_t*)calloc((size_t)V + 1, sizeof(int64_t));
    double* ew = (double*)malloc(sizeof(double) * (E ? E : 1));
    for (int64_t e = 0; e < E; ++e) {
        if (src[e] < 0 || src[e] >= V || dst[e] < 0 || dst[e] >= V) { free(cnt); free(ew); return -1; }
        cnt[src[e] + 1]++;
    }
    offsets[0] = 0;
    for (int64_t v = 0; v < V; ++v) offsets[v + 1] = offsets[v] + cnt[v + 1];
    for (int64_t v = 0; v <= V; ++v) cnt[v] = offsets[v < V ? v : V];
    for (int64_t e = 0; e < E; ++e) {           /* stable: keeps push order per source */
        int64_t p = cnt[src[e]]++;
        targets[p] = dst[e];
        ew[p] = w[e];
    }
    /* degrees: out_degree summed in adjacency order (:431-436), in_degree by a
     * pass over the context array in CSR order (:439-443) */
    for (int64_t v = 0; v < V; ++v) { out_deg[v] = 0.0; in_deg[v] = 0.0; }
    #pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < V; ++v)
        for (int64_t p = offsets[v]; p < offsets[v + 1]; ++p) out_deg[v] += ew[p];
    for (int64_t p = 0; p < E; ++p) in_deg[targets[p]] += ew[p];

    double* dist = (double*)malloc(sizeof(double) * (V ? V : 1));
    /* vertex table (:457-482) */
    for (int64_t v = 0; v < V; ++v) {
        if (vertex_method == ORC_VM_OUT_DEGREES) dist[v] = out_deg[v];
        else if (vertex_method == ORC_VM_NO_DEGREES) dist[v] = out_deg[v] == 0 ? 0 : 1;
        else dist[v] = in_deg[v] + out_deg[v];
    }
    orc_alias_cpp(dist, V, vprob, valias);
    /* negative table (:485-510) */
    for (int64_t v = 0; v < V; ++v) {
        if (negative_method == ORC_NM_DEGREES) dist[v] = in_deg[v] + out_deg[v];
        else if (negative_method == ORC_NM_IN_DEGREES) dist[v] = in_deg[v];
        else dist[v] = in_deg[v] == 0 ? 0 : 1;
    }
    orc_alias_cpp(dist, V, nprob, nalias);
    free(dist);
    /* per-vertex context tables, alias remapped to the target vid (:517-537);
     * the vertices are independent, so they are built by all threads (same
     * result as the sequential loop) */
    #pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t v = 0; v < V; ++v) {
        int64_t off = offsets[v], br = offsets[v + 1] - offsets[v];
        if (br == 0) continue;
        orc_alias_cpp(ew + off, br, cprob + off, calias + off);
        for (int64_t i = 0; i < br; ++i)
            if (calias[off + i] != -1) calias[off + i] = targets[off + calias[off + i]];
    }
    free(cnt); free(ew);
    return 0;
}

/* ========================================================================== */
/* Samplers.                                                                   */
/* ========================================================================== */
/* SourceSample src/proNet.cpp:647-657: p first, then index. */
static inline int32_t source_sample(const orc_graph* g, uint32_t kp, uint32_t ki) {
    uint32_t i = draw_index(ki, (uint64_t)g->V);
    return kp < g->vthr[i] ? (int32_t)i : g->valias[i];
}
/* TargetSample(vid) src/proNet.cpp:671-683: branch 0 -> -1; p first. */
static inline int32_t target_sample(const orc_graph* g, int32_t v, uint32_t kp, uint32_t ki) {
    int64_t off = g->offsets[v], br = g->offsets[v + 1] - off;
    if (br == 0) return -1;
    int64_t i = off + draw_index(ki, (uint64_t)br);
    return kp < g->cthr[i] ? g->targets[i] : g->calias[i];
}
/* NegativeSample src/proNet.cpp:623-633: index FIRST, then p. */
static inline int32_t negative_sample(const orc_graph* g, uint32_t ki, uint32_t kp) {
    uint32_t i = draw_index(ki, (uint64_t)g->V);
    return kp < g->nthr[i] ? (int32_t)i : g->nalias[i];
}

#define MAX_SLOTS 256
/* LINE/MF sample slot layout: 0 src p, 1 src i, 2 tgt p, 3 tgt i,
 * 4+2j neg_j i, 5+2j neg_j p. */
void orc_sample_line(const orc_graph* g, uint64_t seed, uint64_t begin, uint64_t count,
                     int K, int32_t* out) {
    uint32_t w[MAX_SLOTS];
    for (uint64_t t = 0; t < count; ++t) {
        uint64_t s = begin + t;
        orc_words(seed, 0, s, 4 + 2 * K, w);
        int32_t* o = out + t * (2 + K);
        int32_t v = source_sample(g, w[0], w[1]);
        o[0] = v;
        o[1] = target_sample(g, v, w[2], w[3]);
        for (int j = 0; j < K; ++j) o[2 + j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
    }
}

/* BPR slot layout: 0-3 as LINE, 4-5 neg j0 (i,p), 6+2r/7+2r round r+1 neg. */
void orc_sample_bpr(const orc_graph* g, uint64_t seed, uint64_t begin, uint64_t count,
                    int32_t* out) {
    uint32_t w[16];
    for (uint64_t t = 0; t < count; ++t) {
        uint64_t s = begin + t;
        orc_words(seed, 0, s, 14, w);
        int32_t* o = out + t * 7;
        int32_t u = source_sample(g, w[0], w[1]);
        o[0] = u;
        o[1] = target_sample(g, u, w[2], w[3]);
        for (int j = 0; j < 5; ++j) o[2 + j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
    }
}

/* ========================================================================== */
/* fastSigmoid, src/proNet.cpp:52-71 (table of 1001 entries; the reference     */
/* allocates 1000, :54, and writes/reads index 1000 -- the Go port sizes 1001, */
/* pkg/pronet/pronet.go:81).                                                   */
/* ========================================================================== */
void orc_sigmoid_table(double* tab) {
    for (int i = 0; i != 1000 + 1; i++) {
        double x = i * 2.0 * 8.0 / 1000 - 8.0;
        tab[i] = 1.0 / (1.0 + exp(-x));
    }
}

static double g_sig64[1001];
static float g_sig32[1001];
static int g_sig_init = 0;
static void sig_init(void) {
    if (g_sig_init) return;
    orc_sigmoid_table(g_sig64);
    for (int i = 0; i < 1001; ++i) g_sig32[i] = (float)g_sig64[i];
    g_sig_init = 1;
}

static inline int sig_index(double x) { return (int)((x + 8.0) * 1000 / 8.0 / 2); }

double orc_fast_sigmoid(double x) {
    sig_init();
    if (x < -8.0) return 0.0;
    if (x > 8.0) return 1.0;
    return g_sig64[sig_index(x)];
}

/* fp32 spec: f is an fp32 dot; the bucket index is evaluated in fp64 exactly
 * as the reference expression. */
static inline float fast_sigmoid_f32(float f) {
    double x = (double)f;
    if (x < -8.0) return 0.0f;
    if (x > 8.0) return 1.0f;
    return g_sig32[sig_index(x)];
}

/* ========================================================================== */
/* Learning-rate schedules.                                                    */
/* LINE/MF/BPR (src/model/LINE.cpp:166-187, MF.cpp:85-101, BPR.cpp:84-101):    */
/* the sample run with counter value c uses alpha0 while c < 10^4, then        */
/* alpha0 * (1 - cs/total) with cs = (floor(c/10^4) - 1) * 10^4, floored at    */
/* alpha0 * 1e-4.  LINE's counter starts at 1, MF/BPR's at 0.                  */
/* DeepWalk (src/model/DeepWalk.cpp:137-147): walk w uses                       */
/* alpha0 * (1 - floor(w/10^4)*10^4 / total).                                  */
/* ========================================================================== */
double orc_alpha_line(uint64_t c, double alpha0, uint64_t total) {
    uint64_t u = c / 10000;
    if (u == 0) return alpha0;
    uint64_t cs = (u - 1) * 10000;
    double a = alpha0 * (1.0 - (double)cs / total);
    double amin = alpha0 * 0.0001;
    if (a < amin) a = amin;
    return a;
}

double orc_alpha_walk(uint64_t w, double alpha0, uint64_t total) {
    uint64_t u = w / 10000;
    if (u == 0) return alpha0;
    double a = alpha0 * (1.0 - (double)(u * 10000) / total);
    double amin = alpha0 * 0.0001;
    if (a < amin) a = amin;
    return a;
}

/* ========================================================================== */
/* fp64 training: the reference's arithmetic.                                   */
/* ========================================================================== */

/* Opt_SigmoidSGD, src/proNet.cpp:1312-1330 (loss_context aliases w_context). */
static void opt_sigmoid_sgd_f64(const double* wv, double* wc, double label, int dim,
                                double alpha, double* err) {
    double f = 0, g;
    for (int d = 0; d < dim; ++d) f += wv[d] * wc[d];
    f = orc_fast_sigmoid(f);
    g = (label - f) * alpha;
    for (int d = 0; d < dim; ++d) err[d] += g * wc[d];
    for (int d = 0; d < dim; ++d) wc[d] += g * wv[d];
}

/* Opt_SGD, src/proNet.cpp:991-1012 (linear, L2 reg). */
static void opt_sgd_f64(const double* wv, double* wc, double label, double alpha, double reg,
                        int dim, double* err) {
    double f = 0, g;
    for (int d = 0; d < dim; ++d) f += wv[d] * wc[d];
    g = (label - f);
    for (int d = 0; d < dim; ++d) err[d] += alpha * (g * wc[d] - reg * wv[d]);
    for (int d = 0; d < dim; ++d) wc[d] += alpha * (g * wv[d] - reg * wc[d]);
}

/* One LINE-2 / LINE-1 / MF sample with the reference's arithmetic:
 * UpdatePair src/proNet.cpp:1784-1809, UpdateFactorizedPair :2591-2614. */
static void update_edge_f64(int model, double* W, double* C, int dim, int32_t v, int32_t c,
                            const int32_t* negs, int K, double alpha, double reg, double* err) {
    double* wv = W + (int64_t)v * dim;
    double* T = (model == 0) ? C : W;             /* context table */
    for (int d = 0; d < dim; ++d) err[d] = 0.0;
    if (model == 2) {
        opt_sgd_f64(wv, T + (int64_t)c * dim, 1.0, alpha, reg, dim, err);
        for (int j = 0; j < K; ++j) opt_sgd_f64(wv, T + (int64_t)negs[j] * dim, -1.0, alpha, reg, dim, err);
    } else {
        opt_sigmoid_sgd_f64(wv, T + (int64_t)c * dim, 1.0, dim, alpha, err);
        for (int j = 0; j < K; ++j) opt_sigmoid_sgd_f64(wv, T + (int64_t)negs[j] * dim, 0.0, dim, alpha, err);
    }
    for (int d = 0; d < dim; ++d) wv[d] += err[d];
}

/* Driver loops: LINE::Train src/model/LINE.cpp:160-191 (count from 1),
 * MF::Train src/model/MF.cpp:78-101 (count from 0).  Samples [begin, end) of
 * the global sample index s; counter value c = s + (LINE ? 1 : 0). */
int orc_train_edge_f64(const orc_graph* g, int model, double* W, double* C, int dim,
                       int K, double alpha0, double reg, uint64_t total, uint64_t begin,
                       uint64_t end, uint64_t seed) {
    sig_init();
    double* err = (double*)malloc(sizeof(double) * dim);
    uint32_t w[MAX_SLOTS];
    int32_t negs[MAX_SLOTS];
    int skipped = 0;
    uint64_t base = (model == 2) ? 0 : 1;
    for (uint64_t s = begin; s < end; ++s) {
        orc_words(seed, 0, s, 4 + 2 * K, w);
        int32_t v = source_sample(g, w[0], w[1]);
        int32_t c = target_sample(g, v, w[2], w[3]);
        if (c < 0) { skipped++; continue; }       /* reference: UB (index -1) */
        for (int j = 0; j < K; ++j) negs[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
        double alpha = orc_alpha_line(s + base, alpha0, total);
        update_edge_f64(model, W, C, dim, v, c, negs, K, alpha, reg, err);
    }
    free(err);
    return skipped;
}

/* The same loop with OpenMP Hogwild threads over contiguous sample blocks:
 * the reference's own CPU structure (src/model/LINE.cpp:162, racy shared fp64
 * rows) -- bench.py's reference-arithmetic CPU baseline. */
int orc_train_edge_f64_mt(const orc_graph* g, int model, double* W, double* C, int dim,
                          int K, double alpha0, double reg, uint64_t total, uint64_t begin,
                          uint64_t end, uint64_t seed, int threads) {
    if (threads <= 1) return orc_train_edge_f64(g, model, W, C, dim, K, alpha0, reg, total, begin, end, seed);
    int skipped = 0;
#ifdef _OPENMP
    sig_init();
    uint64_t base = (model == 2) ? 0 : 1;
    #pragma omp parallel num_threads(threads) reduction(+:skipped)
    {
        double* err = (double*)malloc(sizeof(double) * dim);
        uint32_t w[MAX_SLOTS];
        int32_t negs[MAX_SLOTS];
        #pragma omp for schedule(static)
        for (int64_t si = (int64_t)begin; si < (int64_t)end; ++si) {
            uint64_t s = (uint64_t)si;
            orc_words(seed, 0, s, 4 + 2 * K, w);
            int32_t v = source_sample(g, w[0], w[1]);
            int32_t c = target_sample(g, v, w[2], w[3]);
            if (c < 0) { skipped++; continue; }
            for (int j = 0; j < K; ++j) negs[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
            double alpha = orc_alpha_line(s + base, alpha0, total);
            update_edge_f64(model, W, C, dim, v, c, negs, K, alpha, reg, err);
        }
        free(err);
    }
#endif
    return skipped;
}

/* UpdateBPRPair src/proNet.cpp:1406-1455 with Opt_BPRSGD :1053-1068; one
 * shared table (BPR::Train passes w_vertex twice, src/model/BPR.cpp:91). */
static void update_bpr_f64(double* W, int dim, int32_t u, int32_t i, const int32_t* js,
                           double alpha, double* verr, double* cerr, double* x) {
    for (int d = 0; d < dim; ++d) verr[d] = 0.0;
    double* wu = W + (int64_t)u * dim;
    double* wi = W + (int64_t)i * dim;
    for (int n = 0; n < 5; ++n) {
        double* wj = W + (int64_t)js[n] * dim;
        for (int d = 0; d < dim; ++d) { cerr[d] = 0.0; x[d] = wi[d] - wj[d]; }
        double f = 0, g;
        for (int d = 0; d < dim; ++d) f += wu[d] * x[d];
        g = orc_fast_sigmoid(0.0 - f) * alpha;
        for (int d = 0; d < dim; ++d) verr[d] += g * x[d];
        for (int d = 0; d < dim; ++d) cerr[d] += g * wu[d];
        for (int d = 0; d < dim; ++d) {
            wi[d] -= alpha * 0.0025 * wi[d];
            wj[d] -= alpha * 0.0025 * wj[d];
            wi[d] += cerr[d];
            wj[d] -= cerr[d];
        }
    }
    for (int d = 0; d < dim; ++d) {
        wu[d] -= alpha * 0.025 * wu[d];
        wu[d] += verr[d];
    }
}

/* BPR::Train src/model/BPR.cpp:77-101 (count from 0). */
int orc_train_bpr_f64(const orc_graph* g, double* W, int dim, double alpha0, uint64_t total,
                      uint64_t begin, uint64_t end, uint64_t seed) {
    sig_init();
    double* buf = (double*)malloc(sizeof(double) * dim * 3);
    uint32_t w[16];
    int32_t js[5];
    int skipped = 0;
    for (uint64_t s = begin; s < end; ++s) {
        orc_words(seed, 0, s, 14, w);
        int32_t u = source_sample(g, w[0], w[1]);
        int32_t i = target_sample(g, u, w[2], w[3]);
        if (i < 0) { skipped++; continue; }
        for (int j = 0; j < 5; ++j) js[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
        double alpha = orc_alpha_line(s, alpha0, total);
        update_bpr_f64(W, dim, u, i, js, alpha, buf, buf + dim, buf + 2 * dim);
    }
    free(buf);
    return skipped;
}

/* ---- DeepWalk ---------------------------------------------------------------
 * Walk w (global index t*V + i over walk_times t and shuffled position i)
 * draws from stream 1, unit w, consecutive slots:
 *   RandomWalk  src/proNet.cpp:704-724: 2 per step taken (p, i);
 *   SkipGrams   src/proNet.cpp:769-809: 1 per walk position (window shrink);
 *   UpdatePairs src/proNet.cpp:2741-2753 -> UpdatePair: 2 per negative (i, p).
 */
typedef struct { uint64_t seed, unit; uint32_t slot; uint32_t buf[4]; uint32_t bufblk; } walk_rng;
static inline uint32_t walk_next(walk_rng* r) {
    uint32_t blk = r->slot >> 2;
    if (blk != r->bufblk) {
        uint32_t ctr[4] = {(uint32_t)r->unit, (uint32_t)(r->unit >> 32), blk, 1u};
        uint32_t key[2] = {(uint32_t)r->seed, (uint32_t)(r->seed >> 32)};
        orc_philox4x32_10(ctr, key, r->buf);
        r->bufblk = blk;
    }
    return r->buf[r->slot++ & 3];
}

static int random_walk(const orc_graph* g, walk_rng* r, int32_t start, int steps, int32_t* walk) {
    int L = 0;
    int32_t next = start;
    walk[L++] = next;
    for (int s = 0; s < steps; ++s) {
        if (g->offsets[next + 1] - g->offsets[next] == 0) {
            if (next == start) return L;
            next = start;
        }
        uint32_t kp = walk_next(r), ki = walk_next(r);
        next = target_sample(g, next, kp, ki);
        walk[L++] = next;
    }
    return L;
}

/* pairs of SkipGrams(walk, window, 0); returns count */
static int skip_grams(walk_rng* r, const int32_t* walk, int L, int window, int32_t* pv, int32_t* pc) {
    int n = 0;
    for (int i = 0; i < L; ++i) {
        int reduce = (int)draw_index(walk_next(r), (uint64_t)window) + 1;
        int left = i - reduce; if (left < 0) left = 0;
        int right = i + reduce; if (right >= L) right = L - 1;
        for (int j = left; j <= right; ++j) {
            if (i == j) continue;
            pv[n] = walk[i]; pc[n] = walk[j]; n++;
        }
    }
    return n;
}

int orc_train_deepwalk_f64(const orc_graph* g, double* W, double* C, int dim,
                           int walk_times, int walk_steps, int window, int K,
                           double alpha0, uint64_t seed, const int64_t* order) {
    sig_init();
    int64_t V = g->V;
    uint64_t total = (uint64_t)walk_times * (uint64_t)V;
    int32_t* walk = (int32_t*)malloc(sizeof(int32_t) * (walk_steps + 1));
    int maxp = 2 * window * (walk_steps + 1) + 1;
    int32_t* pv = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t negs[MAX_SLOTS];
    double* err = (double*)malloc(sizeof(double) * dim);
    for (uint64_t w = 0; w < total; ++w) {
        walk_rng r = {seed, w, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        double alpha = orc_alpha_walk(w, alpha0, total);
        int L = random_walk(g, &r, (int32_t)order[w], walk_steps, walk);
        int np = skip_grams(&r, walk, L, window, pv, pc);
        for (int p = 0; p < np; ++p) {
            for (int j = 0; j < K; ++j) {
                uint32_t ki = walk_next(&r), kp = walk_next(&r);
                negs[j] = negative_sample(g, ki, kp);
            }
            update_edge_f64(0, W, C, dim, pv[p], pc[p], negs, K, alpha, 0.0, err);
        }
    }
    free(walk); free(pv); free(pc); free(err);
    return 0;
}

/* ========================================================================== */
/* fp32 spec (DESIGN.md "Arithmetic spec"), what the HIP kernels compute.      */
/* Rows are padded to dpad (multiple of 4) floats.  A sample is owned by G      */
/* lanes (G = min(64, pow2ceil(dpad/4))); lane l owns the 16-B chunks l, l+G,   */
/* l+2G, ... below dpad/4 (elements 4q .. 4q+3 of chunk q, so one wave          */
/* instruction moves 16G contiguous bytes of a row).  dot = pairwise tree over  */
/* the G lane partials, each an fmaf chain over the lane's elements in          */
/* increasing order from +0.0f.                                                 */
/* ========================================================================== */
int orc_lane_width(int dpad) {
    int nq = dpad / 4, G = 1;
    while (G < nq && G < 64) G <<= 1;
    return G;
}

static float dot_spec(const float* a, const float* b, int dpad) {
    float part[64];
    int G = orc_lane_width(dpad);
    for (int l = 0; l < G; ++l) {
        float p = 0.0f;
        for (int q = l; q < dpad / 4; q += G)
            for (int e = 4 * q; e < 4 * q + 4; ++e) p = fmaf(a[e], b[e], p);
        part[l] = p;
    }
    for (int w = 1; w < G; w <<= 1)
        for (int l = 0; l < G; l += 2 * w) part[l] = part[l] + part[l + w];
    return part[0];
}

/* fp32 LINE-2 / LINE-1 / MF sample.  Per element, in this order:
 *   sigmoid rule (UpdatePair):  g = (label - sig(f)) * alpha
 *                               e = fmaf(g, c, e);  c = fmaf(g, wv, c)
 *   MF rule (Opt_SGD):          g = label - f
 *                               e = fmaf(alpha, g*c - reg*wv, e)
 *                               c = fmaf(alpha, g*wv - reg*c, c)
 *   end:                        wv = wv + e
 * Rows are updated in place, so a repeated id (negative == positive, or
 * v == c in a shared table) sees the earlier update exactly as the
 * reference's in-place vector<double> update does. */
static void update_edge_f32_w(int model, float* W, float* C, int dpad, int32_t v, int32_t c,
                              const int32_t* negs, int K, float alpha, float reg, float* e, float nsc);
static void update_edge_f32(int model, float* W, float* C, int dpad, int32_t v, int32_t c,
                            const int32_t* negs, int K, float alpha, float reg, float* e) {
    update_edge_f32_w(model, W, C, dpad, v, c, negs, K, alpha, reg, e, 1.0f);
}

/* nsc: the negatives' step weight of a block-schedule cell (blocks.cpp
 * cell_args): negative j steps with alpha * nsc (== alpha when nsc == 1) */
static void update_edge_f32_w(int model, float* W, float* C, int dpad, int32_t v, int32_t c,
                              const int32_t* negs, int K, float alpha, float reg, float* e, float nsc) {
    float* wv = W + (int64_t)v * dpad;
    float* T = (model == 0) ? C : W;
    for (int d = 0; d < dpad; ++d) e[d] = 0.0f;
    for (int j = -1; j < K; ++j) {
        int32_t id = j < 0 ? c : negs[j];
        float* cr = T + (int64_t)id * dpad;
        float f = dot_spec(wv, cr, dpad);
        if (model == 2) {
            float label = j < 0 ? 1.0f : -1.0f;
            float gg = label - f;
            for (int d = 0; d < dpad; ++d) {
                float ce = cr[d], we = wv[d];
                float t1 = gg * ce - reg * we;
                float t2 = gg * we - reg * ce;
                e[d] = fmaf(alpha, t1, e[d]);
                cr[d] = fmaf(alpha, t2, ce);
            }
        } else {
            float label = j < 0 ? 1.0f : 0.0f;
            float gg = (label - fast_sigmoid_f32(f)) * (j < 0 ? alpha : alpha * nsc);
            for (int d = 0; d < dpad; ++d) {
                float ce = cr[d], we = wv[d];
                e[d] = fmaf(gg, ce, e[d]);
                cr[d] = fmaf(gg, we, ce);
            }
        }
    }
    for (int d = 0; d < dpad; ++d) wv[d] = wv[d] + e[d];
}

int orc_train_edge_f32(const orc_graph* g, int model, float* W, float* C, int dim,
                       int dpad, int K, double alpha0, double reg, uint64_t total,
                       uint64_t begin, uint64_t end, uint64_t seed, int threads) {
    (void)dim;
    sig_init();
    uint64_t base = (model == 2) ? 0 : 1;
    int skipped = 0;
    if (threads <= 1) {
        float* e = (float*)malloc(sizeof(float) * dpad);
        uint32_t w[MAX_SLOTS];
        int32_t negs[MAX_SLOTS];
        for (uint64_t s = begin; s < end; ++s) {
            orc_words(seed, 0, s, 4 + 2 * K, w);
            int32_t v = source_sample(g, w[0], w[1]);
            int32_t c = target_sample(g, v, w[2], w[3]);
            if (c < 0) { skipped++; continue; }
            for (int j = 0; j < K; ++j) negs[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
            float alpha = (float)orc_alpha_line(s + base, alpha0, total);
            update_edge_f32(model, W, C, dpad, v, c, negs, K, alpha, (float)reg, e);
        }
        free(e);
        return skipped;
    }
#ifdef _OPENMP
    /* Hogwild CPU baseline: the reference's OpenMP structure
     * (src/model/LINE.cpp:162, racy shared rows), contiguous sample blocks. */
    #pragma omp parallel num_threads(threads) reduction(+:skipped)
    {
        float* e = (float*)malloc(sizeof(float) * dpad);
        uint32_t w[MAX_SLOTS];
        int32_t negs[MAX_SLOTS];
        #pragma omp for schedule(static)
        for (int64_t si = (int64_t)begin; si < (int64_t)end; ++si) {
            uint64_t s = (uint64_t)si;
            orc_words(seed, 0, s, 4 + 2 * K, w);
            int32_t v = source_sample(g, w[0], w[1]);
            int32_t c = target_sample(g, v, w[2], w[3]);
            if (c < 0) { skipped++; continue; }
            for (int j = 0; j < K; ++j) negs[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
            float alpha = (float)orc_alpha_line(s + base, alpha0, total);
            update_edge_f32(model, W, C, dpad, v, c, negs, K, alpha, (float)reg, e);
        }
        free(e);
    }
#endif
    return skipped;
}

/* LINE-2 / LINE-1 / MF over explicit sample records {v, c, n_1 .. n_K} (count
 * x (2 + K), ids masked to 30 bits) in order: the update of
 * orc_train_edge_f32 with record i taking the learning rate of global sample
 * begin + i.  The records of the block schedule's cells (smore_block_sample_edges)
 * are checked through it. */
int orc_train_records_f32(int model, float* W, float* C, int dpad, const int32_t* rec, int64_t count, int K,
                          double alpha0, double reg, uint64_t total, uint64_t begin, float neg_scale) {
    sig_init();
    uint64_t base = (model == 2) ? 0 : 1;
    float* e = (float*)malloc(sizeof(float) * dpad);
    int32_t negs[MAX_SLOTS];
    for (int64_t i = 0; i < count; ++i) {
        const int32_t* r = rec + i * (2 + K);
        int32_t v = r[0] & 0x3FFFFFFF, c = r[1];
        if (c < 0) continue;
        c &= 0x3FFFFFFF;
        for (int j = 0; j < K; ++j) negs[j] = r[2 + j] & 0x3FFFFFFF;
        float alpha = (float)orc_alpha_line(begin + (uint64_t)i + base, alpha0, total);
        update_edge_f32_w(model, W, C, dpad, v, c, negs, K, alpha, (float)reg, e, neg_scale);
    }
    free(e);
    return 0;
}

/* fp32 BPR (UpdateBPRPair, src/proNet.cpp:1406-1455).  Per round n, element
 * order as the reference's d-loop:
 *   x = wi - wj;  f = dot(wu, x);  g = sig(0 - f) * alpha   (0-f in fp64 == -f)
 *   ve = fmaf(g, x, ve);  ce = g * wu
 *   wi = fmaf(-r1, wi, wi); wj = fmaf(-r1, wj, wj); wi = wi + ce; wj = wj - ce
 * with r1 = alpha * 0.0025f; end: wu = fmaf(-r2, wu, wu) + ve, r2 = alpha*0.025f. */
static void update_bpr_f32(float* W, int dpad, int32_t u, int32_t i, const int32_t* js,
                           float alpha, float* ve, float* x, float* ce) {
    float* wu = W + (int64_t)u * dpad;
    float* wi = W + (int64_t)i * dpad;
    float r1 = alpha * 0.0025f, r2 = alpha * 0.025f;
    for (int d = 0; d < dpad; ++d) ve[d] = 0.0f;
    for (int n = 0; n < 5; ++n) {
        float* wj = W + (int64_t)js[n] * dpad;
        for (int d = 0; d < dpad; ++d) x[d] = wi[d] - wj[d];
        float f = dot_spec(wu, x, dpad);
        float gg = fast_sigmoid_f32(-f) * alpha;
        for (int d = 0; d < dpad; ++d) { ve[d] = fmaf(gg, x[d], ve[d]); ce[d] = gg * wu[d]; }
        for (int d = 0; d < dpad; ++d) {
            wi[d] = fmaf(-r1, wi[d], wi[d]);
            wj[d] = fmaf(-r1, wj[d], wj[d]);
            wi[d] = wi[d] + ce[d];
            wj[d] = wj[d] - ce[d];
        }
    }
    for (int d = 0; d < dpad; ++d) wu[d] = fmaf(-r2, wu[d], wu[d]) + ve[d];
}

int orc_train_bpr_f32(const orc_graph* g, float* W, int dim, int dpad, double alpha0,
                      uint64_t total, uint64_t begin, uint64_t end, uint64_t seed, int threads) {
    (void)dim;
    sig_init();
    int skipped = 0;
    #pragma omp parallel num_threads(threads > 1 ? threads : 1) reduction(+:skipped)
    {
        float* buf = (float*)malloc(sizeof(float) * dpad * 3);
        uint32_t w[16];
        int32_t js[5];
        #pragma omp for schedule(static)
        for (int64_t si = (int64_t)begin; si < (int64_t)end; ++si) {
            uint64_t s = (uint64_t)si;
            orc_words(seed, 0, s, 14, w);
            int32_t u = source_sample(g, w[0], w[1]);
            int32_t i = target_sample(g, u, w[2], w[3]);
            if (i < 0) { skipped++; continue; }
            for (int j = 0; j < 5; ++j) js[j] = negative_sample(g, w[4 + 2 * j], w[5 + 2 * j]);
            float alpha = (float)orc_alpha_line(s, alpha0, total);
            update_bpr_f32(W, dpad, u, i, js, alpha, buf, buf + dpad, buf + 2 * dpad);
        }
        free(buf);
    }
    return skipped;
}

int orc_train_deepwalk_f32(const orc_graph* g, float* W, float* C, int dim, int dpad,
                           int walk_times, int walk_steps, int window, int K,
                           double alpha0, uint64_t seed, const int64_t* order,
                           uint64_t walk_begin, uint64_t walk_end) {
    (void)dim;
    sig_init();
    uint64_t total = (uint64_t)walk_times * (uint64_t)g->V;
    if (walk_end > total) walk_end = total;
    int32_t* walk = (int32_t*)malloc(sizeof(int32_t) * (walk_steps + 1));
    int maxp = 2 * window * (walk_steps + 1) + 1;
    int32_t* pv = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t negs[MAX_SLOTS];
    float* e = (float*)malloc(sizeof(float) * dpad);
    for (uint64_t w = walk_begin; w < walk_end; ++w) {
        walk_rng r = {seed, w, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        float alpha = (float)orc_alpha_walk(w, alpha0, total);
        int L = random_walk(g, &r, (int32_t)order[w], walk_steps, walk);
        int np = skip_grams(&r, walk, L, window, pv, pc);
        for (int p = 0; p < np; ++p) {
            for (int j = 0; j < K; ++j) {
                uint32_t ki = walk_next(&r), kp = walk_next(&r);
                negs[j] = negative_sample(g, ki, kp);
            }
            update_edge_f32(0, W, C, dpad, pv[p], pc[p], negs, K, alpha, 0.0f, e);
        }
    }
    free(walk); free(pv); free(pc); free(e);
    return 0;
}

/* ---- Walklets --------------------------------------------------------------
 * ScaleSkipGrams(walk, window_min, window_max, 0), src/proNet.cpp:928-987, with
 * its clamping exactly as written: the left range [max(0,i-wmax), max(0,i-wmin)]
 * and the right range [min(i+wmin,L-1), min(i+wmax,L-1)], i itself skipped
 * (a clamped range can pair vertices closer than window_min). No draws. */
static int scale_skip_grams(const int32_t* walk, int L, int wmin, int wmax, int32_t* pv, int32_t* pc) {
    int n = 0;
    for (int i = 0; i < L; ++i) {
        int left = i - wmax; if (left < 0) left = 0;
        int right = i - wmin; if (right < 0) right = 0;
        for (int j = left; j <= right; ++j) {
            if (i == j) continue;
            pv[n] = walk[i]; pc[n] = walk[j]; n++;
        }
        left = i + wmin; if (left >= L) left = L - 1;
        right = i + wmax; if (right >= L) right = L - 1;
        for (int j = left; j <= right; ++j) {
            if (i == j) continue;
            pv[n] = walk[i]; pc[n] = walk[j]; n++;
        }
    }
    return n;
}

static int walklets(const orc_graph* g, double* W64, double* C64, float* W32, float* C32, int dim, int dpad,
                    int walk_times, int walk_steps, int wmin, int wmax, int K, double alpha0, uint64_t seed,
                    uint64_t walk_begin, uint64_t walk_end) {
    sig_init();
    int64_t V = g->V;
    uint64_t total = (uint64_t)walk_times * (uint64_t)V;
    if (walk_end > total) walk_end = total;
    int32_t* walk = (int32_t*)malloc(sizeof(int32_t) * (walk_steps + 1));
    int span = wmax - wmin + 1; if (span < 1) span = 1;
    int maxp = 2 * (span + 1) * (walk_steps + 1) + 1;
    int32_t* pv = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t negs[MAX_SLOTS];
    double* e64 = (double*)malloc(sizeof(double) * (dim > dpad ? dim : dpad));
    float* e32 = (float*)malloc(sizeof(float) * (dpad > 0 ? dpad : 1));
    for (uint64_t w = walk_begin; w < walk_end; ++w) {
        walk_rng r = {seed, w, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        double alpha = orc_alpha_walk(w, alpha0, total);
        int L = random_walk(g, &r, (int32_t)(w % (uint64_t)V), walk_steps, walk);
        int np = scale_skip_grams(walk, L, wmin, wmax, pv, pc);
        for (int p = 0; p < np; ++p) {
            for (int j = 0; j < K; ++j) {
                uint32_t ki = walk_next(&r), kp = walk_next(&r);
                negs[j] = negative_sample(g, ki, kp);
            }
            if (W64) update_edge_f64(0, W64, C64, dim, pv[p], pc[p], negs, K, alpha, 0.0, e64);
            else update_edge_f32(0, W32, C32, dpad, pv[p], pc[p], negs, K, (float)alpha, 0.0f, e32);
        }
    }
    free(walk); free(pv); free(pc); free(e64); free(e32);
    return 0;
}

int orc_train_walklets_f64(const orc_graph* g, double* W, double* C, int dim, int walk_times, int walk_steps,
                           int window_min, int window_max, int K, double alpha0, uint64_t seed) {
    return walklets(g, W, C, NULL, NULL, dim, 0, walk_times, walk_steps, window_min, window_max, K, alpha0, seed, 0,
                    (uint64_t)-1);
}

int orc_train_walklets_f32(const orc_graph* g, float* W, float* C, int dim, int dpad, int walk_times,
                           int walk_steps, int window_min, int window_max, int K, double alpha0, uint64_t seed,
                           uint64_t walk_begin, uint64_t walk_end) {
    return walklets(g, NULL, NULL, W, C, dim, dpad, walk_times, walk_steps, window_min, window_max, K, alpha0, seed,
                    walk_begin, walk_end);
}

/* ---- APP ----------------------------------------------------------------------
 * JumpingRandomWalk(start, jump), src/proNet.cpp:685-701: from `start`, while
 * the current vertex has out-edges: TargetSample (p, index), then stop when
 * random_gen(0.0, 1.0) < jump (the double arguments bind to the int
 * parameters: U[0,1)).  Returns the walk's last vertex (start for a dead
 * start).  The reference has no step bound; this one stops after 2^24 steps
 * (the GPU's bound, where a jump >= 1e-6 ends first with probability
 * 1 - e^-16). */
#define APP_MAX_STEPS (1 << 24)
static int32_t jumping_walk_end(const orc_graph* g, walk_rng* r, int32_t start, double jump) {
    int32_t next = start;
    for (int s = 0; s < APP_MAX_STEPS; ++s) {
        if (g->offsets[next + 1] - g->offsets[next] == 0) return next;
        uint32_t kp = walk_next(r), ki = walk_next(r);
        next = target_sample(g, next, kp, ki);
        if (draw_unit(walk_next(r)) < jump) break;
    }
    return next;
}

void orc_app_pairs(const orc_graph* g, int walk_times, int sample_times, double jump, uint64_t seed,
                   const int64_t* order, uint64_t unit_begin, uint64_t unit_end, int32_t* vc) {
    (void)walk_times;
    for (uint64_t u = unit_begin; u < unit_end; ++u) {
        walk_rng r = {seed, u, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        int32_t start = (int32_t)order[u / (uint64_t)sample_times];
        vc[2 * (u - unit_begin)] = start;
        vc[2 * (u - unit_begin) + 1] = jumping_walk_end(g, &r, start, jump);
    }
}

static int app(const orc_graph* g, double* W64, double* C64, float* W32, float* C32, int dim, int dpad,
               int walk_times, int sample_times, double jump, int K, double alpha0, uint64_t seed,
               const int64_t* order, uint64_t unit_begin, uint64_t unit_end) {
    sig_init();
    uint64_t total = (uint64_t)walk_times * (uint64_t)g->V;
    uint64_t units = total * (uint64_t)sample_times;
    if (unit_end > units) unit_end = units;
    int32_t negs[MAX_SLOTS];
    double* e64 = (double*)malloc(sizeof(double) * (dim > dpad ? dim : dpad));
    float* e32 = (float*)malloc(sizeof(float) * (dpad > 0 ? dpad : 1));
    for (uint64_t u = unit_begin; u < unit_end; ++u) {
        uint64_t w = u / (uint64_t)sample_times;
        walk_rng r = {seed, u, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        double alpha = orc_alpha_walk(w, alpha0, total);
        int32_t v = (int32_t)order[w];
        int32_t c = jumping_walk_end(g, &r, v, jump);
        for (int j = 0; j < K; ++j) {
            uint32_t ki = walk_next(&r), kp = walk_next(&r);
            negs[j] = negative_sample(g, ki, kp);
        }
        if (W64) update_edge_f64(0, W64, C64, dim, v, c, negs, K, alpha, 0.0, e64);
        else update_edge_f32(0, W32, C32, dpad, v, c, negs, K, (float)alpha, 0.0f, e32);
    }
    free(e64); free(e32);
    return 0;
}

int orc_train_app_f64(const orc_graph* g, double* W, double* C, int dim, int walk_times, int sample_times,
                      double jump, int K, double alpha0, uint64_t seed, const int64_t* order) {
    return app(g, W, C, NULL, NULL, dim, 0, walk_times, sample_times, jump, K, alpha0, seed, order, 0,
               (uint64_t)-1);
}

int orc_train_app_f32(const orc_graph* g, float* W, float* C, int dim, int dpad, int walk_times, int sample_times,
                      double jump, int K, double alpha0, uint64_t seed, const int64_t* order,
                      uint64_t unit_begin, uint64_t unit_end) {
    return app(g, NULL, NULL, W, C, dim, dpad, walk_times, sample_times, jump, K, alpha0, seed, order, unit_begin,
               unit_end);
}

/* ---- HPE ----------------------------------------------------------------------
 * Opt_SigmoidRegSGD, src/proNet.cpp:1332-1351 (the caller passes C[c] as the
 * context loss too): f = sig(W.C); g = label - f; first the whole
 * err += alpha*(g*c - reg*w) loop, then c += alpha*(g*w - reg*c). */
static void opt_sigmoid_reg_f64(const double* wv, double* wc, double label, double alpha, double reg, int dim,
                                double* err) {
    double f = 0.0;
    for (int d = 0; d < dim; ++d) f += wv[d] * wc[d];
    f = orc_fast_sigmoid(f);
    double gg = label - f;
    for (int d = 0; d < dim; ++d) err[d] += alpha * (gg * wc[d] - reg * wv[d]);
    for (int d = 0; d < dim; ++d) wc[d] += alpha * (gg * wv[d] - reg * wc[d]);
}

/* fp32 spec of the same step (the MF rule's element form with the sigmoid
 * gradient): e = fmaf(alpha, g*c - reg*w, e); c = fmaf(alpha, g*w - reg*c, c) */
static void opt_sigmoid_reg_f32(const float* wv, float* wc, float label, float alpha, float reg, int dpad, float* e) {
    float f = dot_spec(wv, wc, dpad);
    float gg = label - fast_sigmoid_f32(f);
    for (int d = 0; d < dpad; ++d) {
        float ce = wc[d], we = wv[d];
        float t1 = gg * ce - reg * we;
        float t2 = gg * we - reg * ce;
        e[d] = fmaf(alpha, t1, e[d]);
        wc[d] = fmaf(alpha, t2, ce);
    }
}

typedef struct { uint64_t seed, unit; uint32_t slot; uint32_t buf[4]; uint32_t bufblk; } unit_rng;
static inline uint32_t unit_next(unit_rng* r) {   /* stream 0, consecutive slots of one unit */
    uint32_t blk = r->slot >> 2;
    if (blk != r->bufblk) {
        uint32_t ctr[4] = {(uint32_t)r->unit, (uint32_t)(r->unit >> 32), blk, 0u};
        uint32_t key[2] = {(uint32_t)r->seed, (uint32_t)(r->seed >> 32)};
        orc_philox4x32_10(ctr, key, r->buf);
        r->bufblk = blk;
    }
    return r->buf[r->slot++ & 3];
}
/* TargetSample: no draws on a vertex without out-edges */
static inline int32_t unit_target(const orc_graph* g, unit_rng* r, int32_t v) {
    if (g->offsets[v + 1] - g->offsets[v] == 0) return -1;
    uint32_t kp = unit_next(r), ki = unit_next(r);
    return target_sample(g, v, kp, ki);
}

static int hpe(const orc_graph* g, double* W64, double* C64, float* W32, float* C32, int dim, int dpad,
               int walk_steps, int K, double reg, double alpha0, uint64_t total, uint64_t begin, uint64_t end,
               uint64_t seed) {
    sig_init();
    int skipped = 0;
    int32_t negs[MAX_SLOTS];
    int n = dim > dpad ? dim : dpad;
    double* e64 = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    float* e32 = (float*)malloc(sizeof(float) * (n > 0 ? n : 1));
    for (uint64_t s = begin; s < end; ++s) {
        unit_rng r = {seed, s, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        uint32_t kp = unit_next(&r), ki = unit_next(&r);
        int32_t v1 = source_sample(g, kp, ki);
        int32_t v2 = unit_target(g, &r, v1);
        if (v2 < 0) { skipped++; continue; }
        double alpha = orc_alpha_line(s, alpha0, total);
        int32_t ctx = v2;
        for (int st = 0; st < walk_steps; ++st) {
            if (st != 0) {
                ctx = unit_target(g, &r, ctx);
                if (ctx == -1) break;
            }
            for (int j = 0; j < K; ++j) {
                uint32_t a = unit_next(&r), b = unit_next(&r);
                negs[j] = negative_sample(g, a, b);
            }
            if (W64) {
                double* wv = W64 + (int64_t)v1 * dim;
                for (int d = 0; d < dim; ++d) e64[d] = 0.0;
                opt_sigmoid_reg_f64(wv, C64 + (int64_t)ctx * dim, 1.0, alpha, reg, dim, e64);
                for (int j = 0; j < K; ++j) opt_sigmoid_reg_f64(wv, C64 + (int64_t)negs[j] * dim, 0.0, alpha, reg, dim, e64);
                for (int d = 0; d < dim; ++d) wv[d] += e64[d];
            } else {
                float* wv = W32 + (int64_t)v1 * dpad;
                for (int d = 0; d < dpad; ++d) e32[d] = 0.0f;
                opt_sigmoid_reg_f32(wv, C32 + (int64_t)ctx * dpad, 1.0f, (float)alpha, (float)reg, dpad, e32);
                for (int j = 0; j < K; ++j)
                    opt_sigmoid_reg_f32(wv, C32 + (int64_t)negs[j] * dpad, 0.0f, (float)alpha, (float)reg, dpad, e32);
                for (int d = 0; d < dpad; ++d) wv[d] = wv[d] + e32[d];
            }
        }
        for (int j = 0; j < K; ++j) {
            uint32_t a = unit_next(&r), b = unit_next(&r);
            negs[j] = negative_sample(g, a, b);
        }
        if (W64) update_edge_f64(0, W64, C64, dim, v2, v1, negs, K, alpha, 0.0, e64);
        else update_edge_f32(0, W32, C32, dpad, v2, v1, negs, K, (float)alpha, 0.0f, e32);
    }
    free(e64); free(e32);
    return skipped;
}

int orc_train_hpe_f64(const orc_graph* g, double* W, double* C, int dim, int walk_steps, int K, double reg,
                      double alpha0, uint64_t total, uint64_t begin, uint64_t end, uint64_t seed) {
    return hpe(g, W, C, NULL, NULL, dim, 0, walk_steps, K, reg, alpha0, total, begin, end, seed);
}

int orc_train_hpe_f32(const orc_graph* g, float* W, float* C, int dim, int dpad, int walk_steps, int K, double reg,
                      double alpha0, uint64_t total, uint64_t begin, uint64_t end, uint64_t seed) {
    return hpe(g, NULL, NULL, W, C, dim, dpad, walk_steps, K, reg, alpha0, total, begin, end, seed);
}

/* ========================================================================== */
/* Go semantics (pkg/pronet, internal/models/{line,bpr,deepwalk}).             */
/* No Go toolchain exists here: these restate the Go source and are            */
/* cross-checked against an independent pure-Python restatement               */
/* (tests/go_semantics_ref.py).                                                */
/* ========================================================================== */

/* prefix sums in the Go loop's order: cumWeight += w (pronet.go:275-279) */
void orc_go_cumsum(const int64_t* offsets, int64_t V, const double* w, double* tcum) {
    for (int64_t v = 0; v < V; ++v) {
        double acc = 0.0;
        for (int64_t e = offsets[v]; e < offsets[v + 1]; ++e) { acc += w[e]; tcum[e] = acc; }
    }
}

/* aliasSample (alias.go:93-106): i = Intn(n) first, then r = Float64() */
static inline int32_t go_alias(const uint32_t* thr, const int32_t* alias, int64_t n, uint32_t ki, uint32_t kp) {
    uint32_t i = draw_index(ki, (uint64_t)n);
    return kp < thr[i] ? (int32_t)i : alias[i];
}

/* TargetSample (pronet.go:257-284): r = Float64()*sum(w); first i with r <= cum_i */
static inline int32_t go_target(const orc_go_graph* g, int32_t v, uint32_t kr) {
    int64_t off = g->base.offsets[v], br = g->base.offsets[v + 1] - off;
    if (br == 0) return -1;
    double r = draw_unit(kr) * g->tcum[off + br - 1];
    int64_t lo = 0, hi = br - 1;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (r <= g->tcum[off + mid]) hi = mid; else lo = mid + 1;
    }
    return g->base.targets[off + lo];
}

void orc_go_sample(const orc_go_graph* g, uint64_t seed, uint64_t begin, uint64_t count, int K, int32_t* out) {
    uint32_t w[MAX_SLOTS];
    for (uint64_t t = 0; t < count; ++t) {
        orc_words(seed, 0, begin + t, 3 + 2 * K, w);
        int32_t* o = out + t * (2 + K);
        int32_t v = go_alias(g->base.vthr, g->base.valias, g->base.V, w[0], w[1]);
        o[0] = v;
        o[1] = go_target(g, v, w[2]);
        for (int j = 0; j < K; ++j) o[2 + j] = go_alias(g->base.nthr, g->base.nalias, g->base.V, w[3 + 2 * j], w[4 + 2 * j]);
    }
}

static inline double go_fast_sigmoid(double x) { return orc_fast_sigmoid(x); }   /* pronet.go:98-109 */

/* ---- fp64, the Go arithmetic ------------------------------------------------ */
/* sgdUpdate (optimizer.go:61-84) */
static void go_sgd_f64(const double* ve, const double* ce, double label, double alpha, int dim,
                       double* vg, double* cg) {
    double score = 0.0;
    for (int d = 0; d < dim; ++d) score += ve[d] * ce[d];
    double pred = go_fast_sigmoid(score);
    double grad = alpha * (label - pred);
    for (int d = 0; d < dim; ++d) { vg[d] += grad * ce[d]; cg[d] += grad * ve[d]; }
}

/* UpdatePair (optimizer.go:21-58) */
static void go_update_pair_f64(double* W, double* C, int dim, int32_t v, int32_t c, const int32_t* negs, int K,
                               double alpha, double* vg, double* cg, double* ng) {
    double* wv = W + (int64_t)v * dim;
    double* cc = C + (int64_t)c * dim;
    for (int d = 0; d < dim; ++d) { vg[d] = 0.0; cg[d] = 0.0; }
    go_sgd_f64(wv, cc, 1.0, alpha, dim, vg, cg);
    for (int j = 0; j < K; ++j) {
        if (negs[j] == c) continue;
        double* cn = C + (int64_t)negs[j] * dim;
        for (int d = 0; d < dim; ++d) ng[d] = 0.0;
        go_sgd_f64(wv, cn, 0.0, alpha, dim, vg, ng);
        for (int d = 0; d < dim; ++d) cn[d] += ng[d];
    }
    for (int d = 0; d < dim; ++d) { wv[d] += vg[d]; cc[d] += cg[d]; }
}

/* updateFirstOrder (internal/models/line/line.go:153-200) */
static void go_first_order_f64(double* W, int dim, int32_t s, int32_t t, const int32_t* negs, int K, double alpha,
                               double* vg, double* cg) {
    double* ws = W + (int64_t)s * dim;
    double* wt = W + (int64_t)t * dim;
    double score = 0.0;
    for (int d = 0; d < dim; ++d) score += ws[d] * wt[d];
    double grad = alpha * (1.0 - go_fast_sigmoid(score));
    for (int d = 0; d < dim; ++d) { vg[d] = grad * wt[d]; cg[d] = grad * ws[d]; }
    for (int j = 0; j < K; ++j) {
        int32_t n = negs[j];
        if (n == t || n == s) continue;
        double* wn = W + (int64_t)n * dim;
        double sc = 0.0;
        for (int d = 0; d < dim; ++d) sc += ws[d] * wn[d];
        double gr = alpha * (0.0 - go_fast_sigmoid(sc));
        for (int d = 0; d < dim; ++d) { vg[d] += gr * wn[d]; wn[d] += gr * ws[d]; }
    }
    for (int d = 0; d < dim; ++d) { ws[d] += vg[d]; wt[d] += cg[d]; }
}

/* UpdateBPRPair (optimizer.go:87-117): W users, C items */
static void go_bpr_f64(double* W, double* C, int dim, int32_t u, int32_t i, int32_t j, double alpha, double lambda) {
    double* wu = W + (int64_t)u * dim;
    double* ci = C + (int64_t)i * dim;
    double* cj = C + (int64_t)j * dim;
    double pos = 0.0, neg = 0.0;
    for (int d = 0; d < dim; ++d) { pos += wu[d] * ci[d]; neg += wu[d] * cj[d]; }
    double gc = alpha * go_fast_sigmoid(neg - pos);
    for (int d = 0; d < dim; ++d) {
        double vgr = gc * (ci[d] - cj[d]);
        double pg = gc * wu[d];
        double ngr = -gc * wu[d];
        wu[d] += vgr - lambda * alpha * wu[d];
        ci[d] += pg - lambda * alpha * ci[d];
        cj[d] += ngr - lambda * alpha * cj[d];
    }
}

int orc_go_train_f64(const orc_go_graph* g, int model, double* W, double* C, int dim, int K, double alpha0,
                     double lambda, uint64_t total, uint64_t begin, uint64_t end, uint64_t seed) {
    sig_init();
    double* buf = (double*)malloc(sizeof(double) * dim * 3);
    uint32_t w[MAX_SLOTS];
    int32_t negs[MAX_SLOTS];
    int skipped = 0;
    const int nk = model == 3 ? 1 : K;
    for (uint64_t s = begin; s < end; ++s) {
        orc_words(seed, 0, s, 3 + 2 * nk, w);
        int32_t v = go_alias(g->base.vthr, g->base.valias, g->base.V, w[0], w[1]);
        int32_t c = go_target(g, v, w[2]);
        if (c < 0) { skipped++; continue; }
        for (int j = 0; j < nk; ++j) negs[j] = go_alias(g->base.nthr, g->base.nalias, g->base.V, w[3 + 2 * j], w[4 + 2 * j]);
        double alpha = orc_alpha_walk(s, alpha0, total);
        if (model == 0) go_update_pair_f64(W, C, dim, v, c, negs, K, alpha, buf, buf + dim, buf + 2 * dim);
        else if (model == 1) go_first_order_f64(W, dim, v, c, negs, K, alpha, buf, buf + dim);
        else go_bpr_f64(W, C, dim, v, c, negs[0], alpha, lambda);
    }
    free(buf);
    return skipped;
}

/* ---- fp32 spec of the Go rules (no fused multiply-add: amd64 Go does not fuse) -- */
static void go_update_pair_f32(float* W, float* C, int dpad, int32_t v, int32_t c, const int32_t* negs, int K,
                               float alpha, float* vg, float* cg) {
    float* wv = W + (int64_t)v * dpad;
    float* cc = C + (int64_t)c * dpad;
    float f = dot_spec(wv, cc, dpad);
    float grad = alpha * (1.0f - fast_sigmoid_f32(f));
    for (int d = 0; d < dpad; ++d) { vg[d] = grad * cc[d]; cg[d] = grad * wv[d]; }
    for (int j = 0; j < K; ++j) {
        if (negs[j] == c) continue;
        float* cn = C + (int64_t)negs[j] * dpad;
        float fn = dot_spec(wv, cn, dpad);
        float gr = alpha * (0.0f - fast_sigmoid_f32(fn));
        for (int d = 0; d < dpad; ++d) {
            float ng = gr * wv[d];
            vg[d] = vg[d] + gr * cn[d];
            cn[d] = cn[d] + ng;
        }
    }
    for (int d = 0; d < dpad; ++d) { wv[d] = wv[d] + vg[d]; cc[d] = cc[d] + cg[d]; }
}

static void go_first_order_f32(float* W, int dpad, int32_t s, int32_t t, const int32_t* negs, int K, float alpha,
                               float* vg, float* cg) {
    float* ws = W + (int64_t)s * dpad;
    float* wt = W + (int64_t)t * dpad;
    float grad = alpha * (1.0f - fast_sigmoid_f32(dot_spec(ws, wt, dpad)));
    for (int d = 0; d < dpad; ++d) { vg[d] = grad * wt[d]; cg[d] = grad * ws[d]; }
    for (int j = 0; j < K; ++j) {
        int32_t n = negs[j];
        if (n == t || n == s) continue;
        float* wn = W + (int64_t)n * dpad;
        float gr = alpha * (0.0f - fast_sigmoid_f32(dot_spec(ws, wn, dpad)));
        for (int d = 0; d < dpad; ++d) { vg[d] = vg[d] + gr * wn[d]; wn[d] = wn[d] + gr * ws[d]; }
    }
    for (int d = 0; d < dpad; ++d) { ws[d] = ws[d] + vg[d]; wt[d] = wt[d] + cg[d]; }
}

static void go_bpr_f32(float* W, float* C, int dpad, int32_t u, int32_t i, int32_t j, float alpha, float lambda) {
    float* wu = W + (int64_t)u * dpad;
    float* ci = C + (int64_t)i * dpad;
    float* cj = C + (int64_t)j * dpad;
    float pos = dot_spec(wu, ci, dpad), neg = dot_spec(wu, cj, dpad);
    float gc = alpha * fast_sigmoid_f32(neg - pos);
    float la = lambda * alpha;
    for (int d = 0; d < dpad; ++d) {
        float vgr = gc * (ci[d] - cj[d]);
        float pg = gc * wu[d];
        float ngr = -gc * wu[d];
        wu[d] = wu[d] + (vgr - la * wu[d]);
        ci[d] = ci[d] + (pg - la * ci[d]);
        cj[d] = cj[d] + (ngr - la * cj[d]);
    }
}

int orc_go_train_f32(const orc_go_graph* g, int model, float* W, float* C, int dim, int dpad, int K,
                     double alpha0, double lambda, uint64_t total, uint64_t begin, uint64_t end, uint64_t seed) {
    (void)dim;
    sig_init();
    float* buf = (float*)malloc(sizeof(float) * dpad * 2);
    uint32_t w[MAX_SLOTS];
    int32_t negs[MAX_SLOTS];
    int skipped = 0;
    const int nk = model == 3 ? 1 : K;
    for (uint64_t s = begin; s < end; ++s) {
        orc_words(seed, 0, s, 3 + 2 * nk, w);
        int32_t v = go_alias(g->base.vthr, g->base.valias, g->base.V, w[0], w[1]);
        int32_t c = go_target(g, v, w[2]);
        if (c < 0) { skipped++; continue; }
        for (int j = 0; j < nk; ++j) negs[j] = go_alias(g->base.nthr, g->base.nalias, g->base.V, w[3 + 2 * j], w[4 + 2 * j]);
        float alpha = (float)orc_alpha_walk(s, alpha0, total);
        if (model == 0) go_update_pair_f32(W, C, dpad, v, c, negs, K, alpha, buf, buf + dpad);
        else if (model == 1) go_first_order_f32(W, dpad, v, c, negs, K, alpha, buf, buf + dpad);
        else go_bpr_f32(W, C, dpad, v, c, negs[0], alpha, (float)lambda);
    }
    free(buf);
    return skipped;
}

/* ---- Go DeepWalk ------------------------------------------------------------ */
static int go_random_walk(const orc_go_graph* g, walk_rng* r, int32_t start, int steps, int32_t* walk) {
    int L = 0;
    int32_t cur = start;
    walk[L++] = cur;
    for (int i = 0; i < steps; ++i) {
        if (g->base.offsets[cur + 1] - g->base.offsets[cur] == 0) break;   /* TargetSample -> -1 */
        int32_t next = go_target(g, cur, walk_next(r));
        walk[L++] = next;
        cur = next;
    }
    return L;
}

/* ---- Go node2vec (internal/models/node2vec/node2vec.go) ---------------------- */
typedef struct { const double* w; double inv_p, inv_q; } n2v_params;

/* areNeighbors (:167-175): linear scan of Graph[a] */
static int n2v_adjacent(const orc_go_graph* g, int32_t a, int32_t b) {
    for (int64_t e = g->base.offsets[a]; e < g->base.offsets[a + 1]; ++e)
        if (g->base.targets[e] == b) return 1;
    return 0;
}

/* biasedTargetSample (:114-164) with the draw k already taken */
static int32_t n2v_biased_target(const orc_go_graph* g, const n2v_params* np_, int32_t prev, int32_t cur, uint32_t k) {
    int64_t off = g->base.offsets[cur], deg = g->base.offsets[cur + 1] - off;
    double total = 0.0;
    double* bw = (double*)malloc(sizeof(double) * (size_t)deg);
    for (int64_t i = 0; i < deg; ++i) {
        int32_t nb = g->base.targets[off + i];
        double bias = nb == prev ? np_->inv_p : (n2v_adjacent(g, prev, nb) ? 1.0 : np_->inv_q);
        bw[i] = np_->w[off + i] * bias;
        total += bw[i];
    }
    int32_t out = g->base.targets[off + deg - 1];
    if (total == 0.0) {
        out = g->base.targets[off + draw_index(k, (uint64_t)deg)];
    } else {
        double r = draw_unit(k) * total, cum = 0.0;
        for (int64_t i = 0; i < deg; ++i) {
            cum += bw[i];
            if (r <= cum) { out = g->base.targets[off + i]; break; }
        }
    }
    free(bw);
    return out;
}

/* biasedRandomWalk (:82-110): first step TargetSample, later steps biased;
 * a vertex without out-edges ends the walk before drawing */
static int go_n2v_walk(const orc_go_graph* g, const n2v_params* np_, walk_rng* r, int32_t start, int steps,
                       int32_t* walk) {
    int L = 0;
    walk[L++] = start;
    for (int i = 0; i < steps; ++i) {
        int32_t cur = walk[L - 1];
        if (g->base.offsets[cur + 1] - g->base.offsets[cur] == 0) break;
        uint32_t k = walk_next(r);
        walk[L] = i == 0 ? go_target(g, cur, k) : n2v_biased_target(g, np_, walk[L - 2], cur, k);
        L++;
    }
    return L;
}

int orc_go_node2vec_walk(const orc_go_graph* g, const double* weights, double p, double q, uint64_t seed,
                         uint64_t unit, int32_t start, int steps, int32_t* walk) {
    n2v_params np_ = {weights, 1.0 / p, 1.0 / q};
    walk_rng r = {seed, unit, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
    return go_n2v_walk(g, &np_, &r, start, steps, walk);
}

/* ---- Go metapath2vec (internal/models/metapath2vec, pkg/hetero) -------------- */
typedef struct { const int32_t* ntype; const int32_t* paths; const int32_t* path_off; int npaths; } mp_params;

/* Intn(len(metaPaths)) (metapath2vec.go:184), then MetaPathWalk
 * (hetero_graph.go:221-256) with SampleNeighborByType (:206-214): the
 * neighbours of the wanted type in Edges[cur] order, one picked by Intn */
static int go_mp_walk(const orc_go_graph* g, const mp_params* mp, walk_rng* r, int32_t start, int steps,
                      int32_t* walk) {
    int L = 0;
    walk[L++] = start;
    int pi = (int)draw_index(walk_next(r), (uint64_t)mp->npaths);
    const int32_t* path = mp->paths + mp->path_off[pi];
    int plen = mp->path_off[pi + 1] - mp->path_off[pi];
    if (plen < 2) return L;
    int32_t cur = start;
    for (int idx = 0; L < steps + 1; ++idx) {
        if (mp->ntype[cur] != path[idx % plen]) break;
        int nt = path[(idx + 1) % plen];
        int64_t n = 0;
        for (int64_t e = g->base.offsets[cur]; e < g->base.offsets[cur + 1]; ++e)
            if (mp->ntype[g->base.targets[e]] == nt) n++;
        if (n == 0) break;
        int64_t pick = (int64_t)draw_index(walk_next(r), (uint64_t)n), seen = 0;
        int32_t next = -1;
        for (int64_t e = g->base.offsets[cur]; e < g->base.offsets[cur + 1]; ++e)
            if (mp->ntype[g->base.targets[e]] == nt && seen++ == pick) { next = g->base.targets[e]; break; }
        walk[L++] = next;
        cur = next;
    }
    return L;
}

int orc_go_metapath_walk(const orc_go_graph* g, const int32_t* ntype, const int32_t* paths, const int32_t* path_off,
                         int npaths, uint64_t seed, uint64_t unit, int32_t start, int steps, int32_t* walk) {
    mp_params mp = {ntype, paths, path_off, npaths};
    walk_rng r = {seed, unit, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
    return go_mp_walk(g, &mp, &r, start, steps, walk);
}

/* ---- Go CTDNE (internal/models/ctdne, pkg/temporal) ------------------------- */
typedef struct {
    int64_t V, E;
    int64_t* off;      /* OutEdges per source, time-sorted (stable insertion sort) */
    int32_t* tgt;
    double* ts;
    double* tmin;      /* GetActiveTimeRange */
    double* tmax;
    double max_time, window;
} ct_graph;

static void ct_build(ct_graph* t, int64_t V, int64_t E, const int32_t* src, const int32_t* dst, const double* ts) {
    t->V = V; t->E = E;
    t->off = (int64_t*)calloc((size_t)V + 1, sizeof(int64_t));
    t->tgt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(E + 1));
    t->ts = (double*)malloc(sizeof(double) * (size_t)(E + 1));
    t->tmin = (double*)malloc(sizeof(double) * (size_t)V);
    t->tmax = (double*)malloc(sizeof(double) * (size_t)V);
    for (int64_t i = 0; i < E; ++i) t->off[src[i] + 1]++;
    for (int64_t v = 0; v < V; ++v) t->off[v + 1] += t->off[v];
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(V + 1));
    memcpy(fill, t->off, sizeof(int64_t) * (size_t)V);
    for (int64_t i = 0; i < E; ++i) {   /* append in input order, then insertion-sort by time (stable) */
        int64_t x = fill[src[i]]++;
        int64_t b = t->off[src[i]];
        while (x > b && t->ts[x - 1] > ts[i]) { t->ts[x] = t->ts[x - 1]; t->tgt[x] = t->tgt[x - 1]; x--; }
        t->ts[x] = ts[i]; t->tgt[x] = dst[i];
    }
    free(fill);
    t->max_time = -DBL_MAX;
    for (int64_t v = 0; v < V; ++v) { t->tmin[v] = DBL_MAX; t->tmax[v] = -DBL_MAX; }
    for (int64_t i = 0; i < E; ++i) {
        int32_t ends[2] = {src[i], dst[i]};
        for (int k = 0; k < 2; ++k) {
            if (ts[i] < t->tmin[ends[k]]) t->tmin[ends[k]] = ts[i];
            if (ts[i] > t->tmax[ends[k]]) t->tmax[ends[k]] = ts[i];
        }
        if (ts[i] > t->max_time) t->max_time = ts[i];
    }
    for (int64_t v = 0; v < V; ++v) if (t->tmin[v] == DBL_MAX) t->tmin[v] = t->tmax[v] = 0.0;
}

static void ct_free(ct_graph* t) { free(t->off); free(t->tgt); free(t->ts); free(t->tmin); free(t->tmax); }

/* ctdne.go:159-170 start time + TemporalRandomWalk (temporal_graph.go:225-252)
 * with GetTemporalNeighbors' scan (:181-196) and SampleTemporalNeighbor's
 * timestamp of OutEdges[cur][idx] (:198-208) */
static int go_ct_walk(const ct_graph* t, walk_rng* r, int32_t start, int steps, int32_t* walk) {
    int L = 0;
    walk[L++] = start;
    double lo = t->tmin[start], hi = t->tmax[start];
    if (lo == 0.0 && hi == 0.0) return L;
    double range = hi - lo;
    if (range == 0.0) range = t->window;
    double now = lo + draw_unit(walk_next(r)) * range;
    int32_t cur = start;
    while (L < steps + 1) {
        double end = now + t->window;
        if (end > t->max_time) end = t->max_time;
        int64_t b = t->off[cur], e = t->off[cur + 1], n = 0, first = -1;
        for (int64_t x = b; x < e; ++x) {
            if (t->ts[x] >= now && t->ts[x] <= end) { if (first < 0) first = x; n++; }
            if (t->ts[x] > end) break;
        }
        if (n == 0) break;
        int64_t idx = (int64_t)draw_index(walk_next(r), (uint64_t)n);
        cur = t->tgt[first + idx];
        now = t->ts[b + idx];
        walk[L++] = cur;
    }
    return L;
}

int orc_go_ctdne_walk(int64_t V, int64_t E, const int32_t* src, const int32_t* dst, const double* ts, double window,
                      uint64_t seed, uint64_t unit, int32_t start, int steps, int32_t* walk) {
    ct_graph t;
    ct_build(&t, V, E, src, dst, ts);
    t.window = window;
    walk_rng r = {seed, unit, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
    int L = go_ct_walk(&t, &r, start, steps, walk);
    ct_free(&t);
    return L;
}

static int go_skip_grams(const int32_t* walk, int L, int window, int32_t* pv, int32_t* pc) {
    int n = 0;
    for (int i = 0; i < L; ++i) {
        int start = i - window; if (start < 0) start = 0;
        int end = i + window + 1; if (end > L) end = L;
        for (int j = start; j < end; ++j)
            if (i != j) { pv[n] = walk[i]; pc[n] = walk[j]; n++; }
    }
    return n;
}

static int go_deepwalk(const orc_go_graph* g, double* W64, double* C64, float* W32, float* C32, int dim, int dpad,
                       int walk_times, int walk_steps, int window, int K, double alpha0, uint64_t seed,
                       const int64_t* order, uint64_t walk_begin, uint64_t walk_end, const n2v_params* n2v,
                       const mp_params* mp, const ct_graph* ct) {
    sig_init();
    uint64_t total = (uint64_t)walk_times * (uint64_t)g->base.V;
    if (walk_end > total) walk_end = total;
    int32_t* walk = (int32_t*)malloc(sizeof(int32_t) * (walk_steps + 1));
    int maxp = 2 * window * (walk_steps + 1) + 1;
    int32_t* pv = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * maxp);
    int32_t negs[MAX_SLOTS];
    int n = W64 ? dim : dpad;
    double* b64 = (double*)malloc(sizeof(double) * n * 3);
    float* b32 = (float*)malloc(sizeof(float) * n * 2);
    for (uint64_t wk = walk_begin; wk < walk_end; ++wk) {
        walk_rng r = {seed, wk, 0, {0, 0, 0, 0}, 0xFFFFFFFFu};
        double alpha = orc_alpha_walk(wk, alpha0, total);
        int L = ct    ? go_ct_walk(ct, &r, (int32_t)order[wk], walk_steps, walk)
                : mp  ? go_mp_walk(g, mp, &r, (int32_t)order[wk], walk_steps, walk)
                : n2v ? go_n2v_walk(g, n2v, &r, (int32_t)order[wk], walk_steps, walk)
                      : go_random_walk(g, &r, (int32_t)order[wk], walk_steps, walk);
        int np = go_skip_grams(walk, L, window, pv, pc);
        for (int p = 0; p < np; ++p) {
            for (int j = 0; j < K; ++j) {
                uint32_t ki = walk_next(&r), kp = walk_next(&r);
                negs[j] = go_alias(g->base.nthr, g->base.nalias, g->base.V, ki, kp);
            }
            if (W64) go_update_pair_f64(W64, C64, dim, pv[p], pc[p], negs, K, alpha, b64, b64 + n, b64 + 2 * n);
            else go_update_pair_f32(W32, C32, dpad, pv[p], pc[p], negs, K, (float)alpha, b32, b32 + n);
        }
    }
    free(walk); free(pv); free(pc); free(b64); free(b32);
    return 0;
}

int orc_go_deepwalk_f32(const orc_go_graph* g, float* W, float* C, int dim, int dpad, int walk_times,
                        int walk_steps, int window, int K, double alpha0, uint64_t seed,
                        const int64_t* order, uint64_t walk_begin, uint64_t walk_end) {
    return go_deepwalk(g, NULL, NULL, W, C, dim, dpad, walk_times, walk_steps, window, K, alpha0, seed, order,
                       walk_begin, walk_end, NULL, NULL, NULL);
}

int orc_go_deepwalk_f64(const orc_go_graph* g, double* W, double* C, int dim, int walk_times, int walk_steps,
                        int window, int K, double alpha0, uint64_t seed, const int64_t* order) {
    return go_deepwalk(g, W, C, NULL, NULL, dim, dim, walk_times, walk_steps, window, K, alpha0, seed, order, 0,
                       (uint64_t)-1, NULL, NULL, NULL);
}

/* Go node2vec = Go DeepWalk with biasedRandomWalk (node2vec.go:178-258) */
int orc_go_node2vec_f32(const orc_go_graph* g, const double* weights, float* W, float* C, int dim, int dpad,
                        int walk_times, int walk_steps, int window, int K, double alpha0, double p, double q,
                        uint64_t seed, const int64_t* order, uint64_t walk_begin, uint64_t walk_end) {
    n2v_params np_ = {weights, 1.0 / p, 1.0 / q};
    return go_deepwalk(g, NULL, NULL, W, C, dim, dpad, walk_times, walk_steps, window, K, alpha0, seed, order,
                       walk_begin, walk_end, &np_, NULL, NULL);
}

/* Go metapath2vec = Go DeepWalk's pairs over MetaPathWalk (metapath2vec.go:106-200);
 * negatives from the graph's negative table (the caller sets the uniform one) */
int orc_go_metapath_f32(const orc_go_graph* g, const int32_t* ntype, const int32_t* paths, const int32_t* path_off,
                        int npaths, float* W, float* C, int dim, int dpad, int walk_times, int walk_steps, int window,
                        int K, double alpha0, uint64_t seed, const int64_t* order, uint64_t walk_begin,
                        uint64_t walk_end) {
    mp_params mp = {ntype, paths, path_off, npaths};
    return go_deepwalk(g, NULL, NULL, W, C, dim, dpad, walk_times, walk_steps, window, K, alpha0, seed, order,
                       walk_begin, walk_end, NULL, &mp, NULL);
}

/* Go CTDNE = Go DeepWalk's pairs over the temporal walks (ctdne.go:80-200);
 * negatives from g's negative table (the Go table of the edges, unit weights) */
int orc_go_ctdne_f32(const orc_go_graph* g, int64_t E, const int32_t* src, const int32_t* dst, const double* ts,
                     double window, float* W, float* C, int dim, int dpad, int walk_times, int walk_steps,
                     int win, int K, double alpha0, uint64_t seed, const int64_t* order, uint64_t walk_begin,
                     uint64_t walk_end) {
    ct_graph t;
    ct_build(&t, g->base.V, E, src, dst, ts);
    t.window = window;
    int rc = go_deepwalk(g, NULL, NULL, W, C, dim, dpad, walk_times, walk_steps, win, K, alpha0, seed, order,
                         walk_begin, walk_end, NULL, NULL, &t);
    ct_free(&t);
    return rc;
}

/* ---- caller-supplied pairs: UpdatePairs (src/proNet.cpp:2741-2753; Go
 * pkg/pronet/optimizer.go:8-18) ----------------------------------------------
 * UpdatePair for each pair (v[i], c[i]) in order with a fixed alpha.  Pair i
 * draws its K negatives (NegativeSample: index, then p) from stream 3, unit
 * unit0 + i / ORC_PAIR_BLOCK, slots 2K (i % ORC_PAIR_BLOCK) + 2j, +1 -- the
 * reference's UpdatePairs over blocks of ORC_PAIR_BLOCK pairs with the RNG spec
 * interposed (oracle/ref_harness.cpp "pairs").  go = 0: C++ UpdatePair
 * (src/proNet.cpp:1784-1809); go = 1: Go UpdatePair (optimizer.go:21-58:
 * negatives equal to the context skipped, the context's gradient deferred),
 * both on g's negative table. */
static void pair_negs(const orc_graph* g, uint64_t seed, uint64_t unit0, int64_t i, int K, int32_t* negs) {
    const uint64_t unit = unit0 + (uint64_t)i / ORC_PAIR_BLOCK;
    const uint32_t base = 2u * (uint32_t)K * (uint32_t)((uint64_t)i % ORC_PAIR_BLOCK);
    for (int j = 0; j < K; ++j)
        negs[j] = negative_sample(g, orc_word(seed, 3, unit, base + 2u * j), orc_word(seed, 3, unit, base + 2u * j + 1u));
}

int orc_update_pairs_f64(const orc_graph* g, double* W, double* C, int dim, const int32_t* v, const int32_t* c,
                         int64_t n, int K, double alpha, uint64_t seed, uint64_t unit0, int go) {
    sig_init();
    if (K < 0 || K > MAX_SLOTS) return -1;
    double* buf = (double*)malloc(sizeof(double) * dim * 3);
    int32_t negs[MAX_SLOTS];
    for (int64_t i = 0; i < n; ++i) {
        pair_negs(g, seed, unit0, i, K, negs);
        if (go) go_update_pair_f64(W, C, dim, v[i], c[i], negs, K, alpha, buf, buf + dim, buf + 2 * dim);
        else update_edge_f64(0, W, C, dim, v[i], c[i], negs, K, alpha, 0.0, buf);
    }
    free(buf);
    return 0;
}

int orc_update_pairs_f32(const orc_graph* g, float* W, float* C, int dim, int dpad, const int32_t* v,
                         const int32_t* c, int64_t n, int K, double alpha, uint64_t seed, uint64_t unit0, int go) {
    (void)dim;
    sig_init();
    if (K < 0 || K > MAX_SLOTS) return -1;
    float* buf = (float*)malloc(sizeof(float) * dpad * 2);
    int32_t negs[MAX_SLOTS];
    const float a = (float)alpha;
    for (int64_t i = 0; i < n; ++i) {
        pair_negs(g, seed, unit0, i, K, negs);
        if (go) go_update_pair_f32(W, C, dpad, v[i], c[i], negs, K, a, buf, buf + dpad);
        else update_edge_f32(0, W, C, dpad, v[i], c[i], negs, K, a, 0.0f, buf);
    }
    free(buf);
    return 0;
}
