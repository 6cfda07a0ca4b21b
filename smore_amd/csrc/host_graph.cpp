// host_graph.cpp -- see host_graph.h.
#include "host_graph.h"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unordered_map>

namespace smore {

// d^0.75 as std::pow computes it; 1 and 0 (unit and missing weights, the
// common cases) are exact without the call
static inline double pow075(double x) { return x == 1.0 ? 1.0 : x == 0.0 ? 0.0 : std::pow(x, 0.75); }

void alias_cpp(const double* dist, int64_t n, double* prob, int64_t* alias) {
    // sequential sum in index order, as src/proNet.cpp:556-559
    double sum = 0.0;
    for (int64_t i = 0; i < n; ++i) sum += pow075(dist[i]);
    const double norm = (double)n / sum;
    // per-thread scratch: the context tables call this once per vertex
    thread_local std::vector<double> q;
    thread_local std::vector<int64_t> small, large;
    q.resize((size_t)n);
    small.clear();
    large.clear();
    for (int64_t i = 0; i < n; ++i) {
        q[i] = pow075(dist[i]) * norm;
        prob[i] = 0.0;
        alias[i] = -1;
    }
    for (int64_t i = 0; i < n; ++i) (q[i] < 1 ? small : large).push_back(i);
    while (!small.empty() && !large.empty()) {
        int64_t s = small.back(); small.pop_back();
        int64_t l = large.back(); large.pop_back();
        alias[s] = l;
        prob[s] = q[s];
        q[l] = q[l] + q[s] - 1;
        (q[l] < 1 ? small : large).push_back(l);
    }
    while (!large.empty()) { prob[large.back()] = 1.0; large.pop_back(); }
    while (!small.empty()) { prob[small.back()] = 1.0; small.pop_back(); }
    if (q.capacity() > ((size_t)1 << 24)) {   // do not keep a hub's scratch per thread
        std::vector<double>().swap(q);
        std::vector<int64_t>().swap(small);
        std::vector<int64_t>().swap(large);
    }
}

void alias_encode(const double* prob, const int64_t* alias, int64_t n, const int32_t* self_ids,
                  AliasEntry* out) {
    for (int64_t i = 0; i < n; ++i) {
        const int32_t self = self_ids ? self_ids[i] : (int32_t)i;
        double t = std::ceil(std::ldexp(prob[i], 32));
        if (!(t >= 0)) t = 0;  // NaN: never accept
        if (t >= 4294967296.0) {
            out[i].thresh = 0xFFFFFFFFu;
            out[i].alias = self;
        } else {
            out[i].thresh = (uint32_t)t;
            out[i].alias = alias[i] < 0 ? self : (int32_t)alias[i];
        }
    }
}

void alias_go(const double* dist, int64_t n, double power, double* prob, int64_t* alias) {
    std::vector<double> q((size_t)n);
    double sum = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        q[i] = dist[i] > 0 ? std::pow(dist[i], power) : 0.0;
        sum += q[i];
        prob[i] = 0.0;
        alias[i] = 0;
    }
    if (sum == 0) {
        for (int64_t i = 0; i < n; ++i) { prob[i] = 1.0; alias[i] = i; }
        return;
    }
    for (int64_t i = 0; i < n; ++i) q[i] = q[i] * (double)n / sum;
    std::vector<int64_t> small, large;
    for (int64_t i = 0; i < n; ++i) (q[i] < 1.0 ? small : large).push_back(i);
    while (!small.empty() && !large.empty()) {
        int64_t l = small.back(); small.pop_back();
        int64_t g = large.back(); large.pop_back();
        prob[l] = q[l];
        alias[l] = g;
        q[g] = q[g] + q[l] - 1.0;
        (q[g] < 1.0 ? small : large).push_back(g);
    }
    while (!large.empty()) { int64_t g = large.back(); large.pop_back(); prob[g] = 1.0; alias[g] = g; }
    while (!small.empty()) { int64_t l = small.back(); small.pop_back(); prob[l] = 1.0; alias[l] = l; }
}

void build_go_tables(HostGraph& g, std::vector<double>& tcum) {
    const int64_t V = g.V;
    std::vector<double> dist((size_t)V);
    for (int64_t v = 0; v < V; ++v) dist[v] = g.out_deg[v];
    alias_go(dist.data(), V, 1.0, g.vprob.data(), g.valias.data());
    for (int64_t v = 0; v < V; ++v) dist[v] = g.in_deg[v] + g.out_deg[v];
    alias_go(dist.data(), V, 0.75, g.nprob.data(), g.nalias.data());
    alias_encode(g.vprob.data(), g.valias.data(), V, nullptr, g.vtab.data());
    alias_encode(g.nprob.data(), g.nalias.data(), V, nullptr, g.ntab.data());
    tcum.resize((size_t)std::max<int64_t>(g.E, 1));
    for (int64_t v = 0; v < V; ++v) {
        double acc = 0.0;
        for (int64_t e = g.offsets[v]; e < g.offsets[v + 1]; ++e) { acc += g.weights[e]; tcum[e] = acc; }
    }
}

static void parallel_for(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn) {
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    unsigned nt = (unsigned)std::min<int64_t>(std::min<unsigned>(hw, 16u), (n + grain - 1) / grain);
    if (nt <= 1) { fn(0, n); return; }
    std::vector<std::thread> th;
    int64_t chunk = (n + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        int64_t b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back(fn, b, e);
    }
    for (auto& x : th) x.join();
}

// Stable sort of edge slots by source: LSD radix over the source id (two
// passes up to 2^26 vertices, else 11-bit digits) of packed (src << 32 | slot) words, threads over contiguous slot
// ranges with per-thread digit counts -- stable, so each source keeps its
// push order.  Returns the slot order.
static std::vector<uint64_t> sort_slots_by_source(int64_t V, int64_t E, const int32_t* src) {
    std::vector<uint64_t> a((size_t)E), b((size_t)E);
    parallel_for(E, 1 << 16, [&](int64_t lo, int64_t hi) {
        for (int64_t e = lo; e < hi; ++e) a[e] = ((uint64_t)(uint32_t)src[e] << 32) | (uint64_t)e;
    });
    int bits = 1;
    while (bits < 31 && ((int64_t)1 << bits) < V) ++bits;
    const int D = bits <= 26 ? (bits + 1) / 2 : 11;     // two passes up to 2^26 vertices
    const int NB = 1 << D;
    const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                               E >> 16}));
    const int64_t chunk = (E + nt - 1) / std::max<int64_t>(nt, 1);
    std::vector<int64_t> cnt((size_t)(nt * NB));
    for (int shift = 32; shift < 32 + bits; shift += D) {
        std::fill(cnt.begin(), cnt.end(), 0);
        auto run = [&](auto&& fn) {
            std::vector<std::thread> th;
            for (int64_t t = 0; t < nt; ++t) th.emplace_back(fn, t);
            for (auto& x : th) x.join();
        };
        run([&](int64_t t) {
            int64_t* c = cnt.data() + t * NB;
            for (int64_t e = t * chunk, end = std::min(E, e + chunk); e < end; ++e) c[(a[e] >> shift) & (NB - 1)]++;
        });
        int64_t sum = 0;                               // digit-major, thread-minor offsets
        for (int d = 0; d < NB; ++d)
            for (int64_t t = 0; t < nt; ++t) {
                const int64_t x = cnt[t * NB + d];
                cnt[t * NB + d] = sum;
                sum += x;
            }
        run([&](int64_t t) {
            int64_t* c = cnt.data() + t * NB;
            for (int64_t e = t * chunk, end = std::min(E, e + chunk); e < end; ++e)
                b[c[(a[e] >> shift) & (NB - 1)]++] = a[e];
        });
        a.swap(b);
    }
    return a;
}

bool build_graph(int64_t V, int64_t E, const int32_t* src, const int32_t* dst, const double* w,
                 int vertex_method, int negative_method, HostGraph& g, std::string& err) {
    const bool verbose = getenv("SMORE_LOAD_VERBOSE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!verbose) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[build] %-12s %.2f s\n", what, std::chrono::duration<double>(now - tick).count());
        tick = now;
    };
    if (V <= 0 || V >= (int64_t)1 << 30 || E < 0 || E >= (int64_t)1 << 32) {   // ids carry a tag in bit 30
        err = "bad graph size (V < 2^30, E < 2^32)";
        return false;
    }
    std::vector<int64_t> bad(16, -1);
    {
        std::vector<std::thread> th;
        const int64_t nt = 16, chunk = (E + nt - 1) / nt;
        for (int64_t t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (int64_t e = t * chunk, end = std::min(E, e + chunk); e < end; ++e)
                    if (src[e] < 0 || src[e] >= V || dst[e] < 0 || dst[e] >= V) { bad[t] = e; break; }
            });
        for (auto& x : th) x.join();
    }
    for (int64_t e : bad)
        if (e >= 0) {
            err = "edge " + std::to_string(e) + " has a vertex id out of range";
            return false;
        }
    g.V = V;
    g.E = E;
    g.offsets.assign((size_t)V + 1, 0);
    g.targets.resize((size_t)E);
    g.weights.resize((size_t)E);
    // CSR by a stable sort on the source: per source, targets keep push order
    // (graph[vid1].push_back(vid2), src/proNet.cpp:208-215 and :427-437)
    {
        const std::vector<uint64_t> order = sort_slots_by_source(V, E, src);
        parallel_for(E, 1 << 16, [&](int64_t lo, int64_t hi) {
            for (int64_t p = lo; p < hi; ++p) {
                const int64_t e = (int64_t)(order[p] & 0xFFFFFFFFu);
                g.targets[p] = dst[e];
                g.weights[p] = w[e];
                const int64_t v = (int64_t)(order[p] >> 32);
                if (p == E - 1 || (int64_t)(order[p + 1] >> 32) != v) g.offsets[v + 1] = p + 1;
            }
        });
        for (int64_t v = 0; v < V; ++v)                // sources without edges
            if (g.offsets[v + 1] < g.offsets[v]) g.offsets[v + 1] = g.offsets[v];
    }
    phase("csr");
    // degrees (src/proNet.cpp:431-443): out in adjacency order, in over the CSR
    g.out_deg.assign((size_t)V, 0.0);
    g.in_deg.assign((size_t)V, 0.0);
    parallel_for(V, 1 << 14, [&](int64_t lo, int64_t hi) {
        for (int64_t v = lo; v < hi; ++v)
            for (int64_t p = g.offsets[v]; p < g.offsets[v + 1]; ++p) g.out_deg[v] += g.weights[p];
    });
    // in-degrees sum in CSR order; with integer weights (sums exact in fp64,
    // so any order gives the same bits) threads keep private partial sums
    bool integral = E < ((int64_t)1 << 40);
    for (int64_t p = 0; p < E && integral; ++p)
        integral = g.weights[p] == std::floor(g.weights[p]) && g.weights[p] >= 0 && g.weights[p] < 4096.0;
    const int64_t nt = std::min<int64_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (!integral || E < ((int64_t)1 << 22) || nt == 1) {
        for (int64_t p = 0; p < E; ++p) g.in_deg[g.targets[p]] += g.weights[p];
    } else {
        std::vector<std::vector<double>> part((size_t)nt);
        std::vector<std::thread> th;
        const int64_t chunk = (E + nt - 1) / nt;
        for (int64_t t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                part[t].assign((size_t)V, 0.0);
                for (int64_t p = t * chunk, end = std::min(E, p + chunk); p < end; ++p)
                    part[t][g.targets[p]] += g.weights[p];
            });
        for (auto& x : th) x.join();
        parallel_for(V, 1 << 16, [&](int64_t lo, int64_t hi) {
            for (int64_t t = 0; t < nt; ++t)
                for (int64_t v = lo; v < hi; ++v) g.in_deg[v] += part[t][v];
        });
    }

    phase("degrees");
    g.vertex_method = vertex_method;
    g.negative_method = negative_method;
    g.vprob.resize((size_t)V); g.valias.resize((size_t)V);
    g.nprob.resize((size_t)V); g.nalias.resize((size_t)V);
    g.vtab.resize((size_t)V); g.ntab.resize((size_t)V);
    build_cpp_vn_tables(g);
    phase("v/n tables");
    build_ctx_tables(g);
    phase("ctx tables");
    return true;
}

void build_ctx_tables(HostGraph& g) {
    const int64_t V = g.V, E = g.E;
    // per-vertex context tables, alias remapped to the target vid
    // (src/proNet.cpp:517-537); vertices are independent -> threads
    g.cprob.resize((size_t)E); g.calias.resize((size_t)E);
    g.ctab.resize((size_t)E);
    parallel_for(V, 1 << 14, [&](int64_t b, int64_t e) {
        for (int64_t v = b; v < e; ++v) {
            int64_t off = g.offsets[v], br = g.offsets[v + 1] - off;
            if (br == 0) continue;
            alias_cpp(g.weights.data() + off, br, g.cprob.data() + off, g.calias.data() + off);
            for (int64_t i = 0; i < br; ++i)
                if (g.calias[off + i] != -1) g.calias[off + i] = g.targets[off + g.calias[off + i]];
            alias_encode(g.cprob.data() + off, g.calias.data() + off, br, g.targets.data() + off,
                         g.ctab.data() + off);
        }
    });
}

void build_cpp_vn_tables(HostGraph& g) {
    const int64_t V = g.V;
    std::vector<double> dist((size_t)V);
    // vertex table (src/proNet.cpp:457-482)
    for (int64_t v = 0; v < V; ++v) {
        if (g.vertex_method == 0) dist[v] = g.out_deg[v];
        else if (g.vertex_method == 1) dist[v] = g.out_deg[v] == 0 ? 0 : 1;
        else dist[v] = g.in_deg[v] + g.out_deg[v];
    }
    alias_cpp(dist.data(), V, g.vprob.data(), g.valias.data());
    // negative table (src/proNet.cpp:485-510)
    for (int64_t v = 0; v < V; ++v) {
        if (g.negative_method == 0) dist[v] = g.in_deg[v] + g.out_deg[v];
        else if (g.negative_method == 1) dist[v] = g.in_deg[v];
        else dist[v] = g.in_deg[v] == 0 ? 0 : 1;
    }
    alias_cpp(dist.data(), V, g.nprob.data(), g.nalias.data());
    alias_encode(g.vprob.data(), g.valias.data(), V, nullptr, g.vtab.data());
    alias_encode(g.nprob.data(), g.nalias.data(), V, nullptr, g.ntab.data());
}

static void alias_marginal(const hvec<double>& prob, const hvec<int64_t>& alias, int64_t off,
                           int64_t n, const int32_t* self_ids, double scale, std::vector<double>& p) {
    for (int64_t i = 0; i < n; ++i) {
        const double pr = prob[off + i];
        const int64_t self = self_ids ? self_ids[off + i] : i;
        p[self] += scale * pr;
        if (alias[off + i] >= 0 && pr < 1.0) p[alias[off + i]] += scale * (1.0 - pr);
    }
}

void draw_probabilities(const HostGraph& g, std::vector<double>& p_src, std::vector<double>& p_neg,
                        std::vector<double>& p_ctx, const std::vector<double>* src_law) {
    p_src.assign((size_t)g.V, 0.0);
    p_neg.assign((size_t)g.V, 0.0);
    p_ctx.assign((size_t)g.V, 0.0);
    if (src_law) p_src = *src_law;
    else alias_marginal(g.vprob, g.valias, 0, g.V, nullptr, 1.0 / g.V, p_src);
    alias_marginal(g.nprob, g.nalias, 0, g.V, nullptr, 1.0 / g.V, p_neg);
    for (int64_t v = 0; v < g.V; ++v) {
        const int64_t off = g.offsets[v], br = g.offsets[v + 1] - off;
        if (br == 0 || p_src[v] == 0) continue;
        alias_marginal(g.cprob, g.calias, off, br, g.targets.data(), p_src[v] / br, p_ctx);
    }
}

// ---------------------------------------------------------------- glibc rand
GlibcRand::GlibcRand(uint32_t seed) {
    int32_t r[344];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int32_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = word;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 34; i < 344; ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    for (int i = 0; i < 34; ++i) tbl_[i] = (uint32_t)r[310 + i];
    pos_ = 0;
}

int32_t GlibcRand::next() {
    uint32_t v = tbl_[(pos_ + 3) % 34] + tbl_[(pos_ + 31) % 34];
    tbl_[pos_] = v;
    pos_ = (pos_ + 1) % 34;
    return (int32_t)(v >> 1);
}

void GlibcRand::discard(uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) next();
}

void deepwalk_order(int64_t V, int walk_times, uint64_t skip, int64_t* order) {
    GlibcRand r;
    r.discard(skip);
    for (int t = 0; t < walk_times; ++t) {
        int64_t* keys = order + (int64_t)t * V;
        for (int64_t v = 0; v < V; ++v) keys[v] = v;
        for (int64_t v = 0; v < V; ++v) {
            int rdx = (int)(v + r.next() % (V - v));
            std::swap(keys[v], keys[rdx]);
        }
    }
}

// ---------------------------------------------------------------- warm start
// header of the raw fp32 table dump (save_weights fmt 2)
static const char RAW_MAGIC[8] = {'S', 'M', 'R', 'A', 'W', '1', 0, 0};

bool load_pretrain(const std::string& path, const HostGraph& g, float* table, int dim, int stride,
                   int64_t* loaded, std::string& err) {
    *loaded = 0;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    {   // raw fp32 dump of save_weights fmt 2: rows are vertex ids
        char magic[8];
        if (fread(magic, 1, 8, f) == 8 && std::memcmp(magic, RAW_MAGIC, 8) == 0) {
            int64_t n = 0;
            int32_t hd[2] = {0, 0};
            if (fread(&n, 8, 1, f) != 1 || fread(hd, 4, 2, f) != 2) { fclose(f); err = "truncated " + path; return false; }
            if (hd[0] != dim || n != g.V) { fclose(f); *loaded = -1; return true; }
            std::vector<float> row((size_t)dim);
            for (int64_t v = 0; v < n; ++v) {
                if (fread(row.data(), 4, (size_t)dim, f) != (size_t)dim) { fclose(f); err = "truncated " + path; return false; }
                std::copy(row.begin(), row.end(), table + v * stride);
            }
            fclose(f);
            *loaded = n;
            return true;
        }
        rewind(f);
    }
    std::string line;
    auto getline = [&](std::string& out) -> bool {
        out.clear();
        int ch;
        while ((ch = fgetc(f)) != EOF) {
            if (ch == '\n') return true;
            out.push_back((char)ch);
        }
        return !out.empty();
    };
    if (!getline(line)) { fclose(f); return true; }
    long long n = 0;
    int d = 0;
    if (sscanf(line.c_str(), "%lld %d", &n, &d) != 2 || d != dim) {
        fclose(f);
        *loaded = -1;   // "Dimension not matched, Skip Loading Pre-train model." (:259-262)
        return true;
    }
    std::unordered_map<std::string, int32_t> ids;
    ids.reserve(g.names.size());
    for (size_t i = 0; i < g.names.size(); ++i) ids.emplace(g.names[i], (int32_t)i);
    std::vector<float> row((size_t)dim);
    while (getline(line)) {
        const char* p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        const char* q = p;
        while (*q && *q != ' ' && *q != '\t' && *q != '\r') ++q;
        std::string name(p, q);
        auto it = ids.find(name);
        if (it == ids.end()) continue;
        int got = 0;
        char* endp = nullptr;
        const char* cur = q;
        for (; got < dim; ++got) {
            double x = strtod(cur, &endp);
            if (endp == cur) break;
            row[got] = (float)x;
            cur = endp;
        }
        if (got != dim) continue;   // malformed row: skipped (the reference would index past it)
        std::copy(row.begin(), row.end(), table + (int64_t)it->second * stride);
        ++*loaded;
    }
    fclose(f);
    return true;
}

// ---------------------------------------------------------------- saver
// Rows are formatted by all host threads in blocks (each thread snprintf's its
// block into its own buffer: glibc's exact %g / %.6f), then written in order,
// so the file is byte-identical to a sequential fprintf loop.  fmt 2 writes the
// raw fp32 matrix (RAW_MAGIC, int64 rows, int32 dim, int32 0, rows x dim
// floats) that load_pretrain reads back by vertex id.
bool save_weights(const std::string& path, const HostGraph& g, const float* table, int64_t rows,
                  int dim, int stride, int fmt, std::string& err) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { err = "cannot open " + path; return false; }
    bool ok = true;
    if (fmt == 2) {
        const int64_t r64 = rows;
        const int32_t hd[2] = {dim, 0};
        ok = fwrite(RAW_MAGIC, 1, 8, f) == 8 && fwrite(&r64, 8, 1, f) == 1 && fwrite(hd, 4, 2, f) == 2;
        std::vector<float> buf;
        const int64_t blk = 1 << 16;
        for (int64_t b = 0; ok && b < rows; b += blk) {
            const int64_t n = std::min(blk, rows - b);
            buf.resize((size_t)(n * dim));
            for (int64_t v = 0; v < n; ++v) std::memcpy(&buf[(size_t)(v * dim)], table + (b + v) * stride, dim * 4);
            ok = fwrite(buf.data(), 4, buf.size(), f) == buf.size();
        }
    } else {
        fprintf(f, "%lld %d\n", (long long)rows, dim);
        int threads = (int)std::max(1u, std::thread::hardware_concurrency());
        if (const char* e = getenv("SMORE_SAVE_THREADS")) threads = std::max(1, atoi(e));
        threads = std::min(threads, 64);
        const int64_t blk = 8192;
        std::vector<std::string> out((size_t)threads);
        auto format = [&](int t, int64_t b0) {
            std::string& o = out[(size_t)t];
            o.clear();
            const int64_t lo = b0 + t * blk, hi = std::min(rows, lo + blk);
            char num[64];
            for (int64_t v = lo; v < hi; ++v) {
                if (!g.names.empty()) o += g.names[(size_t)v];
                else o += std::to_string((long long)v);
                const float* r = table + v * stride;
                for (int d = 0; d < dim; ++d) {
                    const int k = snprintf(num, sizeof num, fmt == 1 ? " %.6f" : " %g", (double)r[d]);
                    o.append(num, (size_t)k);
                }
                o.push_back('\n');
            }
        };
        for (int64_t b0 = 0; ok && b0 < rows; b0 += blk * threads) {
            std::vector<std::thread> pool;
            for (int t = 1; t < threads; ++t) pool.emplace_back(format, t, b0);
            format(0, b0);
            for (auto& th : pool) th.join();
            for (int t = 0; ok && t < threads; ++t)
                ok = out[(size_t)t].empty() || fwrite(out[(size_t)t].data(), 1, out[(size_t)t].size(), f) ==
                                                   out[(size_t)t].size();
        }
    }
    ok = (fclose(f) == 0) && ok;
    if (!ok) err = "write failed: " + path;
    return ok;
}

}  // namespace smore
