// ref_harness.cpp -- drives the REFERENCE C++ (compiled unmodified from
// /root/reference/src by oracle/Makefile) to produce golden vectors.
//
// TEST INFRASTRUCTURE ONLY.  Output goes to oracle/_ref/ (git-ignored) and,
// through oracle/gen_golden.py, to tests/golden/*.npz.
//
// Determinism: the reference's random_gen (src/random.cpp:5-13, thread_local
// mt19937 seeded by random_device) is replaced at link time by the definition
// below (the archive member's symbol is weakened with objcopy), which serves
// the build's RNG spec (DESIGN.md "RNG spec"):
//   edge models  : draw n of the run -> unit n / D, slot n % D, stream 0
//   DeepWalk     : proNet::RandomWalk is wrapped (ld --wrap) so each walk
//                  starts unit = walk index, slot 0, stream 1 (Walklets too)
//   APP          : proNet::JumpingRandomWalk is wrapped the same way: each
//                  jumping walk (and its UpdatePair) is one unit
//   HPE          : proNet::SourceSample is wrapped (HPE mode only): each
//                  sample is one unit of stream 0, consecutive slots
//   UpdatePairs  : (caller-supplied pairs) each block of ORC_PAIR_BLOCK pairs
//                  is one unit of stream 3, consecutive slots
//   random_gen(0,1)   -> k * 2^-32
//   random_gen(a,b)   -> a + floor(k * (b-a) / 2^32)
// Weight init keeps the reference's own glibc rand() calls.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "model/APP.h"
#include "model/BPR.h"
#include "model/DeepWalk.h"
#include "model/HPE.h"
#include "model/Walklets.h"
#include "model/LINE.h"
#include "model/MF.h"

extern "C" {
#include "smore_oracle.h"
}

// ---------------------------------------------------------------- interposed RNG
static uint64_t g_seed = 1;
static uint64_t g_D = 1;            // draws per edge sample
static uint64_t g_n = 0;            // draw counter (edge models)
static int g_walk_mode = 0;
static uint64_t g_walk_unit = 0, g_walk_counter = 0;
static uint32_t g_walk_slot = 0;
static uint32_t g_walk_stream = 1;     // walk models: stream 1; HPE: stream 0
static int g_hpe_mode = 0;

double random_gen(const int& min, const int& max) {
    uint32_t k;
    if (g_walk_mode) {
        k = orc_word(g_seed, g_walk_stream, g_walk_unit, g_walk_slot++);
    } else {
        uint64_t s = g_n / g_D, slot = g_n % g_D;
        g_n++;
        k = orc_word(g_seed, 0, s, (uint32_t)slot);
    }
    if (min == 0 && max == 1) return std::ldexp((double)k, -32);
    return (double)min + (double)(((uint64_t)k * (uint64_t)(max - min)) >> 32);
}

// proNet::RandomWalk(long, int) returns vector<long> by value: sret in the
// first integer register, `this` second (SysV x86-64).  Pass-through wrapper.
extern "C" void* __real__ZN6proNet10RandomWalkEli(void* ret, void* self, long start, int steps);
extern "C" void* __wrap__ZN6proNet10RandomWalkEli(void* ret, void* self, long start, int steps) {
    g_walk_unit = g_walk_counter++;
    g_walk_slot = 0;
    return __real__ZN6proNet10RandomWalkEli(ret, self, start, steps);
}

// proNet::JumpingRandomWalk(long, double): same sret convention (jump in xmm0)
extern "C" void* __real__ZN6proNet17JumpingRandomWalkEld(void* ret, void* self, long start, double jump);
extern "C" void* __wrap__ZN6proNet17JumpingRandomWalkEld(void* ret, void* self, long start, double jump) {
    g_walk_unit = g_walk_counter++;
    g_walk_slot = 0;
    return __real__ZN6proNet17JumpingRandomWalkEld(ret, self, start, jump);
}

// proNet::SourceSample(): HPE's sample starts here (a new unit)
extern "C" long __real__ZN6proNet12SourceSampleEv(void* self);
extern "C" long __wrap__ZN6proNet12SourceSampleEv(void* self) {
    if (g_hpe_mode) {
        g_walk_unit = g_walk_counter++;
        g_walk_slot = 0;
    }
    return __real__ZN6proNet12SourceSampleEv(self);
}

// ---------------------------------------------------------------- tiny container
// "SMRF" then records: u32 name_len, name, u8 dtype ('d','q','i','b'),
// u32 ndim, u64 shape[ndim], raw data.
struct Out {
    FILE* f;
    explicit Out(const char* path) {
        f = fopen(path, "wb");
        if (!f) { perror(path); exit(2); }
        fwrite("SMRF", 1, 4, f);
    }
    ~Out() { fclose(f); }
    void put(const char* name, char dt, std::vector<uint64_t> shape, const void* data, size_t esz) {
        uint32_t nl = (uint32_t)strlen(name);
        fwrite(&nl, 4, 1, f);
        fwrite(name, 1, nl, f);
        fwrite(&dt, 1, 1, f);
        uint32_t nd = (uint32_t)shape.size();
        fwrite(&nd, 4, 1, f);
        size_t n = 1;
        for (auto s : shape) { fwrite(&s, 8, 1, f); n *= s; }
        if (n) fwrite(data, esz, n, f);
    }
    void f64(const char* name, const std::vector<double>& v) { put(name, 'd', {v.size()}, v.data(), 8); }
    void i64(const char* name, const std::vector<long>& v) { put(name, 'q', {v.size()}, v.data(), 8); }
    void table(const char* name, const std::vector<std::vector<double>>& t, int dim) {
        std::vector<double> flat;
        flat.reserve(t.size() * dim);
        for (auto& r : t) flat.insert(flat.end(), r.begin(), r.begin() + dim);
        put(name, 'd', {t.size(), (uint64_t)dim}, flat.data(), 8);
    }
};

static std::vector<double> read_dist(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    std::vector<double> v;
    double x;
    while (fread(&x, 8, 1, f) == 1) v.push_back(x);
    fclose(f);
    return v;
}

static void dump_graph(Out& o, proNet& pn) {
    std::vector<long> offset, branch, ctx_vid, valias, nalias, calias;
    std::vector<double> outd, ind, ctx_w, vprob, nprob, cprob;
    for (long v = 0; v < pn.MAX_vid; ++v) {
        offset.push_back(pn.vertex[v].offset);
        branch.push_back(pn.vertex[v].branch);
        outd.push_back(pn.vertex[v].out_degree);
        ind.push_back(pn.vertex[v].in_degree);
        valias.push_back(pn.vertex_AT[v].alias);
        vprob.push_back(pn.vertex_AT[v].prob);
        nalias.push_back(pn.negative_AT[v].alias);
        nprob.push_back(pn.negative_AT[v].prob);
    }
    for (unsigned long long e = 0; e < pn.MAX_line; ++e) {
        ctx_vid.push_back(pn.context[e].vid);
        ctx_w.push_back(pn.context[e].in_degree);
        calias.push_back(pn.context_AT[e].alias);
        cprob.push_back(pn.context_AT[e].prob);
    }
    std::string names;
    std::vector<long> name_off;
    for (long v = 0; v < pn.MAX_vid; ++v) {
        name_off.push_back((long)names.size());
        names += pn.vertex_hash.keys[v];
    }
    name_off.push_back((long)names.size());
    o.i64("offset", offset); o.i64("branch", branch);
    o.f64("out_degree", outd); o.f64("in_degree", ind);
    o.i64("ctx_vid", ctx_vid); o.f64("ctx_w", ctx_w);
    o.f64("vprob", vprob); o.i64("valias", valias);
    o.f64("nprob", nprob); o.i64("nalias", nalias);
    o.f64("cprob", cprob); o.i64("calias", calias);
    o.put("names", 'b', {names.size()}, names.data(), 1);
    o.i64("name_off", name_off);
}

static void usage() {
    fprintf(stderr,
            "ref_harness alias <dist.f64> <out>\n"
            "ref_harness sigmoid <x.f64> <out>\n"
            "ref_harness graph <edges> <undirected> <vertex_method> <negative_method> <out>\n"
            "ref_harness line <edges> <undirected> <order> <dim> <sample_times> <K> <alpha> <seed> <out>\n"
            "ref_harness mf <edges> <dim> <sample_times> <K> <alpha> <reg> <seed> <out>\n"
            "ref_harness bpr <edges> <dim> <sample_times> <alpha> <reg> <seed> <out>\n"
            "ref_harness deepwalk <edges> <undirected> <dim> <walk_times> <walk_steps> <window> <K> <alpha> <seed> <out>\n"
            "ref_harness walklets <edges> <undirected> <dim> <walk_times> <walk_steps> <wmin> <wmax> <K> <alpha> <seed> <out>\n"
            "ref_harness app <edges> <undirected> <dim> <walk_times> <sample_times> <jump> <K> <alpha> <seed> <out>\n"
            "ref_harness hpe <edges> <undirected> <dim> <sample_times> <walk_steps> <K> <reg> <alpha> <seed> <out>\n"
            "ref_harness updates <edges> <undirected> <model:line2|line1|mf|bpr> <dim> <K> <alpha> <reg> <seed> <first> <n> <out>\n"
            "ref_harness pairs <edges> <undirected> <dim> <K> <alpha> <seed> <unit> <pairs.i64> <out>\n");
    exit(1);
}

int main(int argc, char** argv) {
    if (argc < 2) usage();
    std::string mode = argv[1];
    if (mode == "alias" && argc == 4) {
        std::vector<double> d = read_dist(argv[2]);
        proNet pn;
        std::vector<AliasTable> at = pn.AliasMethod(d, 1.0);
        std::vector<double> p; std::vector<long> a;
        for (auto& e : at) { p.push_back(e.prob); a.push_back(e.alias); }
        Out o(argv[3]);
        o.f64("prob", p); o.i64("alias", a);
        return 0;
    }
    if (mode == "sigmoid" && argc == 4) {
        std::vector<double> x = read_dist(argv[2]), y;
        proNet pn;
        for (double v : x) y.push_back(pn.fastSigmoid(v));
        Out o(argv[3]);
        o.f64("x", x); o.f64("y", y);
        return 0;
    }
    if (mode == "graph" && argc == 7) {
        proNet pn;
        pn.SetVertexMethod(argv[4]);
        pn.SetNegativeMethod(argv[5]);
        pn.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        Out o(argv[6]);
        dump_graph(o, pn);
        return 0;
    }
    if (mode == "line" && argc == 11) {
        int order = atoi(argv[4]), dim = atoi(argv[5]), st = atoi(argv[6]), K = atoi(argv[7]);
        double alpha = atof(argv[8]);
        g_seed = strtoull(argv[9], 0, 10);
        LINE m;
        m.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        m.Init(dim, order);
        Out o(argv[10]);
        if (order == 1) o.table("W0", m.w_vertex_o1, dim);
        else { o.table("W0", m.w_vertex, dim); o.table("C0", m.w_context, dim); }
        g_D = 4 + 2 * (uint64_t)K; g_n = 0;
        m.Train(st, K, alpha, 1);
        if (order == 1) o.table("W", m.w_vertex_o1, dim);
        else { o.table("W", m.w_vertex, dim); o.table("C", m.w_context, dim); }
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "mf" && argc == 10) {
        int dim = atoi(argv[3]), st = atoi(argv[4]), K = atoi(argv[5]);
        double alpha = atof(argv[6]), reg = atof(argv[7]);
        g_seed = strtoull(argv[8], 0, 10);
        MF m;
        m.LoadEdgeList(argv[2], 0);
        m.Init(dim);
        Out o(argv[9]);
        o.table("W0", m.w_vertex, dim);
        g_D = 4 + 2 * (uint64_t)K; g_n = 0;
        m.Train(st, K, alpha, reg, 1);
        o.table("W", m.w_vertex, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "bpr" && argc == 9) {
        int dim = atoi(argv[3]), st = atoi(argv[4]);
        double alpha = atof(argv[5]), reg = atof(argv[6]);
        g_seed = strtoull(argv[7], 0, 10);
        BPR m;
        m.LoadEdgeList(argv[2], 0);
        m.Init(dim);
        Out o(argv[8]);
        o.table("W0", m.w_vertex, dim);
        g_D = 14; g_n = 0;
        m.Train(st, 5, alpha, reg, 1);
        o.table("W", m.w_vertex, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "deepwalk" && argc == 12) {
        int dim = atoi(argv[4]), wt = atoi(argv[5]), ws = atoi(argv[6]), win = atoi(argv[7]), K = atoi(argv[8]);
        double alpha = atof(argv[9]);
        g_seed = strtoull(argv[10], 0, 10);
        DeepWalk m;
        m.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        m.Init(dim);
        Out o(argv[11]);
        o.table("W0", m.w_vertex, dim); o.table("C0", m.w_context, dim);
        g_walk_mode = 1; g_walk_counter = 0;
        m.Train(wt, ws, win, K, alpha, 1);
        o.table("W", m.w_vertex, dim); o.table("C", m.w_context, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "walklets" && argc == 13) {
        int dim = atoi(argv[4]), wt = atoi(argv[5]), ws = atoi(argv[6]), wmin = atoi(argv[7]), wmax = atoi(argv[8]);
        int K = atoi(argv[9]);
        double alpha = atof(argv[10]);
        g_seed = strtoull(argv[11], 0, 10);
        Walklets m;
        m.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        m.Init(dim);
        Out o(argv[12]);
        o.table("W0", m.w_vertex, dim); o.table("C0", m.w_context, dim);
        g_walk_mode = 1; g_walk_counter = 0;
        m.Train(wt, ws, wmin, wmax, K, alpha, 1);
        o.table("W", m.w_vertex, dim); o.table("C", m.w_context, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "app" && argc == 12) {
        int dim = atoi(argv[4]), wt = atoi(argv[5]), st = atoi(argv[6]), K = atoi(argv[8]);
        double jump = atof(argv[7]), alpha = atof(argv[9]);
        g_seed = strtoull(argv[10], 0, 10);
        APP m;
        m.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        m.Init(dim);
        Out o(argv[11]);
        o.table("W0", m.w_vertex, dim); o.table("C0", m.w_context, dim);
        g_walk_mode = 1; g_walk_counter = 0;
        m.Train(wt, st, jump, K, alpha, 1);
        o.table("W", m.w_vertex, dim); o.table("C", m.w_context, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "hpe" && argc == 12) {
        int dim = atoi(argv[4]), st = atoi(argv[5]), ws = atoi(argv[6]), K = atoi(argv[7]);
        double reg = atof(argv[8]), alpha = atof(argv[9]);
        g_seed = strtoull(argv[10], 0, 10);
        HPE m;
        m.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        m.Init(dim);
        Out o(argv[11]);
        o.table("W0", m.w_vertex, dim); o.table("C0", m.w_context, dim);
        g_walk_mode = 1; g_walk_stream = 0; g_hpe_mode = 1; g_walk_counter = 0;
        m.Train(st, ws, K, reg, alpha, 1);
        o.table("W", m.w_vertex, dim); o.table("C", m.w_context, dim);
        dump_graph(o, m.pnet);
        return 0;
    }
    if (mode == "updates" && argc == 13) {
        // Single-sample trials (golden G4): from fixed starting tables, apply
        // exactly one sample s = first + t of the driver's loop body.
        std::string model = argv[4];
        int dim = atoi(argv[5]), K = atoi(argv[6]);
        double alpha = atof(argv[7]), reg = atof(argv[8]);
        g_seed = strtoull(argv[9], 0, 10);
        uint64_t first = strtoull(argv[10], 0, 10);
        int n = atoi(argv[11]);
        proNet pn;
        if (model == "mf" || model == "bpr") { char nd[] = "no_degrees"; pn.SetNegativeMethod(nd); }
        pn.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        long V = pn.MAX_vid;
        // starting tables: a fixed LCG, magnitudes U(-0.5, 0.5) so dot products
        // span many sigmoid buckets
        std::vector<std::vector<double>> W0(V, std::vector<double>(dim)), C0 = W0;
        uint64_t lcg = 0x243F6A8885A308D3ull;
        auto nxt = [&]() { lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
                           return std::ldexp((double)(lcg >> 11), -53) - 0.5; };
        for (long v = 0; v < V; ++v) for (int d = 0; d < dim; ++d) W0[v][d] = nxt();
        for (long v = 0; v < V; ++v) for (int d = 0; d < dim; ++d) C0[v][d] = nxt();
        Out o(argv[12]);
        o.table("W0", W0, dim); o.table("C0", C0, dim);
        std::vector<double> Wout, Cout;
        std::vector<long> ids;
        g_D = (model == "bpr") ? 14 : 4 + 2 * (uint64_t)K;
        for (int t = 0; t < n; ++t) {
            uint64_t s = first + t;
            auto W = W0, C = C0;
            g_n = s * g_D;
            long v = pn.SourceSample();
            long c = pn.TargetSample(v);
            ids.push_back((long)s); ids.push_back(v); ids.push_back(c);
            if (c < 0) { fprintf(stderr, "sample %llu has no target\n", (unsigned long long)s); return 3; }
            if (model == "line2") pn.UpdatePair(W, C, v, c, dim, K, alpha);
            else if (model == "line1") pn.UpdatePair(W, W, v, c, dim, K, alpha);
            else if (model == "mf") pn.UpdateFactorizedPair(W, W, v, c, dim, reg, K, alpha);
            else if (model == "bpr") { long j = pn.NegativeSample(); pn.UpdateBPRPair(W, W, v, c, j, dim, reg, alpha); }
            else usage();
            for (auto& r : W) Wout.insert(Wout.end(), r.begin(), r.end());
            for (auto& r : C) Cout.insert(Cout.end(), r.begin(), r.end());
        }
        o.put("W", 'd', {(uint64_t)n, (uint64_t)V, (uint64_t)dim}, Wout.data(), 8);
        o.put("C", 'd', {(uint64_t)n, (uint64_t)V, (uint64_t)dim}, Cout.data(), 8);
        o.put("trial", 'q', {(uint64_t)n, 3}, ids.data(), 8);
        dump_graph(o, pn);
        return 0;
    }
    if (mode == "pairs" && argc == 11) {
        // caller-supplied pairs (smore_train_pairs): proNet::UpdatePairs over
        // the pairs in <pairs.i64> (v, c interleaved) from fixed starting
        // tables (the "updates" LCG); block b of ORC_PAIR_BLOCK pairs draws
        // from stream 3, unit <unit> + b, consecutive slots
        int dim = atoi(argv[4]), K = atoi(argv[5]);
        double alpha = atof(argv[6]);
        g_seed = strtoull(argv[7], 0, 10);
        uint64_t unit0 = strtoull(argv[8], 0, 10);
        std::vector<double> raw = read_dist(argv[9]);   // 8-byte records, reinterpreted below
        std::vector<long> pv, pc;
        for (size_t i = 0; i + 1 < raw.size(); i += 2) {
            long a, b;
            memcpy(&a, &raw[i], 8);
            memcpy(&b, &raw[i + 1], 8);
            pv.push_back(a);
            pc.push_back(b);
        }
        proNet pn;
        pn.LoadEdgeList(argv[2], atoi(argv[3]) != 0);
        long V = pn.MAX_vid;
        std::vector<std::vector<double>> W(V, std::vector<double>(dim)), C = W;
        uint64_t lcg = 0x243F6A8885A308D3ull;
        auto nxt = [&]() { lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
                           return std::ldexp((double)(lcg >> 11), -53) - 0.5; };
        for (long v = 0; v < V; ++v) for (int d = 0; d < dim; ++d) W[v][d] = nxt();
        for (long v = 0; v < V; ++v) for (int d = 0; d < dim; ++d) C[v][d] = nxt();
        Out o(argv[10]);
        o.table("W0", W, dim); o.table("C0", C, dim);
        g_walk_mode = 1; g_walk_stream = 3;
        for (size_t b = 0; b < pv.size(); b += ORC_PAIR_BLOCK) {
            const size_t e = std::min(pv.size(), b + (size_t)ORC_PAIR_BLOCK);
            std::vector<long> bv(pv.begin() + b, pv.begin() + e), bc(pc.begin() + b, pc.begin() + e);
            g_walk_unit = unit0 + b / ORC_PAIR_BLOCK;
            g_walk_slot = 0;
            pn.UpdatePairs(W, C, bv, bc, dim, K, alpha);
        }
        o.table("W", W, dim); o.table("C", C, dim);
        o.i64("pv", pv); o.i64("pc", pc);
        dump_graph(o, pn);
        return 0;
    }
    usage();
    return 1;
}
