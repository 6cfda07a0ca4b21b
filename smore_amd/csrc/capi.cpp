// capi.cpp -- the C ABI (include/smore_hip.h) over the gfx950 kernels.
//
// A context owns one GPU's copy of the graph (CSR, encoded alias tables, the
// fastSigmoid table) and the embedding tables.  Everything on the device is
// uploaded once; training calls only launch kernels on the context stream.
#include "ctx.h"
#include "go_walks.h"
#include "hot_exchange.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using namespace smore_host;

extern "C" {

const char* smore_version(void) { return "smore_hip 0.1 (gfx950)"; }

int smore_create(int device, smore_ctx** out) {
    if (!out) return SMORE_EINVAL;
    *out = nullptr;
    smore_ctx* c = new smore_ctx();
    c->device = device;
    if (device < 0) {  // host-only context: graph/alias building, no device state
        *out = c;
        return SMORE_OK;
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->draw_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_skipped, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(c->d_skipped, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_work, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) {
        delete c;
        return SMORE_EHIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return SMORE_OK;
}

void smore_destroy(smore_ctx* c) {
    if (!c) return;
    smore_exchange_release(c);
    if (c->device >= 0) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    dfree(c->d_offsets); dfree(c->d_targets); dfree(c->d_vtab); dfree(c->d_ntab); dfree(c->d_ctab);
    dfree(c->d_sig); dfree(c->d_skipped); dfree(c->d_work); dfree(c->d_table[0]); dfree(c->d_table[1]);

    dfree(c->d_order); dfree(c->d_walks); dfree(c->d_lens); dfree(c->d_tcum); dfree(c->d_wts); dfree(c->d_nbr_sorted); dfree(c->d_ntype); dfree(c->d_ttargets); dfree(c->d_toff); dfree(c->d_paths); dfree(c->d_path_off); dfree(c->d_t_off); dfree(c->d_t_tgt); dfree(c->d_t_ts); dfree(c->d_t_min); dfree(c->d_t_max); dfree(c->d_sh_hash); dfree(c->d_sh_ids);
    dfree(c->d_rec); dfree(c->d_vt32); dfree(c->d_ct16); dfree(c->d_split);
    dfree(c->d_pcount); dfree(c->d_poff); dfree(c->d_pairs); dfree(c->d_census[0]); dfree(c->d_census[1]);
    dfree(c->d_io_ids[0]); dfree(c->d_io_rows[0]); dfree(c->d_io_ids[1]); dfree(c->d_io_rows[1]);
    blocks_release(c);
    if (c->d_scan_tmp) (void)hipFree(c->d_scan_tmp);
    for (hipEvent_t e : c->phase_ev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->draw_stream) (void)hipStreamDestroy(c->draw_stream);
    for (hipEvent_t e : c->sync_ev) (void)hipEventDestroy(e);
    delete c;
}

const char* smore_last_error(const smore_ctx* c) { return c ? c->err.c_str() : "null context"; }

int smore_set_stream(smore_ctx* c, void* s) {
    if (!c) return SMORE_EINVAL;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return SMORE_OK;
}

int smore_synchronize(smore_ctx* c) {
    if (!c) return SMORE_EINVAL;
    if (c->device < 0) return SMORE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    if ((rc = comm_sync(c))) return rc;   // own communicator: the RCCL failure watch first
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

// ---------------------------------------------------------------- graph
int smore_set_graph_edges(smore_ctx* c, int64_t V, int64_t E, const int32_t* src, const int32_t* dst,
                          const double* w, int vm, int nm) {
    if (!c) return SMORE_EINVAL;
    if ((E > 0 && (!src || !dst || !w)) || vm < 0 || vm > 2 || nm < 0 || nm > 2)
        return fail(c, SMORE_EINVAL, "bad arguments");
    c->g = std::make_shared<HostGraph>();
    c->hot_key.clear();
    c->semantics = SMORE_SEM_CPP;
    if (!build_graph(V, E, src, dst, w, vm, nm, *c->g, c->err)) return SMORE_EINVAL;
    return upload_graph(c);
}

int smore_load_edgelist(smore_ctx* c, const char* path, int undirected, int vm, int nm) {
    if (!c || !path) return SMORE_EINVAL;
    if (vm < 0 || vm > 2 || nm < 0 || nm > 2) return fail(c, SMORE_EINVAL, "bad arguments");
    std::vector<std::string> names;
    std::vector<int32_t> src, dst;
    std::vector<double> w;
    const char* cache = !c->cache_dir.empty() ? c->cache_dir.c_str() : getenv("SMORE_CACHE_DIR");
    const auto t0 = std::chrono::steady_clock::now();
    // with a cache directory: the built graph of this input and these methods,
    // if an earlier load stored it (no parse, no CSR / alias build)
    std::string gfile;
    uint64_t key = 0;
    if (cache && *cache && edgelist_key(path, undirected != 0, &key, c->err)) {
        char name[96];
        snprintf(name, sizeof name, "/%016llx-v%dn%d.smoregc", (unsigned long long)key, vm, nm);
        gfile = std::string(cache) + name;
        auto g = std::make_shared<HostGraph>();
        if (load_graph_cache(gfile, key, vm, nm, *g)) {
            c->g = g;
            c->hot_key.clear();
            c->semantics = SMORE_SEM_CPP;
            c->load_stats = LoadStats();
            c->load_stats.cache_hit = 2;
            c->load_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            return upload_graph(c);
        }
    }
    if (!read_edgelist(path, undirected != 0, names, src, dst, w, c->err, cache, &c->load_stats)) return SMORE_EIO;
    c->load_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (names.empty()) return fail(c, SMORE_EIO, std::string("no edges in ") + path);
    int rc = smore_set_graph_edges(c, (int64_t)names.size(), (int64_t)src.size(), src.data(), dst.data(),
                                   w.data(), vm, nm);
    if (rc == SMORE_OK) c->g->names = std::move(names);
    if (rc == SMORE_OK && !gfile.empty()) (void)save_graph_cache(gfile, key, *c->g);
    return rc;
}

// the built graph (CSR, degrees, alias tables) to / from a binary file: one
// process of a multi-GPU job builds it, the others read it (bench.py at N > 1;
// the same format as the edge-list loader's graph cache, loader.cpp)
static constexpr uint64_t GRAPH_FILE_KEY = 0x534d4f5245475246ull;   // "SMOREGRF"

int smore_save_graph(const smore_ctx* c, const char* path) {
    if (!c || !path) return SMORE_EINVAL;
    if (!c->has_graph) return SMORE_ESTATE;
    return save_graph_cache(path, GRAPH_FILE_KEY, *c->g) ? SMORE_OK : SMORE_EIO;
}

int smore_load_graph(smore_ctx* c, const char* path, int vm, int nm) {
    if (!c || !path || vm < 0 || vm > 2 || nm < 0 || nm > 2) return SMORE_EINVAL;
    auto g = std::make_shared<HostGraph>();
    if (!load_graph_cache(path, GRAPH_FILE_KEY, vm, nm, *g))
        return fail(c, SMORE_EIO, std::string("cannot read a graph file (or other sampling methods): ") + path);
    c->g = g;
    c->hot_key.clear();
    c->semantics = SMORE_SEM_CPP;
    return upload_graph(c);
}

int smore_set_load_cache(smore_ctx* c, const char* dir) {
    if (!c) return SMORE_EINVAL;
    c->cache_dir = dir ? dir : "";
    return SMORE_OK;
}

int smore_last_load_info(const smore_ctx* c, double* seconds, int* threads, int* cache_hit) {
    if (!c) return SMORE_EINVAL;
    if (seconds) *seconds = c->load_seconds;
    if (threads) *threads = c->load_stats.threads;
    if (cache_hit) *cache_hit = c->load_stats.cache_hit;
    return SMORE_OK;
}

int smore_graph_info(const smore_ctx* c, int64_t* V, int64_t* E) {
    if (!c) return SMORE_EINVAL;
    if (V) *V = c->g->V;
    if (E) *E = c->g->E;
    return c->has_graph ? SMORE_OK : SMORE_ESTATE;
}

const char* smore_vertex_name(const smore_ctx* c, int64_t vid) {
    if (!c || vid < 0 || vid >= (int64_t)c->g->names.size()) return nullptr;
    return c->g->names[vid].c_str();
}

int smore_get_csr(const smore_ctx* c, int64_t* offsets, int32_t* targets) {
    if (!c || !c->has_graph) return SMORE_ESTATE;
    if (offsets) memcpy(offsets, c->g->offsets.data(), c->g->offsets.size() * sizeof(int64_t));
    if (targets) memcpy(targets, c->g->targets.data(), c->g->targets.size() * sizeof(int32_t));
    return SMORE_OK;
}

static int apply_partition(smore_ctx* c);   // source partition (below)

int smore_set_alias(smore_ctx* c, int which, const double* prob, const int64_t* alias, int64_t n) {
    if (!c || !prob || !alias) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    HostGraph& g = *c->g;
    int64_t want = which == SMORE_AT_CONTEXT ? g.E : g.V;
    if (which < 0 || which > 2 || n != want) return fail(c, SMORE_EINVAL, "alias table size mismatch");
    int64_t lim = g.V;
    for (int64_t i = 0; i < n; ++i) {
        if (alias[i] >= lim || alias[i] < -1 || !(prob[i] >= 0)) return fail(c, SMORE_EINVAL, "alias entry out of range");
        if (which != SMORE_AT_CONTEXT && alias[i] >= g.V) return fail(c, SMORE_EINVAL, "alias out of range");
    }
    hvec<double>& P = which == 0 ? g.vprob : which == 1 ? g.nprob : g.cprob;
    hvec<int64_t>& A = which == 0 ? g.valias : which == 1 ? g.nalias : g.calias;
    hvec<AliasEntry>& T = which == 0 ? g.vtab : which == 1 ? g.ntab : g.ctab;
    P.assign(prob, prob + n);
    A.assign(alias, alias + n);
    c->hot_key.clear();
    T.resize((size_t)n);
    alias_encode(P.data(), A.data(), n, which == SMORE_AT_CONTEXT ? g.targets.data() : nullptr, T.data());
    if (c->device < 0) return SMORE_OK;
    int rc;
    if ((rc = set_device(c))) return rc;
    AliasEntry*& d = which == 0 ? c->d_vtab : which == 1 ? c->d_ntab : c->d_ctab;
    c->packed_ok = false;
    if ((rc = upload(c, d, T.data(), T.size()))) return rc;
    return which == 0 && c->part_n > 1 ? apply_partition(c) : SMORE_OK;   // the new law, restricted again
}

int smore_get_alias(const smore_ctx* c, int which, double* prob, int64_t* alias, int64_t n) {
    if (!c || !c->has_graph || which < 0 || which > 2) return SMORE_EINVAL;
    const HostGraph& g = *c->g;
    const hvec<double>& P = which == 0 ? g.vprob : which == 1 ? g.nprob : g.cprob;
    const hvec<int64_t>& A = which == 0 ? g.valias : which == 1 ? g.nalias : g.calias;
    if (n != (int64_t)P.size()) return SMORE_EINVAL;
    if (prob) memcpy(prob, P.data(), n * sizeof(double));
    if (alias) memcpy(alias, A.data(), n * sizeof(int64_t));
    return SMORE_OK;
}

int smore_get_alias_encoded(const smore_ctx* c, int which, uint32_t* thresh, int32_t* alias, int64_t n) {
    if (!c || !c->has_graph || which < 0 || which > 2) return SMORE_EINVAL;
    const HostGraph& g = *c->g;
    const hvec<AliasEntry>& T = which == 0 ? g.vtab : which == 1 ? g.ntab : g.ctab;
    if (n != (int64_t)T.size()) return SMORE_EINVAL;
    for (int64_t i = 0; i < n; ++i) {
        if (thresh) thresh[i] = T[i].thresh;
        if (alias) alias[i] = T[i].alias;
    }
    return SMORE_OK;
}

// ---------------------------------------------------------------- tables
int smore_alloc_tables(smore_ctx* c, int dim, int ntables) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (dim <= 0 || dim > 512 || ntables < 1 || ntables > 2) return fail(c, SMORE_EINVAL, "bad dim/ntables");
    int rc;
    if ((rc = set_device(c))) return rc;
    dfree(c->d_table[0]);
    dfree(c->d_table[1]);
    c->dim = dim;
    c->dpad = (dim + 3) / 4 * 4;
    c->ntables = ntables;
    size_t bytes = (size_t)c->g->V * c->dpad * sizeof(float);
    // the C table of a two-table model carries HUB_SLOTS_MAX rows after V: the
    // block schedule's hub slots (blocks.cpp), never part of a rotating block
    c->c_slots = ntables == 2 ? std::min<int64_t>(HUB_SLOTS_MAX, c->g->V) : 0;
    const size_t cbytes = bytes + (size_t)c->c_slots * c->dpad * sizeof(float);
    // The embedding tables live in UNCACHED device memory: every row access is
    // served memory-side (Infinity Cache / HBM), which is coherent across the
    // 8 XCDs.  In the default coarse-grained memory each XCD's L2 keeps its own
    // copy of a row, so a plain-store (Hogwild) update made on one XCD is
    // overwritten by a read-modify-write from another XCD that still holds the
    // old line -- lost updates the reference's cache-coherent CPU Hogwild never
    // has (DESIGN.md "Scatter modes": DeepWalk held-out AUC on 2 blocks 0.82 ->
    // 0.87, the atomic level).  Measured on one box, C4 LINE-2 +2.5 %, C5
    // DeepWalk +8.6 %, C3 BPR equal (rows are random and miss L2 anyway).
    // SMORE_TABLE_MEM=coarse|finegrained|uncached overrides (experiments).
    unsigned flags = hipDeviceMallocUncached;
    if (const char* e = getenv("SMORE_TABLE_MEM")) {
        if (!strcmp(e, "coarse")) flags = hipDeviceMallocDefault;
        else if (!strcmp(e, "finegrained")) flags = hipDeviceMallocFinegrained;
        else if (!strcmp(e, "contiguous")) flags = hipDeviceMallocContiguous;
    }
    for (int t = 0; t < ntables; ++t)
        HIPCHK(c, hipExtMallocWithFlags((void**)&c->d_table[t], t == 1 ? cbytes : bytes, flags));
    for (int t = 0; t < ntables; ++t) HIPCHK(c, hipMemset(c->d_table[t], 0, t == 1 ? cbytes : bytes));
    c->blk.key.clear();   // the block tables' hub slots live in the new C table
    return SMORE_OK;
}

static int check_table(smore_ctx* c, int which) {
    if (!c) return SMORE_EINVAL;
    if (which < 0 || which >= c->ntables || !c->d_table[which]) return fail(c, SMORE_ESTATE, "table not allocated");
    return SMORE_OK;
}

int smore_init_table_glibc(smore_ctx* c, int which, uint64_t skip) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    GlibcRand r;
    r.discard(skip);
    std::vector<float> h((size_t)c->g->V * c->dpad, 0.0f);
    for (int64_t v = 0; v < c->g->V; ++v)
        for (int d = 0; d < c->dim; ++d)
            h[(size_t)v * c->dpad + d] = (float)((r.next() / (double)2147483647 - 0.5) / c->dim);
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipMemcpy(c->d_table[which], h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    return SMORE_OK;
}

int smore_init_table_uniform(smore_ctx* c, int which, uint64_t seed) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, launch_init_uniform(c->d_table[which], c->g->V, c->dim, c->dpad, seed, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_zero_table(smore_ctx* c, int which) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipMemsetAsync(c->d_table[which], 0, (size_t)c->g->V * c->dpad * sizeof(float), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_set_table(smore_ctx* c, int which, const float* host, int64_t rows, int dim) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (!host || rows != c->g->V || dim != c->dim) return fail(c, SMORE_EINVAL, "table shape mismatch");
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy2D(c->d_table[which], c->dpad * sizeof(float), host, dim * sizeof(float),
                          dim * sizeof(float), rows, hipMemcpyHostToDevice));
    return SMORE_OK;
}

int smore_get_table(const smore_ctx* cc, int which, float* host, int64_t rows, int dim) {
    smore_ctx* c = const_cast<smore_ctx*>(cc);
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (!host || rows != c->g->V || dim != c->dim) return fail(c, SMORE_EINVAL, "table shape mismatch");
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy2D(host, dim * sizeof(float), c->d_table[which], c->dpad * sizeof(float),
                          dim * sizeof(float), rows, hipMemcpyDeviceToHost));
    return SMORE_OK;
}

int smore_table_device(smore_ctx* c, int which, void** dptr, int64_t* stride) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (dptr) *dptr = c->d_table[which];
    if (stride) *stride = c->dpad;
    return SMORE_OK;
}

// ---------------------------------------------------------------- source partition
// Part bounds of the current (global) source law: vertex v belongs to the part
// holding the midpoint of its probability mass, so parts are contiguous id
// ranges of (nearly) equal mass; bound[p] .. bound[p + 1] - 1 is part p.
static void source_bounds(const std::vector<double>& ps, int n, std::vector<int64_t>& bound) {
    const int64_t V = (int64_t)ps.size();
    double total = 0.0;
    for (double p : ps) total += p;
    bound.assign((size_t)n + 1, V);
    bound[0] = 0;
    double cum = 0.0;
    int next = 1;
    for (int64_t v = 0; v < V && next < n; ++v) {
        const double mid = (cum + 0.5 * ps[v]) / total;
        const int owner = std::min(n - 1, (int)std::floor(mid * n));
        while (next <= owner && next < n) bound[next++] = v;
        cum += ps[v];
    }
}

// the source law restricted to part i of n and renormalised
static void partition_law(const std::vector<double>& ps, int n, int i, std::vector<double>& law) {
    std::vector<int64_t> bound;
    source_bounds(ps, n, bound);
    law.assign(ps.size(), 0.0);
    double sum = 0.0;
    for (int64_t v = bound[i]; v < bound[i + 1]; ++v) sum += ps[v];
    if (sum > 0.0)
        for (int64_t v = bound[i]; v < bound[i + 1]; ++v) law[v] = ps[v] / sum;
}

// Restrict the device vertex table to this context's part (renormalised, Go
// alias rule with power 1: any valid encoding of the law; N > 1 only, where
// draws are not compared with one GPU's) and upload it.
static int apply_partition(smore_ctx* c) {
    const HostGraph& g = *c->g;
    int rc;
    if ((rc = set_device(c))) return rc;
    c->packed_ok = false;
    c->hot_key.clear();
    if (c->part_n <= 1) {
        c->part_vtab.clear();
        c->part_bounds.clear();
        return upload(c, c->d_vtab, g.vtab.data(), g.vtab.size());
    }
    std::vector<double> ps, pn, pc;
    draw_probabilities(g, ps, pn, pc);
    std::vector<int64_t>& bound = c->part_bounds;
    source_bounds(ps, c->part_n, bound);
    const int64_t lo = bound[c->part_i], hi = bound[c->part_i + 1];
    if (hi <= lo) return fail(c, SMORE_EINVAL, "source partition: an empty part (more parts than vertices with mass)");
    std::vector<double> w((size_t)g.V, 0.0), prob((size_t)g.V);
    std::vector<int64_t> alias((size_t)g.V);
    for (int64_t v = lo; v < hi; ++v) w[v] = ps[v];
    alias_go(w.data(), g.V, 1.0, prob.data(), alias.data());
    c->part_vtab.resize((size_t)g.V);
    alias_encode(prob.data(), alias.data(), g.V, nullptr, c->part_vtab.data());
    return upload(c, c->d_vtab, c->part_vtab.data(), c->part_vtab.size());
}

int smore_source_parts(smore_ctx* c, int nparts, int64_t* bounds) {
    if (!c || !bounds || nparts < 1) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (nparts > c->g->V) return fail(c, SMORE_EINVAL, "more parts than vertices");
    if (c->part_n == nparts && (int)c->part_bounds.size() == nparts + 1) {   // the active partition's
        std::copy(c->part_bounds.begin(), c->part_bounds.end(), bounds);
        return SMORE_OK;
    }
    std::vector<double> ps, pn, pc;
    draw_probabilities(*c->g, ps, pn, pc);
    std::vector<int64_t> bound;
    source_bounds(ps, nparts, bound);
    std::copy(bound.begin(), bound.end(), bounds);
    return SMORE_OK;
}

int smore_set_source_partition(smore_ctx* c, int nparts, int part) {
    if (!c || nparts < 1 || part < 0 || part >= nparts) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (nparts > c->g->V) return fail(c, SMORE_EINVAL, "more parts than vertices");
    if (c->device < 0) return fail(c, SMORE_ESTATE, "host-only context");
    if (c->part_n == nparts && c->part_i == part) return SMORE_OK;   // kept current by the table setters
    c->part_n = nparts;
    c->part_i = part;
    return apply_partition(c);
}

// ---------------------------------------------------------------- hybrid scatter
// A row is "hot" when the expected number of resident sample groups touching
// it at once, M * p(row), exceeds tau; hot rows take float atomics, the rest
// plain stores (DESIGN.md "Scatter modes").
// Hybrid scatter: rows whose expected number of concurrent updates M * p(row)
// exceeds tau are tagged hot in the device graph's id words (device_common.h):
// W-rows through the vertex table, C-rows through the negative and context
// tables and the CSR targets (one union set for shared-table models).  Written
// in place into the existing device arrays; the host graph stays untagged.
constexpr double SH_STALE_MAX = 65536.0;
// automatic drain interval (smore_set_write_combine flush_rounds 0, the
// default): the hottest combined row gathers about M * p_top * flush updates
// that other workgroups cannot see yet; flush = budget / (M * p_top) within
// [8, 32] rounds keeps that at the config-4 level (flush 32) on hotter graphs
constexpr double SH_AUTO_BUDGET = 6144.0;
// the pair-record kernels' budget (and staleness bound): 1024 hidden updates,
// the one-GPU C5 DeepWalk top row's at its 8-round drain.  A walk group runs
// a walk's records in order, so a hub context row's hidden updates come in
// correlated bursts; 4096 (drain 32 at one GPU) cost C5 held-out loss +6 %,
// and under the 2-D block schedule (a cell's rows nb times hotter: the top
// row M p = 512 per round at 2 GPUs) it diverged (loss 2.6e8; budget 1024:
// 0.5308, one GPU 0.5309; profiles/r05/walk_blocks.txt)
constexpr double SH_PAIR_BUDGET = 1024.0;
// the 2-D block schedule's per-cell concurrency cap (blocks.cpp cell_grid):
// at most this many updates per round on a cell's hottest row (0: no cap).
// Walk cells need it: C5 DeepWalk on 8 GPUs (top row M p = 2048 per round)
// diverged without it and reached 1.027 x the one-GPU held-out loss with 512
// (1024: 1.027, 256: 1.024).  LINE-2 cells do not: C2 on 8 GPUs with the
// atomic scatter is at 0.99 x one GPU uncapped; what the hybrid loses there is
// the cold rows' plain stores (HOT_TAU_CELL), and the cap costs the hub cells
// 1.5-3 x (C4, 8 GPUs: predicted speed-up 3.4 x capped vs 4.9 x)
constexpr double CELL_RATE_PAIRS = 512.0, CELL_RATE_EDGES = 0.0;
static double sh_budget(bool pairs) {
    if (const char* e = getenv("SMORE_SH_BUDGET")) return atof(e);
    return pairs ? SH_PAIR_BUDGET : SH_AUTO_BUDGET;
}
// LINE-2 cells of the 2-D block schedule (blocks.cpp block_sh_sets): twice the
// edge budget.  A cell's hub rows are 2N times hotter, so at the edge budget
// they drain every 1-2 rounds and the hub cells are bound by those drains'
// memory-side atomics; C4 on 8 GPUs predicted 4.9 x at 6144, 5.5 x at 9216,
// 5.8 x at 12288, 6.3 x at 24576, for C2 held-out loss 1.019 / 1.031 / 1.037 /
// 1.077 x one GPU (profiles/r05/blocks)
constexpr double SH_CELL_BUDGET = 12288.0;
static double cell_budget(bool walk) {
    if (const char* e = getenv("SMORE_SH_BUDGET")) return atof(e);
    return walk ? SH_PAIR_BUDGET : SH_CELL_BUDGET;
}
// rows whose hidden updates would pass this even at a 1-round drain (edge
// rule) / the budget (pair rule) stay on atomics; SMORE_SH_STALE overrides
static double sh_stale(bool pairs) {
    if (const char* e = getenv("SMORE_SH_STALE")) return atof(e);
    return pairs ? SH_PAIR_BUDGET : SH_STALE_MAX;
}

// hot-row threshold defaults (smore_set_hot_threshold(ctx, -1)): the C++
// rules' edge-record kernel takes 1.0 (C4 / C2 update 4 % / 12 % faster than
// at 0.3, held-out loss +0.1 / +0.2 % of the atomic scatter's); the Go edge
// rules (no faster at 1.0: C4 Go LINE-2 1140 vs 1133 M/s) and the pair-record
// kernels keep 0.3 (on small graphs the walk models' runs of W_v updates need
// the context rows' atomics: Go DeepWalk AUC on the 920-vertex graph 0.881 at
// 1.0 vs 0.900 at 0.3, serial 0.906); DESIGN.md 8, profiles/r03/tau
constexpr double HOT_TAU_EDGE = 1.0, HOT_TAU_WALK = 0.3;
// LINE-2 cells of the 2-D block schedule: a cell's law is its C block's
// (1/2N of the rows) renormalised, so more of its updates land on rows just
// under the threshold, where plain stores collide.  C2 LINE-2 held-out loss
// on 8 GPUs / one GPU: tau 1.0 1.065, 0.5 1.026, 0.3 1.020 (atomic 0.99);
// C4 8-GPU predicted speed-up 4.9 x at 0.3 and 0.5 (profiles/r05/blocks.md)
constexpr double HOT_TAU_CELL = 0.3;

// PAIR_FLUSH_MAX: the pair-record kernels' automatic drain interval (8 rounds,
// the floor, instead of up to 32): a group runs a walk's consecutive records,
// so a combined context row gathers its pending deltas in bursts; C5 DeepWalk
// (d=128, 10 walks per vertex) held-out loss / AUC: drain 32 rounds (the edge
// rule's choice there) 0.5648 / 0.9835 in 2.99 s, 16: 0.5444 / 0.9840 in 3.02
// s, 8: 0.5376 / 0.9847 in 3.20 s, no combining 0.5312 / 0.9843 in 4.28 s,
// atomic 0.5276 / 0.9844 in 6.98 s (profiles/r04/walk_combine.jsonl)
constexpr int EDGE_FLUSH_MAX = 32, PAIR_FLUSH_MAX = 8;

// w_scale / c_scale (the 2-D block schedule, blocks.cpp): a launch then
// draws its W rows from one part of N and its C rows from one block of 2N, so
// the rows it touches are about N / 2N times as likely per sample as under
// the global law; the tags and the write-combined set follow the scaled law.
// The C-row law and the flags are kept on the host (hot_pc, hot_c) for the
// block tables' own tags and write-combined sets.
// drain interval of one write-combined row with M * p expected updates per
// round: the budget of hidden updates over that rate, a power of two in
// [1, cap] (cap a power of two) -- the two-tier drain's unit
static int slot_interval(double Mp, int cap, double budget) {
    int f = 1;
    while (2 * f <= cap && (double)(2 * f) * Mp <= budget) f *= 2;
    return f;
}

// EdgeArgs::sh_lvl of n slots sorted by rate: lvl[j] = the slots whose own
// interval is at most 2^j (and below cap, which every slot drains at)
static void sh_levels(int64_t M, int cap, double budget, const std::pair<double, int32_t>* r, int64_t n,
                      int (&lvl)[8]) {
    for (int j = 0; j < 8; ++j) {
        int64_t k = 0;
        while (k < n && slot_interval((double)M * r[k].first, cap, budget) <= (1 << j) && (1 << j) < cap) ++k;
        lvl[j] = (int)k;
    }
}

static int build_hot_maps(smore_ctx* c, int model, int K, int64_t M, double tau_default,
                          int flush_max = EDGE_FLUSH_MAX, double w_scale = 1.0, double c_scale = 1.0) {
    // Small graphs (the V/16 concurrency cap binds: 16 M >= V, e.g. the test
    // graphs, never C2-C5): with the default threshold every touched row is
    // hot and nothing is write-combined, i.e. the hybrid is the lossless
    // atomic scatter.  There every row is a hub (920 vertices: M p ~ 0.3-3 for
    // most rows), plain stores lose updates at any threshold (caller pairs,
    // C++ rules: held-out loss +2.6 % at tau 0.3, +16 % at 1.0, atomic +0.06 %;
    // profiles/r04/pairs_probe.jsonl), and the tables sit in L2, so the
    // memory-side traffic the hybrid saves does not exist.  An explicit
    // smore_set_hot_threshold keeps its meaning.
    const bool small = c->hot_tau < 0 && 16.0 * (double)M >= (double)c->g->V;
    const double tau = c->hot_tau >= 0 ? c->hot_tau : small ? 0.0 : tau_default;
    char key[128];
    const char* stale_env = getenv("SMORE_SH_STALE");
    // W rows of two-table models stay out of the write-combined set unless
    // SMORE_SH_WROWS=1: combining the hub W rows makes their pending deltas
    // invisible for a whole drain window, which cost Go LINE-2 (source law
    // out_degree^1, ~1 % of samples on one W row) 4.7 % held-out loss at C2
    // (0.7 % without), for +12 % C4 throughput; C++ LINE-2 gains nothing from
    // it (1338 vs 1342 M/s), DESIGN.md 8
    const char* wrows_env = getenv("SMORE_SH_WROWS");
    const bool wrows = wrows_env && atoi(wrows_env) != 0;
    // combined W rows drain on their own interval (SMORE_SH_WFLUSH rounds,
    // default 8; 0 = with the context rows)
    const char* wflush_env = getenv("SMORE_SH_WFLUSH");
    const int wflush = wrows ? (wflush_env ? std::max(0, atoi(wflush_env)) : 8) : 0;
    // per-slot drain levels (EdgeArgs::sh_lvl): the C++ rules' edge and pair
    // kernels; the Go record kernels drain on one interval
    const bool two_tier = c->semantics != SMORE_SEM_GO && c->sh_flush <= 0 && !wrows;
    snprintf(key, sizeof key, "%d/%d/%lld/%.9g/%d/%d/%s/%d/%d/%d/%d/%d/%g/%g/%d", model, K, (long long)M, tau,
             c->sh_max, c->sh_flush, stale_env ? stale_env : "", (int)wrows, c->part_n, c->part_i, flush_max, wflush,
             w_scale, c_scale, (int)two_tier);
    if (c->hot_key == key) return SMORE_OK;
    if (c->g->V >= ((int64_t)1 << 30)) return fail(c, SMORE_EINVAL, "hybrid scatter needs V < 2^30");
    std::vector<double> ps, pn, pc;
    draw_probabilities(*c->g, ps, pn, pc);
    if (c->part_n > 1) {
        // this replica draws its sources from its part only: the hot rows
        // follow the restricted law (its part's W rows N times as hot)
        std::vector<double> law;
        partition_law(ps, c->part_n, c->part_i, law);
        draw_probabilities(*c->g, ps, pn, pc, &law);
    }
    const int64_t V = c->g->V, E = c->g->E;
    std::vector<uint8_t> hw((size_t)V, 0), hc((size_t)V, 0);
    const int negs = model == SMORE_BPR ? 5 : K;
    c->hot_rows[0] = c->hot_rows[1] = 0;
    for (int64_t v = 0; v < V; ++v) {
        double pw, pcx;
        if (model == SMORE_LINE2) { pw = ps[v] * w_scale; pcx = (pc[v] + negs * pn[v]) * c_scale; }
        else { pw = pcx = ps[v] + pc[v] + negs * pn[v]; }
        if ((double)M * pw > tau) { hw[v] = 1; c->hot_rows[0]++; }
        if ((double)M * pcx > tau) { hc[v] = 1; c->hot_rows[1]++; }
    }
    // super-hot rows: the hottest hot context rows, write-combined per block
    {
        // the pair-record kernels (walks) pass PAIR_FLUSH_MAX: their budget
        const bool pairs = flush_max == PAIR_FLUSH_MAX;
        const double stale_max = sh_stale(pairs), budget = sh_budget(pairs);
        std::vector<std::pair<double, int32_t>> r;
        const int flush_cap = c->sh_flush > 0 ? c->sh_flush : flush_max;
        for (int64_t v = 0; v < V; ++v) {
            const double p = model == SMORE_LINE2 ? (pc[v] + negs * pn[v]) * c_scale : ps[v] + pc[v] + negs * pn[v];
            // bounded staleness: a combined row's pending deltas are invisible to
            // other workgroups for up to sh_flush rounds, i.e. about
            // M * p * sh_flush updates; rows above SH_STALE_MAX stay on atomics
            // (on small graphs that is every hot row)
            // (two tiers: each row at its own interval, slot_interval)
            const double f = two_tier ? (double)slot_interval((double)M * p, flush_cap, budget) : (double)flush_cap;
            if (hc[v] && (double)M * p * f <= stale_max) r.push_back({p, (int32_t)v});
            // two tables (SMORE_SH_WROWS=1 only): the hub W rows compete for
            // the same slots (key v | SH_WKEY)
            if (wrows && model == SMORE_LINE2 && hw[v] &&
                (double)M * ps[v] * w_scale * (wflush ? wflush : flush_cap) <= stale_max)
                r.push_back({ps[v] * w_scale, (int32_t)(v | SH_WKEY)});
        }
        const int64_t cap =
            small ? 0 : std::max<int64_t>(0, std::min<int64_t>(c->sh_max, sh_rows_max(c->dpad)));
        const int64_t n = std::min<int64_t>(cap, (int64_t)r.size());
        std::partial_sort(r.begin(), r.begin() + n, r.end(), [](const auto& x, const auto& y) {
            return x.first > y.first || (x.first == y.first && x.second < y.second);
        });
        std::vector<int2> hash(SH_HASH, make_int2(-1, -1));
        std::vector<int32_t> ids((size_t)std::max<int64_t>(n, 1), -1);
        for (int64_t i = 0; i < n; ++i) {
            const int32_t id = r[i].second;
            ids[i] = id;
            uint32_t p = sh_hash_of(id);
            while (hash[p & (SH_HASH - 1)].x >= 0) ++p;
            hash[p & (SH_HASH - 1)] = make_int2(id, (int)i);
        }
        int rc2;
        if ((rc2 = set_device(c))) return rc2;
        if ((rc2 = upload(c, c->d_sh_hash, hash.data(), hash.size()))) return rc2;
        if ((rc2 = upload(c, c->d_sh_ids, ids.data(), ids.size()))) return rc2;
        c->sh_rows = (int)n;
        c->sh_flush_eff = flush_cap;
        c->sh_flush_w_eff = wflush;
        // every slot drains every flush_cap rounds; a slot whose own interval
        // (slot_interval) is shorter also at its own (a prefix per level: r is
        // sorted by rate)
        for (int& x : c->sh_lvl_eff) x = 0;
        if (two_tier) sh_levels(M, flush_cap, budget, r.data(), n, c->sh_lvl_eff);
        if (getenv("SMORE_SH_DEBUG")) {
            const int* l = c->sh_lvl_eff;
            fprintf(stderr, "[sh] global M %lld rows %lld of %zu flush %d lvl %d %d %d %d %d %d %d %d top", (long long)M,
                    (long long)n, r.size(), flush_cap, l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]);
            for (int64_t i = 0; i < std::min<int64_t>(n, 4); ++i)
                fprintf(stderr, " %d:%.3g", r[i].second, (double)M * r[i].first);
            fprintf(stderr, "\n");
        }
        // the automatic interval follows the hottest row drained on it (with
        // their own interval, W rows do not count)
        int64_t top = 0;
        while (top < n && wflush && (r[top].second & SH_WKEY)) ++top;
        if (c->sh_flush <= 0 && top < n && !two_tier) {
            const double f = budget / ((double)M * r[top].first);
            c->sh_flush_eff = (int)std::max(8.0, std::min((double)flush_cap, std::floor(f)));
        }
    }
    const HostGraph& g = *c->g;
    auto tag_tab = [&](const hvec<AliasEntry>& tab, const std::vector<uint8_t>& hot) {
        std::vector<AliasEntry> t(tab.begin(), tab.end());
        for (int64_t i = 0; i < V; ++i) {
            const uint32_t al = (uint32_t)t[i].alias;
            t[i].alias = (int32_t)(al | ((uint32_t)hot[al] << 30) | ((uint32_t)hot[i] << 31));
        }
        return t;
    };
    int rc;
    if ((rc = set_device(c))) return rc;
    {
        const std::vector<AliasEntry> vt = tag_tab(c->part_n > 1 ? c->part_vtab : g.vtab, hw),
                                      nt = tag_tab(g.ntab, hc);
        HIPCHK(c, hipMemcpy(c->d_vtab, vt.data(), V * sizeof(AliasEntry), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_ntab, nt.data(), V * sizeof(AliasEntry), hipMemcpyHostToDevice));
    }
    // targets and context alias words, in slices to bound the host copy
    const int64_t slice = (int64_t)1 << 26;
    std::vector<int32_t> tt;
    std::vector<AliasEntry> ct;
    for (int64_t b = 0; b < E; b += slice) {
        const int64_t n = std::min(slice, E - b);
        tt.resize((size_t)n);
        ct.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const int32_t t = g.targets[b + i];
            tt[i] = t | ((int32_t)hc[t] << 30);
            const AliasEntry e = g.ctab[b + i];
            ct[i] = {e.thresh, e.alias | ((int32_t)hc[e.alias] << 30)};
        }
        HIPCHK(c, hipMemcpy(c->d_targets + b, tt.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_ctab + b, ct.data(), n * sizeof(AliasEntry), hipMemcpyHostToDevice));
    }
    c->hot_key = key;
    c->packed_ok = false;
    // the C-row law and flags for the block tables (blocks.cpp)
    c->hot_c.assign(hc.begin(), hc.end());
    c->hot_w.assign(hw.begin(), hw.end());
    c->hot_pc.resize((size_t)V);
    for (int64_t v = 0; v < V; ++v)
        c->hot_pc[v] = model == SMORE_LINE2 ? (pc[v] + negs * pn[v]) * c_scale : ps[v] + pc[v] + negs * pn[v];
    c->hot_M = M;
    c->hot_small = small;
    return SMORE_OK;
}

// packed draw tables (DevGraph::vt32 / ct16): built on the device from the
// current (tagged) tables; skipped when offsets do not fit 32 bits
static int ensure_packed(smore_ctx* c) {
    if (c->packed_ok) return SMORE_OK;
    const int64_t V = c->g->V, E = c->g->E;
    if (E >= ((int64_t)1 << 32)) return SMORE_OK;
    if (!c->d_vt32) HIPCHK(c, draw_malloc((void**)&c->d_vt32, (size_t)std::max<int64_t>(V, 1) * 2 * sizeof(uint4)));
    if (!c->d_ct16) HIPCHK(c, draw_malloc((void**)&c->d_ct16, (size_t)std::max<int64_t>(E, 1) * sizeof(uint4)));
    HIPCHK(c, launch_pack(dev_graph(c), (uint64_t)E, c->d_vt32, c->d_ct16, c->stream));
    c->packed_ok = true;
    return SMORE_OK;
}

// ---------------------------------------------------------------- training
static const void* go_rec_symbol(const EdgeArgs& a) {
    return a.mode == SMORE_ATOMIC ? go_rec_symbol_a(a) : a.mode == SMORE_HYBRID ? go_rec_symbol_h(a) : go_rec_symbol_s(a);
}

static hipError_t launch_go_rec(const EdgeArgs& a, int grid, hipStream_t st) {
    return a.mode == SMORE_ATOMIC   ? launch_go_rec_a(a, grid, st)
           : a.mode == SMORE_HYBRID ? launch_go_rec_h(a, grid, st)
                                    : launch_go_rec_s(a, grid, st);
}

// kind: 0 the C++ edge/pair kernel, 1 Go records (go_rec_kernel), 2 Go walk
// pairs (go_pair_kernel)
static int edge_grid(smore_ctx* c, const EdgeArgs& a, bool leave_slot = false, int kind = 0) {
    if (a.mode == SMORE_SERIAL) return 1;
    int per_cu = 0;
    const void* sym = kind == 1   ? go_rec_symbol(a)
                      : kind == 2 ? (a.mode == SMORE_ATOMIC   ? go_pair_symbol_a(a)
                                     : a.mode == SMORE_HYBRID ? go_pair_symbol_h(a)
                                                              : go_pair_symbol_s(a))
                                  : edge_kernel_symbol(a);
    if (!sym ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sym, 256, sh_lds_bytes(a.sh_rows, a.dpad)) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    // leave one block slot per CU to the concurrent draw kernel (measured at C4:
    // 3 of 4 update blocks per CU run the update as fast as 4)
    if (leave_slot && per_cu > 1) per_cu -= 1;
    // tuning knob: SMORE_BLOCKS_PER_CU caps the resident blocks per CU
    if (const char* e = getenv("SMORE_BLOCKS_PER_CU")) {
        const int cap = atoi(e);
        if (cap > 0 && cap < per_cu) per_cu = cap;
    }
    int64_t grid = (int64_t)c->cus * per_cu;
    // tuning knob: SMORE_MAX_BLOCKS caps the whole grid
    if (const char* e = getenv("SMORE_MAX_BLOCKS")) {
        const int64_t cap = atoll(e);
        if (cap > 0 && cap < grid) grid = cap;
    }
    const int G = lanes_of(a.dpad);
    const int64_t groups_per_block = 256 / G;
    const int64_t need = ((int64_t)a.count + groups_per_block - 1) / groups_per_block;
    if (need < grid) grid = need;
    // Hogwild concurrency cap: at most V/16 resident sample groups (each keeps
    // two samples in flight), so that on small graphs the expected number of
    // in-flight updates per row stays O(1) as in the reference's few-thread
    // Hogwild; the benchmark graphs (V >= 1M) are far from the cap.
    const int64_t cap_groups = std::max<int64_t>(1, c->g->V / 16);
    const int64_t cap = (cap_groups + groups_per_block - 1) / groups_per_block;
    if (cap < grid) grid = cap;
    return (int)(grid < 1 ? 1 : grid);
}

// the hot/cold record split of the C++ edge models' hybrid scatter (train_draw.hip
// draw_split_kernel): SMORE_SPLIT=1 / 0 overrides the per-model default
static bool split_on(int model) {
    static const int env = [] {
        const char* e = getenv("SMORE_SPLIT");
        return e ? atoi(e) : -1;
    }();
    if (env >= 0) return env != 0;
    (void)model;
    return false;
}

int smore_train_edges_async(smore_ctx* c, int model, uint64_t begin, uint64_t count, uint64_t total, int K,
                            double alpha0, double reg, uint64_t seed, int mode) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (model < 0 || model > 3 || mode < 0 || mode > 3 || K < 0 || K > 20)
        return fail(c, SMORE_EINVAL, "bad model/mode/K");
    const int need_tables = model == SMORE_LINE2 ? 2 : 1;
    if (c->ntables < need_tables) return fail(c, SMORE_ESTATE, "tables not allocated");
    if (total == 0) return fail(c, SMORE_EINVAL, "total == 0");
    if (c->census)
        return fail(c, SMORE_ESTATE, "row census: edge models have exact rates (smore_row_rates with their model)");
    if (count == 0) return SMORE_OK;
    int rc;
    if ((rc = set_device(c))) return rc;
    EdgeArgs a{};
    a.g = dev_graph(c);
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = model == SMORE_LINE2 ? c->d_table[1] : c->d_table[0];
    a.skipped = c->d_skipped;
    a.begin = begin;
    a.count = count;
    a.total = total;
    a.seed = seed;
    a.alpha0 = alpha0;
    a.reg = (float)reg;
    a.dpad = c->dpad;
    a.K = model == SMORE_BPR ? 5 : K;
    a.model = model;
    a.mode = mode;
    a.tcum = c->d_tcum;
    // Go semantics (SMORE_SEM_GO): Go draws into the same records
    // (go_draw_kernel) and the Go rules on them (go_rec.h), with every
    // scatter mode; BPR is Go's two-table, one-negative rule
    const bool go = c->semantics == SMORE_SEM_GO;
    if (go) {
        if (model == SMORE_MF) return fail(c, SMORE_EINVAL, "Go semantics has no MF model");
        if (K > 10) return fail(c, SMORE_EINVAL, "Go semantics: K <= 10");
        if (model == SMORE_BPR && c->ntables < 2) return fail(c, SMORE_ESTATE, "Go BPR needs W (users) and C (items)");
        if (model == SMORE_BPR) {
            a.C = c->d_table[1];
            a.K = 1;
        } else {
            a.K = K;
        }
    }
    // C++ BPR's hybrid runs the plain-store kernel on graphs above the
    // small-graph cap (16 M < V; below it every row is hot and the hybrid is
    // the atomic scatter): C3 at 2^28 samples, held-out BPR objective +0.11 %
    // of the atomic scatter's and the same ranking accuracy (0.82548 vs
    // 0.82549), update 80.3 ms per 2^26 against the tagged kernel's 97.6 -- its
    // ~170 hot rows are hub items drawn as positives, whose collisions cost
    // less than the hybrid kernel's code shape (2 blocks per CU against 3;
    // DESIGN.md 8, profiles/r05/bpr).  SMORE_BPR_SCATTER=tagged keeps the
    // tagged hybrid kernel.
    if (model == SMORE_BPR && !go && mode == SMORE_HYBRID) {
        const char* e = getenv("SMORE_BPR_SCATTER");
        EdgeArgs t = a;
        t.sh_rows = 0;
        const int64_t Mb = (int64_t)edge_grid(c, t, false, 0) * (256 / lanes_of(c->dpad));
        const bool small = c->hot_tau < 0 && 16.0 * (double)Mb >= (double)c->g->V;
        if (!small && !(e && !strcmp(e, "tagged"))) a.mode = mode = SMORE_HOGWILD;
    }
    // C++ BPR combines its hub rows only with SMORE_BPR_COMBINE=1 (measured in
    // the hub items are positives, the negatives are uniform)
    const char* bpr_comb = getenv("SMORE_BPR_COMBINE");
    const bool combine = mode == SMORE_HYBRID && (go || model != SMORE_BPR || (bpr_comb && atoi(bpr_comb) != 0));
    a.sh_rows = combine ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;   // LDS bound for the grid
    const int grid = edge_grid(c, a, false, go ? 1 : 0);
    if (mode == SMORE_HYBRID) {
        const int64_t M = (int64_t)grid * (256 / lanes_of(c->dpad));
        // Go BPR has two tables (users W, items C): the LINE-2 row roles
        const int hot_model = go && model == SMORE_BPR ? SMORE_LINE2 : model;
        if ((rc = build_hot_maps(c, hot_model, a.K, M, go ? HOT_TAU_WALK : HOT_TAU_EDGE))) return rc;
    }
    a.sh_rows = combine ? c->sh_rows : 0;
    a.sh_hash = c->d_sh_hash;
    a.sh_ids = c->d_sh_ids;
    a.sh_flush = std::max(1, c->sh_flush_eff);
    a.sh_flush_w = c->sh_flush_w_eff;
    std::copy(std::begin(c->sh_lvl_eff), std::end(c->sh_lvl_eff), a.sh_lvl);
    // edge models: draw kernel -> update kernel per chunk of samples.  With
    // several chunks the draws of chunk k+1 run on a second stream while
    // chunk k updates (two record buffers; the update kernel leaves one block
    // slot per CU for them).  Both kernels are bound by HBM, so the overlap
    // buys little (C4 hybrid, 2^25-sample chunks: 120.4 ms per 2^27 samples
    // vs 122 sequential; plain stores 116.6 vs 108): chunks default to 2^27
    // samples (SMORE_DRAW_CHUNK overrides), i.e. sequential for a bench step.
    const int RW = rec_width(kmax_of(a.K));
    uint64_t chunk_max = (uint64_t)1 << 27;
    if (const char* e = getenv("SMORE_DRAW_CHUNK")) chunk_max = std::max<uint64_t>(1024, strtoull(e, nullptr, 10));
    if (a.mode == SMORE_SERIAL) chunk_max = ((uint64_t)1 << 30) / (uint64_t)RW;
    const uint64_t chunk = std::min<uint64_t>(count, chunk_max);
    const int nch = (int)((count + chunk - 1) / chunk);
    const int nbuf = nch > 1 ? 2 : 1;
    if (c->rec_cap < chunk * RW * nbuf) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * RW * nbuf * sizeof(int32_t)));
        c->rec_cap = chunk * RW * nbuf;
    }
    auto grow = [&](std::vector<hipEvent_t>& v, size_t n) -> int {
        while (v.size() < n) {
            hipEvent_t e;
            HIPCHK(c, hipEventCreate(&e));
            v.push_back(e);
        }
        return SMORE_OK;
    };
    if ((rc = grow(c->phase_ev, 2 * (size_t)nch + 1))) return rc;
    if ((rc = grow(c->sync_ev, 2 * (size_t)nch))) return rc;
    if ((rc = ensure_packed(c))) return rc;
    const DevGraph dg = dev_graph(c);
    // hot/cold record split (C++ rules, hybrid): records touching no hot row
    // run through the plain-store kernel (train_draw.hip draw_split_kernel);
    // SMORE_SPLIT=1/0 forces it on / off, default split_default()
    const bool split = mode == SMORE_HYBRID && !go && dg.vt32 && split_on(model);
    if (split && !c->d_split) HIPCHK(c, hipMalloc((void**)&c->d_split, 4 * sizeof(unsigned long long)));
    // tuning knob: SMORE_DRAW_LEAVE=0 keeps the update kernel's full grid
    // while the next chunk's draws run beside it
    const char* leave_env = getenv("SMORE_DRAW_LEAVE");
    const bool leave = !leave_env || atoi(leave_env) != 0;
    const int ugrid = nch > 1 ? edge_grid(c, a, leave, go ? 1 : 0) : grid;
    hipStream_t ds = nch > 1 ? c->draw_stream : c->stream;
    auto recbuf = [&](int k) { return c->d_rec + (size_t)(k % nbuf) * chunk * RW; };
    auto draw = [&](int k) -> int {
        const uint64_t b = (uint64_t)k * chunk, n = std::min<uint64_t>(chunk, count - b);
        if (k >= 2) HIPCHK(c, hipStreamWaitEvent(ds, c->sync_ev[2 * (k - 2) + 1], 0));   // buffer free
        if (go) HIPCHK(c, launch_go_draw(dg, c->d_tcum, c->go_unit_w, seed, begin + b, n, a.K, recbuf(k), c->d_skipped, ds));
        else if (split) {
            unsigned long long* cnt = c->d_split + 2 * (k % nbuf);
            HIPCHK(c, hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned long long), ds));
            HIPCHK(c, launch_draw_split(dg, seed, begin + b, n, a.K, alpha0, total,
                                        model == SMORE_MF || model == SMORE_BPR ? 0 : 1, recbuf(k), c->d_skipped, cnt,
                                        ds));
        } else HIPCHK(c, launch_draw(dg, seed, begin + b, n, a.K, recbuf(k), c->d_skipped, ds));
        HIPCHK(c, hipEventRecord(c->sync_ev[2 * k], ds));
        return SMORE_OK;
    };
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, hipEventRecord(c->phase_ev[0], c->stream));
    if (ds != c->stream) HIPCHK(c, hipStreamWaitEvent(ds, c->phase_ev[0], 0));   // after earlier work
    if ((rc = draw(0))) return rc;
    for (int k = 0; k < nch; ++k) {
        if (k + 1 < nch && (rc = draw(k + 1))) return rc;
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->sync_ev[2 * k], 0));
        HIPCHK(c, hipEventRecord(c->phase_ev[2 * k + 1], c->stream));
        const uint64_t b = (uint64_t)k * chunk, n = std::min<uint64_t>(chunk, count - b);
        EdgeArgs ak = a;
        ak.begin = begin + b;
        ak.count = n;
        ak.rec = recbuf(k);
        ak.work = c->d_work;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        if (go) HIPCHK(c, launch_go_rec(ak, ugrid, c->stream));
        else if (split) {
            // hot records [0, h) on the hybrid kernel, cold [h, n) on the
            // plain-store kernel; both read their rate from the record
            unsigned long long* cnt = c->d_split + 2 * (k % nbuf);
            ak.alpha_rec = 2;
            ak.count_dev = reinterpret_cast<const uint64_t*>(cnt);
            HIPCHK(c, launch_edge_train(ak, ugrid, c->stream));
            EdgeArgs ac = ak;
            ac.mode = SMORE_HOGWILD;
            ac.sh_rows = 0;
            ac.count_dev = nullptr;
            ac.rec_base = reinterpret_cast<const uint64_t*>(cnt);
            HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
            HIPCHK(c, launch_edge_train(ac, edge_grid(c, ac), c->stream));
        } else HIPCHK(c, launch_edge_train(ak, ugrid, c->stream));
        HIPCHK(c, hipEventRecord(c->phase_ev[2 * k + 2], c->stream));
        HIPCHK(c, hipEventRecord(c->sync_ev[2 * k + 1], c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = nch;
    return SMORE_OK;
}

int smore_last_phase_ms(const smore_ctx* c, float* draw_ms, float* update_ms, int* launches) {
    if (!c || !c->timed || c->phase_n <= 0) return SMORE_ESTATE;
    float d = 0.0f, u = 0.0f, ms = 0.0f;
    if (hipEventSynchronize(c->phase_ev[2 * c->phase_n]) != hipSuccess) return SMORE_EHIP;
    for (int k = 0; k < c->phase_n; ++k) {
        if (hipEventElapsedTime(&ms, c->phase_ev[2 * k], c->phase_ev[2 * k + 1]) != hipSuccess) return SMORE_EHIP;
        d += ms;
        if (hipEventElapsedTime(&ms, c->phase_ev[2 * k + 1], c->phase_ev[2 * k + 2]) != hipSuccess) return SMORE_EHIP;
        u += ms;
    }
    if (draw_ms) *draw_ms = d;
    if (update_ms) *update_ms = u;
    if (launches) *launches = c->phase_n;
    return SMORE_OK;
}

int smore_train_edges(smore_ctx* c, int model, uint64_t begin, uint64_t count, uint64_t total, int K,
                      double alpha0, double reg, uint64_t seed, int mode) {
    int rc = smore_train_edges_async(c, model, begin, count, total, K, alpha0, reg, seed, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipGetLastError());
    return SMORE_OK;
}

int smore_set_semantics(smore_ctx* c, int semantics) {
    if (!c || (semantics != SMORE_SEM_CPP && semantics != SMORE_SEM_GO)) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (semantics == c->semantics) return SMORE_OK;
    c->packed_ok = false;
    std::vector<double> tcum;
    if (semantics == SMORE_SEM_GO) build_go_tables(*c->g, tcum);
    else build_cpp_vn_tables(*c->g);
    c->go_unit_w = 1;
    for (int64_t e = 0; e < c->g->E && c->go_unit_w; ++e)
        if (c->g->weights[e] != 1.0) c->go_unit_w = 0;
    c->semantics = semantics;
    c->hot_key.clear();
    if (c->device < 0) return SMORE_OK;
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = upload(c, c->d_vtab, c->g->vtab.data(), c->g->vtab.size()))) return rc;
    if ((rc = upload(c, c->d_ntab, c->g->ntab.data(), c->g->ntab.size(), true))) return rc;
    if (semantics == SMORE_SEM_GO) {
        if ((rc = upload(c, c->d_tcum, tcum.data(), tcum.size()))) return rc;
    } else {
        dfree(c->d_tcum);
    }
    return c->part_n > 1 ? apply_partition(c) : SMORE_OK;   // the semantics' source law, restricted
}

int smore_set_hot_threshold(smore_ctx* c, double tau) {
    if (!c || tau != tau) return SMORE_EINVAL;
    if (tau < 0) tau = -1.0;   // the per-path defaults
    c->hot_tau = tau;
    return SMORE_OK;
}

int smore_set_write_combine(smore_ctx* c, int rows, int flush_rounds) {
    if (!c || rows < 0 || rows > 1024 || flush_rounds < 0) return SMORE_EINVAL;
    c->sh_max = rows;
    c->sh_flush = flush_rounds;
    c->hot_key.clear();
    return SMORE_OK;
}

int smore_write_combine_info(const smore_ctx* c, int* rows, int* flush_rounds) {
    if (!c) return SMORE_EINVAL;
    if (rows) *rows = c->sh_rows;
    if (flush_rounds) *flush_rounds = c->sh_flush_eff;
    return SMORE_OK;
}

// the n rows of table `which` (0: W, 1: C) with the highest expected touches
// per sample under the context's samplers and the model's row roles (LINE-2 /
// Go BPR: W = sources, C = contexts + K x negatives; one-table models: the
// union), highest first -- the rows the replica exchange syncs every launch
int smore_row_rates(smore_ctx* c, int model, int K, int which, int64_t n, double* rate) {
    if (!c || !rate || which < 0 || which > 1 || ((model < 0 || model > 3) && model != SMORE_CENSUS) || K < 0)
        return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    const int64_t V = c->g->V;
    if (n != V) return fail(c, SMORE_EINVAL, "row_rates: n must be the vertex count");
    if (model == SMORE_CENSUS) {
        if (!c->census_ok || (int64_t)c->census_rate[which].size() != V)
            return fail(c, SMORE_ESTATE, "row_rates: no census (smore_census_begin / _end)");
        std::copy(c->census_rate[which].begin(), c->census_rate[which].end(), rate);
        return SMORE_OK;
    }
    std::vector<double> ps, pn, pc;
    draw_probabilities(*c->g, ps, pn, pc);
    const bool two = model == SMORE_LINE2 || (model == SMORE_BPR && c->semantics == SMORE_SEM_GO);
    const int negs = model == SMORE_BPR ? (c->semantics == SMORE_SEM_GO ? 1 : 5) : K;
    for (int64_t v = 0; v < V; ++v)
        rate[v] = two ? (which == 0 ? ps[v] : pc[v] + negs * pn[v]) : ps[v] + pc[v] + negs * pn[v];
    return SMORE_OK;
}

int smore_hot_row_ids(smore_ctx* c, int model, int K, int which, int64_t n, int32_t* ids) {
    if (!c || !ids || n < 0 || which < 0 || which > 1 || ((model < 0 || model > 3) && model != SMORE_CENSUS) || K < 0)
        return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    const int64_t V = c->g->V;
    if (n > V) return fail(c, SMORE_EINVAL, "more hot rows than vertices");
    std::vector<double> rate((size_t)V);
    int rc;
    if ((rc = smore_row_rates(c, model, K, which, V, rate.data()))) return rc;
    std::vector<int32_t> order((size_t)V);
    for (int64_t v = 0; v < V; ++v) order[v] = (int32_t)v;
    std::partial_sort(order.begin(), order.begin() + n, order.end(), [&](int32_t a, int32_t b) {
        return rate[a] > rate[b] || (rate[a] == rate[b] && a < b);
    });
    std::copy(order.begin(), order.begin() + n, ids);
    return SMORE_OK;
}

int smore_hot_rows(const smore_ctx* c, int64_t* hot_w, int64_t* hot_c) {
    if (!c) return SMORE_EINVAL;
    if (hot_w) *hot_w = c->hot_rows[0];
    if (hot_c) *hot_c = c->hot_rows[1];
    return SMORE_OK;
}

int smore_skipped(smore_ctx* c, uint64_t* skipped) {
    if (!c || !skipped) return SMORE_EINVAL;
    int rc;
    if ((rc = set_device(c))) return rc;
    unsigned long long h = 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(&h, c->d_skipped, sizeof(h), hipMemcpyDeviceToHost));
    *skipped = h;
    return SMORE_OK;
}

// streaming-copy bandwidth of this GPU (membw.hip): two fresh buffers of
// `bytes`, one warm-up copy, then `reps` timed copies per variant (grid-
// stride default policy / non-temporal at 4 and 8 blocks per CU, one word per
// thread over the whole buffer); the best variant's (read +
// written bytes) / time.  Measurement only: nothing of the context changes.
int smore_copy_bandwidth(smore_ctx* c, uint64_t bytes, int reps, double* gbs) {
    if (!c || !gbs || reps < 1 || bytes < 4096) return SMORE_EINVAL;
    if (c->device < 0) return fail(c, SMORE_ESTATE, "host-only context");
    int rc;
    if ((rc = set_device(c))) return rc;
    const uint64_t n16 = bytes / 16;
    void *src = nullptr, *dst = nullptr;
    HIPCHK(c, hipMalloc(&src, n16 * 16));
    if (hipMalloc(&dst, n16 * 16) != hipSuccess) {
        (void)hipFree(src);
        return fail(c, SMORE_EHIP, "copy buffer allocation");
    }
    double best = 0.0;
    hipError_t e = hipMemsetAsync(src, 0x3c, n16 * 16, c->stream);
    for (int variant = 0; variant < 3 && e == hipSuccess; ++variant)
        for (int per_cu = 4; per_cu <= (variant == 2 ? 4 : 8) && e == hipSuccess; per_cu *= 2) {
            const int blocks = c->cus * per_cu;
            e = launch_copy(src, dst, n16, blocks, variant, c->stream);
            if (e == hipSuccess) e = hipEventRecord(c->ev0, c->stream);
            for (int r = 0; r < reps && e == hipSuccess; ++r) e = launch_copy(src, dst, n16, blocks, variant, c->stream);
            if (e == hipSuccess) e = hipEventRecord(c->ev1, c->stream);
            if (e == hipSuccess) e = hipEventSynchronize(c->ev1);
            float ms = 0.0f;
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, c->ev0, c->ev1);
            if (e == hipSuccess && ms > 0) best = std::max(best, 2.0 * (double)n16 * 16 * reps / (ms * 1e-3) / 1e9);
        }
    (void)hipFree(src);
    (void)hipFree(dst);
    c->timed = false;
    if (e != hipSuccess) return fail(c, SMORE_EHIP, hipGetErrorString(e));
    *gbs = best;
    return SMORE_OK;
}

int smore_last_mode(const smore_ctx* c) { return c ? c->last_mode : -1; }

float smore_last_kernel_ms(const smore_ctx* c) {
    if (!c || !c->timed) return -1.0f;
    float ms = -1.0f;
    if (hipEventSynchronize(c->ev1) != hipSuccess) return -1.0f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.0f;
    return ms;
}

int smore_deepwalk_order(int64_t V, int walk_times, uint64_t skip, int64_t* order) {
    if (V <= 0 || walk_times < 0 || !order) return SMORE_EINVAL;
    deepwalk_order(V, walk_times, skip, order);
    return SMORE_OK;
}

int smore_sample_edges(smore_ctx* c, int model, uint64_t begin, uint64_t count, int K, uint64_t seed,
                       int32_t* out) {
    if (!c || !out) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (K < 0 || K > 20) return fail(c, SMORE_EINVAL, "bad K");
    if (count == 0) return SMORE_OK;
    int rc;
    if ((rc = set_device(c))) return rc;
    const int bpr = model == SMORE_BPR;
    const size_t width = c->semantics == SMORE_SEM_GO ? (bpr ? 3 : 2 + K) : (bpr ? 7 : 2 + K);
    int32_t* d = nullptr;
    HIPCHK(c, hipMalloc((void**)&d, count * width * sizeof(int32_t)));
    hipError_t e = c->semantics == SMORE_SEM_GO
                       ? launch_go_sample(dev_graph(c), c->d_tcum, seed, begin, count, bpr ? 1 : K, d, c->stream)
                       : launch_sample(dev_graph(c), seed, begin, count, K, bpr, d, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d, count * width * sizeof(int32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, SMORE_EHIP, std::string("sample: ") + hipGetErrorString(e));
    return SMORE_OK;
}

int smore_load_pretrain(smore_ctx* c, int which, const char* path) {
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (!path) return SMORE_EINVAL;
    if (c->g->names.empty()) return fail(c, SMORE_ESTATE, "warm start needs vertex names (load an edge list)");
    std::vector<float> h((size_t)c->g->V * c->dpad);
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h.data(), c->d_table[which], h.size() * sizeof(float), hipMemcpyDeviceToHost));
    int64_t loaded = 0;
    if (!load_pretrain(path, *c->g, h.data(), c->dim, c->dpad, &loaded, c->err)) return SMORE_EIO;
    c->last_loaded = loaded;
    HIPCHK(c, hipMemcpy(c->d_table[which], h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    return SMORE_OK;
}

int smore_save_weights(const smore_ctx* cc, int which, const char* path, int fmt) {
    smore_ctx* c = const_cast<smore_ctx*>(cc);
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (!path || fmt < 0 || fmt > 2) return fail(c, SMORE_EINVAL, "save_weights: bad path or format");
    std::vector<float> h((size_t)c->g->V * c->dpad);
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h.data(), c->d_table[which], h.size() * sizeof(float), hipMemcpyDeviceToHost));
    if (!save_weights(path, *c->g, h.data(), c->g->V, c->dim, c->dpad, fmt, c->err)) return SMORE_EIO;
    return SMORE_OK;
}

// Walk models on the record path: DeepWalk (rule 0) and Walklets (rule 1)
// walks -> skip-gram pair records -> update kernel.  `order` holds the walk
// start of every walk index (DeepWalk's shuffled keys; Walklets: vid).
// node2vec's device tables: the raw CSR edge weights (biasedTargetSample's
// base weights) and every vertex's CSR targets sorted (areNeighbors), built
// once per graph by all host threads.
static int ensure_n2v_tables(smore_ctx* c) {
    if (c->d_wts && c->d_nbr_sorted) return SMORE_OK;
    const HostGraph& g = *c->g;
    const int64_t V = g.V, E = g.E;
    std::vector<int32_t> nbr(g.targets.data(), g.targets.data() + E);
    const int nt = std::max(1, std::min(64, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int64_t v = V * t / nt; v < V * (t + 1) / nt; ++v)
                std::sort(nbr.begin() + g.offsets[v], nbr.begin() + g.offsets[v + 1]);
        });
    for (auto& x : th) x.join();
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = upload(c, c->d_nbr_sorted, nbr.data(), nbr.size()))) return rc;
    return upload(c, c->d_wts, g.weights.data(), (size_t)E);
}

// metapath2vec's typed neighbour index: NeighborsByType (pkg/hetero/
// hetero_graph.go:164-177) as every vertex's CSR targets stably grouped by the
// neighbour's type, with per-(vertex, type) offsets.
int smore_set_node_types(smore_ctx* c, const int32_t* node_type, int ntypes) {
    if (!c || !node_type || ntypes <= 0) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    const HostGraph& g = *c->g;
    const int64_t V = g.V, T = ntypes;
    for (int64_t v = 0; v < V; ++v)
        if (node_type[v] < 0 || node_type[v] >= ntypes) return fail(c, SMORE_EINVAL, "node type out of range");
    std::vector<int64_t> toff((size_t)(V * (T + 1)));
    std::vector<int32_t> tt((size_t)std::max<int64_t>(1, g.E));
    for (int64_t v = 0; v < V; ++v) {
        int64_t* o = toff.data() + v * (T + 1);
        const int64_t b = g.offsets[v], e = g.offsets[v + 1];
        std::vector<int64_t> cnt((size_t)T, 0);
        for (int64_t x = b; x < e; ++x) cnt[node_type[g.targets[x]]]++;
        o[0] = b;
        for (int64_t t = 0; t < T; ++t) o[t + 1] = o[t] + cnt[t];
        std::vector<int64_t> pos(o, o + T);
        for (int64_t x = b; x < e; ++x) {
            const int32_t n = g.targets[x];
            tt[pos[node_type[n]]++] = n;
        }
    }
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = upload(c, c->d_ntype, node_type, (size_t)V))) return rc;
    if ((rc = upload(c, c->d_toff, toff.data(), toff.size()))) return rc;
    if ((rc = upload(c, c->d_ttargets, tt.data(), tt.size()))) return rc;
    c->ntypes = ntypes;
    return SMORE_OK;
}

// CTDNE's temporal graph (pkg/temporal/temporal_graph.go:60-170, 254-288):
// OutEdges per source sorted by timestamp (stable: Go's sort.Slice leaves the
// order of equal timestamps unspecified), the active time range of every
// vertex over its out- and in-edges ({0, 0} without edges), Min/MaxTime.
int smore_set_temporal_edges(smore_ctx* c, int64_t E, const int32_t* src, const int32_t* dst, const double* ts) {
    if (!c || E < 0 || (E > 0 && (!src || !dst || !ts))) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    const int64_t V = c->g->V;
    for (int64_t i = 0; i < E; ++i)
        if (src[i] < 0 || src[i] >= V || dst[i] < 0 || dst[i] >= V)
            return fail(c, SMORE_EINVAL, "temporal edge id out of range");
    std::vector<int64_t> off((size_t)V + 1, 0);
    for (int64_t i = 0; i < E; ++i) off[(size_t)src[i] + 1]++;
    for (int64_t v = 0; v < V; ++v) off[v + 1] += off[v];
    std::vector<int64_t> slot(off.begin(), off.end() - 1), perm((size_t)std::max<int64_t>(1, E));
    for (int64_t i = 0; i < E; ++i) perm[slot[src[i]]++] = i;
    std::vector<int32_t> tgt((size_t)std::max<int64_t>(1, E));
    std::vector<double> tts((size_t)std::max<int64_t>(1, E));
    std::vector<double> tmin((size_t)V, std::numeric_limits<double>::max());
    std::vector<double> tmax((size_t)V, -std::numeric_limits<double>::max());
    double lo = std::numeric_limits<double>::max(), hi = -std::numeric_limits<double>::max();
    for (int64_t v = 0; v < V; ++v) {
        std::stable_sort(perm.begin() + off[v], perm.begin() + off[v + 1],
                         [&](int64_t a, int64_t b) { return ts[a] < ts[b]; });
        for (int64_t x = off[v]; x < off[v + 1]; ++x) {
            tgt[x] = dst[perm[x]];
            tts[x] = ts[perm[x]];
        }
    }
    for (int64_t i = 0; i < E; ++i) {
        for (int32_t v : {src[i], dst[i]}) {
            tmin[v] = std::min(tmin[v], ts[i]);
            tmax[v] = std::max(tmax[v], ts[i]);
        }
        lo = std::min(lo, ts[i]);
        hi = std::max(hi, ts[i]);
    }
    for (int64_t v = 0; v < V; ++v)
        if (tmin[v] == std::numeric_limits<double>::max()) tmin[v] = tmax[v] = 0.0;
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = upload(c, c->d_t_off, off.data(), off.size()))) return rc;
    if ((rc = upload(c, c->d_t_tgt, tgt.data(), tgt.size()))) return rc;
    if ((rc = upload(c, c->d_t_ts, tts.data(), tts.size()))) return rc;
    if ((rc = upload(c, c->d_t_min, tmin.data(), tmin.size()))) return rc;
    if ((rc = upload(c, c->d_t_max, tmax.data(), tmax.size()))) return rc;
    c->t_min_time = lo;
    c->t_max_time = hi;
    c->has_temporal = true;
    return SMORE_OK;
}

static int train_walks(smore_ctx* c, int rule, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                       int window, int window_min, int K, double alpha0, uint64_t seed, const int64_t* order,
                       uint64_t order_base, int mode, double n2v_p = 1.0, double n2v_q = 1.0,
                       int npaths = 0, double time_window = 0.0) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->ntables < 2) return fail(c, SMORE_ESTATE, "walk models need W and C tables");
    if ((!order && rule != 1) || walk_times <= 0 || walk_steps < 0 || window <= 0 || K < 0 || K > 10 || mode < 0 || mode > 3)
        return fail(c, SMORE_EINVAL, "bad DeepWalk / Walklets arguments");
    if (rule == 1 && (window_min < 0 || window_min > window))
        return fail(c, SMORE_EINVAL, "Walklets: need 0 <= window_min <= window_max");
    if (rule == 1 && c->semantics == SMORE_SEM_GO) return fail(c, SMORE_EINVAL, "Walklets has no Go semantics");
    if (rule == 2 && c->semantics != SMORE_SEM_GO)
        return fail(c, SMORE_EINVAL, "node2vec is a Go model: smore_set_semantics(ctx, SMORE_SEM_GO) first");
    if (rule == 2 && !(n2v_p > 0 && n2v_q > 0)) return fail(c, SMORE_EINVAL, "node2vec: need p > 0 and q > 0");
    if (rule == 4 && c->semantics != SMORE_SEM_GO)
        return fail(c, SMORE_EINVAL, "CTDNE is a Go model: smore_set_semantics(ctx, SMORE_SEM_GO) first");
    if (rule == 4 && !c->has_temporal) return fail(c, SMORE_ESTATE, "CTDNE: no temporal edges");
    if (rule == 4 && time_window <= 0) time_window = (c->t_max_time - c->t_min_time) * 0.1;   // ctdne.go:45-49
    if (rule == 3 && c->semantics != SMORE_SEM_GO)
        return fail(c, SMORE_EINVAL, "metapath2vec is a Go model: smore_set_semantics(ctx, SMORE_SEM_GO) first");
    if (rule == 3 && (c->ntypes <= 0 || npaths <= 0 || !c->d_paths))
        return fail(c, SMORE_ESTATE, "metapath2vec: node types and meta-paths not set");
    const uint64_t total = (uint64_t)walk_times * (uint64_t)c->g->V;
    if (walk_end > total) walk_end = total;
    if (walk_begin >= walk_end) return SMORE_OK;
    // only this call's walks [walk_begin, walk_end) are read: validate and
    // upload that slice on every call (no caching by host pointer)
    const uint64_t nw_call = walk_end - walk_begin;
    int rc;
    if (order) {
        if (walk_begin < order_base) return fail(c, SMORE_EINVAL, "walk order slice does not cover the range");
        order -= order_base;   // order[w] is walk w's start
        for (uint64_t i = walk_begin; i < walk_end; ++i)
            if (order[i] < 0 || order[i] >= c->g->V) return fail(c, SMORE_EINVAL, "walk start out of range");
    }
    if ((rc = set_device(c))) return rc;
    if (rule == 2 && (rc = ensure_n2v_tables(c))) return rc;
    if (!order) {
        // starts computed on the device (walk mod V)
    } else if (c->order_cap < nw_call) {
        dfree(c->d_order);
        c->order_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_order, nw_call * sizeof(int64_t)));
        c->order_cap = nw_call;
    }
    if (order)
        HIPCHK(c, hipMemcpyAsync(c->d_order, order + walk_begin, nw_call * sizeof(int64_t), hipMemcpyHostToDevice,
                                 c->stream));
    // walks -> pair records -> update kernel (C++: edge_kernels.h over the
    // pair_emit records; Go: go_rec.h go_pair_kernel over go_pair_emit's);
    // chunks of up to 2^18 walks whose pair records (sized by the per-walk
    // upper bound, so no host read-back of the pair count) stay under 4 GiB
    const bool go = c->semantics == SMORE_SEM_GO;
    const int RW = rec_width(kmax_of(K));
    const uint64_t pb = std::max<uint64_t>(1, pair_bound(walk_steps, window, rule, window_min));
    uint64_t chunk_cap = (uint64_t)1 << 18;
    chunk_cap = std::max<uint64_t>(1, std::min<uint64_t>(chunk_cap, ((uint64_t)1 << 30) / (pb * RW)));
    const uint64_t chunk = std::min<uint64_t>(nw_call, chunk_cap);
    const size_t need = chunk * (size_t)(walk_steps + 1);
    if (c->walk_buf_n < need) {
        dfree(c->d_walks);
        c->walk_buf_n = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_walks, need * sizeof(int32_t)));
        c->walk_buf_n = need;
    }
    if (c->walk_lens_n < chunk) {
        dfree(c->d_lens);
        c->walk_lens_n = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_lens, chunk * sizeof(int32_t)));
        c->walk_lens_n = chunk;
    }
    EdgeArgs a{};
    a.g = dev_graph(c);
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = c->d_table[1];
    a.skipped = c->d_skipped;
    a.begin = 0; a.count = 0; a.total = total; a.seed = seed; a.alpha0 = alpha0; a.reg = 0.0f;
    a.dpad = c->dpad; a.K = K; a.model = SMORE_LINE2; a.mode = mode;
    // Go walks on a unit-weight graph: O(1) CDF target (go_target, tcum null)
    a.tcum = go && c->go_unit_w ? nullptr : c->d_tcum;
    EdgeArgs ar = a;   // the update kernel over pair records
    if (c->pair_walks < chunk + 1) {
        dfree(c->d_pcount);
        dfree(c->d_poff);
        c->pair_walks = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_pcount, (chunk + 1) * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc((void**)&c->d_poff, (chunk + 1) * sizeof(uint64_t)));
        c->pair_walks = chunk + 1;
    }
    if (c->rec_cap < chunk * pb * RW) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * pb * RW * sizeof(int32_t)));
        c->rec_cap = chunk * pb * RW;
    }
    const bool combine = mode == SMORE_HYBRID;
    ar.sh_rows = combine ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;
    ar.alpha_rec = 1;
    ar.work = c->d_work;
    ar.count = chunk * pb;   // grid for the most pairs a chunk can have
    const int ugrid = edge_grid(c, ar, false, go ? 2 : 0);
    if (mode == SMORE_HYBRID) {
        const int64_t M = (int64_t)ugrid * (256 / lanes_of(c->dpad));
        if ((rc = build_hot_maps(c, SMORE_LINE2, K, M, HOT_TAU_WALK, PAIR_FLUSH_MAX))) return rc;
    }
    ar.g = dev_graph(c);
    ar.sh_rows = combine ? c->sh_rows : 0;
    ar.sh_hash = c->d_sh_hash;
    ar.sh_ids = c->d_sh_ids;
    ar.sh_flush = std::max(1, c->sh_flush_eff);
    ar.sh_flush_w = c->sh_flush_w_eff;
    std::copy(std::begin(c->sh_lvl_eff), std::end(c->sh_lvl_eff), ar.sh_lvl);
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    for (uint64_t b = walk_begin; b < walk_end; b += chunk) {
        WalkArgs w;
        w.order = order ? c->d_order : nullptr;
        w.order_base = walk_begin;
        w.walks = c->d_walks;
        w.lens = c->d_lens;
        w.walk_begin = b;
        w.nwalks = std::min<uint64_t>(chunk, walk_end - b);
        w.total_walks = total;
        w.steps = walk_steps;
        w.window = window;
        w.rule = rule;
        w.window_min = window_min;
        w.inv_p = 1.0 / n2v_p;   // node2vec.go:136,142 (fp64 1.0 / p)
        w.inv_q = 1.0 / n2v_q;
        w.wts = c->d_wts;
        w.nbr_sorted = c->d_nbr_sorted;
        w.ntype = c->d_ntype;
        w.ttargets = c->d_ttargets;
        w.toff = c->d_toff;
        w.paths = c->d_paths;
        w.path_off = c->d_path_off;
        w.ntypes = c->ntypes;
        w.npaths = npaths;
        w.slot_extra = rule >= 3 ? 1 : 0;   // metapath2vec: the path pick; CTDNE: the start time
        if (c->own_hi >= 0) {
            w.own_lo = (int32_t)c->own_lo;
            w.own_hi = (int32_t)c->own_hi;
        }
        // walks, then their pair counts plus a zero at n: the exclusive scan's
        // entry n is the chunk's pair total, which the update kernel reads on
        // the device (no host round trip between chunks)
        if (rule == 4) {
            TemporalArgs tg{c->d_t_off, c->d_t_tgt, c->d_t_ts, c->d_t_min, c->d_t_max, c->t_max_time, time_window};
            HIPCHK(c, launch_go_ctdne_walk(tg, w, seed, c->stream));
        } else if (go) {
            HIPCHK(c, launch_go_walk(a, w, 1, c->stream));
        } else {
            HIPCHK(c, launch_walk_gen(ar.g, w, seed, c->stream));
        }
        HIPCHK(c, hipMemsetAsync(c->d_pcount + w.nwalks, 0, sizeof(uint32_t), c->stream));
        if (go) HIPCHK(c, launch_go_pair_count(w, c->d_pcount, c->stream));
        else HIPCHK(c, launch_pair_count(w, seed, c->d_pcount, c->stream));
        HIPCHK(c, scan_pair_counts(c->d_pcount, c->d_poff, w.nwalks + 1, &c->d_scan_tmp, &c->scan_tmp_bytes,
                                   c->stream));
        if (go)
            HIPCHK(c, launch_go_pair_emit(ar.g, w, seed, K, alpha0, c->d_poff, c->d_rec, mode == SMORE_HYBRID,
                                          c->stream));
        else HIPCHK(c, launch_pair_emit(ar.g, w, seed, K, alpha0, c->d_poff, c->d_rec, c->stream));
        EdgeArgs ak = ar;
        ak.begin = 0;
        ak.count = w.nwalks * pb;
        ak.count_dev = c->d_poff + w.nwalks;
        ak.rec = c->d_rec;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        const int g = mode == SMORE_SERIAL ? 1 : ugrid;
        if (c->census)
            HIPCHK(c, launch_row_census(ak.rec, ak.count, ak.count_dev, RW, K, c->d_census[0], c->d_census[1], c->cus,
                                        c->stream));
        else if (!go) HIPCHK(c, launch_edge_train(ak, g, c->stream));
        else if (mode == SMORE_ATOMIC) HIPCHK(c, launch_go_pair_a(ak, g, c->stream));
        else if (mode == SMORE_HYBRID) HIPCHK(c, launch_go_pair_h(ak, g, c->stream));
        else HIPCHK(c, launch_go_pair_s(ak, g, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = 0;
    return SMORE_OK;
}

int smore_train_deepwalk_async(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, uint64_t seed, const int64_t* order,
                               int mode) {
    return train_walks(c, 0, walk_begin, walk_end, walk_times, walk_steps, window, 0, K, alpha0, seed, order, 0,
                       mode);
}

int smore_train_node2vec_async(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, double p, double q, uint64_t seed,
                               const int64_t* order, int mode) {
    return train_walks(c, 2, walk_begin, walk_end, walk_times, walk_steps, window, 0, K, alpha0, seed, order, 0, mode,
                       p, q);
}

int smore_train_metapath2vec_async(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                                   int walk_steps, int window, int K, double alpha0, const int32_t* paths,
                                   const int32_t* path_lens, int npaths, uint64_t seed, const int64_t* order,
                                   int mode) {
    if (!c) return SMORE_EINVAL;
    if (!paths || !path_lens || npaths <= 0) return fail(c, SMORE_EINVAL, "metapath2vec: no meta-paths");
    std::vector<int32_t> off((size_t)npaths + 1, 0);
    for (int p = 0; p < npaths; ++p) {
        if (path_lens[p] < 0) return fail(c, SMORE_EINVAL, "metapath2vec: bad path length");
        off[p + 1] = off[p] + path_lens[p];
    }
    for (int32_t i = 0; i < off[npaths]; ++i)
        if (paths[i] < 0 || paths[i] >= c->ntypes) return fail(c, SMORE_EINVAL, "metapath2vec: unknown type in path");
    int rc;
    if ((rc = set_device(c))) return rc;
    std::vector<int32_t> key(path_lens, path_lens + npaths);
    key.insert(key.end(), paths, paths + off[npaths]);
    if (key != c->path_host || !c->d_paths) {
        // the previous call's kernels may still read the paths: reallocate
        // only after the stream has drained
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if ((rc = upload(c, c->d_paths, paths, (size_t)off[npaths]))) return rc;
        if ((rc = upload(c, c->d_path_off, off.data(), off.size()))) return rc;
        c->path_host.swap(key);
    }
    return train_walks(c, 3, walk_begin, walk_end, walk_times, walk_steps, window, 0, K, alpha0, seed, order, 0, mode,
                       1.0, 1.0, npaths);
}

int smore_train_metapath2vec(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                             int window, int K, double alpha0, const int32_t* paths, const int32_t* path_lens,
                             int npaths, uint64_t seed, const int64_t* order, int mode) {
    int rc = smore_train_metapath2vec_async(c, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, paths,
                                            path_lens, npaths, seed, order, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_ctdne_async(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                            int window, int K, double alpha0, double time_window, uint64_t seed, const int64_t* order,
                            int mode) {
    return train_walks(c, 4, walk_begin, walk_end, walk_times, walk_steps, window, 0, K, alpha0, seed, order, 0, mode,
                       1.0, 1.0, 0, time_window);
}

int smore_train_ctdne(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps, int window,
                      int K, double alpha0, double time_window, uint64_t seed, const int64_t* order, int mode) {
    int rc = smore_train_ctdne_async(c, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, time_window,
                                     seed, order, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_node2vec(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                         int window, int K, double alpha0, double p, double q, uint64_t seed, const int64_t* order,
                         int mode) {
    int rc = smore_train_node2vec_async(c, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, p, q,
                                        seed, order, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_walklets_async(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                               int window_min, int window_max, int K, double alpha0, uint64_t seed, int mode) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (walk_times <= 0) return fail(c, SMORE_EINVAL, "bad DeepWalk / Walklets arguments");
    // Walklets::Train walks from vid itself (src/model/Walklets.cpp:45): no
    // order array, the walk kernel starts walk w at w mod V
    return train_walks(c, 1, walk_begin, walk_end, walk_times, walk_steps, window_max, window_min, K, alpha0, seed,
                       nullptr, 0, mode);
}

int smore_train_walklets(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                         int window_min, int window_max, int K, double alpha0, uint64_t seed, int mode) {
    int rc = smore_train_walklets_async(c, walk_begin, walk_end, walk_times, walk_steps, window_min, window_max, K,
                                        alpha0, seed, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_app_async(smore_ctx* c, uint64_t unit_begin, uint64_t unit_end, int walk_times, int sample_times,
                          double jump, int K, double alpha0, uint64_t seed, const int64_t* order, int mode) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->ntables < 2) return fail(c, SMORE_ESTATE, "APP needs W and C tables");
    if (c->semantics == SMORE_SEM_GO) return fail(c, SMORE_EINVAL, "APP has no Go semantics");
    // jump <= 0 never ends a walk on a graph without dead ends (the reference
    // loops forever); the device walk is bounded, but reject it up front
    if (!order || walk_times <= 0 || sample_times <= 0 || !(jump > 0.0) || K < 0 || K > 10 || mode < 0 || mode > 3)
        return fail(c, SMORE_EINVAL, "bad APP arguments");
    const uint64_t total = (uint64_t)walk_times * (uint64_t)c->g->V;
    const uint64_t units = total * (uint64_t)sample_times;
    if (unit_end > units) unit_end = units;
    if (unit_begin >= unit_end) return SMORE_OK;
    const uint64_t w0 = unit_begin / (uint64_t)sample_times, w1 = (unit_end - 1) / (uint64_t)sample_times + 1;
    for (uint64_t w = w0; w < w1; ++w)
        if (order[w] < 0 || order[w] >= c->g->V) return fail(c, SMORE_EINVAL, "walk start out of range");
    int rc;
    if ((rc = set_device(c))) return rc;
    if (c->order_cap < w1 - w0) {
        dfree(c->d_order);
        c->order_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_order, (w1 - w0) * sizeof(int64_t)));
        c->order_cap = w1 - w0;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_order, order + w0, (w1 - w0) * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    const int RW = rec_width(kmax_of(K));
    const uint64_t chunk = std::min<uint64_t>(unit_end - unit_begin, (uint64_t)1 << 25);
    if (c->rec_cap < chunk * RW) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * RW * sizeof(int32_t)));
        c->rec_cap = chunk * RW;
    }
    EdgeArgs a{};
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = c->d_table[1];
    a.skipped = c->d_skipped;
    a.total = total; a.seed = seed; a.alpha0 = alpha0; a.reg = 0.0f;
    a.dpad = c->dpad; a.K = K; a.model = SMORE_LINE2; a.mode = mode;
    a.tcum = c->d_tcum;
    a.alpha_rec = 1;
    a.work = c->d_work;
    a.count = chunk;
    const int combine = mode == SMORE_HYBRID;
    a.sh_rows = combine ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;
    const int grid = edge_grid(c, a);
    if (mode == SMORE_HYBRID) {
        const int64_t M = (int64_t)grid * (256 / lanes_of(c->dpad));
        if ((rc = build_hot_maps(c, SMORE_LINE2, K, M, HOT_TAU_WALK, PAIR_FLUSH_MAX))) return rc;
    }
    a.g = dev_graph(c);
    a.sh_rows = combine ? c->sh_rows : 0;
    a.sh_hash = c->d_sh_hash;
    a.sh_ids = c->d_sh_ids;
    a.sh_flush = std::max(1, c->sh_flush_eff);
    a.sh_flush_w = c->sh_flush_w_eff;
    std::copy(std::begin(c->sh_lvl_eff), std::end(c->sh_lvl_eff), a.sh_lvl);
    a.rec = c->d_rec;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    for (uint64_t b = unit_begin; b < unit_end; b += chunk) {
        AppArgs p;
        p.order = c->d_order;
        p.order_base = w0;
        p.unit_begin = b;
        p.n = std::min<uint64_t>(chunk, unit_end - b);
        p.total_walks = total;
        p.sample_times = sample_times;
        p.jump = jump;
        HIPCHK(c, launch_app_records(a.g, p, seed, K, alpha0, c->d_rec, c->stream));
        EdgeArgs ak = a;
        ak.begin = 0;
        ak.count = p.n;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        if (c->census)
            HIPCHK(c, launch_row_census(ak.rec, ak.count, nullptr, RW, K, c->d_census[0], c->d_census[1], c->cus,
                                        c->stream));
        else HIPCHK(c, launch_edge_train(ak, mode == SMORE_SERIAL ? 1 : grid, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = 0;
    return SMORE_OK;
}

int smore_train_app(smore_ctx* c, uint64_t unit_begin, uint64_t unit_end, int walk_times, int sample_times,
                    double jump, int K, double alpha0, uint64_t seed, const int64_t* order, int mode) {
    int rc = smore_train_app_async(c, unit_begin, unit_end, walk_times, sample_times, jump, K, alpha0, seed, order,
                                   mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_hpe_async(smore_ctx* c, uint64_t begin, uint64_t count, uint64_t total, int walk_steps, int K,
                          double reg, double alpha0, uint64_t seed, int mode) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->ntables < 2) return fail(c, SMORE_ESTATE, "HPE needs W and C tables");
    if (c->semantics == SMORE_SEM_GO) return fail(c, SMORE_EINVAL, "HPE in Go semantics is the Go LINE-2 rule (internal/models/hpe/hpe.go:72-124): smore_train_edges with SMORE_LINE2");
    if (walk_steps < 1 || walk_steps > 4096 || K < 0 || K > 10 || mode < 0 || mode > 3 || total == 0)
        return fail(c, SMORE_EINVAL, "bad HPE arguments");
    if (count == 0) return SMORE_OK;
    int rc;
    if ((rc = set_device(c))) return rc;
    const int RW = rec_width(kmax_of(K));
    const uint64_t nrec = (uint64_t)walk_steps + 1;
    const uint64_t chunk = std::min<uint64_t>(count, std::max<uint64_t>(1, ((uint64_t)1 << 27) / nrec));
    if (c->rec_cap < chunk * nrec * RW) {
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * nrec * RW * sizeof(int32_t)));
        c->rec_cap = chunk * nrec * RW;
    }
    EdgeArgs a{};
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = c->d_table[1];
    a.skipped = c->d_skipped;
    a.total = total; a.seed = seed; a.alpha0 = alpha0; a.reg = (float)reg;
    a.dpad = c->dpad; a.K = K; a.model = SMORE_LINE2; a.mode = mode;
    a.tcum = c->d_tcum;
    a.alpha_rec = 1;
    a.work = c->d_work;
    a.count = chunk * nrec;
    const int combine = mode == SMORE_HYBRID;
    a.sh_rows = combine ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;
    const int grid = edge_grid(c, a);
    if (mode == SMORE_HYBRID) {
        const int64_t M = (int64_t)grid * (256 / lanes_of(c->dpad));
        if ((rc = build_hot_maps(c, SMORE_LINE2, K, M, HOT_TAU_WALK, PAIR_FLUSH_MAX))) return rc;
    }
    a.g = dev_graph(c);
    a.sh_rows = combine ? c->sh_rows : 0;
    a.sh_hash = c->d_sh_hash;
    a.sh_ids = c->d_sh_ids;
    a.sh_flush = std::max(1, c->sh_flush_eff);
    a.sh_flush_w = c->sh_flush_w_eff;
    std::copy(std::begin(c->sh_lvl_eff), std::end(c->sh_lvl_eff), a.sh_lvl);
    a.rec = c->d_rec;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    for (uint64_t b = begin; b < begin + count; b += chunk) {
        HpeArgs p;
        p.begin = b;
        p.n = std::min<uint64_t>(chunk, begin + count - b);
        p.total = total;
        p.walk_steps = walk_steps;
        HIPCHK(c, launch_hpe_records(a.g, p, seed, K, alpha0, c->d_rec, c->d_skipped, c->stream));
        EdgeArgs ak = a;
        ak.begin = 0;
        ak.count = p.n * nrec;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        if (c->census)
            HIPCHK(c, launch_row_census(ak.rec, ak.count, nullptr, RW, K, c->d_census[0], c->d_census[1], c->cus,
                                        c->stream));
        else HIPCHK(c, launch_edge_train(ak, mode == SMORE_SERIAL ? 1 : grid, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = 0;
    return SMORE_OK;
}

int smore_train_hpe(smore_ctx* c, uint64_t begin, uint64_t count, uint64_t total, int walk_steps, int K, double reg,
                    double alpha0, uint64_t seed, int mode) {
    int rc = smore_train_hpe_async(c, begin, count, total, walk_steps, K, reg, alpha0, seed, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

int smore_train_deepwalk(smore_ctx* c, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                         int window, int K, double alpha0, uint64_t seed, const int64_t* order, int mode) {
    int rc = smore_train_deepwalk_async(c, walk_begin, walk_end, walk_times, walk_steps, window, K, alpha0, seed,
                                        order, mode);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SMORE_OK;
}

// ---------------------------------------------------------------- caller pairs
// proNet::UpdatePairs (src/proNet.cpp:2741-2753) / Go (*ProNet).UpdatePairs
// (pkg/pronet/optimizer.go:8-18): the caller's pairs become records
// (caller_pair_kernel, negatives drawn on the device) for the pair kernels --
// pair_train_kernel (C++ UpdatePair; serial: edge_train_kernel's in-order
// path) or go_pair_kernel (Go UpdatePair) -- in chunks of up to 2^24 pairs.
static int train_pairs_core(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, double alpha,
                            uint64_t seed, uint64_t unit, int mode);

int smore_train_pairs(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, double alpha,
                      uint64_t seed, uint64_t unit, int mode) {
    int rc = train_pairs_core(c, v, cc, n, K, alpha, seed, unit, mode);
    if (rc || !c || n == 0) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipGetLastError());
    return SMORE_OK;
}

// smore_train_pairs queued on the stream (the caller synchronizes)
static int train_pairs_core(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, double alpha,
                            uint64_t seed, uint64_t unit, int mode) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->ntables < 2) return fail(c, SMORE_ESTATE, "UpdatePairs needs W and C tables");
    if (n < 0 || (n > 0 && (!v || !cc)) || K < 0 || K > 10 || mode < 0 || mode > 3)
        return fail(c, SMORE_EINVAL, "bad UpdatePairs arguments");
    if (n == 0) return SMORE_OK;
    const int64_t V = c->g->V;
    for (int64_t i = 0; i < n; ++i)
        if (v[i] < 0 || v[i] >= V || cc[i] < 0 || cc[i] >= V) return fail(c, SMORE_EINVAL, "pair id out of range");
    int rc;
    if ((rc = set_device(c))) return rc;
    const bool go = c->semantics == SMORE_SEM_GO;
    const int RW = rec_width(kmax_of(K));
    const uint64_t chunk = std::min<uint64_t>((uint64_t)n, (uint64_t)1 << 24);
    if (c->pairs_cap < chunk) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dfree(c->d_pairs);
        c->pairs_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_pairs, 2 * chunk * sizeof(int32_t)));
        c->pairs_cap = chunk;
    }
    if (c->rec_cap < chunk * RW) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dfree(c->d_rec);
        c->rec_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_rec, chunk * RW * sizeof(int32_t)));
        c->rec_cap = chunk * RW;
    }
    EdgeArgs a{};
    a.sig = c->d_sig;
    a.W = c->d_table[0];
    a.C = c->d_table[1];
    a.skipped = c->d_skipped;
    a.total = 1; a.seed = seed; a.alpha0 = alpha; a.reg = 0.0f;
    a.dpad = c->dpad; a.K = K; a.model = SMORE_LINE2; a.mode = mode;
    a.tcum = c->d_tcum;
    a.alpha_rec = 1;
    a.work = c->d_work;
    a.count = chunk;
    const bool combine = mode == SMORE_HYBRID;
    a.sh_rows = combine ? std::min(c->sh_max, sh_rows_max(c->dpad)) : 0;
    const int grid = edge_grid(c, a, false, go ? 2 : 0);
    if (mode == SMORE_HYBRID) {
        const int64_t M = (int64_t)grid * (256 / lanes_of(c->dpad));
        if ((rc = build_hot_maps(c, SMORE_LINE2, K, M, HOT_TAU_WALK, PAIR_FLUSH_MAX))) return rc;
    }
    a.g = dev_graph(c);
    a.sh_rows = combine ? c->sh_rows : 0;
    a.sh_hash = c->d_sh_hash;
    a.sh_ids = c->d_sh_ids;
    a.sh_flush = std::max(1, c->sh_flush_eff);
    a.sh_flush_w = c->sh_flush_w_eff;
    std::copy(std::begin(c->sh_lvl_eff), std::end(c->sh_lvl_eff), a.sh_lvl);
    a.rec = c->d_rec;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    for (uint64_t b = 0; b < (uint64_t)n; b += chunk) {
        const uint64_t m = std::min<uint64_t>(chunk, (uint64_t)n - b);
        // the previous chunk's kernels read d_pairs / d_rec: the copies are
        // ordered after them on the stream
        HIPCHK(c, hipMemcpyAsync(c->d_pairs, v + b, m * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->d_pairs + chunk, cc + b, m * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, launch_caller_pairs(a.g, c->d_pairs, c->d_pairs + chunk, m, b, K, (float)alpha, seed, unit, go ? 1 : 0,
                                      mode == SMORE_HYBRID, c->d_rec, c->stream));
        EdgeArgs ak = a;
        ak.begin = 0;
        ak.count = m;
        // a small batch (one walk's pairs, the Go callers' unit): short
        // slices so that every pair gets a group of its own; the
        // CH_ROUNDS-record slices keep W_v in registers over a long batch
        const uint64_t groups = (uint64_t)grid * (uint64_t)(256 / lanes_of(c->dpad));
        if (m < groups * CH_ROUNDS) ak.pair_slice = (uint32_t)std::max<uint64_t>(1, (m + groups - 1) / groups);
        const int g = mode == SMORE_SERIAL ? 1 : grid;
        HIPCHK(c, hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
        if (c->census)
            HIPCHK(c, launch_row_census(ak.rec, m, nullptr, RW, K, c->d_census[0], c->d_census[1], c->cus, c->stream));
        else if (!go) HIPCHK(c, launch_edge_train(ak, g, c->stream));
        else if (mode == SMORE_ATOMIC) HIPCHK(c, launch_go_pair_a(ak, g, c->stream));
        else if (mode == SMORE_HYBRID) HIPCHK(c, launch_go_pair_h(ak, g, c->stream));
        else HIPCHK(c, launch_go_pair_s(ak, g, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mode = mode;
    c->phase_n = 0;
    return SMORE_OK;
}

// ---------------------------------------------------------------- touched rows
// The Philox spec on the host (device_common.h philox_block):
// the negatives smore_train_pairs will draw, without a device round trip.
static uint32_t philox_word(uint64_t seed, uint32_t stream, uint64_t unit, uint32_t slot) {
    uint32_t c0 = (uint32_t)unit, c1 = (uint32_t)(unit >> 32), c2 = slot >> 2, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    const uint32_t w[4] = {c0, c1, c2, c3};
    return w[slot & 3];
}

int smore_pairs_rows(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, uint64_t seed,
                     uint64_t unit, int32_t* w_ids, int64_t* nw, int32_t* c_ids, int64_t* nc) {
    if (!c || !nw || !nc || (n > 0 && (!v || !cc || !w_ids || !c_ids)) || n < 0 || K < 0 || K > 10)
        return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    const HostGraph& g = *c->g;
    const int64_t V = g.V;
    std::vector<int32_t> ws, cs;
    ws.reserve((size_t)n);
    cs.reserve((size_t)n * (K + 1));
    for (int64_t i = 0; i < n; ++i) {
        if (v[i] < 0 || v[i] >= V || cc[i] < 0 || cc[i] >= V) return fail(c, SMORE_EINVAL, "pair id out of range");
        ws.push_back(v[i]);
        cs.push_back(cc[i]);
        // caller_pair_kernel's draws: stream 3, unit + i / PAIR_BLOCK, slots
        // 2K (i % PAIR_BLOCK) + 2q (index), + 1 (p)
        const uint64_t u = unit + (uint64_t)i / PAIR_BLOCK;
        const uint32_t base = 2u * (uint32_t)K * (uint32_t)((uint64_t)i % PAIR_BLOCK);
        for (int q = 0; q < K; ++q) {
            const uint32_t ki = philox_word(seed, 3, u, base + 2u * (uint32_t)q);
            const uint32_t kp = philox_word(seed, 3, u, base + 2u * (uint32_t)q + 1u);
            const uint32_t ni = (uint32_t)(((uint64_t)ki * (uint64_t)V) >> 32);
            const AliasEntry e = g.ntab[ni];
            cs.push_back(kp < e.thresh ? (int32_t)ni : (e.alias & ID_MASK));
        }
    }
    std::sort(ws.begin(), ws.end());
    ws.erase(std::unique(ws.begin(), ws.end()), ws.end());
    std::sort(cs.begin(), cs.end());
    cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
    std::copy(ws.begin(), ws.end(), w_ids);
    std::copy(cs.begin(), cs.end(), c_ids);
    *nw = (int64_t)ws.size();
    *nc = (int64_t)cs.size();
    return SMORE_OK;
}

// rows `ids` of table `which` from (to_table) / to a host buffer, through the
// device buffers of slot `which`, queued on the context stream (the host
// buffer is read / written when the stream gets there: synchronize first)
static int rows_io_async(smore_ctx* c, int which, const int32_t* ids, int64_t n, float* rows, bool to_table) {
    if (!c || n < 0 || (n > 0 && (!ids || !rows))) return SMORE_EINVAL;
    int rc;
    if ((rc = check_table(c, which))) return rc;
    if (n == 0) return SMORE_OK;
    for (int64_t i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= c->g->V) return fail(c, SMORE_EINVAL, "row id out of range");
    if ((rc = set_device(c))) return rc;
    if (c->io_cap[which] < (size_t)n) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dfree(c->d_io_ids[which]);
        dfree(c->d_io_rows[which]);
        c->io_cap[which] = 0;
        const size_t cap = std::max<size_t>((size_t)n, 4096);
        HIPCHK(c, hipMalloc((void**)&c->d_io_ids[which], cap * sizeof(int32_t)));
        HIPCHK(c, hipMalloc((void**)&c->d_io_rows[which], cap * c->dim * sizeof(float)));
        c->io_cap[which] = cap;
    }
    const size_t bytes = (size_t)n * c->dim * sizeof(float);
    HIPCHK(c, hipMemcpyAsync(c->d_io_ids[which], ids, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    if (to_table) HIPCHK(c, hipMemcpyAsync(c->d_io_rows[which], rows, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_rows_io(c->d_table[which], c->d_io_ids[which], (uint64_t)n, c->dpad, c->dim, c->d_io_rows[which],
                             to_table ? 1 : 0, c->stream));
    if (!to_table) HIPCHK(c, hipMemcpyAsync(rows, c->d_io_rows[which], bytes, hipMemcpyDeviceToHost, c->stream));
    return SMORE_OK;
}

int smore_set_rows(smore_ctx* c, int which, const int32_t* ids, int64_t n, const float* rows) {
    int rc = rows_io_async(c, which, ids, n, const_cast<float*>(rows), true);
    if (rc == SMORE_OK && c && n > 0) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int smore_get_rows(smore_ctx* c, int which, const int32_t* ids, int64_t n, float* rows) {
    int rc = rows_io_async(c, which, ids, n, rows, false);
    if (rc == SMORE_OK && c && n > 0) HIPCHK(c, hipStreamSynchronize(c->stream));
    return rc;
}

int smore_train_pairs_rows(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, double alpha,
                           uint64_t seed, uint64_t unit, int mode, const int32_t* w_ids, int64_t nw, float* w_rows,
                           const int32_t* c_ids, int64_t nc, float* c_rows) {
    int rc;
    if (!c) return SMORE_EINVAL;
    if ((rc = rows_io_async(c, 0, w_ids, nw, w_rows, true))) return rc;
    if ((rc = rows_io_async(c, 1, c_ids, nc, c_rows, true))) return rc;
    if ((rc = train_pairs_core(c, v, cc, n, K, alpha, seed, unit, mode))) return rc;
    if ((rc = rows_io_async(c, 0, w_ids, nw, w_rows, false))) return rc;
    if ((rc = rows_io_async(c, 1, c_ids, nc, c_rows, false))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipGetLastError());
    return SMORE_OK;
}

// ---------------------------------------------------------------- combining
// The reference's callers run UpdatePairs from `workers` goroutines at once,
// each on its own walk's ~380 pairs (internal/models/deepwalk/deepwalk.go:
// 96-120; pkg/pronet/optimizer.go:8-18).  A GPU call per batch costs a
// synchronisation and two small transfers whatever the batch, so a serialised
// hook loses to the CPU path once two goroutines run.  Flat combining: every
// caller copies its batch (pairs, row ids, rows) into a pinned staging slot of
// its own -- in parallel with the other callers -- and queues it; whichever
// finds the context idle becomes the leader, takes every request queued so far
// and runs them as ONE device call: per request in queue order, its rows up
// (asynchronous from pinned memory; rows an earlier request of the call
// already brought are NOT uploaded again, so each batch sees the rows the
// earlier ones wrote -- the serial order of the queue), its pairs, its rows
// back; one synchronisation; then every caller copies its rows out of its
// slot, again in parallel.  A request's rows come back as they are after its
// own batch.
struct PairSlot {   // pinned staging of one request; capacities in elements
    float *w_rows = nullptr, *c_rows = nullptr;
    int32_t *w_ids = nullptr, *c_ids = nullptr, *v = nullptr, *cc = nullptr, *w_sel = nullptr, *c_sel = nullptr;
    size_t cap[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

struct PairReq {
    int64_t n;
    int K;
    double alpha;
    uint64_t seed, unit;
    int mode;
    int64_t nw, nc;
    PairSlot* slot;
    int64_t msel_w = 0, msel_c = 0;   // rows this request uploads (not already on the device in this call)
    int rc = SMORE_OK;
    bool done = false;
};

struct PairCombiner {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<PairReq*> q;
    bool busy = false;
    uint64_t calls = 0, requests = 0;   // combined device calls, requests served
    std::mutex pool_mu;                 // the free slots
    std::vector<PairSlot*> pool;
    std::vector<PairSlot*> all;
    std::vector<uint8_t> seen[2];       // the leader's marks of the rows already brought (cleared after use)
    bool seen_dirty = false;            // a call failed before clearing its marks
    // device staging of one combined call
    float* d_rows = nullptr;
    int32_t *d_ids = nullptr, *d_sel = nullptr;
    size_t rows_cap = 0;   // rows
    ~PairCombiner() {
        for (PairSlot* p : all) {
            for (void* x : {(void*)p->w_rows, (void*)p->c_rows, (void*)p->w_ids, (void*)p->c_ids, (void*)p->v,
                            (void*)p->cc, (void*)p->w_sel, (void*)p->c_sel})
                if (x) (void)hipHostFree(x);
            delete p;
        }
        if (d_rows) (void)hipFree(d_rows);
        if (d_ids) (void)hipFree(d_ids);
        if (d_sel) (void)hipFree(d_sel);
    }
};

namespace {
// a pinned host buffer of at least `need` elements of `size` bytes
bool host_grow(void** p, size_t& cap, size_t need, size_t size) {
    if (need <= cap && *p) return true;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    cap = 0;
    const size_t n = std::max<size_t>(need, 1024);
    if (hipHostMalloc(p, n * size, hipHostMallocDefault) != hipSuccess) return false;
    cap = n;
    return true;
}

PairSlot* slot_acquire(PairCombiner& pc, int64_t n, int64_t nw, int64_t nc, int dim) {
    PairSlot* s = nullptr;
    {
        std::lock_guard<std::mutex> g(pc.pool_mu);
        if (!pc.pool.empty()) {
            s = pc.pool.back();
            pc.pool.pop_back();
        } else {
            s = new PairSlot();
            pc.all.push_back(s);
        }
    }
    const size_t need[8] = {(size_t)nw * dim, (size_t)nc * dim, (size_t)nw, (size_t)nc, (size_t)n, (size_t)n,
                            (size_t)nw, (size_t)nc};
    void** buf[8] = {(void**)&s->w_rows, (void**)&s->c_rows, (void**)&s->w_ids, (void**)&s->c_ids, (void**)&s->v,
                     (void**)&s->cc, (void**)&s->w_sel, (void**)&s->c_sel};
    bool ok = true;
    for (int k = 0; k < 8 && ok; ++k) ok = host_grow(buf[k], s->cap[k], need[k], k < 2 ? sizeof(float) : sizeof(int32_t));
    if (!ok) {
        std::lock_guard<std::mutex> g(pc.pool_mu);
        pc.pool.push_back(s);
        return nullptr;
    }
    return s;
}

void slot_release(PairCombiner& pc, PairSlot* s) {
    std::lock_guard<std::mutex> g(pc.pool_mu);
    pc.pool.push_back(s);
}

// the leader: every request of the call, in queue order, on the stream
int combined_call(smore_ctx* c, PairCombiner& pc, const std::vector<PairReq*>& reqs) {
    const int dim = c->dim;
    size_t rows = 0;
    for (const PairReq* q : reqs) rows += (size_t)(q->nw + q->nc);
    if (pc.rows_cap < rows) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (pc.d_rows) (void)hipFree(pc.d_rows);
        if (pc.d_ids) (void)hipFree(pc.d_ids);
        if (pc.d_sel) (void)hipFree(pc.d_sel);
        pc.d_rows = nullptr;
        pc.d_ids = pc.d_sel = nullptr;
        pc.rows_cap = 0;
        const size_t cap = std::max<size_t>(rows * 2, 1 << 16);
        HIPCHK(c, hipMalloc((void**)&pc.d_rows, cap * dim * sizeof(float)));
        HIPCHK(c, hipMalloc((void**)&pc.d_ids, cap * sizeof(int32_t)));
        HIPCHK(c, hipMalloc((void**)&pc.d_sel, cap * sizeof(int32_t)));
        pc.rows_cap = cap;
    }
    // the rows each request must bring: those no earlier request of the call brought
    auto& seen = pc.seen;
    const int64_t V = c->g->V;
    for (auto& x : seen)
        if ((int64_t)x.size() != V || pc.seen_dirty) x.assign((size_t)V, 0);
    pc.seen_dirty = true;
    for (PairReq* q : reqs) {
        PairSlot* s = q->slot;
        q->msel_w = q->msel_c = 0;
        for (int64_t i = 0; i < q->nw; ++i)
            if (!seen[0][s->w_ids[i]]) {
                seen[0][s->w_ids[i]] = 1;
                s->w_sel[q->msel_w++] = (int32_t)i;
            }
        for (int64_t i = 0; i < q->nc; ++i)
            if (!seen[1][s->c_ids[i]]) {
                seen[1][s->c_ids[i]] = 1;
                s->c_sel[q->msel_c++] = (int32_t)i;
            }
    }
    int rc;
    size_t off = 0;
    for (PairReq* q : reqs) {
        PairSlot* s = q->slot;
        for (int t = 0; t < 2; ++t) {
            const int64_t n = t ? q->nc : q->nw, m = t ? q->msel_c : q->msel_w;
            if (n == 0) continue;
            float* dr = pc.d_rows + (off + (t ? (size_t)q->nw : 0)) * dim;
            int32_t* di = pc.d_ids + off + (t ? (size_t)q->nw : 0);
            int32_t* ds = pc.d_sel + off + (t ? (size_t)q->nw : 0);
            HIPCHK(c, hipMemcpyAsync(di, t ? s->c_ids : s->w_ids, n * sizeof(int32_t), hipMemcpyHostToDevice,
                                     c->stream));
            if (m > 0) {
                HIPCHK(c, hipMemcpyAsync(ds, t ? s->c_sel : s->w_sel, m * sizeof(int32_t), hipMemcpyHostToDevice,
                                         c->stream));
                HIPCHK(c, hipMemcpyAsync(dr, t ? s->c_rows : s->w_rows, (size_t)n * dim * sizeof(float),
                                         hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, launch_rows_put_sel(c->d_table[t], di, ds, (uint64_t)m, c->dpad, dim, dr, c->stream));
            }
        }
        q->rc = train_pairs_core(c, s->v, s->cc, q->n, q->K, q->alpha, q->seed, q->unit, q->mode);
        if (q->rc) return q->rc;
        for (int t = 0; t < 2; ++t) {
            const int64_t n = t ? q->nc : q->nw;
            if (n == 0) continue;
            float* dr = pc.d_rows + (off + (t ? (size_t)q->nw : 0)) * dim;
            int32_t* di = pc.d_ids + off + (t ? (size_t)q->nw : 0);
            HIPCHK(c, launch_rows_io(c->d_table[t], di, (uint64_t)n, c->dpad, dim, dr, 0, c->stream));
            HIPCHK(c, hipMemcpyAsync(t ? s->c_rows : s->w_rows, dr, (size_t)n * dim * sizeof(float),
                                     hipMemcpyDeviceToHost, c->stream));
        }
        off += (size_t)(q->nw + q->nc);
    }
    for (PairReq* q : reqs) {   // clear the marks this call set
        for (int64_t i = 0; i < q->msel_w; ++i) seen[0][q->slot->w_ids[q->slot->w_sel[i]]] = 0;
        for (int64_t i = 0; i < q->msel_c; ++i) seen[1][q->slot->c_ids[q->slot->c_sel[i]]] = 0;
    }
    pc.seen_dirty = false;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)rc;
    return SMORE_OK;
}
}  // namespace

int smore_train_pairs_rows_mt(smore_ctx* c, const int32_t* v, const int32_t* cc, int64_t n, int K, double alpha,
                              uint64_t seed, uint64_t unit, int mode, const int32_t* w_ids, int64_t nw, float* w_rows,
                              const int32_t* c_ids, int64_t nc, float* c_rows) {
    if (!c) return SMORE_EINVAL;
    if (n < 0 || nw < 0 || nc < 0 || (n > 0 && (!v || !cc)) || (nw > 0 && (!w_ids || !w_rows)) ||
        (nc > 0 && (!c_ids || !c_rows)))
        return SMORE_EINVAL;
    if (!c->has_graph || c->ntables < 2 || c->dim <= 0) return fail(c, SMORE_ESTATE, "pairs: no graph or tables");
    const int64_t V = c->g->V;
    for (int64_t i = 0; i < nw; ++i)
        if (w_ids[i] < 0 || w_ids[i] >= V) return fail(c, SMORE_EINVAL, "row id out of range");
    for (int64_t i = 0; i < nc; ++i)
        if (c_ids[i] < 0 || c_ids[i] >= V) return fail(c, SMORE_EINVAL, "row id out of range");
    std::shared_ptr<PairCombiner> pc;
    {
        static std::mutex create_mu;   // the context's combiner, made once
        std::lock_guard<std::mutex> g(create_mu);
        if (!c->pair_comb) c->pair_comb = std::make_shared<PairCombiner>();
        pc = c->pair_comb;
    }
    const int dim = c->dim;
    PairSlot* slot = slot_acquire(*pc, n, nw, nc, dim);
    if (!slot) return fail(c, SMORE_EHIP, "pairs: pinned staging");
    // this caller's copies into its slot (in parallel with the other callers)
    std::copy(v, v + n, slot->v);
    std::copy(cc, cc + n, slot->cc);
    std::copy(w_ids, w_ids + nw, slot->w_ids);
    std::copy(c_ids, c_ids + nc, slot->c_ids);
    std::copy(w_rows, w_rows + (size_t)nw * dim, slot->w_rows);
    std::copy(c_rows, c_rows + (size_t)nc * dim, slot->c_rows);
    PairReq me{n, K, alpha, seed, unit, mode, nw, nc, slot};
    std::unique_lock<std::mutex> lk(pc->mu);
    pc->q.push_back(&me);
    pc->cv.wait(lk, [&] { return me.done || !pc->busy; });
    if (!me.done) {
        // leader: every queued request (its own among them) in one device call
        pc->busy = true;
        std::vector<PairReq*> reqs;
        reqs.swap(pc->q);
        lk.unlock();
        const int rc = set_device(c) ? SMORE_EHIP : combined_call(c, *pc, reqs);
        lk.lock();
        for (PairReq* q : reqs) {
            if (rc && !q->rc) q->rc = rc;
            q->done = true;
        }
        pc->calls++;
        pc->requests += reqs.size();
        pc->busy = false;
        lk.unlock();
        pc->cv.notify_all();
    } else {
        lk.unlock();
    }
    if (me.rc == SMORE_OK) {   // this caller's rows out of its slot (in parallel)
        std::copy(slot->w_rows, slot->w_rows + (size_t)nw * dim, w_rows);
        std::copy(slot->c_rows, slot->c_rows + (size_t)nc * dim, c_rows);
    }
    slot_release(*pc, slot);
    return me.rc;
}

int smore_pairs_combine_stats(const smore_ctx* c, uint64_t* calls, uint64_t* requests) {
    if (!c) return SMORE_EINVAL;
    std::shared_ptr<PairCombiner> pc = c->pair_comb;
    if (calls) *calls = pc ? pc->calls : 0;
    if (requests) *requests = pc ? pc->requests : 0;
    return SMORE_OK;
}

// ---------------------------------------------------------------- row census
int smore_census_begin(smore_ctx* c) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    int rc;
    if ((rc = set_device(c))) return rc;
    const size_t V = (size_t)std::max<int64_t>(1, c->g->V);
    for (auto*& p : c->d_census) {
        if (!p) HIPCHK(c, hipMalloc((void**)&p, V * sizeof(unsigned long long)));
        HIPCHK(c, hipMemsetAsync(p, 0, V * sizeof(unsigned long long), c->stream));
    }
    c->census = true;
    c->census_ok = false;
    return SMORE_OK;
}

int smore_census_end(smore_ctx* c, double units) {
    if (!c) return SMORE_EINVAL;
    if (!c->census) return fail(c, SMORE_ESTATE, "no census in progress (smore_census_begin)");
    c->census = false;
    if (!(units > 0.0)) return fail(c, SMORE_EINVAL, "census: units must be > 0");
    int rc;
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t V = (size_t)c->g->V;
    std::vector<unsigned long long> h(V);
    for (int t = 0; t < 2; ++t) {
        if (V) HIPCHK(c, hipMemcpy(h.data(), c->d_census[t], V * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        c->census_rate[t].resize(V);
        for (size_t i = 0; i < V; ++i) c->census_rate[t][i] = (double)h[i] / units;
    }
    c->census_ok = true;
    c->census_gen++;
    return SMORE_OK;
}

// ---------------------------------------------------------------- walk partition
int smore_set_walk_owner(smore_ctx* c, int64_t lo, int64_t hi) {
    if (!c) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (hi < 0) {
        c->own_lo = 0;
        c->own_hi = -1;
        return SMORE_OK;
    }
    if (lo < 0 || lo > hi || hi > c->g->V) return fail(c, SMORE_EINVAL, "walk owner range outside [0, V]");
    c->own_lo = lo;
    c->own_hi = hi;
    return SMORE_OK;
}

int smore_walk_parts(smore_ctx* c, int nparts, int64_t* bounds) {
    if (!c || !bounds || nparts < 1) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (nparts > c->g->V) return fail(c, SMORE_EINVAL, "more parts than vertices");
    if (!c->census_ok) return fail(c, SMORE_ESTATE, "walk parts need a row census (smore_census_begin / _end)");
    std::vector<int64_t> bound;
    source_bounds(c->census_rate[0], nparts, bound);
    std::copy(bound.begin(), bound.end(), bounds);
    return SMORE_OK;
}

// ---------------------------------------------------------------- replica exchange
static int delta_args(smore_ctx* c, const void* T, const void* S, const void* D, const void* R, int64_t n) {
    if (!c || !T || !S || !D || !R || n < 0 || (n & 3)) return fail(c, SMORE_EINVAL, "delta: bad buffers");
    for (const void* p : {T, S, D, R})
        if ((uintptr_t)p & 15) return fail(c, SMORE_EINVAL, "delta: buffers must be 16-byte aligned");
    return set_device(c);
}

int smore_delta_begin(smore_ctx* c, const void* T, void* S, void* D, void* R, int64_t n) {
    int rc;
    if ((rc = delta_args(c, T, S, D, R, n))) return rc;
    HIPCHK(c, launch_delta_begin((const float*)T, (float*)S, (float*)D, (float*)R, (uint64_t)n, c->cus, c->stream));
    return SMORE_OK;
}

int smore_delta_end(smore_ctx* c, void* T, void* S, const void* D, const void* R, float scale, int64_t n) {
    int rc;
    if ((rc = delta_args(c, T, S, D, R, n))) return rc;
    HIPCHK(c, launch_delta_end((float*)T, (float*)S, (const float*)D, (const float*)R, scale, (uint64_t)n, c->cus,
                               c->stream));
    return SMORE_OK;
}

int smore_delta_cycle(smore_ctx* c, void* T, void* S, void* D, void* R, float scale, int64_t n) {
    int rc;
    if ((rc = delta_args(c, T, S, D, R, n))) return rc;
    HIPCHK(c, launch_delta_cycle((float*)T, (float*)S, (float*)D, (float*)R, scale, (uint64_t)n, c->cus, c->stream));
    return SMORE_OK;
}

static int delta_rows_args(smore_ctx* c, const void* T, const void* S, const void* D, const void* R,
                           const void* scale, int64_t rows, int64_t stride) {
    if (!c || !scale || rows < 0 || stride <= 0 || (stride & 3) || stride > (1 << 20))
        return fail(c, SMORE_EINVAL, "delta rows: bad shape");
    if ((uintptr_t)scale & 3) return fail(c, SMORE_EINVAL, "delta rows: scale must be 4-byte aligned");
    return delta_args(c, T, S, D, R, rows * stride);
}

int smore_delta_end_rows(smore_ctx* c, void* T, void* S, const void* D, const void* R, const void* scale,
                         int64_t rows, int64_t stride) {
    int rc;
    if ((rc = delta_rows_args(c, T, S, D, R, scale, rows, stride))) return rc;
    HIPCHK(c, launch_delta_end_rows((float*)T, (float*)S, (const float*)D, (const float*)R, (const float*)scale,
                                    (uint64_t)rows, (int)stride, c->cus, c->stream));
    return SMORE_OK;
}

int smore_delta_cycle_rows(smore_ctx* c, void* T, void* S, void* D, void* R, const void* scale, int64_t rows,
                           int64_t stride) {
    int rc;
    if ((rc = delta_rows_args(c, T, S, D, R, scale, rows, stride))) return rc;
    HIPCHK(c, launch_delta_cycle_rows((float*)T, (float*)S, (float*)D, (float*)R, (const float*)scale,
                                      (uint64_t)rows, (int)stride, c->cus, c->stream));
    return SMORE_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- shared with blocks.cpp
namespace smore_host {
void part_bounds(const std::vector<double>& ps, int n, std::vector<int64_t>& bound) { source_bounds(ps, n, bound); }
int hot_maps(smore_ctx* c, int model, int K, int64_t M, bool walk, double w_scale, double c_scale) {
    return build_hot_maps(c, model, K, M, walk ? HOT_TAU_WALK : HOT_TAU_EDGE, walk ? PAIR_FLUSH_MAX : EDGE_FLUSH_MAX,
                          w_scale, c_scale);
}
int launch_grid(smore_ctx* c, const EdgeArgs& a) { return edge_grid(c, a, false, 0); }
int sh_flush_max(bool walk) { return walk ? PAIR_FLUSH_MAX : EDGE_FLUSH_MAX; }
int sh_slot_interval(double Mp, int cap, bool walk) { return slot_interval(Mp, cap, cell_budget(walk)); }
void sh_slot_levels(int64_t M, int cap, bool walk, const std::pair<double, int32_t>* r, int64_t n, int (&lvl)[8]) {
    sh_levels(M, cap, cell_budget(walk), r, n, lvl);
}
double hot_tau_default(bool walk) { return walk ? HOT_TAU_WALK : HOT_TAU_EDGE; }
double hot_tau_cell_default(bool walk) { return walk ? HOT_TAU_WALK : HOT_TAU_CELL; }
double cell_rate_default(bool walk) { return walk ? CELL_RATE_PAIRS : CELL_RATE_EDGES; }
double sh_stale_max(bool walk) { return sh_stale(walk); }
}  // namespace smore_host
