// host_graph.h -- host-side graph construction for the MI355X hot path.
//
// Everything here runs once per run on the host (not in the metric): edge-list
// loading, CSR build, Vose alias tables and their device encoding, glibc
// rand() initialisation and the text saver.  Each function cites the
// reference code it replaces (RainBoltz/smore, C++ proNet-core).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace smore {

struct AliasEntry {          // device encoding of one alias-table entry (8 B)
    uint32_t thresh;         // accept iff k < thresh (k = 32-bit uniform word)
    int32_t alias;           // id returned otherwise (self when always accepted)
};

// std::allocator whose value-less construct() default-initialises: resize()
// of a trivial element type leaves the memory untouched, so multi-GB graph
// arrays are first touched (page-faulted) by the threads that fill them
template <class T>
struct UninitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = UninitAlloc<U>;
    };
    UninitAlloc() = default;
    template <class U>
    UninitAlloc(const UninitAlloc<U>&) {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
        else ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using hvec = std::vector<T, UninitAlloc<T>>;

struct HostGraph {
    int64_t V = 0, E = 0;
    int vertex_method = 0, negative_method = 0;
    std::vector<std::string> names;          // empty when built from ids
    hvec<int64_t> offsets;                   // V+1
    hvec<int32_t> targets;                   // E, push order per source
    hvec<double> weights;                    // E
    hvec<double> out_deg, in_deg;            // V
    // reference representation (prob, alias with -1 = none)
    hvec<double> vprob, nprob, cprob;
    hvec<int64_t> valias, nalias, calias;
    // device encoding
    hvec<AliasEntry> vtab, ntab, ctab;
};

// Vose alias method, C++ rule (src/proNet.cpp:544-620): q = d^0.75 * n / sum
// (power argument ignored, :558,564), LIFO stacks, leftovers prob 1 alias -1.
void alias_cpp(const double* dist, int64_t n, double* prob, int64_t* alias);

// Vose alias method, Go rule (pkg/pronet/alias.go:10-90): q = d^power (0 for
// d <= 0), sum 0 -> uniform, leftovers alias = self.
void alias_go(const double* dist, int64_t n, double power, double* prob, int64_t* alias);

// Go-semantics tables (pkg/pronet/pronet.go:191-249): VertexAT = alias_go(out,
// 1.0), NegativeAT = alias_go(in+out, 0.75) written into vprob/valias/vtab and
// nprob/nalias/ntab; tcum = per-vertex sequential prefix sums of the edge
// weights (TargetSample's CDF scan, pronet.go:257-284).
void build_go_tables(HostGraph& g, std::vector<double>& tcum);

// {prob, alias} -> {ceil(prob * 2^32), alias}; always-accept entries store
// {0xFFFFFFFF, self}; alias -1 -> self.  self_ids == nullptr: self = index.
void alias_encode(const double* prob, const int64_t* alias, int64_t n, const int32_t* self_ids,
                  AliasEntry* out);

// CSR + degrees + all three alias tables from directed edge slots in the
// reference's push order (src/proNet.cpp:208-215, 410-542).  Returns false on
// an id out of range.
bool build_graph(int64_t V, int64_t E, const int32_t* src, const int32_t* dst, const double* w,
                 int vertex_method, int negative_method, HostGraph& g, std::string& err);

// (Re)build the C++-rule vertex and negative tables from the degrees and the
// stored methods (src/proNet.cpp:457-510).
void build_cpp_vn_tables(HostGraph& g);

// (Re)build the per-vertex context tables (cprob, calias remapped to target
// ids, ctab) from the CSR and the weights (src/proNet.cpp:517-537), threaded
// over vertices; deterministic, so a graph file need not store them.
void build_ctx_tables(HostGraph& g);

// Text edge list(s) -> names + directed slots (src/proNet.cpp:115-236), parsed
// in parallel (loader.cpp); with a cache directory, a binary copy keyed by the
// input's content hash is written on the first load and read on later ones.
struct LoadStats {
    int threads = 0;
    size_t bytes = 0;
    int cache_hit = 0, cache_written = 0;
};
bool read_edgelist(const std::string& path, bool undirected, std::vector<std::string>& names,
                   std::vector<int32_t>& src, std::vector<int32_t>& dst, std::vector<double>& w,
                   std::string& err, const char* cache_dir = nullptr, LoadStats* stats = nullptr);
// Built-graph cache (names, CSR, degrees, all alias tables) of one input and
// sampling methods, keyed by the same content hash: <dir>/<key>-v<vm>n<nm>.smoregc.
bool edgelist_key(const std::string& path, bool undirected, uint64_t* key, std::string& err);
bool save_graph_cache(const std::string& file, uint64_t key, const HostGraph& g);
bool load_graph_cache(const std::string& file, uint64_t key, int vm, int nm, HostGraph& g);

// glibc TYPE_3 rand() stream after srand(1) (the reference's Init).
class GlibcRand {
  public:
    explicit GlibcRand(uint32_t seed = 1);
    int32_t next();
    void discard(uint64_t n);
  private:
    uint32_t tbl_[34];
    int pos_ = 0;
};

// Exact per-draw probabilities encoded by the alias tables: source
// (vertex_AT), negative (negative_AT) and the marginal context-target
// probability sum_v p_src(v) * P(target | v).  src_law: use this source law
// instead of vertex_AT's (a replica's restricted law, capi source partition).
void draw_probabilities(const HostGraph& g, std::vector<double>& p_src, std::vector<double>& p_neg,
                        std::vector<double>& p_ctx, const std::vector<double>* src_law = nullptr);

// DeepWalk walk-start order (src/model/DeepWalk.cpp:122-131).
void deepwalk_order(int64_t V, int walk_times, uint64_t skip, int64_t* order);

// LoadPreTrain (src/proNet.cpp:238-286): "N dim" header, then "name v1..vdim"
// rows; rows whose name is a vertex of g overwrite table[vid] (stride floats
// per row); a dim mismatch skips the file (returns true, *loaded = -1).
bool load_pretrain(const std::string& path, const HostGraph& g, float* table, int dim, int stride,
                   int64_t* loaded, std::string& err);

// SaveWeights text format (src/model/LINE.cpp:13-47 / Go line.go:209-233).
bool save_weights(const std::string& path, const HostGraph& g, const float* table, int64_t rows,
                  int dim, int stride, int fmt, std::string& err);

}  // namespace smore
