// loader.cpp -- parallel edge-list loader with a binary cache.
//
// Replaces proNet::LoadEdgeList's text pass (src/proNet.cpp:115-236; Go
// (*ProNet).LoadEdgeList pkg/pronet/pronet.go:112-174) with the same result:
// "v1 v2 w" per line (the first three whitespace-separated fields; lines with
// fewer, or an unparsable weight, are skipped), vertex ids in order of first
// appearance (v1 before v2 within a line), one directed slot per line plus
// the reverse slot right after it when undirected; a directory is read file
// by file in readdir order.
//
// Two parallel passes over the memory-mapped text:
//   1. chunks cut at line ends; every thread interns its tokens into a
//      sharded hash table (string views into the mapping, per-shard locks),
//      keeping each key's earliest global position and counting valid lines;
//   2. keys sorted by first position -> ids 0..V-1; every thread re-parses
//      its chunk and writes src/dst/w at its lines' global slots.
// The result is byte-identical to a sequential first-appearance pass.
//
// Binary cache: names + directed slots keyed by a 64-bit hash of the input
// bytes (all files, in order), their sizes and the undirected flag, written to
// <cache_dir>/<key>.smorelc and read back instead of parsing.
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#include "host_graph.h"

namespace smore {

namespace {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    bool ok(std::string& err, const std::string& fn) {
        fd = open(fn.c_str(), O_RDONLY);
        if (fd < 0) { err = "cannot open " + fn; return false; }
        struct stat st;
        if (fstat(fd, &st) != 0) { err = "cannot stat " + fn; return false; }
        n = (size_t)st.st_size;
        if (n == 0) return true;
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { err = "cannot map " + fn; return false; }
        madvise(m, n, MADV_SEQUENTIAL);
        p = (const char*)m;
        return true;
    }
    ~Mapped() {
        if (p) munmap((void*)p, n);
        if (fd >= 0) close(fd);
    }
};

inline bool ws(char c) { return c == ' ' || c == '\t' || c == '\r'; }

inline uint64_t hash_bytes(const char* s, size_t n) {   // FNV-1a 64 + final mix
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)s[i]) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
}

// one line "a b w ..." -> tokens; false if fewer than 3 fields or w unparsable
inline bool parse_line(const char* s, const char* e, const char*& a, size_t& al, const char*& b, size_t& bl,
                       double& w) {
    const char* tok[3];
    size_t len[3];
    int nt = 0;
    const char* p = s;
    while (p < e && nt < 3) {
        while (p < e && ws(*p)) ++p;
        if (p >= e) break;
        const char* q = p;
        while (q < e && !ws(*q)) ++q;
        tok[nt] = p;
        len[nt] = (size_t)(q - p);
        ++nt;
        p = q;
    }
    if (nt < 3) return false;
    char wb[64];
    const size_t wl = std::min<size_t>(len[2], 63);
    memcpy(wb, tok[2], wl);
    wb[wl] = 0;
    char* endp;
    w = strtod(wb, &endp);
    if (endp == wb) return false;
    a = tok[0]; al = len[0];
    b = tok[1]; bl = len[1];
    return true;
}

// sharded token table: open addressing over 64-B slots that hold the key's
// hash, length, first 28 bytes and earliest position (one cache line per
// probe); records are numbered in insertion order, a token's reference is
// (shard << 24 | record).  Slot arrays are huge-page backed.
struct Shard {
    struct alignas(64) Slot {
        uint64_t h;
        uint64_t first;      // earliest global position (2 * line + side)
        uint32_t n;
        uint32_t rec;        // record + 1; 0 = empty
        char inl[32];        // first 32 bytes of the key
    };
    static_assert(sizeof(Slot) == 64, "one cache line per slot");
    Slot* slot = nullptr;
    size_t cap = 0, used = 0;
    std::atomic<Slot*> pub_slot{nullptr};       // for lock-free prefetches
    std::atomic<size_t> pub_mask{0};
    std::vector<const char*> ptr;               // record -> key bytes in the mapping
    std::vector<int32_t> ids;                   // record -> vertex id
    std::mutex mu;
    static Slot* alloc(size_t n) {
        const size_t bytes = n * sizeof(Slot);
        void* p = nullptr;
        if (posix_memalign(&p, 1 << 21, bytes) != 0) return nullptr;
        if (bytes >= (1 << 21)) madvise(p, bytes, MADV_HUGEPAGE);
        memset(p, 0, bytes);
        return (Slot*)p;
    }
    Shard() { resize(1 << 10); }
    ~Shard() { free(slot); }
    void resize(size_t n) {
        Slot* old = slot;
        const size_t oc = cap;
        slot = alloc(n);
        cap = n;
        for (size_t k = 0; k < oc; ++k)
            if (old[k].rec) {
                size_t i = (size_t)old[k].h & (cap - 1);
                while (slot[i].rec) i = (i + 1) & (cap - 1);
                slot[i] = old[k];
            }
        free(old);
        pub_slot.store(slot, std::memory_order_release);
        pub_mask.store(cap - 1, std::memory_order_release);
    }
    bool same(const Slot& e, uint64_t h, const char* p, size_t n) const {
        return e.h == h && e.n == n && memcmp(e.inl, p, std::min<size_t>(n, sizeof e.inl)) == 0 &&
               (n <= sizeof e.inl || memcmp(ptr[e.rec - 1], p, n) == 0);
    }
    size_t find(uint64_t h, const char* p, size_t n) const {
        for (size_t i = (size_t)h & (cap - 1);; i = (i + 1) & (cap - 1))
            if (!slot[i].rec || same(slot[i], h, p, n)) return i;
    }
    void prefetch(uint64_t h) const {
        const Slot* b = pub_slot.load(std::memory_order_relaxed);
        if (b) __builtin_prefetch(b + ((size_t)h & pub_mask.load(std::memory_order_relaxed)));
    }
    // the token's record index (new tokens appended), first position lowered to pos
    uint32_t intern(uint64_t h, const char* p, size_t n, uint64_t pos) {
        std::lock_guard<std::mutex> lk(mu);
        size_t i = find(h, p, n);
        if (slot[i].rec) {
            if (pos < slot[i].first) slot[i].first = pos;
            return slot[i].rec - 1;
        }
        if ((used + 1) * 10 > cap * 7) {
            resize(cap * 2);
            i = find(h, p, n);
        }
        Slot& e = slot[i];
        e.h = h; e.first = pos; e.n = (uint32_t)n;
        memcpy(e.inl, p, std::min<size_t>(n, sizeof e.inl));
        ptr.push_back(p);
        e.rec = (uint32_t)ptr.size();
        ++used;
        return e.rec - 1;
    }
};

constexpr int NSHARD = 256;

unsigned threads_for(size_t bytes) {
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    if (const char* e = getenv("SMORE_LOAD_THREADS")) hw = std::max(1, atoi(e));
    hw = std::min(hw, 64u);
    return (unsigned)std::max<size_t>(1, std::min<size_t>(hw, bytes / (1 << 20) + 1));
}

void run_threads(unsigned n, const std::function<void(unsigned)>& fn) {
    if (n <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < n; ++t) th.emplace_back(fn, t);
    for (auto& x : th) x.join();
}

std::vector<std::string> input_files(const std::string& path, std::string& err) {
    std::vector<std::string> files;
    struct stat st;
    if (stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) {   // src/proNet.cpp:124-134, readdir order
        DIR* d = opendir(path.c_str());
        if (!d) { err = "cannot open directory " + path; return files; }
        while (struct dirent* ent = readdir(d)) {
            std::string f = path + "/" + ent->d_name;
            struct stat s2;
            if (stat(f.c_str(), &s2) == 0 && !S_ISDIR(s2.st_mode)) files.push_back(f);
        }
        closedir(d);
    } else {
        files.push_back(path);
    }
    return files;
}

// ---------------------------------------------------------------- cache file
constexpr char CACHE_MAGIC[8] = {'S', 'M', 'O', 'R', 'E', 'L', 'C', '1'};

bool write_all(FILE* f, const void* p, size_t n) { return n == 0 || fwrite(p, 1, n, f) == n; }
bool read_all(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

bool save_cache(const std::string& fn, uint64_t key, const std::vector<std::string>& names,
                const std::vector<int32_t>& src, const std::vector<int32_t>& dst, const std::vector<double>& w) {
    const std::string tmp = fn + ".tmp" + std::to_string((long)getpid());
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    uint64_t hdr[4] = {key, (uint64_t)names.size(), (uint64_t)src.size(), 0};
    std::string blob;
    for (const auto& s : names) { blob += s; blob.push_back('\n'); }
    hdr[3] = blob.size();
    bool all_one = true;
    for (double x : w) if (x != 1.0) { all_one = false; break; }
    const uint8_t flag = all_one ? 1 : 0;
    bool ok = write_all(f, CACHE_MAGIC, 8) && write_all(f, hdr, sizeof hdr) && write_all(f, &flag, 1) &&
              write_all(f, blob.data(), blob.size()) && write_all(f, src.data(), src.size() * 4) &&
              write_all(f, dst.data(), dst.size() * 4) && (all_one || write_all(f, w.data(), w.size() * 8));
    ok = (fclose(f) == 0) && ok;
    if (ok) ok = rename(tmp.c_str(), fn.c_str()) == 0;
    if (!ok) unlink(tmp.c_str());
    return ok;
}

bool load_cache(const std::string& fn, uint64_t key, std::vector<std::string>& names, std::vector<int32_t>& src,
                std::vector<int32_t>& dst, std::vector<double>& w) {
    FILE* f = fopen(fn.c_str(), "rb");
    if (!f) return false;
    char magic[8];
    uint64_t hdr[4];
    uint8_t flag = 0;
    bool ok = read_all(f, magic, 8) && memcmp(magic, CACHE_MAGIC, 8) == 0 && read_all(f, hdr, sizeof hdr) &&
              hdr[0] == key && read_all(f, &flag, 1);
    if (ok) {
        std::string blob(hdr[3], '\0');
        src.resize(hdr[2]);
        dst.resize(hdr[2]);
        ok = read_all(f, &blob[0], blob.size()) && read_all(f, src.data(), src.size() * 4) &&
             read_all(f, dst.data(), dst.size() * 4);
        if (ok) {
            if (flag) w.assign(hdr[2], 1.0);
            else { w.resize(hdr[2]); ok = read_all(f, w.data(), w.size() * 8); }
        }
        if (ok) {
            names.clear();
            names.reserve(hdr[1]);
            size_t s = 0;
            for (size_t i = 0; i < blob.size(); ++i)
                if (blob[i] == '\n') { names.emplace_back(blob, s, i - s); s = i + 1; }
            ok = names.size() == hdr[1];
        }
    }
    fclose(f);
    return ok;
}

// The key is a pure function of the bytes, the file sizes and the undirected
// flag: every file is hashed in fixed 64-MiB pieces (the host's thread count
// only decides how many pieces are hashed at once) and the piece hashes are
// folded in file order.
constexpr size_t KEY_PIECE = (size_t)1 << 26;
uint64_t content_key(const std::vector<std::unique_ptr<Mapped>>& maps, bool undirected, unsigned nt) {
    uint64_t key = hash_bytes(undirected ? "u1" : "u0", 2);
    for (const auto& m : maps) {
        const size_t parts = std::max<size_t>(1, (m->n + KEY_PIECE - 1) / KEY_PIECE);
        std::vector<uint64_t> ph(parts);
        std::atomic<size_t> next(0);
        run_threads((unsigned)std::max<size_t>(1, std::min<size_t>(nt, parts)), [&](unsigned) {
            for (size_t i; (i = next++) < parts;) {
                const size_t b = i * KEY_PIECE, e = std::min(m->n, b + KEY_PIECE);
                ph[i] = hash_bytes(m->p + b, e - b);
            }
        });
        for (uint64_t h : ph) key = (key ^ h) * 0x9E3779B97F4A7C15ull + (uint64_t)m->n;
    }
    return key;
}

// ---------------------------------------------------------------- built-graph cache
// The HostGraph of one (input, undirected, vertex method, negative method):
// names, CSR, degrees, weights, the vertex and negative alias tables.  The
// per-edge context tables (cprob, calias, ctab: 20 of the 24 bytes per slot)
// are rebuilt on load (build_ctx_tables, deterministic): C4's file is 2.3 GB
// instead of 11.9, which a tmpfs write takes ~12 s for (bench.py N > 1: one
// rank builds, the others read).  Arrays are read back with parallel pread()s.
constexpr char GRAPH_MAGIC[8] = {'S', 'M', 'O', 'R', 'E', 'G', 'C', '2'};
// Version of the rules that produce a HostGraph (build_graph's CSR order, the
// degree methods, alias_cpp, alias_encode).  Bump it whenever one of them
// changes: a cache written under other rules is then rebuilt, never reused.
constexpr uint64_t GRAPH_BUILDER_VERSION = 4;

// cheap consistency checks of a graph read back from a cache file (a truncated
// or corrupted file must not drive out-of-bounds device reads)
bool graph_sane(const HostGraph& g) {
    const int64_t V = g.V, E = g.E;
    if (g.offsets[0] != 0 || g.offsets[V] != E) return false;
    std::atomic<bool> ok(true);
    const unsigned nt = std::max(1u, std::min<unsigned>(threads_for((size_t)E * 4), 32u));
    run_threads(nt, [&](unsigned t) {
        const int64_t vb = V * t / nt, ve = V * (t + 1) / nt;
        for (int64_t v = vb; v < ve && ok; ++v)
            if (g.offsets[v + 1] < g.offsets[v]) ok = false;
        for (int64_t v = vb; v < ve && ok; ++v)
            if (g.valias[v] < -1 || g.valias[v] >= V || g.nalias[v] < -1 || g.nalias[v] >= V) ok = false;
        const int64_t eb = E * t / nt, ee = E * (t + 1) / nt;
        for (int64_t e = eb; e < ee && ok; ++e)
            if (g.targets[e] < 0 || g.targets[e] >= V || !(g.weights[e] >= 0.0)) ok = false;
    });
    return ok;
}

struct Blk {   // one array of the file
    void* p;
    size_t bytes;
};

std::vector<Blk> graph_blocks(HostGraph& g, std::string& names_blob, bool weights_one) {
    const size_t V = (size_t)g.V, E = (size_t)g.E;
    std::vector<Blk> b = {{&names_blob[0], names_blob.size()},
                          {g.offsets.data(), (V + 1) * 8}, {g.targets.data(), E * 4},
                          {g.out_deg.data(), V * 8}, {g.in_deg.data(), V * 8},
                          {g.vprob.data(), V * 8}, {g.valias.data(), V * 8},
                          {g.nprob.data(), V * 8}, {g.nalias.data(), V * 8},
                          {g.vtab.data(), V * 8}, {g.ntab.data(), V * 8}};
    if (!weights_one) b.push_back({g.weights.data(), E * 8});
    return b;
}

}  // namespace

bool edgelist_key(const std::string& path, bool undirected, uint64_t* key, std::string& err) {
    const std::vector<std::string> files = input_files(path, err);
    if (files.empty()) return false;
    std::vector<std::unique_ptr<Mapped>> maps;
    size_t total = 0;
    for (const auto& fn : files) {
        maps.emplace_back(new Mapped());
        if (!maps.back()->ok(err, fn)) return false;
        total += maps.back()->n;
    }
    *key = content_key(maps, undirected, threads_for(total));
    return true;
}

bool save_graph_cache(const std::string& fn, uint64_t key, const HostGraph& gc) {
    HostGraph& g = const_cast<HostGraph&>(gc);
    const std::string tmp = fn + ".tmp" + std::to_string((long)getpid());
    const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return false;
    std::string blob;
    for (const auto& s : g.names) { blob += s; blob.push_back('\n'); }
    bool one = true;
    for (double x : g.weights) if (x != 1.0) { one = false; break; }
    const uint64_t hdr[9] = {key, (uint64_t)g.V, (uint64_t)g.E, (uint64_t)g.vertex_method,
                             (uint64_t)g.negative_method, (uint64_t)blob.size(), one ? 1ull : 0ull,
                             (uint64_t)g.names.size(), GRAPH_BUILDER_VERSION};
    bool ok = pwrite(fd, GRAPH_MAGIC, 8, 0) == 8 && pwrite(fd, hdr, sizeof hdr, 8) == (ssize_t)sizeof hdr;
    if (blob.empty()) blob.push_back('\0');   // graph_blocks takes &blob[0]; 0-byte blocks write nothing
    std::vector<Blk> blks = graph_blocks(g, blob, one);
    blks[0].bytes = (size_t)hdr[5];
    // the arrays in <= 64-MiB pieces written by all host threads
    struct Piece { size_t off; const char* src; size_t n; };
    std::vector<Piece> pcs;
    size_t off = 8 + sizeof hdr;
    for (const Blk& b : blks) {
        for (size_t o = 0; o < b.bytes; o += (size_t)1 << 26)
            pcs.push_back({off + o, (const char*)b.p + o, std::min<size_t>((size_t)1 << 26, b.bytes - o)});
        off += b.bytes;
    }
    std::atomic<size_t> next(0);
    std::atomic<bool> good(ok);
    run_threads(std::max(1u, std::min<unsigned>(threads_for(off), 16u)), [&](unsigned) {
        for (size_t i; good && (i = next++) < pcs.size();) {
            size_t done = 0;
            while (done < pcs[i].n) {
                const ssize_t r = pwrite(fd, pcs[i].src + done, pcs[i].n - done, (off_t)(pcs[i].off + done));
                if (r <= 0) { good = false; return; }
                done += (size_t)r;
            }
        }
    });
    ok = (close(fd) == 0) && good;
    if (ok) ok = rename(tmp.c_str(), fn.c_str()) == 0;
    if (!ok) unlink(tmp.c_str());
    return ok;
}

bool load_graph_cache(const std::string& fn, uint64_t key, int vm, int nm, HostGraph& g) {
    const bool verbose = getenv("SMORE_LOAD_VERBOSE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!verbose) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[graph cache] %-10s %.2f s\n", what, std::chrono::duration<double>(now - tick).count());
        tick = now;
    };
    const int fd = open(fn.c_str(), O_RDONLY);
    if (fd < 0) return false;
    char magic[8];
    uint64_t hdr[9];
    bool ok = pread(fd, magic, 8, 0) == 8 && memcmp(magic, GRAPH_MAGIC, 8) == 0 &&
              pread(fd, hdr, sizeof hdr, 8) == (ssize_t)sizeof hdr && hdr[0] == key && hdr[3] == (uint64_t)vm &&
              hdr[4] == (uint64_t)nm && hdr[8] == GRAPH_BUILDER_VERSION && hdr[1] < ((uint64_t)1 << 31) &&
              hdr[2] < ((uint64_t)1 << 40);
    if (!ok) { close(fd); return false; }
    const size_t V = hdr[1], E = hdr[2];
    g.V = (int64_t)V; g.E = (int64_t)E; g.vertex_method = vm; g.negative_method = nm;
    g.offsets.resize(V + 1); g.targets.resize(E); g.weights.resize(E);
    g.out_deg.resize(V); g.in_deg.resize(V);
    g.vprob.resize(V); g.valias.resize(V); g.nprob.resize(V); g.nalias.resize(V);
    g.vtab.resize(V); g.ntab.resize(V);
    std::string blob(std::max<uint64_t>(hdr[5], 1), '\0');
    phase("allocate");
    std::vector<Blk> blks = graph_blocks(g, blob, hdr[6] != 0);
    blks[0].bytes = (size_t)hdr[5];
    // (file offset, destination, bytes) pieces of <= 64 MiB over all host threads
    struct Piece { size_t off; char* dst; size_t n; };
    std::vector<Piece> pcs;
    size_t off = 8 + sizeof hdr;
    for (const Blk& b : blks) {
        for (size_t o = 0; o < b.bytes; o += (size_t)1 << 26)
            pcs.push_back({off + o, (char*)b.p + o, std::min<size_t>((size_t)1 << 26, b.bytes - o)});
        off += b.bytes;
    }
    std::atomic<size_t> next(0);
    std::atomic<bool> good(true);
    run_threads(std::max(1u, std::min<unsigned>(threads_for(off), 32u)), [&](unsigned) {
        for (size_t i; (i = next++) < pcs.size();) {
            size_t done = 0;
            while (done < pcs[i].n) {
                const ssize_t r = pread(fd, pcs[i].dst + done, pcs[i].n - done, (off_t)(pcs[i].off + done));
                if (r <= 0) { good = false; return; }
                done += (size_t)r;
            }
        }
    });
    close(fd);
    phase("read");
    if (!good) { if (verbose) fprintf(stderr, "[graph cache] short read\n"); return false; }
    if (hdr[6]) {   // all-one weights are not stored: fill them on every thread
        const unsigned nf = std::max(1u, std::min<unsigned>(threads_for(E * 8), 32u));
        run_threads(nf, [&](unsigned t) {
            std::fill(g.weights.begin() + (ptrdiff_t)(E * t / nf), g.weights.begin() + (ptrdiff_t)(E * (t + 1) / nf),
                      1.0);
        });
    }
    if (!graph_sane(g)) { if (verbose) fprintf(stderr, "[graph cache] inconsistent arrays\n"); return false; }
    build_ctx_tables(g);
    phase("ctx tables");
    // names: newline-separated; threads take byte ranges, count their lines,
    // then fill their slice of the pre-sized vector
    const size_t nb = (size_t)hdr[5];
    const unsigned nt = std::max(1u, std::min<unsigned>(threads_for(nb), 32u));
    std::vector<size_t> lo(nt + 1), cnt(nt + 1, 0);
    for (unsigned t = 0; t <= nt; ++t) {   // range starts just after a newline
        size_t b = nb * t / nt;
        while (b > 0 && b < nb && blob[b - 1] != '\n') ++b;
        lo[t] = t == nt ? nb : b;
    }
    run_threads(nt, [&](unsigned t) {
        for (size_t i = lo[t]; i < lo[t + 1]; ++i) cnt[t + 1] += blob[i] == '\n';
    });
    for (unsigned t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
    if (cnt[nt] != hdr[7]) return false;
    g.names.clear();
    g.names.resize(hdr[7]);
    run_threads(nt, [&](unsigned t) {
        size_t k = cnt[t], st = lo[t];
        for (size_t i = lo[t]; i < lo[t + 1]; ++i)
            if (blob[i] == '\n') { g.names[k++].assign(blob, st, i - st); st = i + 1; }
    });
    phase("names");
    return true;
}

bool read_edgelist(const std::string& path, bool undirected, std::vector<std::string>& names,
                   std::vector<int32_t>& src, std::vector<int32_t>& dst, std::vector<double>& w,
                   std::string& err, const char* cache_dir, LoadStats* stats) {
    const std::vector<std::string> files = input_files(path, err);
    if (files.empty()) {
        if (err.empty()) err = "no input files in " + path;
        return false;
    }
    std::vector<std::unique_ptr<Mapped>> maps;
    size_t total_bytes = 0;
    for (const auto& fn : files) {
        maps.emplace_back(new Mapped());
        if (!maps.back()->ok(err, fn)) return false;
        total_bytes += maps.back()->n;
    }
    const unsigned nt = threads_for(total_bytes);
    if (stats) { *stats = LoadStats(); stats->threads = (int)nt; stats->bytes = total_bytes; }

    // cache key: content hash of every file (parallel per file slice) + sizes + flag
    std::string cache_file;
    uint64_t key = 0;
    if (cache_dir && *cache_dir) {
        key = content_key(maps, undirected, nt);
        char name[64];
        snprintf(name, sizeof name, "/%016llx.smorelc", (unsigned long long)key);
        cache_file = std::string(cache_dir) + name;
        if (load_cache(cache_file, key, names, src, dst, w)) {
            if (stats) stats->cache_hit = 1;
            return true;
        }
    }

    names.clear(); src.clear(); dst.clear(); w.clear();
    const bool verbose = getenv("SMORE_LOAD_VERBOSE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!verbose) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[loader] %-12s %.2f s\n", what, std::chrono::duration<double>(now - tick).count());
        tick = now;
    };
    std::vector<Shard> shards(NSHARD);
    // chunks over all files: {file, begin, end} cut after '\n'
    struct Chunk { int file; size_t b, e; uint64_t line0; uint64_t lines; uint64_t valid0; uint64_t valid; };
    std::vector<Chunk> chunks;
    for (size_t fi = 0; fi < maps.size(); ++fi) {
        const Mapped& m = *maps[fi];
        const size_t pieces = std::max<size_t>(1, std::min<size_t>(4 * nt, m.n / (1 << 20) + 1));
        size_t b = 0;
        for (size_t k = 1; k <= pieces && b < m.n; ++k) {
            size_t e = k == pieces ? m.n : m.n * k / pieces;
            if (e < b) e = b;
            while (e < m.n && m.p[e - 1] != '\n') ++e;
            if (e > b) chunks.push_back({(int)fi, b, e, 0, 0, 0, 0});
            b = e;
        }
    }
    // line counts per chunk -> global line index of each chunk's first line
    run_threads(nt, [&](unsigned t) {
        for (size_t c = t; c < chunks.size(); c += nt) {
            const char* p = maps[chunks[c].file]->p;
            uint64_t n = 0;
            for (size_t i = chunks[c].b; i < chunks[c].e; ++i) n += p[i] == '\n';
            if (chunks[c].e > chunks[c].b && p[chunks[c].e - 1] != '\n') ++n;   // last line without '\n'
            chunks[c].lines = n;
        }
    });
    uint64_t acc = 0;
    for (auto& c : chunks) { c.line0 = acc; acc += c.lines; }
    phase("lines");

    // pass 1: intern tokens with their earliest position (2 * line + side);
    // every valid line leaves its two token references and its weight
    std::vector<std::vector<uint32_t>> refs(chunks.size());
    std::vector<std::vector<double>> wts(chunks.size());
    std::atomic<int> bad{0};
    run_threads(nt, [&](unsigned t) {
        // tokens this thread has interned already: its chunks come in increasing
        // position order, so a repeat can never lower the key's first position
        // and needs no shard lock (the hub vertices of a power-law graph)
        struct Seen { uint64_t h; const char* p; uint32_t n; uint32_t ref; };
        const bool use_seen = getenv("SMORE_LOAD_NOSEEN") == nullptr;
        std::vector<Seen> seen(1 << 18, Seen{0, nullptr, 0, 0});
        auto intern = [&](uint64_t h, const char* q, size_t n, uint64_t pos) -> uint32_t {
            Seen& e = seen[(h >> 7) & ((1 << 18) - 1)];
            if (use_seen && e.p && e.h == h && e.n == n && memcmp(e.p, q, n) == 0) return e.ref;
            const uint32_t sh = (uint32_t)(h >> 56);
            const uint32_t rec = shards[sh].intern(h, q, n, pos);
            if (rec >= (1u << 24)) bad = 2;
            const uint32_t ref = (sh << 24) | (rec & 0xFFFFFF);
            e = Seen{h, q, (uint32_t)n, ref};
            return ref;
        };
        // lines are parsed in batches whose slots are prefetched before the
        // lookups (many misses in flight instead of one at a time)
        constexpr int B = 16;
        struct Tok { uint64_t h; const char* p; uint32_t n; };
        Tok tk[2 * B];
        double tw[B];
        uint64_t tl[B];
        for (size_t c = t; c < chunks.size(); c += nt) {
            const char* p = maps[chunks[c].file]->p;
            const char* s = p + chunks[c].b;
            const char* end = p + chunks[c].e;
            uint64_t line = chunks[c].line0;
            std::vector<uint32_t>& rf = refs[c];
            std::vector<double>& wv = wts[c];
            rf.reserve(2 * chunks[c].lines);
            wv.reserve(chunks[c].lines);
            while (s < end) {
                int nb = 0;
                while (s < end && nb < B) {
                    const char* nl = (const char*)memchr(s, '\n', (size_t)(end - s));
                    const char* le = nl ? nl : end;
                    const char *a, *b;
                    size_t al, bl;
                    double x;
                    if (parse_line(s, le, a, al, b, bl, x)) {
                        if (al >= (1u << 31) || bl >= (1u << 31)) { bad = 1; return; }
                        tk[2 * nb] = Tok{hash_bytes(a, al), a, (uint32_t)al};
                        tk[2 * nb + 1] = Tok{hash_bytes(b, bl), b, (uint32_t)bl};
                        tw[nb] = x;
                        tl[nb] = line;
                        ++nb;
                    }
                    ++line;
                    s = le + 1;
                }
                for (int k = 0; k < 2 * nb; ++k) {
                    shards[tk[k].h >> 56].prefetch(tk[k].h);
                    __builtin_prefetch(&seen[(tk[k].h >> 7) & ((1 << 18) - 1)]);
                }
                for (int k = 0; k < nb; ++k) {
                    rf.push_back(intern(tk[2 * k].h, tk[2 * k].p, tk[2 * k].n, 2 * tl[k]));
                    rf.push_back(intern(tk[2 * k + 1].h, tk[2 * k + 1].p, tk[2 * k + 1].n, 2 * tl[k] + 1));
                    wv.push_back(tw[k]);
                }
            }
            chunks[c].valid = wv.size();
        }
    });
    if (bad) { err = bad == 1 ? "token too long" : "too many vertices"; return false; }
    phase("intern");
    // ids in first-appearance order
    size_t nkeys = 0;
    for (auto& sh : shards) nkeys += sh.used;
    if (nkeys >= ((size_t)1 << 31) - 1) { err = "too many vertices"; return false; }
    std::vector<std::pair<uint64_t, uint32_t>> keys;   // (first position, reference)
    keys.reserve(nkeys);
    for (uint32_t k = 0; k < (uint32_t)NSHARD; ++k) {
        Shard& sh = shards[k];
        sh.ids.assign(sh.used, -1);
        std::vector<uint32_t> len(sh.used);
        for (size_t i = 0; i < sh.cap; ++i)
            if (sh.slot[i].rec) {
                keys.push_back({sh.slot[i].first, (k << 24) | (sh.slot[i].rec - 1)});
                len[sh.slot[i].rec - 1] = sh.slot[i].n;
            }
        // key lengths ride in ids until the ids are assigned
        for (size_t r = 0; r < sh.used; ++r) sh.ids[r] = (int32_t)len[r];
    }
    std::sort(keys.begin(), keys.end());
    names.resize(keys.size());
    for (size_t i = 0; i < keys.size(); ++i) {
        Shard& sh = shards[keys[i].second >> 24];
        const uint32_t r = keys[i].second & 0xFFFFFF;
        names[i].assign(sh.ptr[r], (size_t)sh.ids[r]);
        sh.ids[r] = (int32_t)i;
    }
    phase("ids");
    // pass 2: references -> ids at each chunk's first valid line
    acc = 0;
    for (auto& c : chunks) { c.valid0 = acc; acc += c.valid; }
    const size_t per = undirected ? 2 : 1;
    src.resize(acc * per);
    dst.resize(acc * per);
    w.resize(acc * per);
    run_threads(nt, [&](unsigned t) {
        for (size_t c = t; c < chunks.size(); c += nt) {
            const std::vector<uint32_t>& rf = refs[c];
            const std::vector<double>& wv = wts[c];
            size_t o = chunks[c].valid0 * per;
            for (size_t l = 0; l < wv.size(); ++l) {
                const uint32_t ra = rf[2 * l], rb = rf[2 * l + 1];
                const int32_t ia = shards[ra >> 24].ids[ra & 0xFFFFFF];
                const int32_t ib = shards[rb >> 24].ids[rb & 0xFFFFFF];
                src[o] = ia; dst[o] = ib; w[o] = wv[l]; ++o;
                if (undirected) { src[o] = ib; dst[o] = ia; w[o] = wv[l]; ++o; }
            }
            std::vector<uint32_t>().swap(refs[c]);
            std::vector<double>().swap(wts[c]);
        }
    });
    phase("slots");
    if (!cache_file.empty() && save_cache(cache_file, key, names, src, dst, w) && stats) stats->cache_written = 1;
    phase("cache write");
    return true;
}

}  // namespace smore
