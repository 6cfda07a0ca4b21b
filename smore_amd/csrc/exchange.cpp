// exchange.cpp -- multi-GPU replicas over RCCL in the C ABI.
//
// The reference scales one training run over CPU threads sharing the tables
// (LINE::Train's `#pragma omp parallel for` over workers, src/model/LINE.cpp:162;
// Go goroutines, internal/models/line/line.go:96-146).  Here every GPU holds a
// replica of the graph and of the tables, trains a disjoint range of global
// sample indices, and the replicas exchange table deltas over RCCL (xGMI):
//
//   begin  (after a step, context stream):  D = T - S;  R = D;  S = T
//          all-reduce R (SUM) on the exchange stream, overlapping the next step
//   end    (before the next begin):         X = scale*R - D;  T += X;  S += X
//          (end fused with the next begin: delta_cycle, replica_sync.hip)
//
// so every sample's update lands on every replica one exchange late, and the
// next D is again only this replica's own updates.  Two ways to drive it:
//   * one process per GPU: smore_comm_unique_id / smore_comm_init, then
//     smore_exchange_reset / _begin / _end around the training calls;
//   * one process, N GPUs: smore_group_* (ncclCommInitAll, one host thread
//     enqueues every replica's work; the collectives of all replicas go out in
//     one ncclGroupStart/End).
// RCCL is loaded on first use (dlopen librccl.so.1): single-GPU users and the
// host-only context never load it.  A group whose replicas all sit on ONE
// device (smore_group_create with a repeated device id) runs the same rounds
// with its collectives as device passes on that GPU (local_sum_kernel, stream-
// ordered copies) and no RCCL: the multi-replica path on a one-GPU machine
// (tests, the replica-quality runs of DESIGN.md 10).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <initializer_list>
#include <mutex>

#include "comm_watch.h"
#include "ctx.h"
#include "hot_exchange.h"

using namespace smore_host;

namespace {

// the RCCL table (comm_watch.h): loaded on first use


double g_comm_timeout = -1.0;   // smore_set_comm_timeout; < 0: comm_timeout_default()

double comm_timeout() { return g_comm_timeout > 0 ? g_comm_timeout : comm_timeout_default(); }

Rccl* rccl() {
    static Rccl r;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.err = std::string("cannot load RCCL: ") + dlerror();
            return;
        }
#define SMORE_SYM(field, name)                                          \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, #name));     \
    if (!r.field) {                                                     \
        r.err = "RCCL lacks " #name;                                    \
        return;                                                         \
    }
        SMORE_SYM(get_unique_id, ncclGetUniqueId)
        SMORE_SYM(init_rank, ncclCommInitRank)
        SMORE_SYM(init_all, ncclCommInitAll)
        SMORE_SYM(destroy, ncclCommDestroy)
        SMORE_SYM(abort, ncclCommAbort)
        SMORE_SYM(async_error, ncclCommGetAsyncError)
        SMORE_SYM(all_reduce, ncclAllReduce)
        SMORE_SYM(broadcast, ncclBroadcast)
        SMORE_SYM(send, ncclSend)
        SMORE_SYM(recv, ncclRecv)
        SMORE_SYM(group_start, ncclGroupStart)
        SMORE_SYM(group_end, ncclGroupEnd)
        SMORE_SYM(error_string, ncclGetErrorString)
#undef SMORE_SYM
        ok = true;
    });
    return ok ? &r : nullptr;
}

int nccl_fail(smore_ctx* c, const char* what, ncclResult_t r) {
    Rccl* L = rccl();
    return fail(c, SMORE_EHIP, std::string(what) + ": " + (L ? L->error_string(r) : "RCCL unavailable"));
}

#define NCCLCHK(c, what, expr)                                   \
    do {                                                         \
        ncclResult_t r_ = (expr);                                \
        if (r_ != ncclSuccess) return nccl_fail((c), what, r_);  \
    } while (0)

size_t table_floats(const smore_ctx* c) { return (size_t)c->g->V * (size_t)c->dpad; }

// exchange buffers S, D, R per table and the exchange stream / events
int ensure_exchange(smore_ctx* c) {
    int rc;
    if ((rc = set_device(c))) return rc;
    if (!c->comm_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    if (!c->ex_ready) HIPCHK(c, hipEventCreateWithFlags(&c->ex_ready, hipEventDisableTiming));
    if (!c->ex_done) HIPCHK(c, hipEventCreateWithFlags(&c->ex_done, hipEventDisableTiming));
    const size_t n = table_floats(c);
    if (c->ex_n == n && c->ex_tables == c->ntables) return SMORE_OK;
    for (auto& t : c->ex_buf)
        for (float*& p : t) dfree(p);
    c->ex_n = 0;
    c->ex_tables = 0;
    c->ex_pending = false;
    for (int t = 0; t < c->ntables; ++t)
        for (float*& p : c->ex_buf[t]) HIPCHK(c, hipMalloc((void**)&p, std::max<size_t>(n, 4) * sizeof(float)));
    c->ex_n = n;
    c->ex_tables = c->ntables;
    return SMORE_OK;
}

int check_comm(smore_ctx* c) {
    if (!c) return SMORE_EINVAL;
    if (!c->comm) return fail(c, SMORE_ESTATE, "no communicator (smore_comm_init / smore_group_create)");
    if (c->ntables < 1 || !c->d_table[0]) return fail(c, SMORE_ESTATE, "tables not allocated");
    return ensure_exchange(c);
}

// S = T for every table: the replicas start from identical tables
int exchange_reset(smore_ctx* c) {
    int rc;
    if ((rc = check_comm(c))) return rc;
    if (c->ex_pending) {
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ex_done, 0));
        c->ex_pending = false;
    }
    for (int t = c->ex_t0; t < c->ntables; ++t)
        HIPCHK(c, hipMemcpyAsync(c->ex_buf[t][0], c->d_table[t], c->ex_n * sizeof(float), hipMemcpyDeviceToDevice,
                                 c->stream));
    return SMORE_OK;
}

// the uniform scale of the summed deltas under the in-flight exchange's rule
float rule_scale(const smore_ctx* c) { return c->ex_mode == SMORE_SYNC_MEAN ? 1.0f / (float)c->nranks : 1.0f; }

// the fused passes of an exchange's begin on the context stream (folding the
// in-flight exchange in first), then the hand-off event for the collective
int exchange_passes(smore_ctx* c, int mode) {
    int rc;
    if ((rc = set_device(c))) return rc;
    if (mode < SMORE_SYNC_SUM || mode > SMORE_SYNC_ADAPTIVE) return fail(c, SMORE_EINVAL, "bad exchange rule");
    if (mode == SMORE_SYNC_ADAPTIVE && !c->ex_scale[0])
        return fail(c, SMORE_ESTATE, "adaptive exchange without row scales (smore_exchange_set_adaptive)");
    if (c->ex_pending) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ex_done, 0));
    for (int t = c->ex_t0; t < c->ntables; ++t) {
        float* T = c->d_table[t];
        float* const* b = c->ex_buf[t];
        if (!c->ex_pending) HIPCHK(c, launch_delta_begin(T, b[0], b[1], b[2], c->ex_n, c->cus, c->stream));
        else if (c->ex_mode == SMORE_SYNC_ADAPTIVE)
            HIPCHK(c, launch_delta_cycle_rows(T, b[0], b[1], b[2], c->ex_scale[t], (uint64_t)c->g->V, c->dpad, c->cus,
                                              c->stream));
        else HIPCHK(c, launch_delta_cycle(T, b[0], b[1], b[2], rule_scale(c), c->ex_n, c->cus, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ex_ready, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->comm_stream, c->ex_ready, 0));
    c->ex_mode = mode;
    return SMORE_OK;
}

int exchange_collective(smore_ctx* c) {
    Rccl* L = rccl();
    for (int t = c->ex_t0; t < c->ntables; ++t)
        NCCLCHK(c, "ncclAllReduce",
                L->all_reduce(c->ex_buf[t][2], c->ex_buf[t][2], c->ex_n, ncclFloat32, ncclSum, (ncclComm_t)c->comm,
                              c->comm_stream));
    c->coll_queued = true;
    return SMORE_OK;
}

int exchange_posted(smore_ctx* c) {
    int rc;
    if ((rc = set_device(c))) return rc;
    HIPCHK(c, hipEventRecord(c->ex_done, c->comm_stream));
    c->ex_pending = true;
    return SMORE_OK;
}

int exchange_end(smore_ctx* c) {
    int rc;
    if ((rc = check_comm(c))) return rc;
    if (!c->ex_pending) return SMORE_OK;
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ex_done, 0));
    for (int t = c->ex_t0; t < c->ntables; ++t) {
        float* const* b = c->ex_buf[t];
        if (c->ex_mode == SMORE_SYNC_ADAPTIVE)
            HIPCHK(c, launch_delta_end_rows(c->d_table[t], b[0], b[1], b[2], c->ex_scale[t], (uint64_t)c->g->V,
                                            c->dpad, c->cus, c->stream));
        else HIPCHK(c, launch_delta_end(c->d_table[t], b[0], b[1], b[2], rule_scale(c), c->ex_n, c->cus, c->stream));
    }
    c->ex_pending = false;
    return SMORE_OK;
}

// the adaptive rule's per-row scales (smore_hip.h SMORE_SYNC_ADAPTIVE) for
// `updates` samples of `model` per rank per exchange over `nranks` ranks, from
// the sampler marginals of c's graph
int adaptive_scales(smore_ctx* c, int model, int K, double updates, double c0, int nranks,
                    std::vector<float> (&out)[2]) {
    const int64_t V = c->g->V;
    std::vector<double> rate((size_t)V);
    for (int t = 0; t < c->ntables; ++t) {
        int rc;
        if ((rc = smore_row_rates(c, model, K, t, V, rate.data()))) return rc;
        out[t].resize((size_t)V);
        for (int64_t v = 0; v < V; ++v) {
            const double k = rate[v] * updates * nranks;
            const double sv = k > c0 ? c0 / k : 1.0;
            out[t][v] = (float)(sv + (1.0 - sv) / nranks);
        }
    }
    return SMORE_OK;
}

int upload_scales(smore_ctx* c, const std::vector<float> (&sc)[2], const std::string& key) {
    int rc;
    if ((rc = set_device(c))) return rc;
    // an in-flight exchange's end reads the old scales on the stream: replace
    // them only after it drained
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int t = 0; t < 2; ++t) {
        dfree(c->ex_scale[t]);
        if (t < c->ntables && (rc = upload(c, c->ex_scale[t], sc[t].data(), sc[t].size()))) return rc;
    }
    c->ex_scale_key = key;
    return SMORE_OK;
}

std::string scale_key(int model, int K, double updates, double c0, int nranks, const smore_ctx* c) {
    char key[160];
    snprintf(key, sizeof key, "%d/%d/%.17g/%.17g/%d/%lld/%d/%llu", model, K, updates, c0, nranks, (long long)c->g->V,
             c->ntables, model == SMORE_CENSUS ? (unsigned long long)c->census_gen : 0ull);
    return key;
}

}  // namespace

void smore_exchange_release(smore_ctx* c) {
    if (!c) return;
    if (c->device >= 0) (void)hipSetDevice(c->device);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    for (auto& t : c->ex_buf)
        for (float*& p : t) dfree(p);
    for (int t = 0; t < 2; ++t) {
        dfree(c->hot_idx[t]);
        dfree(c->hot_buf[t][0]);
        dfree(c->hot_buf[t][1]);
    }
    c->hot_n = 0;
    c->hot_ex_key.clear();
    for (float*& p : c->ex_scale) dfree(p);
    c->ex_scale_key.clear();
    if (c->comm && c->own_comm) {
        ncclComm_t cm = (ncclComm_t)c->comm;
        comm_release(rccl(), &cm, 1);
    }
    c->comm = nullptr;
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->ex_ready) (void)hipEventDestroy(c->ex_ready);
    if (c->ex_done) (void)hipEventDestroy(c->ex_done);
    c->comm_stream = nullptr;
    c->ex_ready = c->ex_done = nullptr;
}

struct smore_group {
    std::vector<smore_ctx*> ctx;
    std::vector<ncclComm_t> comms;
    std::string err;
    // hub-row exchange (smore_group_set_hot_exchange): rows per table (-1:
    // automatic, 0: off) and training launches per exchange round
    int64_t hot_rows = -1;
    int launches = 8;
    double c0 = -1.0;   // adaptive exchange (smore_group_set_adaptive); -1: 2048 with the source partition, else 64
    int partition = 1;  // LINE-2: W rows partitioned by source (smore_group_set_partition)
    int walk_partition = 0;   // walk models: W rows partitioned by walk center (smore_group_set_walk_partition)
    // every replica on one device: collectives as device passes, ordered by
    // events between the replicas' streams (no RCCL)
    bool local = false;
    std::vector<hipEvent_t> lev;   // one per replica
    hipEvent_t ldone = nullptr;
    // the 2-D block schedule (smore_group_set_schedule): per replica the
    // compute-done event of a sub-round and the receive-done events of the
    // last two rotations (by sub-round parity)
    int schedule = SMORE_SCHED_BLOCKS;   // include/smore_hip.h: the default
    std::vector<hipEvent_t> bdone, brecv;
    // the block schedule's hub slots (blocks.cpp): per replica the event
    // after its exchange pass (compute stream) and after the all-reduce
    std::vector<hipEvent_t> hready, hdone;
    // same-device studies (SMORE_LOCAL_SERIAL=1): the replicas' cells run one
    // after another, each with the whole GPU as on its own device
    std::vector<hipEvent_t> lser;
};

namespace {

int gfail(smore_group* g, int rank, int rc) {
    if (g && rc != SMORE_OK && rank >= 0) g->err = "replica " + std::to_string(rank) + ": " + g->ctx[rank]->err;
    return rc;
}

// ---- the group's collectives over per-replica buffers, each replica's part
// on its own stream (RCCL: one grouped call; local: device passes)
int coll_allreduce(smore_group* g, const std::vector<float*>& buf, size_t n, const std::vector<hipStream_t>& st,
                   const char* what) {
    const size_t R = g->ctx.size();
    if (g->local) {
        smore_ctx* c0 = g->ctx[0];
        int rc;
        if ((rc = set_device(c0))) return gfail(g, 0, rc);
        // the sum runs on replica 0's stream after every replica's stream
        // reached this point; every stream continues after the sum
        for (size_t r = 1; r < R; ++r) {
            if (hipEventRecord(g->lev[r], st[r]) != hipSuccess || hipStreamWaitEvent(st[0], g->lev[r], 0) != hipSuccess)
                return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, std::string(what) + ": event"));
        }
        if (launch_local_sum(buf.data(), (int)R, n, c0->cus, st[0]) != hipSuccess)
            return gfail(g, 0, fail(c0, SMORE_EHIP, std::string(what) + ": local sum"));
        if (hipEventRecord(g->ldone, st[0]) != hipSuccess) return gfail(g, 0, fail(c0, SMORE_EHIP, what));
        for (size_t r = 1; r < R; ++r)
            if (hipStreamWaitEvent(st[r], g->ldone, 0) != hipSuccess)
                return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, what));
        return SMORE_OK;
    }
    Rccl* L = rccl();
    ncclResult_t nr = L->group_start();
    for (size_t r = 0; r < R && nr == ncclSuccess; ++r) {
        (void)hipSetDevice(g->ctx[r]->device);
        nr = L->all_reduce(buf[r], buf[r], n, ncclFloat32, ncclSum, (ncclComm_t)g->ctx[r]->comm, st[r]);
    }
    ncclResult_t ne = L->group_end();
    if (nr == ncclSuccess) nr = ne;
    if (nr != ncclSuccess) return gfail(g, 0, nccl_fail(g->ctx[0], what, nr));
    return SMORE_OK;
}

int coll_broadcast(smore_group* g, const std::vector<float*>& buf, size_t n, int root,
                   const std::vector<hipStream_t>& st, const char* what) {
    const size_t R = g->ctx.size();
    if (g->local) {
        int rc;
        if ((rc = set_device(g->ctx[0]))) return gfail(g, 0, rc);
        if (hipEventRecord(g->ldone, st[root]) != hipSuccess) return gfail(g, root, fail(g->ctx[root], SMORE_EHIP, what));
        for (size_t r = 0; r < R; ++r) {
            if ((int)r == root) continue;
            // the copy waits for the root's stream; the root's stream waits
            // for the copy before it writes the rows again
            if (hipStreamWaitEvent(st[r], g->ldone, 0) != hipSuccess ||
                hipMemcpyAsync(buf[r], buf[root], n * sizeof(float), hipMemcpyDeviceToDevice, st[r]) != hipSuccess ||
                hipEventRecord(g->lev[r], st[r]) != hipSuccess || hipStreamWaitEvent(st[root], g->lev[r], 0) != hipSuccess)
                return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, std::string(what) + ": local copy"));
        }
        return SMORE_OK;
    }
    Rccl* L = rccl();
    ncclResult_t nr = L->group_start();
    for (size_t r = 0; r < R && nr == ncclSuccess; ++r) {
        (void)hipSetDevice(g->ctx[r]->device);
        nr = L->broadcast(buf[r], buf[r], n, ncclFloat32, root, (ncclComm_t)g->ctx[r]->comm, st[r]);
    }
    ncclResult_t ne = L->group_end();
    if (nr == ncclSuccess) nr = ne;
    if (nr != ncclSuccess) return gfail(g, 0, nccl_fail(g->ctx[0], what, nr));
    return SMORE_OK;
}

std::vector<hipStream_t> compute_streams(const smore_group* g) {
    std::vector<hipStream_t> st;
    for (smore_ctx* c : g->ctx) st.push_back(c->stream);
    return st;
}

// every replica adopts replica 0's (shared) host graph and uploads it
int replicate_graph(smore_group* g) {
    smore_ctx* c0 = g->ctx[0];
    for (size_t r = 1; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        c->g = c0->g;
        c->hot_key.clear();
        c->semantics = SMORE_SEM_CPP;
        int rc = upload_graph(c);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int group_exchange_begin(smore_group* g, int rule) {
    int rc;
    const size_t R = g->ctx.size();
    for (size_t r = 0; r < R; ++r)
        if ((rc = exchange_passes(g->ctx[r], rule))) return gfail(g, (int)r, rc);
    std::vector<hipStream_t> st;
    for (smore_ctx* c : g->ctx) st.push_back(c->comm_stream);
    for (int t = g->ctx[0]->ex_t0; t < g->ctx[0]->ntables; ++t) {
        std::vector<float*> buf;
        for (smore_ctx* c : g->ctx) buf.push_back(c->ex_buf[t][2]);
        if ((rc = coll_allreduce(g, buf, g->ctx[0]->ex_n, st, "ncclAllReduce"))) return rc;
    }
    for (size_t r = 0; r < R; ++r)
        if ((rc = exchange_posted(g->ctx[r]))) return gfail(g, (int)r, rc);
    return SMORE_OK;
}

// the hub rows of every exchanged table of every replica (replica 0's host
// graph: all replicas share it); keyed by the rows' law and the tables (the
// key is cleared with the graph, upload_graph)
int ensure_hot(smore_group* g, int model, int K, int64_t rows) {
    smore_ctx* c0 = g->ctx[0];
    const std::string key = std::to_string(model) + "/" + std::to_string(K) + "/" + std::to_string(rows) + "/" +
                            std::to_string(c0->dpad) + "/" + std::to_string(c0->ntables) + "/" +
                            std::to_string(c0->ex_t0) + "/" + std::to_string(c0->g->V) + "/" +
                            std::to_string(c0->g->E) + "/" + c0->census_key;
    bool same = true;
    for (smore_ctx* c : g->ctx) same = same && c->hot_ex_key == key;
    if (same) return SMORE_OK;
    std::vector<int32_t> ids[2];
    for (int t = c0->ex_t0; t < c0->ntables; ++t) {
        ids[t].resize((size_t)rows);
        int rc = smore_hot_row_ids(c0, model, K, t, rows, ids[t].data());
        if (rc) return gfail(g, 0, rc);
    }
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        int rc;
        if ((rc = set_device(c))) return gfail(g, (int)r, rc);
        for (int t = 0; t < 2; ++t) {
            dfree(c->hot_idx[t]);
            dfree(c->hot_buf[t][0]);
            dfree(c->hot_buf[t][1]);
        }
        for (int t = c->ex_t0; t < c->ntables; ++t) {
            if ((rc = upload(c, c->hot_idx[t], ids[t].data(), ids[t].size()))) return gfail(g, (int)r, rc);
            for (float*& p : c->hot_buf[t])
                if (hipMalloc((void**)&p, (size_t)rows * c->dpad * sizeof(float)) != hipSuccess)
                    return gfail(g, (int)r, fail(c, SMORE_EHIP, "hub-row exchange buffers"));
        }
        c->hot_n = rows;
        c->hot_ex_key = key;
    }
    return SMORE_OK;
}

// the synchronous hub-row exchange of the exchanged tables on every replica's
// compute stream (a table outside [ex_t0, ntables) has no snapshot to pack against)
int group_hot_exchange(smore_group* g) {
    int rc;
    const int t0 = g->ctx[0]->ex_t0;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        if ((rc = set_device(c))) return gfail(g, (int)r, rc);
        for (int t = t0; t < c->ntables; ++t)
            if (launch_hot_pack(c->d_table[t], c->ex_buf[t][0], c->hot_idx[t], (uint64_t)c->hot_n, c->dpad,
                                c->hot_buf[t][0], c->hot_buf[t][1], c->cus, c->stream) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "hot_pack"));
    }
    const std::vector<hipStream_t> st = compute_streams(g);
    for (int t = t0; t < g->ctx[0]->ntables; ++t) {
        std::vector<float*> buf;
        for (smore_ctx* c : g->ctx) buf.push_back(c->hot_buf[t][1]);
        if ((rc = coll_allreduce(g, buf, (size_t)g->ctx[0]->hot_n * g->ctx[0]->dpad, st, "hub-row ncclAllReduce")))
            return rc;
    }
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        if ((rc = set_device(c))) return gfail(g, (int)r, rc);
        for (int t = t0; t < c->ntables; ++t)
            if (launch_hot_unpack(c->d_table[t], c->ex_buf[t][0], c->hot_idx[t], (uint64_t)c->hot_n, c->dpad,
                                  c->hot_buf[t][0], c->hot_buf[t][1], c->cus, c->stream) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "hot_unpack"));
    }
    return SMORE_OK;
}

// every replica gets every part's W rows from the part's owner (replica p
// owns rows [b[p], b[p+1]): the source partition's or the walk partition's
// parts): one in-place broadcast per part
int gather_sources(smore_group* g, const std::vector<int64_t>& b) {
    const size_t n = g->ctx.size();
    int rc;
    const std::vector<hipStream_t> st = compute_streams(g);
    for (size_t p = 0; p < n; ++p) {
        if (b[p + 1] <= b[p]) continue;
        std::vector<float*> rows;
        for (smore_ctx* c : g->ctx) rows.push_back(c->d_table[0] + (size_t)b[p] * c->dpad);
        if ((rc = coll_broadcast(g, rows, (size_t)(b[p + 1] - b[p]) * g->ctx[0]->dpad, (int)p, st,
                                 "W gather ncclBroadcast")))
            return rc;
    }
    return SMORE_OK;
}

// the end of a group call: with RCCL communicators the host waits for every
// replica's stream under the failure watch (comm_watch.h: async errors
// polled, the wait bounded, communicators aborted on failure)
int group_sync(smore_group* g) {
    int rc;
    if (!g->local && !g->comms.empty()) {
        std::string why;
        int bad = -1;
        auto ready = [&]() -> int {
            for (size_t r = 0; r < g->ctx.size(); ++r) {
                (void)hipSetDevice(g->ctx[r]->device);
                const hipError_t e = hipStreamQuery(g->ctx[r]->stream);
                if (e == hipErrorNotReady) return 0;
                if (e != hipSuccess) {
                    bad = (int)r;
                    return -1;
                }
            }
            return 1;
        };
        if (comm_watch(rccl(), g->comms.data(), (int)g->comms.size(), ready, comm_timeout(), why)) {
            // the communicators are aborted (freed): no replica may use its
            // handle again, and the group's teardown skips them
            for (smore_ctx* c : g->ctx) c->comm = nullptr;
            return gfail(g, bad < 0 ? 0 : bad, fail(g->ctx[bad < 0 ? 0 : bad], SMORE_EHIP, why));
        }
    }
    for (size_t r = 0; r < g->ctx.size(); ++r)
        if ((rc = smore_synchronize(g->ctx[r]))) return gfail(g, (int)r, rc);
    return SMORE_OK;
}

// ---- the 2-D block schedule's group side (blocks.cpp holds one replica's):
// sub-round s trains cell (r, (2r + s) mod nb) on replica r; after it replica
// r sends that C block to r - 1, which trains it at sub-round s + 2, and
// receives the block r + 1 just trained.  Replica r's stream waits for the
// receive of the rotation two sub-rounds back before its sub-round, so a
// transfer overlaps one whole sub-round.  No row is replicated while it
// trains: nothing is all-reduced.
int ensure_block_events(smore_group* g) {
    const size_t n = g->ctx.size();
    if (g->bdone.size() == n) return SMORE_OK;
    g->bdone.assign(n, nullptr);
    g->brecv.assign(2 * n, nullptr);
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        int rc;
        if ((rc = set_device(c))) return gfail(g, (int)r, rc);
        if (!c->comm_stream && hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking) != hipSuccess)
            return gfail(g, (int)r, fail(c, SMORE_EHIP, "block schedule: comm stream"));
        for (hipEvent_t* e : {&g->bdone[r], &g->brecv[2 * r], &g->brecv[2 * r + 1]})
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "block schedule: events"));
    }
    return SMORE_OK;
}

float* block_rows(smore_ctx* c, int b) { return c->d_table[1] + (size_t)c->blk.cb[b] * c->dpad; }
size_t block_floats(const smore_ctx* c, int b) { return (size_t)(c->blk.cb[b + 1] - c->blk.cb[b]) * c->dpad; }

int group_rotate(smore_group* g, uint64_t s) {
    const size_t n = g->ctx.size();
    const int nb = 2 * (int)n;
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        (void)hipSetDevice(c->device);
        if (hipEventRecord(g->bdone[r], c->stream) != hipSuccess)
            return gfail(g, (int)r, fail(c, SMORE_EHIP, "block rotation: event"));
    }
    if (g->local) {
        for (size_t r = 0; r < n; ++r) {
            smore_ctx *c = g->ctx[r], *d = g->ctx[(r + n - 1) % n];
            const int b = (int)((2 * r + s) % (uint64_t)nb);
            hipEvent_t done = g->brecv[2 * ((r + n - 1) % n) + (s & 1)];
            if (hipStreamWaitEvent(d->comm_stream, g->bdone[r], 0) != hipSuccess ||
                hipMemcpyAsync(block_rows(d, b), block_rows(c, b), block_floats(c, b) * sizeof(float),
                               hipMemcpyDeviceToDevice, d->comm_stream) != hipSuccess ||
                hipEventRecord(done, d->comm_stream) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "block rotation: local copy"));
        }
        return SMORE_OK;
    }
    Rccl* L = rccl();
    for (size_t r = 0; r < n; ++r) {
        (void)hipSetDevice(g->ctx[r]->device);
        if (hipStreamWaitEvent(g->ctx[r]->comm_stream, g->bdone[r], 0) != hipSuccess)
            return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "block rotation: wait"));
    }
    ncclResult_t nr = L->group_start();
    for (size_t r = 0; r < n && nr == ncclSuccess; ++r) {
        smore_ctx* c = g->ctx[r];
        (void)hipSetDevice(c->device);
        const int b = (int)((2 * r + s) % (uint64_t)nb), b2 = (b + 2) % nb;
        nr = L->send(block_rows(c, b), block_floats(c, b), ncclFloat32, (int)((r + n - 1) % n), (ncclComm_t)c->comm,
                     c->comm_stream);
        if (nr == ncclSuccess)
            nr = L->recv(block_rows(c, b2), block_floats(c, b2), ncclFloat32, (int)((r + 1) % n), (ncclComm_t)c->comm,
                         c->comm_stream);
    }
    ncclResult_t ne = L->group_end();
    if (nr == ncclSuccess) nr = ne;
    if (nr != ncclSuccess) return gfail(g, 0, nccl_fail(g->ctx[0], "block rotation ncclSend/ncclRecv", nr));
    for (size_t r = 0; r < n; ++r) {
        (void)hipSetDevice(g->ctx[r]->device);
        if (hipEventRecord(g->brecv[2 * r + (s & 1)], g->ctx[r]->comm_stream) != hipSuccess)
            return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "block rotation: event"));
    }
    return SMORE_OK;
}

// replica r's stream waits for the block it trains at sub-round s
int block_wait(smore_group* g, size_t r, uint64_t s) {
    if (s < 2) return SMORE_OK;
    smore_ctx* c = g->ctx[r];
    (void)hipSetDevice(c->device);
    if (hipStreamWaitEvent(c->stream, g->brecv[2 * r + (s & 1)], 0) != hipSuccess)
        return gfail(g, (int)r, fail(c, SMORE_EHIP, "block schedule: wait"));
    return SMORE_OK;
}

int hub_ex_finish(smore_group* g);

// after the last rotation: every transfer done before the tables are read;
// then every replica gets the W parts from their owners and the C blocks from
// their holders (after S sub-rounds block b sits on replica ((b - S) mod nb) / 2)
int block_finish(smore_group* g, uint64_t S) {
    const size_t n = g->ctx.size();
    const int nb = 2 * (int)n;
    int rc;
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        (void)hipSetDevice(c->device);
        for (size_t q = 0; q < n; ++q) {
            if (!g->local && q != r) continue;   // RCCL: own transfers (send and receive) on own comm stream
            if (hipStreamWaitEvent(c->stream, g->brecv[2 * q], 0) != hipSuccess ||
                hipStreamWaitEvent(c->stream, g->brecv[2 * q + 1], 0) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "block schedule: drain"));
        }
    }
    // the hub slots back into their rows only now: the last rotation's
    // transfer carries the block's stale copy of those rows and would
    // overwrite a store queued ahead of the drain
    if ((rc = hub_ex_finish(g))) return rc;
    const std::vector<hipStream_t> st = compute_streams(g);
    smore_ctx* c0 = g->ctx[0];
    for (size_t p = 0; p < n; ++p) {
        std::vector<float*> rows;
        for (smore_ctx* c : g->ctx) rows.push_back(c->d_table[0] + (size_t)c0->blk.wb[p] * c->dpad);
        if ((rc = coll_broadcast(g, rows, (size_t)(c0->blk.wb[p + 1] - c0->blk.wb[p]) * c0->dpad, (int)p, st,
                                 "W parts ncclBroadcast")))
            return rc;
    }
    for (int b = 0; b < nb; ++b) {
        const int holder = (int)(((uint64_t)b + (uint64_t)nb - S % (uint64_t)nb) % (uint64_t)nb) / 2;
        std::vector<float*> rows;
        for (smore_ctx* c : g->ctx) rows.push_back(block_rows(c, b));
        if ((rc = coll_broadcast(g, rows, block_floats(c0, b), holder, st, "C blocks ncclBroadcast"))) return rc;
    }
    return group_sync(g);
}

// ---- the hub slots of the LINE-2 block schedule (blocks.cpp): every part
// trains its own copy of the H hub C rows in every cell; after each
// sub-round the copies' deltas are all-reduced one late (begin / cycle / end
// of replica_sync.hip on the slot rows, per-slot adaptive scales), on the
// comm streams ahead of the rotation
// the slots' adaptive rule's c0: LINE-2 2048 (the source-partitioned replica
// exchange's); walk models 64 (theirs: a C5 run is ~2000 pair updates per
// row in all, so a hub's copies are averaged sooner -- c0 2048 cost 1.11x
// one GPU's held-out loss at 8 parts, 64 1.026x)
double hub_c0(const smore_group* g) {
    const char* e = getenv("SMORE_HUB_C0");
    const double v = e ? atof(e) : 0.0;
    if (v > 0) return v;
    return g->ctx[0]->blk.model == SMORE_CENSUS ? 64.0 : 2048.0;
}

float* hub_slots(smore_ctx* c) { return c->d_table[1] + (size_t)c->g->V * c->dpad; }

int hub_ex_start(smore_group* g, double samples_per_exchange) {
    const size_t n = g->ctx.size();
    if (!g->ctx[0]->blk.H) return SMORE_OK;
    if (g->hready.size() != n) {
        g->hready.assign(n, nullptr);
        g->hdone.assign(n, nullptr);
        for (size_t r = 0; r < n; ++r) {
            (void)hipSetDevice(g->ctx[r]->device);
            if (hipEventCreateWithFlags(&g->hready[r], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g->hdone[r], hipEventDisableTiming) != hipSuccess)
                return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "hub exchange: events"));
        }
    }
    const double c0 = hub_c0(g);
    char key[96];
    snprintf(key, sizeof key, "%.17g/%.17g", samples_per_exchange, c0);
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        auto& B = c->blk;
        int rc;
        if ((rc = set_device(c))) return gfail(g, (int)r, rc);
        const size_t nf = (size_t)B.H * c->dpad;
        for (float*& p : B.d_hub_ex)
            if (!p && hipMalloc((void**)&p, nf * sizeof(float)) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "hub exchange buffers"));
        if (B.hub_scale_key != key) {
            std::vector<float> sc((size_t)B.H);
            hub_scales(B, samples_per_exchange, c0, sc.data());
            if ((rc = upload(c, B.d_hub_scale, sc.data(), sc.size()))) return gfail(g, (int)r, rc);
            B.hub_scale_key = key;
        }
        if ((rc = smore_block_hubs_load(c))) return gfail(g, (int)r, rc);
        if (hipMemcpyAsync(B.d_hub_ex[0], hub_slots(c), nf * sizeof(float), hipMemcpyDeviceToDevice, c->stream) !=
            hipSuccess)
            return gfail(g, (int)r, fail(c, SMORE_EHIP, "hub exchange: snapshot"));
        B.hub_pending = false;
    }
    return SMORE_OK;
}

// after every replica's cell of a sub-round: the exchange pass on the compute
// stream, then the all-reduce of the slots' deltas on the comm streams
int hub_ex_post(smore_group* g) {
    const size_t n = g->ctx.size();
    if (!g->ctx[0]->blk.H) return SMORE_OK;
    std::vector<float*> bufs;
    std::vector<hipStream_t> st;
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        auto& B = c->blk;
        (void)hipSetDevice(c->device);
        float* const* x = B.d_hub_ex;
        hipError_t e = hipSuccess;
        if (B.hub_pending) {
            e = hipStreamWaitEvent(c->stream, g->hdone[r], 0);
            if (e == hipSuccess)
                e = launch_delta_cycle_rows(hub_slots(c), x[0], x[1], x[2], B.d_hub_scale, (uint64_t)B.H, c->dpad,
                                            c->cus, c->stream);
        } else {
            e = launch_delta_begin(hub_slots(c), x[0], x[1], x[2], (uint64_t)B.H * c->dpad, c->cus, c->stream);
        }
        if (e == hipSuccess) e = hipEventRecord(g->hready[r], c->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->comm_stream, g->hready[r], 0);
        if (e != hipSuccess) return gfail(g, (int)r, fail(c, SMORE_EHIP, "hub exchange pass"));
        bufs.push_back(x[2]);
        st.push_back(c->comm_stream);
    }
    int rc;
    if ((rc = coll_allreduce(g, bufs, (size_t)g->ctx[0]->blk.H * g->ctx[0]->dpad, st, "hub ncclAllReduce"))) return rc;
    for (size_t r = 0; r < n; ++r) {
        (void)hipSetDevice(g->ctx[r]->device);
        if (hipEventRecord(g->hdone[r], g->ctx[r]->comm_stream) != hipSuccess)
            return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "hub exchange: event"));
        g->ctx[r]->blk.hub_pending = true;
    }
    return SMORE_OK;
}

// the last exchange's end (every copy of the slots equal again), then the
// slots back into the hub rows, before block_finish gathers the blocks
int hub_ex_finish(smore_group* g) {
    if (!g->ctx[0]->blk.H) return SMORE_OK;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        auto& B = c->blk;
        (void)hipSetDevice(c->device);
        if (B.hub_pending) {
            float* const* x = B.d_hub_ex;
            if (hipStreamWaitEvent(c->stream, g->hdone[r], 0) != hipSuccess ||
                launch_delta_end_rows(hub_slots(c), x[0], x[1], x[2], B.d_hub_scale, (uint64_t)B.H, c->dpad, c->cus,
                                      c->stream) != hipSuccess)
                return gfail(g, (int)r, fail(c, SMORE_EHIP, "hub exchange end"));
            B.hub_pending = false;
        }
        int rc;
        if ((rc = smore_block_hubs_store(c))) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

// SMORE_LOCAL_SERIAL=1 on a same-device group: replica r's next launch
// waits for the previous launch of replica r - 1 (of replica n - 1 for r = 0),
// so cells never share the GPU -- each runs with the whole device's
// concurrency, as on N GPUs (the quality studies' fidelity knob)
bool local_serial(const smore_group* g) {
    const char* e = getenv("SMORE_LOCAL_SERIAL");
    return g->local && e && atoi(e) != 0;
}

int serial_before(smore_group* g, size_t r) {
    if (!local_serial(g)) return SMORE_OK;
    const size_t n = g->ctx.size();
    if (g->lser.size() != n) {
        g->lser.assign(n, nullptr);
        for (size_t q = 0; q < n; ++q)
            if (hipEventCreateWithFlags(&g->lser[q], hipEventDisableTiming) != hipSuccess)
                return gfail(g, (int)q, fail(g->ctx[q], SMORE_EHIP, "serial events"));
        for (size_t q = 0; q < n; ++q) (void)hipEventRecord(g->lser[q], g->ctx[q]->stream);
    }
    const size_t p = (r + n - 1) % n;
    if (hipStreamWaitEvent(g->ctx[r]->stream, g->lser[p], 0) != hipSuccess)
        return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "serial wait"));
    return SMORE_OK;
}

int serial_after(smore_group* g, size_t r) {
    if (!local_serial(g)) return SMORE_OK;
    if (hipEventRecord(g->lser[r], g->ctx[r]->stream) != hipSuccess)
        return gfail(g, (int)r, fail(g->ctx[r], SMORE_EHIP, "serial record"));
    return SMORE_OK;
}

// samples per row per replica per epoch of the LINE-2 block schedule (the C4
// bench's one epoch per 2^27-sample step: 13.4 per row)
constexpr double EDGE_BLOCK_PER_ROW = 13.42;
constexpr uint64_t WALK_BLOCK_ROUND = (uint64_t)1 << 18;   // walks per epoch (blocks.cpp's round cap)

int group_block_edges(smore_group* g, uint64_t begin, uint64_t count, uint64_t per, uint64_t total, int K,
                      double alpha0, uint64_t seed, int mode) {
    const size_t n = g->ctx.size();
    const int nb = 2 * (int)n;
    int rc;
    if (count == 0) return SMORE_OK;
    for (size_t r = 0; r < n; ++r)
        if ((rc = smore_block_setup(g->ctx[r], SMORE_LINE2, (int)n, (int)r, K, mode))) return gfail(g, (int)r, rc);
    if ((rc = ensure_block_events(g))) return rc;
    const int64_t V = g->ctx[0]->g->V;
    if (per == 0)
        per = (uint64_t)std::min(134217728.0, std::max(1024.0 * nb, std::round(EDGE_BLOCK_PER_ROW * (double)V)));
    const uint64_t round_units = per > count / n ? count : per * (uint64_t)n;
    const uint64_t rounds = (count + round_units - 1) / round_units;
    auto round_lo = [&](uint64_t k) { return (uint64_t)(((unsigned __int128)count * k) / rounds); };
    std::vector<std::vector<uint64_t>> cnt(n, std::vector<uint64_t>((size_t)nb));
    std::vector<uint64_t> cur(n), share(n);
    // a round's samples go to the replicas in proportion to their parts'
    // source mass, so the union of the parts draws SourceSample's law
    const std::vector<double>& pm = g->ctx[0]->blk.part_mass;
    const int split = cell_launches(g->ctx[0]->blk);
    if ((rc = hub_ex_start(g, (double)std::min<uint64_t>(per, count / n) / nb / split))) return rc;
    uint64_t S = 0;
    for (uint64_t k = 0; k < rounds; ++k) {
        const uint64_t lo = round_lo(k), m = round_lo(k + 1) - lo;
        largest_remainder(m, pm.data(), (int)n, share.data());
        uint64_t b = lo;
        for (size_t r = 0; r < n; ++r) {
            if ((rc = smore_block_counts(g->ctx[r], share[r], cnt[r].data()))) return gfail(g, (int)r, rc);
            cur[r] = b;
            b += share[r];
        }
        for (int s = 0; s < nb; ++s, ++S) {
            // a cell in `split` launches, the hub slots exchanged after each
            // (blocks.cpp cell_launches)
            for (int q = 0; q < split; ++q) {
                for (size_t r = 0; r < n; ++r) {
                    const int bk = (int)((2 * r + (size_t)s) % (size_t)nb);
                    if (q == 0 && (rc = block_wait(g, r, S))) return rc;
                    const uint64_t x0 = cnt[r][bk] * q / split, x = cnt[r][bk] * (q + 1) / split - x0;
                    if ((rc = serial_before(g, r))) return rc;
                    if (x && (rc = smore_block_train_edges_async(g->ctx[r], bk, begin + cur[r] + x0, x, total, K,
                                                                 alpha0, seed, mode)))
                        return gfail(g, (int)r, rc);
                    if ((rc = serial_after(g, r))) return rc;
                }
                if ((rc = hub_ex_post(g))) return rc;
            }
            for (size_t r = 0; r < n; ++r) cur[r] += cnt[r][(2 * r + (size_t)s) % (size_t)nb];
            if ((rc = group_rotate(g, S))) return rc;
        }
    }
    return block_finish(g, S);   // hub_ex_finish after the drain
}

int group_block_walks(smore_group* g, int rule, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                      int walk_steps, int window, int window_min, int K, double alpha0, uint64_t seed,
                      const int64_t* order, int mode, uint64_t per) {
    const size_t n = g->ctx.size();
    const int nb = 2 * (int)n;
    int rc;
    const uint64_t total = (uint64_t)walk_times * (uint64_t)g->ctx[0]->g->V;
    if (walk_end > total) walk_end = total;
    if (walk_begin >= walk_end) return SMORE_OK;
    for (size_t r = 0; r < n; ++r)
        if ((rc = smore_block_setup(g->ctx[r], SMORE_CENSUS, (int)n, (int)r, K, mode))) return gfail(g, (int)r, rc);
    if ((rc = ensure_block_events(g))) return rc;
    if (per == 0 || per > WALK_BLOCK_ROUND) per = WALK_BLOCK_ROUND;
    {   // the hub slots' exchange: pair records per replica per sub-round
        const int L = walk_steps + 1;
        double ppw = 0.0;   // expected pairs per walk (SkipGrams' random shrink / Walklets' two ranges)
        for (int i = 0; i < L; ++i) {
            if (rule == 1) {
                ppw += (double)(std::min(L - 1, i + window) - std::min(L - 1, i + window_min - 1)) +
                       (double)(std::max(0, i - window_min + 1) - std::max(0, i - window));
            } else {
                for (int r = 1; r <= window; ++r)
                    ppw += (double)(std::min(L - 1, i + r) - std::max(0, i - r)) / window;
            }
        }
        const double walks = (double)std::min<uint64_t>(per, walk_end - walk_begin);
        const double launches = (double)cell_launches(g->ctx[0]->blk);
        if ((rc = hub_ex_start(g, std::max(1.0, walks * ppw / (double)(n * nb) / launches)))) return rc;
    }
    uint64_t S = 0;
    const char* ga = getenv("SMORE_WALK_GEN_ALL");
    const bool split_gen = !(ga && atoi(ga) != 0);
    for (uint64_t lo = walk_begin; lo < walk_end; lo += per) {
        const uint64_t hi = std::min(walk_end, lo + per), nw = hi - lo;
        // walk-partitioned generation: replica r walks its 1/N of the round,
        // every replica gets every walk (one broadcast of each slice from its
        // walker), then each buckets its own centres' pairs.  SMORE_WALK_GEN_ALL=1:
        // every replica walks every walk (round 5)
        for (size_t r = 0; r < n; ++r) {
            const uint64_t glo = split_gen ? lo + nw * r / n : lo, ghi = split_gen ? lo + nw * (r + 1) / n : hi;
            if ((rc = block_walks_gen(g->ctx[r], rule, lo, hi, glo, ghi, walk_times, walk_steps, window, window_min, K,
                                      alpha0, seed, order, 0, mode)))
                return gfail(g, (int)r, rc);
        }
        if (split_gen && n > 1) {
            const std::vector<hipStream_t> st = compute_streams(g);
            const size_t L = (size_t)walk_steps + 1;
            for (size_t q = 0; q < n; ++q) {
                const uint64_t o = nw * q / n, m = nw * (q + 1) / n - o;
                if (!m) continue;
                std::vector<float*> wb, lb;
                for (smore_ctx* c : g->ctx) {
                    wb.push_back(reinterpret_cast<float*>(c->d_walks + o * L));
                    lb.push_back(reinterpret_cast<float*>(c->d_lens + o));
                }
                if ((rc = coll_broadcast(g, wb, m * L, (int)q, st, "walks ncclBroadcast"))) return rc;
                if ((rc = coll_broadcast(g, lb, m, (int)q, st, "walk lengths ncclBroadcast"))) return rc;
            }
        }
        for (size_t r = 0; r < n; ++r)
            if ((rc = block_walks_emit(g->ctx[r]))) return gfail(g, (int)r, rc);
        const int L = cell_launches(g->ctx[0]->blk);
        for (int s = 0; s < nb; ++s, ++S) {
            for (int q = 0; q < L; ++q) {
                for (size_t r = 0; r < n; ++r) {
                    if (q == 0 && (rc = block_wait(g, r, S))) return rc;
                    if ((rc = serial_before(g, r))) return rc;
                    if ((rc = smore_block_train_walks_part_async(g->ctx[r], (int)((2 * r + (size_t)s) % (size_t)nb),
                                                                 q, L)))
                        return gfail(g, (int)r, rc);
                    if ((rc = serial_after(g, r))) return rc;
                }
                if ((rc = hub_ex_post(g))) return rc;
            }
            if ((rc = group_rotate(g, S))) return rc;
        }
    }
    return block_finish(g, S);   // hub_ex_finish after the drain
}

}  // namespace

// The group training round structure.  The range [begin, end) is cut into
// R = ceil(count / (per * N)) rounds of equal size (+-1); round k's units are
// split evenly over the N replicas (replica r gets the r-th of N equal
// slices, so every replica trains a share of every call -- with the source
// partition a replica that got nothing would leave its part's W rows
// untrained).  Replica r queues its slice on its stream (run(ctx, b, e) must
// not synchronize), then the group folds the previous exchange in and starts
// this round's all-reduce, which overlaps round k+1.  rule: SMORE_SYNC_*; the
// adaptive rule's row scales are made for `model` with K negatives at the
// replicas' actual units per round (count / (R N)) * upu updates per replica
// per exchange (upu: updates per unit).  model SMORE_CENSUS (the walk models):
// the rows' touches per unit come from a census of the call's first round on
// replica 0 (run in census mode: records generated, rows counted, nothing
// trained; smore_census_begin), redone only when census_key changes.  With
// the hub-row exchange on (sum rule), each replica's slice runs as
// g->launches launches and the hub rows are synced after each.
//
// part (LINE-2): the source partition.  walkpart (the walk models whose pairs
// come from pair_emit / go_pair_emit): the walk partition -- every replica
// runs the whole round and trains the pairs whose center it owns
// (smore_set_walk_owner over smore_walk_parts of the census), only C is
// exchanged, W is gathered from the owners at the end.
// Default exchange periods (per = 0): measured on config 2's graph for LINE-2
// (tools/replica_study.py + tools/samples_to_loss.py: 6.7 samples per row per
// replica per exchange gives the best effective 8-GPU speed-up, 4.4-5.4x
// counting the exchange passes; 13.4: 3.7-5.1x) and on config 5's for
// DeepWalk (4 pair updates per row per replica, c0 64: 1.02 / 1.07 / 1.35x
// one replica's held-out loss at 2 / 4 / 8 replicas; 54, about the old 2^18
// walks, drain 32: 1.09 / 1.79 / 3.75x), profiles/r04/replica
constexpr double EDGE_PER_ROW = 6.71, EDGE_PER_MIN = 4096.0, EDGE_PER_MAX = 134217728.0, WALK_PER_ROW = 4.0;

template <class F>
static int group_rounds(smore_group* g, uint64_t begin, uint64_t end, uint64_t per, int rule, F&& run,
                        int model = SMORE_LINE2, int K = 5, double upu = 1.0, bool part = false,
                        const std::string& census_key = std::string(), bool walkpart = false) {
    const size_t n = g->ctx.size();
    int rc;
    if (end <= begin) return SMORE_OK;
    if (rule < SMORE_SYNC_SUM || rule > SMORE_SYNC_ADAPTIVE) return gfail(g, 0, fail(g->ctx[0], SMORE_EINVAL, "bad exchange rule"));
    // LINE-2 with the source partition: replica r draws its sources from part
    // r, owns those W rows, and only C is exchanged (W gathered at the end)
    part = part && g->partition && n > 1;
    walkpart = walkpart && !part && g->walk_partition && n > 1;
    for (size_t r = 0; r < n; ++r) {
        smore_ctx* c = g->ctx[r];
        if ((rc = smore_set_source_partition(c, part ? (int)n : 1, part ? (int)r : 0))) return gfail(g, (int)r, rc);
        if ((rc = smore_set_walk_owner(c, 0, -1))) return gfail(g, (int)r, rc);
        c->ex_t0 = part || walkpart ? 1 : 0;
        if ((rc = exchange_reset(c))) return gfail(g, (int)r, rc);
    }
    const uint64_t count = end - begin;
    int64_t rows = g->hot_rows < 0 ? std::min<int64_t>(65536, g->ctx[0]->g->V / 8) : g->hot_rows;
    rows = std::min<int64_t>(rows, g->ctx[0]->g->V);
    const bool hot = rule == SMORE_SYNC_SUM && rows > 0 && g->launches > 1;
    const int64_t V = g->ctx[0]->g->V;
    if (model == SMORE_CENSUS && (rule == SMORE_SYNC_ADAPTIVE || hot || walkpart || per == 0)) {
        smore_ctx* c0 = g->ctx[0];
        const std::string key = census_key + "/" + std::to_string(c0->semantics);
        if (c0->census_key != key || !c0->census_ok) {
            // the first round (or 2^16 units at least, so that the hub rows'
            // rates are well measured on small rounds, or the call)
            const uint64_t m = std::min<uint64_t>(count, std::max<uint64_t>(per * (uint64_t)n, (uint64_t)1 << 16));
            if ((rc = smore_census_begin(c0))) return gfail(g, 0, rc);
            // m units in 16 slices spread evenly over [begin, end), not the
            // leading m: walks without a start order begin at walk mod V, so a
            // prefix would census one contiguous id block's neighbourhood only
            // 
            const uint64_t ns = std::min<uint64_t>(16, m);
            rc = SMORE_OK;
            for (uint64_t k = 0; k < ns && !rc; ++k) {
                const uint64_t lo = begin + (uint64_t)(((unsigned __int128)count * k) / ns);
                const uint64_t len = m * (k + 1) / ns - m * k / ns;
                if (len) rc = run(c0, lo, lo + len);
            }
            const int rc2 = smore_census_end(c0, (double)m);
            if (rc || rc2) return gfail(g, 0, rc ? rc : rc2);
            c0->census_key = key;
            for (size_t r = 1; r < n; ++r) g->ctx[r]->census_key.clear();
        }
    }
    if (per == 0) {
        // the default exchange period, relative to the graph:
        // edge models EDGE_PER_ROW samples per row per replica, walk models
        // WALK_PER_ROW W updates (pairs) per row per replica, from the census
        if (model == SMORE_CENSUS) {
            double upr = 0.0;   // W touches (pairs) per unit
            for (double x : g->ctx[0]->census_rate[0]) upr += x;
            per = (uint64_t)std::max(1.0, std::round(WALK_PER_ROW * (double)V / std::max(upr, 1e-30)));
        } else {
            per = (uint64_t)std::min(EDGE_PER_MAX, std::max(EDGE_PER_MIN, std::round(EDGE_PER_ROW * (double)V)));
        }
    }
    const uint64_t round_units = per > count / n ? count : per * (uint64_t)n;   // no overflow: per * n <= count
    const uint64_t rounds = (count + round_units - 1) / round_units;
    auto round_lo = [&](uint64_t k) { return (uint64_t)(((unsigned __int128)count * k) / rounds); };
    const double share = (double)count / ((double)rounds * (double)n);   // units per replica per exchange
    std::vector<int64_t> bounds((size_t)n + 1);
    if (part && (rc = smore_source_parts(g->ctx[0], (int)n, bounds.data()))) return gfail(g, 0, rc);
    if (walkpart) {
        if ((rc = smore_walk_parts(g->ctx[0], (int)n, bounds.data()))) return gfail(g, 0, rc);
        for (size_t r = 0; r < n; ++r)
            if ((rc = smore_set_walk_owner(g->ctx[r], bounds[r], bounds[r + 1]))) return gfail(g, (int)r, rc);
    }
    const double c0v = g->c0 > 0 ? g->c0 : (part ? 2048.0 : 64.0);
    if (rule == SMORE_SYNC_ADAPTIVE) {
        const double updates = share * upu;
        const std::string key = scale_key(model, K, updates, c0v, (int)n, g->ctx[0]) + "/" + g->ctx[0]->census_key;
        bool same = true;
        for (smore_ctx* c : g->ctx) same = same && c->ex_scale_key == key;
        if (!same) {
            std::vector<float> sc[2];
            if ((rc = adaptive_scales(g->ctx[0], model, K, updates, c0v, (int)n, sc))) return gfail(g, 0, rc);
            for (size_t r = 0; r < n; ++r)
                if ((rc = upload_scales(g->ctx[r], sc, key))) return gfail(g, (int)r, rc);
        }
    }
    if (hot && (rc = ensure_hot(g, model, K, rows))) return rc;
    const int sub = hot ? g->launches : 1;
    for (uint64_t k = 0; k < rounds; ++k) {
        const uint64_t lo = round_lo(k), m = round_lo(k + 1) - lo;
        for (int j = 0; j < sub; ++j) {
            for (size_t r = 0; r < n; ++r) {
                // the walk partition: every replica runs the whole round (its pairs)
                const uint64_t b = walkpart ? lo : lo + (uint64_t)(((unsigned __int128)m * r) / n);
                const uint64_t e = walkpart ? lo + m : lo + (uint64_t)(((unsigned __int128)m * (r + 1)) / n);
                const uint64_t bj = b + (e - b) * (uint64_t)j / sub, ej = b + (e - b) * (uint64_t)(j + 1) / sub;
                if (ej > bj && (rc = run(g->ctx[r], begin + bj, begin + ej))) return gfail(g, (int)r, rc);
            }
            if (hot && (rc = group_hot_exchange(g))) return rc;
        }
        if ((rc = group_exchange_begin(g, rule))) return rc;
    }
    for (size_t r = 0; r < n; ++r)
        if ((rc = exchange_end(g->ctx[r]))) return gfail(g, (int)r, rc);
    if ((part || walkpart) && (rc = gather_sources(g, bounds))) return rc;
    if ((rc = group_sync(g))) return rc;
    for (size_t r = 0; walkpart && r < n; ++r)
        if ((rc = smore_set_walk_owner(g->ctx[r], 0, -1))) return gfail(g, (int)r, rc);
    return SMORE_OK;
}

// the block schedule applies: asked for (the default), more than one replica,
// and the C++ rules (the Go rules keep the replicas)
static bool blocks_for(const smore_group* g) {
    return g->schedule == SMORE_SCHED_BLOCKS && g->ctx.size() > 1 && g->ctx[0]->semantics == SMORE_SEM_CPP;
}

// the census key of a walk-model call: the model and every argument that
// changes which rows its records touch (walk law, window, K, seed)
static std::string census_key(const char* model, std::initializer_list<double> args) {
    std::string k = model;
    char b[40];
    for (double a : args) {
        snprintf(b, sizeof b, "/%.17g", a);
        k += b;
    }
    return k;
}

namespace smore_host {
// smore_synchronize of a context with its own communicator (one process per
// GPU): the stream's completion under the failure watch -- only when a
// collective was queued since the last watched sync (a long training call
// with no collective in flight is not a stuck peer)
int comm_sync(smore_ctx* c) {
    if (!c->comm || !c->own_comm || !c->coll_queued) return SMORE_OK;
    ncclComm_t cm = (ncclComm_t)c->comm;
    std::string why;
    auto ready = [&]() -> int {
        const hipError_t e = hipStreamQuery(c->stream);
        return e == hipSuccess ? 1 : e == hipErrorNotReady ? 0 : -1;
    };
    if (comm_watch(rccl(), &cm, 1, ready, comm_timeout(), why)) {
        c->comm = nullptr;   // aborted (freed): smore_exchange_release must not destroy it
        c->own_comm = false;
        return fail(c, SMORE_EHIP, why);
    }
    c->coll_queued = false;
    return SMORE_OK;
}
}  // namespace smore_host

extern "C" {

int smore_set_comm_timeout(double seconds) {
    if (!(seconds > 0.0) && seconds != -1.0) return SMORE_EINVAL;
    g_comm_timeout = seconds;
    return SMORE_OK;
}

int smore_comm_unique_id(unsigned char* id) {
    if (!id) return SMORE_EINVAL;
    Rccl* L = rccl();
    if (!L) return SMORE_EHIP;
    ncclUniqueId u;
    if (L->get_unique_id(&u) != ncclSuccess) return SMORE_EHIP;
    memcpy(id, u.internal, SMORE_COMM_ID_BYTES);
    return SMORE_OK;
}

int smore_comm_init(smore_ctx* c, int nranks, int rank, const unsigned char* id) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return SMORE_EINVAL;
    int rc;
    if ((rc = set_device(c))) return rc;
    Rccl* L = rccl();
    if (!L) return fail(c, SMORE_EHIP, "RCCL unavailable");
    if (c->comm) return fail(c, SMORE_ESTATE, "context already has a communicator");
    ncclUniqueId u;
    memcpy(u.internal, id, SMORE_COMM_ID_BYTES);
    ncclComm_t comm = nullptr;
    NCCLCHK(c, "ncclCommInitRank", L->init_rank(&comm, nranks, u, rank));
    c->comm = comm;
    c->own_comm = true;
    c->nranks = nranks;
    c->rank = rank;
    return SMORE_OK;
}

int smore_exchange_reset(smore_ctx* c) { return exchange_reset(c); }

int smore_exchange_begin(smore_ctx* c, int mean) {
    int rc;
    if ((rc = check_comm(c))) return rc;
    if (c->local_comm) return fail(c, SMORE_ESTATE, "a same-device group's replica: use the smore_group_* calls");
    if ((rc = exchange_passes(c, mean))) return rc;
    if ((rc = exchange_collective(c))) return rc;
    return exchange_posted(c);
}

int smore_exchange_end(smore_ctx* c) { return exchange_end(c); }

int smore_exchange_set_adaptive(smore_ctx* c, int model, int K, double updates, double c0) {
    if (!c || !(updates > 0.0) || !(c0 > 0.0)) return SMORE_EINVAL;
    if (!c->has_graph) return fail(c, SMORE_ESTATE, "no graph");
    if (c->ntables < 1) return fail(c, SMORE_ESTATE, "tables not allocated");
    // the scales depend on the world size: only after smore_comm_init
    if (!c->comm) return fail(c, SMORE_ESTATE, "adaptive exchange before smore_comm_init");
    // an in-flight exchange's end applies the scales it was begun with
    if (c->ex_pending) return fail(c, SMORE_ESTATE, "adaptive scales changed while an exchange is in flight");
    const std::string key = scale_key(model, K, updates, c0, c->nranks, c);
    if (c->ex_scale_key == key) return SMORE_OK;
    std::vector<float> sc[2];
    int rc;
    if ((rc = adaptive_scales(c, model, K, updates, c0, c->nranks, sc))) return rc;
    return upload_scales(c, sc, key);
}

// ---------------------------------------------------------------- one process, N GPUs
int smore_group_create(const int* devices, int n, smore_group** out) {
    if (!out || !devices || n < 1 || n > 64) return SMORE_EINVAL;
    *out = nullptr;
    // all replicas on one device (a repeated id): local collectives, no RCCL;
    // otherwise every device must be distinct (one RCCL rank per GPU)
    bool local = n > 1, distinct = true;
    for (int r = 1; r < n; ++r) local = local && devices[r] == devices[0];
    for (int r = 0; r < n; ++r)
        for (int q = 0; q < r; ++q) distinct = distinct && devices[q] != devices[r];
    if (n > 1 && !local && !distinct) return SMORE_EINVAL;
    smore_group* g = new smore_group();
    for (int r = 0; r < n; ++r) {
        smore_ctx* c = nullptr;
        const int rc = smore_create(devices[r], &c);
        if (rc) {
            smore_group_destroy(g);
            return rc;
        }
        g->ctx.push_back(c);
    }
    if (local) {
        g->local = true;
        g->lev.assign((size_t)n, nullptr);
        bool ok = hipSetDevice(devices[0]) == hipSuccess &&
                  hipEventCreateWithFlags(&g->ldone, hipEventDisableTiming) == hipSuccess;
        for (int r = 0; r < n && ok; ++r) ok = hipEventCreateWithFlags(&g->lev[r], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            smore_group_destroy(g);
            return SMORE_EHIP;
        }
        for (int r = 0; r < n; ++r) {
            g->ctx[r]->comm = g;   // non-null: the exchange buffers are usable; never passed to RCCL
            g->ctx[r]->own_comm = false;
            g->ctx[r]->local_comm = true;
            g->ctx[r]->nranks = n;
            g->ctx[r]->rank = r;
        }
    } else if (n > 1) {
        Rccl* L = rccl();
        if (!L) {
            smore_group_destroy(g);
            return SMORE_EHIP;
        }
        g->comms.assign((size_t)n, nullptr);
        if (L->init_all(g->comms.data(), n, devices) != ncclSuccess) {
            g->comms.clear();
            smore_group_destroy(g);
            return SMORE_EHIP;
        }
        for (int r = 0; r < n; ++r) {
            g->ctx[r]->comm = g->comms[r];
            g->ctx[r]->own_comm = false;
            g->ctx[r]->nranks = n;
            g->ctx[r]->rank = r;
        }
    }
    *out = g;
    return SMORE_OK;
}

void smore_group_destroy(smore_group* g) {
    if (!g) return;
    for (smore_ctx* c : g->ctx) {
        smore_exchange_release(c);
        smore_destroy(c);
    }
    if (!g->comms.empty()) comm_release(rccl(), g->comms.data(), (int)g->comms.size());
    for (hipEvent_t e : g->lev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->bdone)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->brecv)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->hready)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->hdone)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->lser)
        if (e) (void)hipEventDestroy(e);
    if (g->ldone) (void)hipEventDestroy(g->ldone);
    delete g;
}

int smore_group_size(const smore_group* g) { return g ? (int)g->ctx.size() : 0; }

int smore_group_set_adaptive(smore_group* g, double c0) {
    if (!g || !(c0 > 0.0 || c0 == -1.0)) return SMORE_EINVAL;
    g->c0 = c0;
    return SMORE_OK;
}

int smore_group_set_partition(smore_group* g, int on) {
    if (!g) return SMORE_EINVAL;
    g->partition = on != 0;
    return SMORE_OK;
}

int smore_group_set_walk_partition(smore_group* g, int on) {
    if (!g) return SMORE_EINVAL;
    g->walk_partition = on != 0;
    return SMORE_OK;
}

int smore_group_set_schedule(smore_group* g, int schedule) {
    if (!g || (schedule != SMORE_SCHED_REPLICAS && schedule != SMORE_SCHED_BLOCKS)) return SMORE_EINVAL;
    g->schedule = schedule;
    return SMORE_OK;
}

int smore_group_set_hot_exchange(smore_group* g, int64_t rows, int launches) {
    if (!g || launches < 1) return SMORE_EINVAL;
    g->hot_rows = rows < 0 ? -1 : rows;
    g->launches = launches;
    return SMORE_OK;
}

smore_ctx* smore_group_ctx(smore_group* g, int rank) {
    if (!g || rank < 0 || rank >= (int)g->ctx.size()) return nullptr;
    return g->ctx[rank];
}

const char* smore_group_last_error(const smore_group* g) { return g ? g->err.c_str() : "null group"; }

int smore_group_load_edgelist(smore_group* g, const char* path, int undirected, int vm, int nm) {
    if (!g) return SMORE_EINVAL;
    int rc = smore_load_edgelist(g->ctx[0], path, undirected, vm, nm);
    if (rc) return gfail(g, 0, rc);
    return replicate_graph(g);
}

int smore_group_set_graph_edges(smore_group* g, int64_t V, int64_t E, const int32_t* src, const int32_t* dst,
                                const double* w, int vm, int nm) {
    if (!g) return SMORE_EINVAL;
    int rc = smore_set_graph_edges(g->ctx[0], V, E, src, dst, w, vm, nm);
    if (rc) return gfail(g, 0, rc);
    return replicate_graph(g);
}

int smore_group_set_semantics(smore_group* g, int semantics) {
    if (!g) return SMORE_EINVAL;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        // the host tables are shared: replica 0 rebuilds them, the builders are
        // idempotent, every replica uploads its own device copy
        int rc = smore_set_semantics(g->ctx[r], semantics);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int smore_group_set_alias(smore_group* g, int which, const double* prob, const int64_t* alias, int64_t n) {
    if (!g) return SMORE_EINVAL;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        int rc = smore_set_alias(g->ctx[r], which, prob, alias, n);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int smore_group_set_node_types(smore_group* g, const int32_t* node_type, int ntypes) {
    if (!g) return SMORE_EINVAL;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        int rc = smore_set_node_types(g->ctx[r], node_type, ntypes);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int smore_group_set_temporal_edges(smore_group* g, int64_t E, const int32_t* src, const int32_t* dst,
                                   const double* ts) {
    if (!g) return SMORE_EINVAL;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        int rc = smore_set_temporal_edges(g->ctx[r], E, src, dst, ts);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int smore_group_alloc_tables(smore_group* g, int dim, int ntables) {
    if (!g) return SMORE_EINVAL;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        int rc = smore_alloc_tables(g->ctx[r], dim, ntables);
        if (rc) return gfail(g, (int)r, rc);
    }
    return SMORE_OK;
}

int smore_group_broadcast_tables(smore_group* g) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1) return SMORE_OK;
    int rc;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        smore_ctx* c = g->ctx[r];
        if (c->ntables < 1 || !c->d_table[0]) return gfail(g, (int)r, fail(c, SMORE_ESTATE, "tables not allocated"));
        if ((rc = smore_synchronize(c))) return gfail(g, (int)r, rc);
    }
    const size_t n = table_floats(g->ctx[0]);
    const std::vector<hipStream_t> st = compute_streams(g);
    for (int t = 0; t < g->ctx[0]->ntables; ++t) {
        std::vector<float*> buf;
        for (smore_ctx* c : g->ctx) buf.push_back(c->d_table[t]);
        if ((rc = coll_broadcast(g, buf, n, 0, st, "ncclBroadcast"))) return rc;
    }
    return group_sync(g);
}

int smore_group_train_edges(smore_group* g, int model, uint64_t begin, uint64_t count, uint64_t total, int K,
                            double alpha0, double reg, uint64_t seed, int mode, uint64_t sync_samples, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_edges(g->ctx[0], model, begin, count, total, K, alpha0, reg, seed, mode));
    if (blocks_for(g) && model == SMORE_LINE2)
        return group_block_edges(g, begin, count, sync_samples, total, K, alpha0, seed, mode);
    return group_rounds(g, begin, begin + count, sync_samples, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_edges_async(c, model, b, e - b, total, K, alpha0, reg, seed, mode);
                        },
                        model, K, 1.0, model == SMORE_LINE2);
}

int smore_group_train_deepwalk(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, uint64_t seed, const int64_t* order,
                               int mode, uint64_t sync_walks, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_deepwalk(g->ctx[0], walk_begin, walk_end, walk_times, walk_steps, window, K,
                                                alpha0, seed, order, mode));
    if (blocks_for(g))
        return group_block_walks(g, 0, walk_begin, walk_end, walk_times, walk_steps, window, 0, K, alpha0, seed, order,
                                 mode, sync_walks);
    return group_rounds(g, walk_begin, walk_end, sync_walks, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_deepwalk_async(c, b, e, walk_times, walk_steps, window, K, alpha0,
                                                              seed, order, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("deepwalk", {(double)walk_times, (double)walk_steps, (double)window, (double)K, (double)seed}), true);
}

int smore_group_train_node2vec(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, double p, double q, uint64_t seed,
                               const int64_t* order, int mode, uint64_t sync_walks, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_node2vec(g->ctx[0], walk_begin, walk_end, walk_times, walk_steps, window, K,
                                                alpha0, p, q, seed, order, mode));
    return group_rounds(g, walk_begin, walk_end, sync_walks, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_node2vec_async(c, b, e, walk_times, walk_steps, window, K, alpha0, p,
                                                              q, seed, order, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("node2vec", {(double)walk_times, (double)walk_steps, (double)window, (double)K, p, q, (double)seed}), true);
}

int smore_group_train_metapath2vec(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                                   int walk_steps, int window, int K, double alpha0, const int32_t* paths,
                                   const int32_t* path_lens, int npaths, uint64_t seed, const int64_t* order,
                                   int mode, uint64_t sync_walks, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_metapath2vec(g->ctx[0], walk_begin, walk_end, walk_times, walk_steps, window,
                                                    K, alpha0, paths, path_lens, npaths, seed, order, mode));
    return group_rounds(g, walk_begin, walk_end, sync_walks, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_metapath2vec_async(c, b, e, walk_times, walk_steps, window, K,
                                                                  alpha0, paths, path_lens, npaths, seed, order,
                                                                  mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("metapath2vec", {(double)walk_times, (double)walk_steps, (double)window, (double)K, (double)npaths, (double)seed}), true);
}

int smore_group_train_ctdne(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                            int window, int K, double alpha0, double time_window, uint64_t seed,
                            const int64_t* order, int mode, uint64_t sync_walks, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_ctdne(g->ctx[0], walk_begin, walk_end, walk_times, walk_steps, window, K,
                                             alpha0, time_window, seed, order, mode));
    return group_rounds(g, walk_begin, walk_end, sync_walks, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_ctdne_async(c, b, e, walk_times, walk_steps, window, K, alpha0,
                                                           time_window, seed, order, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("ctdne", {(double)walk_times, (double)walk_steps, (double)window, (double)K, time_window, (double)seed}), true);
}

int smore_group_train_walklets(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                               int window_min, int window_max, int K, double alpha0, uint64_t seed, int mode,
                               uint64_t sync_walks, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_walklets(g->ctx[0], walk_begin, walk_end, walk_times, walk_steps, window_min,
                                                window_max, K, alpha0, seed, mode));
    if (blocks_for(g))
        return group_block_walks(g, 1, walk_begin, walk_end, walk_times, walk_steps, window_max, window_min, K, alpha0,
                                 seed, nullptr, mode, sync_walks);
    return group_rounds(g, walk_begin, walk_end, sync_walks, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_walklets_async(c, b, e, walk_times, walk_steps, window_min,
                                                              window_max, K, alpha0, seed, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("walklets", {(double)walk_times, (double)walk_steps, (double)window_min, (double)window_max, (double)K, (double)seed}), true);
}

int smore_group_train_app(smore_group* g, uint64_t unit_begin, uint64_t unit_end, int walk_times, int sample_times,
                          double jump, int K, double alpha0, uint64_t seed, const int64_t* order, int mode,
                          uint64_t sync_units, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_app(g->ctx[0], unit_begin, unit_end, walk_times, sample_times, jump, K, alpha0,
                                           seed, order, mode));
    return group_rounds(g, unit_begin, unit_end, sync_units, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_app_async(c, b, e, walk_times, sample_times, jump, K, alpha0, seed,
                                                         order, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("app", {(double)walk_times, (double)sample_times, jump, (double)K, (double)seed}));
}

int smore_group_train_hpe(smore_group* g, uint64_t begin, uint64_t count, uint64_t total, int walk_steps, int K,
                          double reg, double alpha0, uint64_t seed, int mode, uint64_t sync_samples, int mean) {
    if (!g) return SMORE_EINVAL;
    if (g->ctx.size() == 1)
        return gfail(g, 0, smore_train_hpe(g->ctx[0], begin, count, total, walk_steps, K, reg, alpha0, seed, mode));
    return group_rounds(g, begin, begin + count, sync_samples, mean,
                        [&](smore_ctx* c, uint64_t b, uint64_t e) {
                            return smore_train_hpe_async(c, b, e - b, total, walk_steps, K, reg, alpha0, seed, mode);
                        },
                        SMORE_CENSUS, K, 1.0, false,
                        census_key("hpe", {(double)walk_steps, (double)K, (double)total, (double)seed}));
}

}  // extern "C"
