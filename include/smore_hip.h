/*
 * smore_hip.h -- C ABI of the MI355X-native SMORe hot path (libsmore_hip.so).
 *
 * The drop-in boundary: plain pointers and sizes, int status codes, no torch
 * and no HIP types in the signatures.  A context owns device memory on ONE GPU;
 * N GPUs are N replicas exchanging table deltas over RCCL, driven either one
 * process per GPU (smore_comm_init / smore_exchange_*) or from one process
 * (smore_group_*).  Calls are synchronous unless named *_async; a context is
 * not thread-safe.  Host buffers are owned by the caller and copied in/out.
 *
 * Each entry point names the reference interface it replaces
 * (RainBoltz/smore paths; C++ proNet-core unless marked Go).
 * The cgo / ctypes bindings a maintainer adds are shown in INTEGRATION.md.
 */
#ifndef SMORE_HIP_H
#define SMORE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct smore_ctx smore_ctx;

/* status codes */
#define SMORE_OK 0
#define SMORE_EINVAL 1   /* bad argument (ids out of range, sizes, state)   */
#define SMORE_EHIP 2     /* HIP runtime / kernel launch failure              */
#define SMORE_ENOMEM 3   /* device or host allocation failure                */
#define SMORE_ESTATE 4   /* call out of order (no graph, no tables, ...)     */
#define SMORE_EIO 5      /* file open / parse / write failure                */

/* sampling distributions (proNet::SetVertexMethod / SetNegativeMethod,
 * src/proNet.cpp:20-25; distributions built at src/proNet.cpp:457-510) */
#define SMORE_VM_OUT_DEGREES 0
#define SMORE_VM_NO_DEGREES 1
#define SMORE_VM_DEGREES 2
#define SMORE_NM_DEGREES 0
#define SMORE_NM_IN_DEGREES 1
#define SMORE_NM_NO_DEGREES 2

/* alias tables (proNet::vertex_AT / negative_AT / context_AT, src/proNet.h:143-145) */
#define SMORE_AT_VERTEX 0
#define SMORE_AT_NEGATIVE 1
#define SMORE_AT_CONTEXT 2

/* embedding tables: W = w_vertex, C = w_context (src/model/LINE.h:22-24) */
#define SMORE_W 0
#define SMORE_C 1

/* update rules */
#define SMORE_LINE2 0   /* UpdatePair(W, C, ...)  src/proNet.cpp:1784-1809 (LINE 2nd, DeepWalk pairs) */
#define SMORE_LINE1 1   /* UpdatePair(W, W, ...)  src/model/LINE.cpp:126-157 */
#define SMORE_MF 2      /* UpdateFactorizedPair(W, W, ...) src/proNet.cpp:2591-2614 */
#define SMORE_BPR 3     /* UpdateBPRPair(W, W, ...) src/proNet.cpp:1406-1455 */

/* scatter modes for the row updates */
#define SMORE_HOGWILD 0  /* lock-free read-modify-write stores (the reference's Hogwild) */
#define SMORE_ATOMIC 1   /* read, then float atomic add of each row's delta            */
#define SMORE_SERIAL 2   /* one lane group, samples strictly in order (parity mode)    */
#define SMORE_HYBRID 3   /* atomic adds for rows hot enough to collide, stores elsewhere */

/* ---- context --------------------------------------------------------------- */
/* replaces: construction of proNet / LINE / BPR / MF / DeepWalk
 * (src/proNet.cpp:3-15, Go pronet.NewProNet pkg/pronet/pronet.go:77) */
int smore_create(int device, smore_ctx** out);
void smore_destroy(smore_ctx* ctx);
/* last error message of this context (empty string if none) */
const char* smore_last_error(const smore_ctx* ctx);
/* run on an external HIP stream (hipStream_t passed as void*); NULL = own stream */
int smore_set_stream(smore_ctx* ctx, void* hip_stream);
int smore_synchronize(smore_ctx* ctx);
/* library version string */
const char* smore_version(void);

/* ---- graph ------------------------------------------------------------------ */
/* replaces: proNet::LoadEdgeList (src/proNet.cpp:115-236; Go LoadEdgeList
 * pkg/pronet/pronet.go:112-174).  Text edge list "v1 v2 w" per line (a file
 * or a directory of files); ids in first-appearance order; undirected lines
 * add both directions.  Builds CSR + alias tables and uploads them. */
int smore_load_edgelist(smore_ctx* ctx, const char* path, int undirected,
                        int vertex_method, int negative_method);
/* loader options (new): the text is parsed by all host threads
 * (ids still in order of first appearance).  With a cache directory (this call,
 * or $SMORE_CACHE_DIR), the parsed names and edge slots are stored there under
 * a hash of the input bytes, and the built graph (CSR, degrees, alias tables)
 * under that hash and the sampling methods; later loads of the same input read
 * the built graph back (or, for other methods, the edge slots).
 * dir NULL or "" = no cache. */
int smore_set_load_cache(smore_ctx* ctx, const char* dir);
/* the last smore_load_edgelist: wall seconds of the text/cache stage, parser
 * threads, cache_hit 1 = edge slots from the cache, 2 = the built graph */
int smore_last_load_info(const smore_ctx* ctx, double* seconds, int* threads, int* cache_hit);
/* replaces: the graph half of LoadEdgeList + BuildAliasMethod
 * (src/proNet.cpp:410-542) for callers that already hold ids: E directed
 * edge slots (src[e] -> dst[e], weight w[e]) in push order. */
int smore_set_graph_edges(smore_ctx* ctx, int64_t V, int64_t E, const int32_t* src,
                          const int32_t* dst, const double* w, int vertex_method,
                          int negative_method);
/* new (multi-GPU start-up): the built graph -- CSR, degrees, the three alias
 * tables -- to a binary file and back (the edge-list loader's graph-cache
 * format), so one process of an N-GPU job builds it and the others read it;
 * smore_load_graph fails (SMORE_EIO) on another format or sampling methods. */
int smore_save_graph(const smore_ctx* ctx, const char* path);
int smore_load_graph(smore_ctx* ctx, const char* path, int vertex_method, int negative_method);
/* graph sizes (MAX_vid, MAX_line) */
int smore_graph_info(const smore_ctx* ctx, int64_t* V, int64_t* E);
/* vertex name of id (proNet::vertex_hash.keys / Go GetVertexName
 * pkg/pronet/pronet.go:336); NULL when the graph was given by ids */
const char* smore_vertex_name(const smore_ctx* ctx, int64_t vid);
/* host copies of the CSR (offsets: V+1, targets: E) */
int smore_get_csr(const smore_ctx* ctx, int64_t* offsets, int32_t* targets);
/* replaces: direct assignment of proNet::*_AT / Go ProNet.NegativeAT
 * (internal/models/ctdne/ctdne.go:109-122).  prob/alias in the reference's
 * representation (alias -1 = none); for SMORE_AT_CONTEXT, n == E and alias
 * holds target vids.  Re-encodes and re-uploads the table. */
int smore_set_alias(smore_ctx* ctx, int which, const double* prob, const int64_t* alias,
                    int64_t n);
/* reference-representation copy of an alias table (prob, alias; n entries) */
int smore_get_alias(const smore_ctx* ctx, int which, double* prob, int64_t* alias, int64_t n);
/* device-encoded copy: accept threshold (u32) + alias id (i32) per entry */
int smore_get_alias_encoded(const smore_ctx* ctx, int which, uint32_t* thresh, int32_t* alias,
                            int64_t n);

/* ---- embedding tables ---------------------------------------------------------- */
/* allocate W (and C when ntables == 2) as [V][dpad] fp32, dpad = dim rounded up
 * to a multiple of 4 (rows 16-byte aligned); 1 <= dim <= 512.  Tables start zeroed. */
int smore_alloc_tables(smore_ctx* ctx, int dim, int ntables);
/* replaces: the rand() initialisation in LINE/MF/BPR/DeepWalk::Init
 * (src/model/LINE.cpp:83, MF.cpp:50, BPR.cpp:49, DeepWalk.cpp:47,54):
 * table[v][d] = (rand()/RAND_MAX - 0.5)/dim with glibc rand() seeded by srand(1),
 * skipping the first `skip` draws (so W then C reproduce the reference order). */
int smore_init_table_glibc(smore_ctx* ctx, int which, uint64_t skip);
/* on-device init (Philox stream 2): (u - 0.5)/dim, u uniform in [0,1) */
int smore_init_table_uniform(smore_ctx* ctx, int which, uint64_t seed);
int smore_zero_table(smore_ctx* ctx, int which);
/* host <-> device copies, host rows unpadded [rows][dim] */
int smore_set_table(smore_ctx* ctx, int which, const float* host, int64_t rows, int dim);
int smore_get_table(const smore_ctx* ctx, int which, float* host, int64_t rows, int dim);
/* device pointer + padded row stride (floats) of a table, for collectives */
int smore_table_device(smore_ctx* ctx, int which, void** dptr, int64_t* stride);

/* ---- benchmark inputs (not a reference interface) ------------------- */
/* Seeded power-law edge list: both endpoints of each of `lines` records ~ Zipf(s)
 * over V ranks, ranks mapped through a seeded permutation, weight 1.  Undirected:
 * slots 2l, 2l+1 = (a,b), (b,a) (the loaders' push order); src/dst hold
 * lines*(undirected ? 2 : 1) ids.  Independent of the host thread count. */
int smore_gen_powerlaw(int64_t V, int64_t lines, int undirected, double s, uint64_t seed, int32_t* src,
                       int32_t* dst);

/* semantics of the sampling and update rules (SURVEY.md 8a "C++ vs Go"):
 * SMORE_SEM_CPP (default) = src/proNet.cpp; SMORE_SEM_GO = pkg/pronet +
 * internal/models: source alias out_degree^1, negatives (in+out)^0.75 with the Go
 * alias rule, CDF target draws, Go UpdatePair (skip duplicate negatives,
 * deferred positive context), Go updateFirstOrder (LINE1), Go UpdateBPRPair
 * (BPR: W users, C items, 1 negative, reg = lambda), Go DeepWalk (dead-end
 * stop, fixed window).  Rebuilds the vertex/negative tables in place.
 * (replaces the choice of binary: cli/ C++ vs cmd/ Go) */
#define SMORE_SEM_CPP 0
#define SMORE_SEM_GO 1
int smore_set_semantics(smore_ctx* ctx, int semantics);

/* ---- training -------------------------------------------------------------------- */
/* replaces: the hot loops of LINE::Train (src/model/LINE.cpp:160-191),
 * MF::Train (src/model/MF.cpp:78-101), BPR::Train (src/model/BPR.cpp:77-101);
 * Go (*LINE).Train internal/models/line/line.go:73-150.
 * Runs global samples [begin, begin+count) of a run of `total` samples
 * (learning-rate schedule of the reference from the global sample index).
 * model: SMORE_LINE2 | SMORE_LINE1 | SMORE_MF | SMORE_BPR; K negatives
 * (BPR: fixed 5 rounds, K ignored as in the reference); reg: MF only.
 * mode: SMORE_HOGWILD | SMORE_ATOMIC | SMORE_HYBRID | SMORE_SERIAL.  Asynchronous on the
 * context stream; *_sync waits and reports launch errors. */
int smore_train_edges_async(smore_ctx* ctx, int model, uint64_t begin, uint64_t count,
                            uint64_t total, int K, double alpha0, double reg, uint64_t seed,
                            int mode);
int smore_train_edges(smore_ctx* ctx, int model, uint64_t begin, uint64_t count,
                      uint64_t total, int K, double alpha0, double reg, uint64_t seed,
                      int mode);
/* SMORE_HYBRID: a row takes float atomics when (resident sample groups) x
 * (its per-sample touch probability) > tau; tau < 0 (the default) = 1.0 for the
 * C++ rules' edge-record models (LINE, MF, BPR), 0.3 for the Go rules and the
 * pair-record models (DeepWalk, Walklets, APP, HPE, the Go walks); DESIGN.md 8 */
int smore_set_hot_threshold(smore_ctx* ctx, double tau);
/* rows marked hot in W and C by the last hybrid launch */
/* hybrid scatter: the `rows` hottest hot context rows (default 128; 0 = off; at
 * most 8192/dim) are write-combined per workgroup in LDS and drained to HBM every
 * `flush_rounds` rounds of a wave's loop -- bounded extra staleness on those rows
 * only (rows whose expected updates per flush window exceed 65536 stay on
 * atomics), in exchange for not serialising every sample's atomic adds on the
 * same few HBM lines.  flush_rounds 0 (default) = automatic: 8..32 rounds, fewer
 * the hotter the hottest combined row (same expected staleness as config 4 at 32). */
int smore_set_write_combine(smore_ctx* ctx, int rows, int flush_rounds);
/* the combined rows and the drain interval the last hybrid launch used */
int smore_write_combine_info(const smore_ctx* ctx, int* rows, int* flush_rounds);
int smore_hot_rows(const smore_ctx* ctx, int64_t* hot_w, int64_t* hot_c);
/* multi-GPU: the n rows of table `which` (0 = W, 1 = C) with
 * the highest expected touches per sample of `model` with K negatives (the
 * sampler marginals of the context's graph), highest first: the hub rows the
 * replica exchange also syncs after every launch (smore_hot_exchange) */
int smore_hot_row_ids(smore_ctx* ctx, int model, int K, int which, int64_t n, int32_t* ids);
/* samples whose source had no out-edge (reference: TargetSample -> -1) */
int smore_skipped(smore_ctx* ctx, uint64_t* skipped);
/* milliseconds of the last training launch (HIP events on the launch stream) */
float smore_last_kernel_ms(const smore_ctx* ctx);
/* the scatter the last training call actually ran (SMORE_HOGWILD / _ATOMIC /
 * _SERIAL / _HYBRID; -1 before any): a call asked for SMORE_HYBRID may run
 * another (C++ BPR above the small-graph cap runs the plain-store kernel) */
int smore_last_mode(const smore_ctx* ctx);
/* measurement (SURVEY.md 8d "the measured copy bandwidth on the box"): the
 * best (read + written bytes) / time of `reps` float4 device-to-device copies of
 * `bytes` over a few cache policies and grid sizes, in GB/s.  Allocates and
 * frees its own buffers; the context's tables and graph are untouched. */
int smore_copy_bandwidth(smore_ctx* ctx, uint64_t bytes, int reps, double* gbs);
/* the last LINE/MF edge call split by phase (HIP events on the context stream):
 * update_ms = total time of its `launches` update-kernel launches (gather/update/
 * scatter), draw_ms = time the context stream waited for draw kernels
 * (train_draw.hip) that did not overlap an update (the draws of chunk k+1 run on
 * a second stream during the update of chunk k); SMORE_ESTATE if the last call
 * was not an edge call */
int smore_last_phase_ms(const smore_ctx* ctx, float* draw_ms, float* update_ms, int* launches);

/* ---- multi-GPU replica exchange (new: the reference is single-process Hogwild,
 * src/model/LINE.cpp:162) -------------------------------------------
 * Fused passes around an all-reduce of R, on the context stream, over n floats
 * of device memory laid out like a table (n % 4 == 0, 16-byte aligned):
 *   begin:  D = T - S;  R = D;  S = T          (this rank's delta since the last exchange)
 *   end:    X = scale*R - D;  T += X;  S += X  (R = sum over ranks; scale 1 or 1/world)
 * Driven by smore_amd/dist.py (RCCL all-reduce overlapping the next step). */
int smore_delta_begin(smore_ctx* ctx, const void* T, void* S, void* D, void* R, int64_t n);
int smore_delta_end(smore_ctx* ctx, void* T, void* S, const void* D, const void* R, float scale, int64_t n);
/* end of one exchange fused with the begin of the next (one pass instead of two):
 * X = scale*R - D; T += X; then D = T - S (the rank's delta since the last begin),
 * R = D, S = T */
int smore_delta_cycle(smore_ctx* ctx, void* T, void* S, void* D, void* R, float scale, int64_t n);
/* the same two passes with a per-row scale: row i (`stride` floats, stride % 4
 * == 0, n = rows * stride) uses scale[i] (device, `rows` floats) -- the
 * adaptive exchange (SMORE_SYNC_ADAPTIVE below) */
int smore_delta_end_rows(smore_ctx* ctx, void* T, void* S, const void* D, const void* R, const void* scale,
                         int64_t rows, int64_t stride);
int smore_delta_cycle_rows(smore_ctx* ctx, void* T, void* S, void* D, void* R, const void* scale, int64_t rows,
                           int64_t stride);
/* Source partition of the replicas: the vertex ids cut into
 * nparts contiguous ranges of equal source mass under the current source law
 * (bounds[p] .. bounds[p + 1] - 1 is part p; bounds has nparts + 1 entries) */
int smore_source_parts(smore_ctx* ctx, int nparts, int64_t* bounds);
/* this context draws its sources from part `part` only (the source law
 * restricted and renormalised; W rows of other parts are never touched by its
 * LINE-2 samples, so replicas own disjoint W rows and exchange only C).
 * nparts 1 = the global law again.  Re-applied after smore_set_semantics /
 * smore_set_alias(SMORE_AT_VERTEX); cleared by a new graph. */
int smore_set_source_partition(smore_ctx* ctx, int nparts, int part);
/* expected touches per sample of every row of table `which` (0 = W, 1 = C)
 * under `model` with K negatives (the sampler marginals of the context's graph;
 * the ranking smore_hot_row_ids sorts by); rate[V] */
int smore_row_rates(smore_ctx* ctx, int model, int K, int which, int64_t n, double* rate);
/* (model SMORE_CENSUS: the last census's touches per unit, see smore_census_begin) */
/* Exchange rules (the `mean` argument of smore_exchange_begin and the group
 * training calls):
 *   SMORE_SYNC_SUM       scale 1: every rank's update lands once on every replica
 *   SMORE_SYNC_MEAN      scale 1/N: model averaging
 *   SMORE_SYNC_ADAPTIVE  per row: with k = the row's expected updates per
 *                        exchange over all ranks (rate * samples per exchange * N),
 *                        s = min(1, c0 / k), scale = s + (1 - s) / N -- the sum for
 *                        rows updated a few times per exchange, towards the mean for
 *                        the hub rows whose summed one-late deltas overshoot
 *                        (the default; c0 = 64, smore_group_set_adaptive) */
#define SMORE_SYNC_SUM 0
#define SMORE_SYNC_MEAN 1
#define SMORE_SYNC_ADAPTIVE 2
/* the row scales of the adaptive rule for `updates` samples of `model` per rank
 * per exchange (smore_exchange_begin with SMORE_SYNC_ADAPTIVE needs them); after
 * smore_comm_init (they depend on the world size) and smore_alloc_tables;
 * model SMORE_CENSUS: the census rates, `updates` = units per rank per exchange.
 * SMORE_ESTATE while an exchange is in flight (call smore_exchange_end first). */
int smore_exchange_set_adaptive(smore_ctx* ctx, int model, int K, double updates, double c0);

/* ---- multi-GPU replicas over RCCL, in the library (smore_amd/csrc/exchange.cpp) ------
 * replaces: the fan-out of one training run over the reference's workers
 * (LINE::Train `#pragma omp parallel for`, src/model/LINE.cpp:162; MF.cpp /
 * BPR.cpp / DeepWalk.cpp Train likewise; Go goroutines per worker,
 * internal/models/line/line.go:96-146) -- here across GPUs.  Every GPU holds a
 * replica of graph and tables and trains a disjoint range of global sample
 * indices; the replicas exchange table deltas (all-reduce over xGMI), one
 * exchange late, overlapping the next step:
 *   begin: D = T - S; R = D; S = T; all-reduce(R) on the exchange stream
 *   end:   X = scale*R - D; T += X; S += X          (scale 1, or 1/nranks if mean)
 * One process per GPU: every rank calls smore_comm_init with the same id (made
 * by one rank with smore_comm_unique_id and shared out of band), then after the
 * tables are initialised smore_exchange_reset (S = T), after each training step
 * smore_exchange_begin (an in-flight exchange is folded in first), and at the
 * end smore_exchange_end.  RCCL is loaded on first use (librccl.so.1). */
#define SMORE_COMM_ID_BYTES 128
int smore_comm_unique_id(unsigned char* id /* SMORE_COMM_ID_BYTES */);
int smore_comm_init(smore_ctx* ctx, int nranks, int rank, const unsigned char* id);
int smore_exchange_reset(smore_ctx* ctx);
int smore_exchange_begin(smore_ctx* ctx, int mean /* SMORE_SYNC_* */);
int smore_exchange_end(smore_ctx* ctx);
/* RCCL failure detection (new -- the reference has no failure
 * path): where the host waits on work behind a collective -- smore_synchronize
 * of a context with its own communicator, the end of every group call over
 * RCCL -- it polls ncclCommGetAsyncError between completion checks and bounds
 * the wait (`seconds`; -1 = the default, $SMORE_COMM_TIMEOUT or 1800 s).  On an
 * asynchronous error, a failed stream or the deadline the communicators are
 * aborted (ncclCommAbort) and the call returns SMORE_EHIP with the reason in
 * smore_last_error / smore_group_last_error.  No in-process restart. */
int smore_set_comm_timeout(double seconds);

/* One process driving N GPUs (`smore_create(dev_ids, n_dev)` with
 * internal fan-out): a group of N contexts with one communicator each
 * (ncclCommInitAll).  Replica 0 is the primary: graph / table / save calls that
 * are not group calls go to smore_group_ctx(g, 0); smore_group_broadcast_tables
 * then copies its tables to every replica.  Group training splits the global
 * sample (walk) range in rounds: in round k replica r runs
 * [begin + (k*N + r)*per, +per), then all replicas exchange; the last exchange
 * completes before the call returns, when all replicas agree (float rounding). */
typedef struct smore_group smore_group;
int smore_group_create(const int* devices, int n, smore_group** out);
void smore_group_destroy(smore_group* g);
int smore_group_size(const smore_group* g);
/* the hub-row exchange of the sum exchange: each replica's
 * share of an exchange round runs as `launches` training launches, and after
 * each the `rows` hub rows per table (smore_hot_row_ids) are all-reduced
 * synchronously.  rows -1 = automatic (min(65536, V/8), the default), 0 = off
 * (then one launch per round); launches >= 1 (default 8). */
int smore_group_set_hot_exchange(smore_group* g, int64_t rows, int launches);
/* c0 of the adaptive exchange (-1 = default: 2048 with the source partition,
 * 64 without) */
int smore_group_set_adaptive(smore_group* g, double c0);
/* LINE-2 group training partitions the W rows by source (default on): replica
 * r draws its sources from part r (smore_set_source_partition, left set after
 * the call), only C is exchanged, and the W parts are broadcast from their
 * owners before the call returns. */
int smore_group_set_partition(smore_group* g, int on);
/* the walk models (DeepWalk, Walklets, node2vec, metapath2vec, CTDNE) with
 * W partitioned by walk center (default off: measured worse than replicated
 * tables): every replica runs every walk of a round and trains
 * the pairs whose center it owns (smore_walk_parts of the call's first-round
 * census, smore_set_walk_owner; reset after the call), only C is exchanged, W
 * is gathered from the owners.  APP and HPE always replicate both tables. */
int smore_group_set_walk_partition(smore_group* g, int on);
/* The multi-GPU schedule of LINE-2, DeepWalk and Walklets (C++ rules):
 *   SMORE_SCHED_REPLICAS  replicated tables, deltas exchanged (the rules above);
 *   SMORE_SCHED_BLOCKS    the 2-D block schedule (smore_block_setup below): no
 *                         row is replicated while it trains, C blocks rotate
 *                         between the replicas (ncclSend / ncclRecv), nothing is
 *                         all-reduced.  `per` of the training calls = samples
 *                         (walks) per replica per epoch (nb sub-rounds); 0 = the
 *                         default.  The other models keep the replicas.
 * Default: SMORE_SCHED_BLOCKS. */
#define SMORE_SCHED_REPLICAS 0
#define SMORE_SCHED_BLOCKS 1
int smore_group_set_schedule(smore_group* g, int schedule);
smore_ctx* smore_group_ctx(smore_group* g, int rank);
const char* smore_group_last_error(const smore_group* g);
int smore_group_load_edgelist(smore_group* g, const char* path, int undirected, int vertex_method,
                              int negative_method);
int smore_group_set_graph_edges(smore_group* g, int64_t V, int64_t E, const int32_t* src, const int32_t* dst,
                                const double* w, int vertex_method, int negative_method);
int smore_group_set_semantics(smore_group* g, int semantics);
/* per-replica copies of smore_set_alias / smore_set_node_types / smore_set_temporal_edges */
int smore_group_set_alias(smore_group* g, int which, const double* prob, const int64_t* alias, int64_t n);
int smore_group_set_node_types(smore_group* g, const int32_t* node_type, int ntypes);
int smore_group_set_temporal_edges(smore_group* g, int64_t E, const int32_t* src, const int32_t* dst,
                                   const double* ts);
int smore_group_alloc_tables(smore_group* g, int dim, int ntables);
int smore_group_broadcast_tables(smore_group* g);
/* per = samples per replica per exchange (0: the default, 6.71 x V clamped to
 * [2^12, 2^27]: 6.7 samples per row per replica per exchange); mean = SMORE_SYNC_* */
int smore_group_train_edges(smore_group* g, int model, uint64_t begin, uint64_t count, uint64_t total, int K,
                            double alpha0, double reg, uint64_t seed, int mode, uint64_t per, int mean);
/* per = walks per replica per exchange (0: the default, 4 pair updates per row
 * per replica per exchange: 4 V / the pairs per walk of the call's row census) */
int smore_group_train_deepwalk(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, uint64_t seed,
                               const int64_t* order, int mode, uint64_t per, int mean);
/* per = walks / APP units / HPE samples per replica per exchange (0: 4 W updates
 * per row per replica per exchange, from the call's row census) */
int smore_group_train_node2vec(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, double p, double q,
                               uint64_t seed, const int64_t* order, int mode, uint64_t per, int mean);
int smore_group_train_metapath2vec(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                                   int walk_steps, int window, int K, double alpha0, const int32_t* paths,
                                   const int32_t* path_lens, int npaths, uint64_t seed, const int64_t* order,
                                   int mode, uint64_t per, int mean);
int smore_group_train_ctdne(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                            int window, int K, double alpha0, double time_window, uint64_t seed,
                            const int64_t* order, int mode, uint64_t per, int mean);
int smore_group_train_walklets(smore_group* g, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window_min, int window_max, int K, double alpha0,
                               uint64_t seed, int mode, uint64_t per, int mean);
int smore_group_train_app(smore_group* g, uint64_t unit_begin, uint64_t unit_end, int walk_times,
                          int sample_times, double jump, int K, double alpha0, uint64_t seed,
                          const int64_t* order, int mode, uint64_t per, int mean);
int smore_group_train_hpe(smore_group* g, uint64_t begin, uint64_t count, uint64_t total, int walk_steps,
                          int K, double reg, double alpha0, uint64_t seed, int mode, uint64_t per, int mean);

/* replaces: DeepWalk::Train (src/model/DeepWalk.cpp:98-155): walks
 * [walk_begin, walk_end) of walk_times*V, start vertices order[] (host,
 * walk_times*V entries, see smore_deepwalk_order), RandomWalk + SkipGrams +
 * UpdatePairs per walk on the GPU. */
int smore_train_deepwalk(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end,
                         int walk_times, int walk_steps, int window, int K, double alpha0,
                         uint64_t seed, const int64_t* order, int mode);
/* the same, returning once the work is queued on the context stream (order[]
 * must stay valid until the context synchronizes) */
int smore_train_deepwalk_async(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end,
                               int walk_times, int walk_steps, int window, int K, double alpha0,
                               uint64_t seed, const int64_t* order, int mode);
/* replaces: (*Node2Vec).Train (Go, internal/models/node2vec/node2vec.go:178-258):
 * walks [walk_begin, walk_end) of walk_times*V from order[] (as DeepWalk),
 * biasedRandomWalk (:82-164: first step TargetSample, later steps weight *
 * 1/p back to the previous vertex, * 1 to its neighbours, * 1/q otherwise),
 * Go SkipGrams + UpdatePairs.  Go semantics only (smore_set_semantics(ctx,
 * SMORE_SEM_GO) first; SMORE_EINVAL otherwise); p, q > 0; mode serial,
 * atomic or hogwild.  Draws: stream 1, unit w: 1 slot per step, then 2K per
 * pair (as Go DeepWalk). */
int smore_train_node2vec(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                         int walk_steps, int window, int K, double alpha0, double p, double q,
                         uint64_t seed, const int64_t* order, int mode);
int smore_train_node2vec_async(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window, int K, double alpha0, double p, double q,
                               uint64_t seed, const int64_t* order, int mode);
/* replaces: pkg/hetero's typed neighbour index (hetero_graph.go:164-177
 * buildTypeIndices / NodeTypes) for metapath2vec: node_type[V] in
 * [0, ntypes) of the graph set by smore_set_graph_edges (the Go caller keeps
 * its hetero loader and passes the ids it assigned). */
int smore_set_node_types(smore_ctx* ctx, const int32_t* node_type, int ntypes);
/* replaces: (*Metapath2Vec).Train (Go, internal/models/metapath2vec/
 * metapath2vec.go:106-200): walks [walk_begin, walk_end) of walk_times*V from
 * order[], each picks one of the npaths meta-paths (type ids, paths[] holds
 * them back to back, path_lens[p] each), MetaPathWalk (pkg/hetero/
 * hetero_graph.go:221-256), Go SkipGrams + UpdatePairs.  The negative table
 * is the context's (set the Go model's uniform BuildAliasMethod(1, 0.75) with
 * smore_set_alias).  Go semantics only; smore_set_node_types first.  Draws:
 * stream 1, unit w: slot 0 the path, 1 slot per step, then 2K per pair. */
int smore_train_metapath2vec(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                             int walk_steps, int window, int K, double alpha0, const int32_t* paths,
                             const int32_t* path_lens, int npaths, uint64_t seed, const int64_t* order,
                             int mode);
int smore_train_metapath2vec_async(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                                   int walk_steps, int window, int K, double alpha0, const int32_t* paths,
                                   const int32_t* path_lens, int npaths, uint64_t seed,
                                   const int64_t* order, int mode);
/* replaces: pkg/temporal's OutEdges / GetActiveTimeRange (temporal_graph.go:
 * 60-170, 254-288) for CTDNE: E timestamped directed edges src->dst (ids of
 * the graph set by smore_set_graph_edges; the Go caller keeps its temporal
 * loader).  Out-edges are sorted by timestamp per source (stable). */
int smore_set_temporal_edges(smore_ctx* ctx, int64_t E, const int32_t* src, const int32_t* dst,
                             const double* ts);
/* replaces: (*CTDNE).Train (Go, internal/models/ctdne/ctdne.go:80-200): walks
 * [walk_begin, walk_end) of walk_times*V from order[]; a start without edges
 * trains nothing; startTime = min + Float64()*(max - min, or time_window when
 * 0); TemporalRandomWalk (temporal_graph.go:225-252, incl. its timestamp of
 * OutEdges[cur][idx]); Go SkipGrams + UpdatePairs with the context's
 * negative table (CTDNE's BuildAliasMethod(activity, 0.75) is the Go table of
 * the temporal edges given unit weights).  time_window <= 0: 0.1 x the time
 * span (ctdne.go:45-49).  Go semantics only.  Draws: stream 1, unit w: slot 0
 * the start time, 1 slot per step, then 2K per pair. */
int smore_train_ctdne(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times, int walk_steps,
                      int window, int K, double alpha0, double time_window, uint64_t seed,
                      const int64_t* order, int mode);
int smore_train_ctdne_async(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                            int walk_steps, int window, int K, double alpha0, double time_window,
                            uint64_t seed, const int64_t* order, int mode);
/* the reference's walk start order: per walk_time a Fisher-Yates shuffle with
 * glibc rand() after `skip` Init draws (src/model/DeepWalk.cpp:122-131) */
int smore_deepwalk_order(int64_t V, int walk_times, uint64_t skip, int64_t* order);

/* replaces: Walklets::Train (src/model/Walklets.cpp:24-63): walks [walk_begin,
 * walk_end) of walk_times*V, walk w starting at vertex w mod V (the reference
 * walks from vid itself), pairs of ScaleSkipGrams(walk, window_min, window_max,
 * 0) (src/proNet.cpp:928-987, its clamping included), UpdatePair per pair.
 * Draws: stream 1, unit w: the walk's 2 per step, then 2K per pair. */
int smore_train_walklets(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                         int walk_steps, int window_min, int window_max, int K, double alpha0,
                         uint64_t seed, int mode);
/* replaces: APP::Train (src/model/APP.cpp:59-120): units [unit_begin, unit_end)
 * of walk_times*V*sample_times; unit u = w*sample_times + s runs
 * JumpingRandomWalk(order[w], jump) (src/proNet.cpp:685-701) and
 * UpdatePair(order[w], walk end) with K negatives.  order[]: walk_times*V start
 * vertices (host; APP shuffles like DeepWalk: smore_deepwalk_order).  Draws:
 * stream 1, unit u: per step p, index, jump test, then 2K.  jump must be > 0
 * (the reference never ends a walk with jump 0 on a graph without dead ends);
 * a walk stops after 2^24 steps. */
int smore_train_app(smore_ctx* ctx, uint64_t unit_begin, uint64_t unit_end, int walk_times,
                    int sample_times, double jump, int K, double alpha0, uint64_t seed,
                    const int64_t* order, int mode);
/* replaces: HPE::Train (src/model/HPE.cpp:94-150): samples [begin, begin+count)
 * of total (= sample_times * 10^6): v1 = SourceSample, v2 = TargetSample(v1),
 * UpdateCommunity(v1, v2, walk_steps) (src/proNet.cpp:3018-3054, the
 * regularised Opt_SigmoidRegSGD, :1332-1351) then UpdatePair(v2, v1).  Draws:
 * stream 0, unit = sample index, consecutive slots.  alpha: count from 0
 * (src/model/HPE.cpp:133-137).  Sources without out-edges are skipped and
 * counted (smore_skipped). */
int smore_train_hpe(smore_ctx* ctx, uint64_t begin, uint64_t count, uint64_t total, int walk_steps,
                    int K, double reg, double alpha0, uint64_t seed, int mode);
/* the same three, returning once the work is queued on the context stream
 * (order[] must stay valid until the context synchronizes) */
int smore_train_walklets_async(smore_ctx* ctx, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                               int walk_steps, int window_min, int window_max, int K, double alpha0,
                               uint64_t seed, int mode);
int smore_train_app_async(smore_ctx* ctx, uint64_t unit_begin, uint64_t unit_end, int walk_times,
                          int sample_times, double jump, int K, double alpha0, uint64_t seed,
                          const int64_t* order, int mode);
int smore_train_hpe_async(smore_ctx* ctx, uint64_t begin, uint64_t count, uint64_t total, int walk_steps,
                          int K, double reg, double alpha0, uint64_t seed, int mode);

/* replaces: proNet::UpdatePairs (src/proNet.cpp:2741-2753) and Go
 * (*ProNet).UpdatePairs (pkg/pronet/optimizer.go:8-18): UpdatePair for each
 * caller-supplied pair (v[i], c[i]), i = 0 .. n-1 in order, with K <= 10
 * negatives and the fixed learning rate alpha, under the context's semantics
 * (C++: UpdatePair src/proNet.cpp:1784-1809, the context row updated in place;
 * Go: optimizer.go:21-58, negatives equal to the context skipped, the
 * context's gradient deferred).  v, c: host arrays of ids < V (copied in).
 * Draws: pair i takes its K negatives (index, then p) from stream 3, unit
 * `unit` + i / 2^20, slots 2K (i mod 2^20) + 2j, +1 -- a serial run equals
 * the reference's UpdatePairs over blocks of 2^20 pairs with the RNG spec
 * interposed.  mode as the training calls; synchronous. */
int smore_train_pairs(smore_ctx* ctx, const int32_t* v, const int32_t* c, int64_t n, int K, double alpha,
                      uint64_t seed, uint64_t unit, int mode);
/* new (the Go UpdatePairs hook, go/pkg/pronet/hip.go): a batch costs
 * O(pairs x dim) instead of O(MaxVid x dim) when only the rows it touches
 * move.  smore_pairs_rows: the sorted unique W rows (the vertices) and C rows
 * (the contexts and the K negatives smore_train_pairs will draw for this
 * batch with this seed / unit -- stream 3, computed on the host) of a batch;
 * w_ids holds n, c_ids n (K + 1) entries.  smore_set_rows / smore_get_rows:
 * rows `ids` of a table from / to a dense host buffer [n][dim]. */
int smore_pairs_rows(smore_ctx* ctx, const int32_t* v, const int32_t* c, int64_t n, int K, uint64_t seed,
                     uint64_t unit, int32_t* w_ids, int64_t* nw, int32_t* c_ids, int64_t* nc);
int smore_set_rows(smore_ctx* ctx, int which, const int32_t* ids, int64_t n, const float* rows);
int smore_get_rows(smore_ctx* ctx, int which, const int32_t* ids, int64_t n, float* rows);
/* the three in one synchronisation: W rows w_ids (nw x dim, w_rows) and C rows
 * c_ids (c_rows) up, smore_train_pairs, the same rows back into w_rows /
 * c_rows (ids from smore_pairs_rows) */
int smore_train_pairs_rows(smore_ctx* ctx, const int32_t* v, const int32_t* c, int64_t n, int K, double alpha,
                           uint64_t seed, uint64_t unit, int mode, const int32_t* w_ids, int64_t nw, float* w_rows,
                           const int32_t* c_ids, int64_t nc, float* c_rows);
/* smore_train_pairs_rows for CONCURRENT callers (the one thread-safe entry
 * point; the reference's UpdatePairs runs from `workers` goroutines,
 * internal/models/deepwalk/deepwalk.go:96-120): requests queued while the
 * context is busy are combined into one device call -- the union of their
 * rows up once (each from the earliest request holding it), the batches in
 * queue order, the union back -- and each caller gets its rows and status.
 * One caller alone: the same result as smore_train_pairs_rows.  No other call
 * may use the context meanwhile. */
int smore_train_pairs_rows_mt(smore_ctx* ctx, const int32_t* v, const int32_t* c, int64_t n, int K, double alpha,
                              uint64_t seed, uint64_t unit, int mode, const int32_t* w_ids, int64_t nw, float* w_rows,
                              const int32_t* c_ids, int64_t nc, float* c_rows);
/* device calls made by smore_train_pairs_rows_mt and the requests they served */
int smore_pairs_combine_stats(const smore_ctx* ctx, uint64_t* calls, uint64_t* requests);

/* ---- row census (the walk models' multi-GPU exchange rates) ---------------
 * Between smore_census_begin and smore_census_end the walk-model calls of this
 * context (DeepWalk, Walklets, APP, HPE, node2vec, metapath2vec, CTDNE,
 * smore_train_pairs) generate their walks and records as usual but COUNT the
 * rows each record would update -- W at its vertex, C at its context and at
 * each negative -- instead of training (the tables are untouched; edge models
 * have exact marginals and are rejected).  smore_census_end divides the counts
 * by `units` (the walks / APP units / HPE samples / pairs the calls covered):
 * expected row touches per unit, which smore_row_rates(ctx, SMORE_CENSUS, ...)
 * returns and smore_exchange_set_adaptive(ctx, SMORE_CENSUS, K, units per rank
 * per exchange, c0) scales by.  A new graph clears the census. */
#define SMORE_CENSUS 16
int smore_census_begin(smore_ctx* ctx);
int smore_census_end(smore_ctx* ctx, double units);

/* ---- walk partition (the walk models' multi-GPU W ownership) ---------------
 * new in this build (the reference's walk models run on one shared table:
 * DeepWalk::Train src/model/DeepWalk.cpp:128-155).  A skip-gram pair updates
 * W only at its center walk[i].  smore_set_walk_owner(ctx, lo, hi): the
 * context's DeepWalk / Walklets / node2vec / metapath2vec / CTDNE calls emit
 * only the pairs whose center is in [lo, hi) -- every pair still takes its
 * draws, so N contexts with disjoint ranges covering [0, V) that all run the
 * same walks train exactly the one-context records between them, each W row
 * on one context only.  hi < 0: every pair (the default); a new graph resets.
 * smore_walk_parts: nparts contiguous ranges of equal W-touch mass from the
 * last row census (bounds[nparts + 1], as smore_source_parts). */
int smore_set_walk_owner(smore_ctx* ctx, int64_t lo, int64_t hi);
int smore_walk_parts(smore_ctx* ctx, int nparts, int64_t* bounds);

/* ---- 2-D block schedule (one replica's side) ------------------------------
 * new in this build: SURVEY.md 8e's conflict-free multi-GPU layout for the
 * reference's one shared table pair (src/model/LINE.cpp:160-191,
 * src/model/DeepWalk.cpp:128-155).  Context `part` of `nparts` (N <= 16) owns
 * the W rows of part r (smore_block_bounds wb: N + 1 bounds of equal source
 * mass); the C table is cut into nb = 2N blocks (cb: nb + 1 bounds of equal
 * negative mass).  Sub-round s trains cell (r, b = (2r + s) mod nb) on every
 * replica; then replica r hands block b to replica r - 1 (which trains it at
 * sub-round s + 2) -- the drivers: smore_group_set_schedule, smore_amd/dist.py
 * BlockSync.  A cell draws the one-context law restricted to the cell: LINE-2
 * (v, c) from an alias table over the part's TargetSample outcomes whose
 * context is in block b, negatives from the negative law restricted to block b;
 * walk models: every replica runs every walk of a round and keeps its centers'
 * pairs, bucketed by the context's block (negatives likewise in the block).
 * model: SMORE_LINE2 or SMORE_CENSUS (the C++ walk models DeepWalk /
 * Walklets); K and mode must match the training calls.  nparts 1 = off. */
int smore_block_setup(smore_ctx* ctx, int model, int nparts, int part, int K, int mode);
int smore_block_info(const smore_ctx* ctx, int* nparts, int* part, int* nblocks);
int smore_block_bounds(const smore_ctx* ctx, int64_t* wb, int64_t* cb);
/* LINE-2: this part's sample mass per C block (nb doubles, sum 1), and
 * `samples` split over the blocks by it (largest remainder; nb counts) */
int smore_block_mass(const smore_ctx* ctx, double* mass);
int smore_block_counts(const smore_ctx* ctx, uint64_t samples, uint64_t* counts);
/* LINE-2: every part's share of the global source law (nparts doubles, sum 1):
 * a round's samples are split over the replicas by it (largest remainder), so
 * an epoch draws SourceSample's law even when the parts' masses differ */
int smore_block_part_mass(const smore_ctx* ctx, double* mass);
/* LINE-2: the weight cell (part, block) gives its negative steps (an fp32
 * value; 1 with SMORE_NEG_LAW=0): NegativeSample's share of the block over the
 * cell's share of the part's samples -- the epoch's negatives then follow
 * NegativeSample's law */
int smore_block_neg_scale(const smore_ctx* ctx, int block, double* weight);
/* LINE-2 hub C rows: the `hubs` C rows with the most expected
 * touches per sample are taken out of the rotating blocks; every cell draws
 * them (contexts and negatives, with 1/nb of their mass) on its part's own
 * copy in the C table's slot rows V .. V + H - 1, kept equal over the parts by
 * an exchange after every launch.  -1: automatic (none at 2 parts, else
 * 4096, at most V / 8nb), 0: none.  Takes effect at the next
 * smore_block_setup.  (Walk models: also the walk pairs' hub contexts.) */
int smore_block_set_hubs(smore_ctx* ctx, int64_t hubs);
/* the setup's hubs: count, the first slot row (V), their C rows and expected
 * touches per sample (each array H entries, or null) */
int smore_block_hubs(const smore_ctx* ctx, int64_t* hubs, int64_t* first_slot, int32_t* rows, double* rates);
/* slots <- hub rows (before a run's first cell) / hub rows <- slots (after its
 * last exchange), on the context stream */
int smore_block_hubs_load(smore_ctx* ctx);
int smore_block_hubs_store(smore_ctx* ctx);
/* the slots' exchange scales for `samples` per part per exchange and c0 (the
 * adaptive rule of SMORE_SYNC_ADAPTIVE over the nparts parts; H floats) */
int smore_block_hub_scales(const smore_ctx* ctx, double samples, double c0, float* scales);
/* launches per cell of the setup (4 with hub slots, else 1;
 * $SMORE_CELL_LAUNCHES overrides): a cell's samples are trained in this many
 * consecutive launches with the hub slots exchanged after each */
int smore_block_cell_launches(const smore_ctx* ctx);
/* LINE-2: samples [begin, begin + count) (Philox units; LINE's learning rate
 * from the global index as smore_train_edges) drawn from cell (part, block) and
 * trained, asynchronously on the context stream */
int smore_block_train_edges_async(smore_ctx* ctx, int block, uint64_t begin, uint64_t count, uint64_t total, int K,
                                  double alpha0, uint64_t seed, int mode);
/* the draws of a cell: out count x (2 + K) {v, c, n1..nK} (parity tests) */
int smore_block_sample_edges(smore_ctx* ctx, int block, uint64_t seed, uint64_t begin, uint64_t count, int K,
                             int32_t* out);
/* walk models: a round of walks [walk_begin, walk_end) (<= 2^18; rule 0
 * DeepWalk with its start order, 1 Walklets with window_min) -> this part's
 * pair records bucketed by block; then smore_block_train_walks_async per
 * block; smore_block_walk_records: a bucket's record count (synchronises) */
int smore_block_prepare_walks(smore_ctx* ctx, int rule, uint64_t walk_begin, uint64_t walk_end, int walk_times,
                              int walk_steps, int window, int window_min, int K, double alpha0, uint64_t seed,
                              const int64_t* order, uint64_t order_base, int mode);
/* the same round in two steps, for walk-partitioned generation (the group
 * driver's default): smore_block_walks_generate walks only [gen_lo, gen_hi)
 * of the round [walk_begin, walk_end) into the context's round buffer
 * (smore_block_walks_buffer: device pointers of the walks, int32 [walks][stride],
 * and their lengths, int32 [walks]); the host fills in the other parts' walks
 * (each part walks 1/N, then every slice is broadcast from its walker), then
 * smore_block_walks_emit buckets every walk's owned pairs */
int smore_block_walks_generate(smore_ctx* ctx, int rule, uint64_t walk_begin, uint64_t walk_end, uint64_t gen_lo,
                               uint64_t gen_hi, int walk_times, int walk_steps, int window, int window_min, int K,
                               double alpha0, uint64_t seed, const int64_t* order, uint64_t order_base, int mode);
int smore_block_walks_buffer(smore_ctx* ctx, void** walks, void** lens, int64_t* stride);
int smore_block_walks_emit(smore_ctx* ctx);
int smore_block_train_walks_async(smore_ctx* ctx, int block);
/* one part of the bucket: records [n part / parts, n (part + 1) / parts) of
 * its n (the group's launches per cell, the hub slots exchanged after each) */
int smore_block_train_walks_part_async(smore_ctx* ctx, int block, int part, int parts);
int smore_block_walk_records(smore_ctx* ctx, int block, uint64_t* n);
/* a bucket's records to the host (parity tests): *n records of *width int32
 * each -- W id | tag, C id | tag, the K negatives (-1 padded), alpha's bits;
 * out may be NULL (count and width only), else it holds cap records */
int smore_block_walk_records_copy(smore_ctx* ctx, int block, int32_t* out, uint64_t cap, uint64_t* n, int* width);

/* ---- samplers (parity tests) -------------------------------------------------------- */
/* replaces: SourceSample/TargetSample/NegativeSample (src/proNet.cpp:623-683):
 * draws of samples [begin, begin+count) as the training kernels draw them.
 * out: count x (2+K) int32 {v, c, n1..nK} (model != BPR) or count x 7 {u,i,j0..j4};
 * Go semantics: count x (2+K), BPR count x 3 {u, i, j}. */
int smore_sample_edges(smore_ctx* ctx, int model, uint64_t begin, uint64_t count, int K,
                       uint64_t seed, int32_t* out);

/* ---- warm start / output --------------------------------------------------------------- */
/* replaces: proNet::LoadPreTrain (src/proNet.cpp:238-286), DeepWalk -load_v /
 * -load_c (cli/deepwalk.cpp:61-62): rows of a SaveWeights-format file whose
 * names are vertices of the loaded graph overwrite those rows of the table;
 * a file whose dimension differs is skipped, as in the reference.  A raw
 * dump (smore_save_weights fmt 2) is read by vertex id. */
int smore_load_pretrain(smore_ctx* ctx, int which, const char* path);
/* replaces: SaveWeights (src/model/LINE.cpp:13-47; Go line.go:209-233):
 * "V dim" header then "name v1 ... vdim" per vertex.  fmt 0 = C++ ostream
 * default (%g, 6 significant digits), fmt 1 = Go "%.6f"; rows are formatted by
 * all host threads ($SMORE_SAVE_THREADS), byte-identical to a sequential loop.
 * fmt 2 (new; checkpoint/resume): the raw fp32 table, "SMRAW1\0\0", int64 V,
 * int32 dim, int32 0, then V x dim floats in vertex-id order;
 * smore_load_pretrain reads it back (same V and dim, else skipped). */
int smore_save_weights(const smore_ctx* ctx, int which, const char* path, int fmt);

#ifdef __cplusplus
}
#endif
#endif
