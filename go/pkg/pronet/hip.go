//go:build smore_hip

// hip.go -- the MI355X drop-in under the Go models' training loops.
//
// Drop this file into pkg/pronet of the Go tree (RainBoltz/smore) and build
// with `-tags smore_hip`; point cgo at this repository's header and library:
//
//	CGO_CFLAGS="-I<repo>/include" \
//	CGO_LDFLAGS="-L<repo>/smore_amd/lib -Wl,-rpath,<repo>/smore_amd/lib" \
//	go build -tags smore_hip ./cmd/line ./cmd/bpr ./cmd/deepwalk
//
// What stays Go: NewProNet, LoadEdgeList (pkg/pronet/pronet.go:77,112), the
// models' Init and SaveWeights.  (*ProNet).UpdatePairs (optimizer.go:8-18) also
// runs on the GPU under this tag (pairs_hook.go + the patch): a caller that
// builds its own pairs gets one library call per batch.  What moves to the GPU: the per-sample loops of
// (*LINE).Train (internal/models/line/line.go:73-150), (*BPR).Train
// (internal/models/bpr/bpr.go:61-135) and (*DeepWalk).Train
// (internal/models/deepwalk/deepwalk.go:61-141), i.e. SourceSample /
// TargetSample / NegativeSample (pronet.go:252-289) and UpdatePair /
// UpdateBPRPair (optimizer.go:21-117) -- one C call per training run instead
// of one Go call per sample.  The library runs them with the GO rules
// (smore_set_semantics(SMORE_SEM_GO)): source ~ out_degree^1, CDF target scan
// over the adjacency order of pn.Graph, NegativeAT from pn (so callers that
// assign their own NegativeAT keep it), duplicate negatives skipped, deferred
// positive context, BPR on W (users) and C (items) with lambda, fixed-window
// SkipGrams.  Draws come from the library's seeded Philox stream instead of
// time-seeded math/rand; tables are fp32 on the GPU.
//
// cgo may not hold Go memory that contains Go pointers, so the [][]float64
// tables are flattened into C-allocated fp32 buffers and copied back.
package pronet

/*
#cgo LDFLAGS: -lsmore_hip
#include <stdlib.h>
#include "smore_hip.h"
*/
import "C"

import (
	"fmt"
	"math/rand"
	"os"
	"strconv"
	"sync"
	"unsafe"
)

// HIP models (include/smore_hip.h)
const (
	HIPLine2 = int(C.SMORE_LINE2) // UpdatePair(W, C)       -- LINE 2nd order, DeepWalk pairs
	HIPLine1 = int(C.SMORE_LINE1) // updateFirstOrder(W)    -- LINE 1st order
	HIPBPR   = int(C.SMORE_BPR)   // UpdateBPRPair(W, C, λ) -- BPR
)

// HIP scatter modes: hybrid (the default: atomic adds for the hub rows, the
// hottest write-combined in LDS, plain stores for the rest; trains like the
// lossless atomic mode), Hogwild plain stores, float atomics, strict serial
// order (parity runs).
const (
	HIPHybrid  = int(C.SMORE_HYBRID)
	HIPHogwild = int(C.SMORE_HOGWILD)
	HIPAtomic  = int(C.SMORE_ATOMIC)
	HIPSerial  = int(C.SMORE_SERIAL)
)

// the exchange rule of the group training calls (smore_hip.h SMORE_SYNC_*)
func (h *HIP) mean() C.int {
	switch h.cfg.Sync {
	case "sum":
		return C.SMORE_SYNC_SUM
	case "mean":
		return C.SMORE_SYNC_MEAN
	}
	return C.SMORE_SYNC_ADAPTIVE
}

// HIPConfig selects the GPUs and the scatter mode of a run.
type HIPConfig struct {
	Device int    // first GPU
	GPUs   int    // replicas on Device .. Device+GPUs-1 (tables all-reduced over RCCL)
	Mode   int    // HIPHybrid unless set
	Seed   uint64 // Philox seed of the draws
	Sync   string // GPUs > 1: exchange rule, "adaptive" (default), "mean" or "sum" (diverges at >= 4 GPUs)
}

// HIPConfigFromEnv reads SMORE_HIP_DEVICE, SMORE_HIP_GPUS, SMORE_HIP_MODE
// (hybrid|atomic|hogwild|serial), SMORE_HIP_SEED and SMORE_SYNC
// (adaptive|mean|sum); defaults 0, 1, hybrid, seed, adaptive.
func HIPConfigFromEnv(seed uint64) HIPConfig {
	c := HIPConfig{Device: 0, GPUs: 1, Mode: HIPHybrid, Seed: seed}
	if v, err := strconv.Atoi(os.Getenv("SMORE_HIP_DEVICE")); err == nil {
		c.Device = v
	}
	if v, err := strconv.Atoi(os.Getenv("SMORE_HIP_GPUS")); err == nil && v > 0 {
		c.GPUs = v
	}
	switch os.Getenv("SMORE_HIP_MODE") {
	case "hogwild":
		c.Mode = HIPHogwild
	case "atomic":
		c.Mode = HIPAtomic
	case "serial":
		c.Mode = HIPSerial
	}
	c.Sync = os.Getenv("SMORE_SYNC")
	if v, err := strconv.ParseUint(os.Getenv("SMORE_HIP_SEED"), 10, 64); err == nil {
		c.Seed = v
	}
	return c
}

// HIP is one library context (or a replica group) holding pn's graph.
type HIP struct {
	group  *C.smore_group
	ctx    *C.smore_ctx // replica 0
	maxVid int64
	cfg    HIPConfig
	dim    int
	ntab   int
}

func (h *HIP) err(what string) error {
	if h.group != nil {
		return fmt.Errorf("%s: %s", what, C.GoString(C.smore_group_last_error(h.group)))
	}
	return fmt.Errorf("%s: %s", what, C.GoString(C.smore_last_error(h.ctx)))
}

// NewHIP uploads pn's graph to the GPUs of cfg in Go semantics: the directed
// edge slots of pn.Graph / pn.EdgeWeights in vertex order (the adjacency order
// TargetSample's CDF scan walks, pronet.go:257-284), then pn.NegativeAT.
func (pn *ProNet) NewHIP(cfg HIPConfig) (*HIP, error) {
	if cfg.GPUs < 1 {
		cfg.GPUs = 1
	}
	h := &HIP{maxVid: pn.MaxVid, cfg: cfg}
	devs := make([]C.int, cfg.GPUs)
	for i := range devs {
		devs[i] = C.int(cfg.Device + i)
	}
	if rc := C.smore_group_create(&devs[0], C.int(cfg.GPUs), &h.group); rc != C.SMORE_OK {
		return nil, fmt.Errorf("smore_group_create(%d GPUs from %d): status %d", cfg.GPUs, cfg.Device, int(rc))
	}
	h.ctx = C.smore_group_ctx(h.group, 0)
	E := 0
	for v := int64(0); v < pn.MaxVid; v++ {
		E += len(pn.Graph[v])
	}
	n := E
	if n == 0 {
		n = 1
	}
	src := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	dst := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	wgt := (*[1 << 40]C.double)(C.malloc(C.size_t(8 * n)))[:n:n]
	defer C.free(unsafe.Pointer(&src[0]))
	defer C.free(unsafe.Pointer(&dst[0]))
	defer C.free(unsafe.Pointer(&wgt[0]))
	e := 0
	for v := int64(0); v < pn.MaxVid; v++ {
		ws := pn.EdgeWeights[v]
		for i, t := range pn.Graph[v] {
			src[e], dst[e], wgt[e] = C.int32_t(v), C.int32_t(t), C.double(ws[i])
			e++
		}
	}
	if rc := C.smore_group_set_graph_edges(h.group, C.int64_t(pn.MaxVid), C.int64_t(E), &src[0], &dst[0], &wgt[0],
		C.SMORE_VM_OUT_DEGREES, C.SMORE_NM_DEGREES); rc != C.SMORE_OK {
		h.Close()
		return nil, h.err("smore_group_set_graph_edges")
	}
	if rc := C.smore_group_set_semantics(h.group, C.SMORE_SEM_GO); rc != C.SMORE_OK {
		h.Close()
		return nil, h.err("smore_group_set_semantics")
	}
	if int64(len(pn.NegativeAT)) == pn.MaxVid && pn.MaxVid > 0 {
		prob := (*[1 << 40]C.double)(C.malloc(C.size_t(8 * pn.MaxVid)))[:pn.MaxVid:pn.MaxVid]
		alias := (*[1 << 40]C.int64_t)(C.malloc(C.size_t(8 * pn.MaxVid)))[:pn.MaxVid:pn.MaxVid]
		defer C.free(unsafe.Pointer(&prob[0]))
		defer C.free(unsafe.Pointer(&alias[0]))
		for i, a := range pn.NegativeAT {
			prob[i], alias[i] = C.double(a.Prob), C.int64_t(a.Alias)
		}
		for r := 0; r < cfg.GPUs; r++ {
			c := C.smore_group_ctx(h.group, C.int(r))
			if rc := C.smore_set_alias(c, C.SMORE_AT_NEGATIVE, &prob[0], &alias[0], C.int64_t(pn.MaxVid)); rc != C.SMORE_OK {
				err := fmt.Errorf("smore_set_alias: %s", C.GoString(C.smore_last_error(c)))
				h.Close()
				return nil, err
			}
		}
	}
	return h, nil
}

// NewHIPEdges uploads a graph that is not a *ProNet -- the typed graph of
// pkg/hetero (metapath2vec) or the temporal graph of pkg/temporal (CTDNE) --
// as V vertices and the directed slots src[i] -> dst[i] with weights w[i] in
// adjacency order, switches to the Go rules and injects negativeAT (the table
// the Go model's Train builds with BuildAliasMethod; nil keeps the library's
// Go table of this graph).
func NewHIPEdges(V int64, src, dst []int64, w []float64, negativeAT []AliasTable, cfg HIPConfig) (*HIP, error) {
	pn := &ProNet{MaxVid: V, Graph: make(map[int64][]int64), EdgeWeights: make(map[int64][]float64)}
	for i := range src {
		pn.Graph[src[i]] = append(pn.Graph[src[i]], dst[i])
		pn.EdgeWeights[src[i]] = append(pn.EdgeWeights[src[i]], w[i])
	}
	pn.NegativeAT = negativeAT
	return pn.NewHIP(cfg)
}

// SetNodeTypes hands pkg/hetero's node types over (type ids in [0, ntypes))
// for TrainMetapath2Vec: the library groups every vertex's neighbours by type
// in adjacency order, as buildTypeIndices does (hetero_graph.go:169-183).
func (h *HIP) SetNodeTypes(types []int64, ntypes int) error {
	n := len(types)
	if int64(n) != h.maxVid || n == 0 {
		return fmt.Errorf("SetNodeTypes: %d types for %d vertices", n, h.maxVid)
	}
	t := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	defer C.free(unsafe.Pointer(&t[0]))
	for i, x := range types {
		t[i] = C.int32_t(x)
	}
	if rc := C.smore_group_set_node_types(h.group, &t[0], C.int(ntypes)); rc != C.SMORE_OK {
		return h.err("smore_group_set_node_types")
	}
	return nil
}

// SetTemporalEdges hands pkg/temporal's out-edge lists over for TrainCTDNE:
// the slots src[i] -> dst[i] at time ts[i], each source's edges in the order
// of tg.OutEdges[src] (already sorted by timestamp by the Go loader; the
// library's per-source stable sort keeps that order, ties included).
func (h *HIP) SetTemporalEdges(src, dst []int64, ts []float64) error {
	n := len(src)
	if n == 0 {
		return fmt.Errorf("SetTemporalEdges: no edges")
	}
	s := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	d := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	t := (*[1 << 40]C.double)(C.malloc(C.size_t(8 * n)))[:n:n]
	defer C.free(unsafe.Pointer(&s[0]))
	defer C.free(unsafe.Pointer(&d[0]))
	defer C.free(unsafe.Pointer(&t[0]))
	for i := 0; i < n; i++ {
		s[i], d[i], t[i] = C.int32_t(src[i]), C.int32_t(dst[i]), C.double(ts[i])
	}
	if rc := C.smore_group_set_temporal_edges(h.group, C.int64_t(n), &s[0], &d[0], &t[0]); rc != C.SMORE_OK {
		return h.err("smore_group_set_temporal_edges")
	}
	return nil
}

// Close releases the GPUs.
func (h *HIP) Close() {
	if h.group != nil {
		C.smore_group_destroy(h.group)
	}
	h.group, h.ctx = nil, nil
}

func (h *HIP) alloc(dim, ntab int) error {
	if h.dim == dim && h.ntab == ntab {
		return nil
	}
	if rc := C.smore_group_alloc_tables(h.group, C.int(dim), C.int(ntab)); rc != C.SMORE_OK {
		return h.err("smore_group_alloc_tables")
	}
	h.dim, h.ntab = dim, ntab
	return nil
}

// put copies Go tables into replica 0 (fp64 -> fp32), get copies them back.
func (h *HIP) transfer(tables [][][]float64, toGPU bool) error {
	n := int(h.maxVid) * h.dim
	if n == 0 {
		return nil
	}
	buf := (*[1 << 40]C.float)(C.malloc(C.size_t(4 * n)))[:n:n]
	defer C.free(unsafe.Pointer(&buf[0]))
	for which, t := range tables {
		if t == nil {
			continue
		}
		if toGPU {
			for v := 0; v < int(h.maxVid); v++ {
				row := t[v]
				for d := 0; d < h.dim; d++ {
					buf[v*h.dim+d] = C.float(row[d])
				}
			}
			if rc := C.smore_set_table(h.ctx, C.int(which), &buf[0], C.int64_t(h.maxVid), C.int(h.dim)); rc != C.SMORE_OK {
				return h.err("smore_set_table")
			}
		} else {
			if rc := C.smore_get_table(h.ctx, C.int(which), &buf[0], C.int64_t(h.maxVid), C.int(h.dim)); rc != C.SMORE_OK {
				return h.err("smore_get_table")
			}
			for v := 0; v < int(h.maxVid); v++ {
				row := t[v]
				for d := 0; d < h.dim; d++ {
					row[d] = float64(buf[v*h.dim+d])
				}
			}
		}
	}
	if toGPU {
		if rc := C.smore_group_broadcast_tables(h.group); rc != C.SMORE_OK {
			return h.err("smore_group_broadcast_tables")
		}
	}
	return nil
}

// hipChunk: samples per replica per library call (progress granularity)
const hipChunk = uint64(1) << 27

// TrainEdges runs samples [0, total) of an edge model (HIPLine2 on w, c;
// HIPLine1 on w; HIPBPR on w = users, c = items with lambda; K negatives, 1 for
// BPR) with the Go learning-rate schedule over `total`, and copies the trained
// tables back.  progress(done) is called between library calls.
func (h *HIP) TrainEdges(model int, w, c [][]float64, dim int, total uint64, K int, alpha, lambda float64,
	progress func(done uint64)) error {
	ntab := 2
	if model == HIPLine1 {
		ntab, c = 1, nil
	}
	if err := h.alloc(dim, ntab); err != nil {
		return err
	}
	if err := h.transfer([][][]float64{w, c}, true); err != nil {
		return err
	}
	step := hipChunk * uint64(h.cfg.GPUs)
	for done := uint64(0); done < total; {
		n := total - done
		if n > step {
			n = step
		}
		if rc := C.smore_group_train_edges(h.group, C.int(model), C.uint64_t(done), C.uint64_t(n), C.uint64_t(total),
			C.int(K), C.double(alpha), C.double(lambda), C.uint64_t(h.cfg.Seed), C.int(h.cfg.Mode), 0, h.mean()); rc != C.SMORE_OK {
			return h.err("smore_group_train_edges")
		}
		done += n
		if progress != nil {
			progress(done)
		}
	}
	return h.transfer([][][]float64{w, c}, false)
}

// trainWalks: tables up, walks [0, len(order)) in library calls of `step`
// walks per replica (progress granularity), tables back.  call runs walks
// [done, done+n) with the start order in C memory.
func (h *HIP) trainWalks(w, c [][]float64, dim int, order []int64, name string,
	call func(done, n uint64, ord *C.int64_t) C.int, progress func(done uint64)) error {
	if err := h.alloc(dim, 2); err != nil {
		return err
	}
	if err := h.transfer([][][]float64{w, c}, true); err != nil {
		return err
	}
	total := uint64(len(order))
	if total == 0 {
		return nil
	}
	ord := (*[1 << 40]C.int64_t)(C.malloc(C.size_t(8 * total)))[:total:total]
	defer C.free(unsafe.Pointer(&ord[0]))
	for i, v := range order {
		ord[i] = C.int64_t(v)
	}
	step := uint64(1<<20) * uint64(h.cfg.GPUs)
	for done := uint64(0); done < total; {
		n := total - done
		if n > step {
			n = step
		}
		if rc := call(done, n, &ord[0]); rc != C.SMORE_OK {
			return h.err(name)
		}
		done += n
		if progress != nil {
			progress(done)
		}
	}
	return h.transfer([][][]float64{w, c}, false)
}

// TrainDeepWalk runs walks [0, len(order)) of the Go DeepWalk (walk from
// order[i], dead-end stop, fixed-window SkipGrams, UpdatePair per pair) and
// copies W and C back.  order holds walkTimes x MaxVid start vertices, built
// by the caller exactly as (*DeepWalk).Train shuffles them.
func (h *HIP) TrainDeepWalk(w, c [][]float64, dim int, order []int64, walkTimes, walkSteps, window, K int,
	alpha float64, progress func(done uint64)) error {
	return h.trainWalks(w, c, dim, order, "smore_group_train_deepwalk", func(done, n uint64, ord *C.int64_t) C.int {
		return C.smore_group_train_deepwalk(h.group, C.uint64_t(done), C.uint64_t(done+n), C.int(walkTimes),
			C.int(walkSteps), C.int(window), C.int(K), C.double(alpha), C.uint64_t(h.cfg.Seed), ord,
			C.int(h.cfg.Mode), 0, h.mean())
	}, progress)
}

// TrainNode2Vec is TrainDeepWalk with node2vec's biased second-order walk
// (internal/models/node2vec/node2vec.go:82-175: 1/p back to the previous
// vertex, 1 to its neighbours, 1/q otherwise) in place of RandomWalk.
func (h *HIP) TrainNode2Vec(w, c [][]float64, dim int, order []int64, walkTimes, walkSteps, window, K int,
	alpha, p, q float64, progress func(done uint64)) error {
	return h.trainWalks(w, c, dim, order, "smore_group_train_node2vec", func(done, n uint64, ord *C.int64_t) C.int {
		return C.smore_group_train_node2vec(h.group, C.uint64_t(done), C.uint64_t(done+n), C.int(walkTimes),
			C.int(walkSteps), C.int(window), C.int(K), C.double(alpha), C.double(p), C.double(q),
			C.uint64_t(h.cfg.Seed), ord, C.int(h.cfg.Mode), 0, h.mean())
	}, progress)
}

// TrainMetapath2Vec is (*Metapath2Vec).Train's loop
// (internal/models/metapath2vec/metapath2vec.go:147-200) on the GPUs: walk i
// starts at order[i] and picks one of metaPaths (node-type ids, SetNodeTypes
// first) uniformly, MetaPathWalk (pkg/hetero/hetero_graph.go:221-256), then
// fixed-window SkipGrams and UpdatePairs.
func (h *HIP) TrainMetapath2Vec(w, c [][]float64, dim int, order []int64, metaPaths [][]int64,
	walkTimes, walkSteps, window, K int, alpha float64, progress func(done uint64)) error {
	np, tot := len(metaPaths), 0
	for _, p := range metaPaths {
		tot += len(p)
	}
	if np == 0 || tot == 0 {
		return fmt.Errorf("TrainMetapath2Vec: no meta-paths")
	}
	paths := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * tot)))[:tot:tot]
	lens := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * np)))[:np:np]
	defer C.free(unsafe.Pointer(&paths[0]))
	defer C.free(unsafe.Pointer(&lens[0]))
	k := 0
	for i, p := range metaPaths {
		lens[i] = C.int32_t(len(p))
		for _, t := range p {
			paths[k] = C.int32_t(t)
			k++
		}
	}
	return h.trainWalks(w, c, dim, order, "smore_group_train_metapath2vec", func(done, n uint64, ord *C.int64_t) C.int {
		return C.smore_group_train_metapath2vec(h.group, C.uint64_t(done), C.uint64_t(done+n), C.int(walkTimes),
			C.int(walkSteps), C.int(window), C.int(K), C.double(alpha), &paths[0], &lens[0], C.int(np),
			C.uint64_t(h.cfg.Seed), ord, C.int(h.cfg.Mode), 0, h.mean())
	}, progress)
}

// TrainCTDNE is (*CTDNE).Train's loop (internal/models/ctdne/ctdne.go:133-200)
// on the GPUs: a start without edges trains nothing, the start time is drawn in
// its active range, TemporalRandomWalk with timeWindow (pkg/temporal/
// temporal_graph.go:225-252; SetTemporalEdges first), then fixed-window
// SkipGrams and UpdatePairs.
func (h *HIP) TrainCTDNE(w, c [][]float64, dim int, order []int64, walkTimes, walkSteps, window, K int,
	alpha, timeWindow float64, progress func(done uint64)) error {
	return h.trainWalks(w, c, dim, order, "smore_group_train_ctdne", func(done, n uint64, ord *C.int64_t) C.int {
		return C.smore_group_train_ctdne(h.group, C.uint64_t(done), C.uint64_t(done+n), C.int(walkTimes),
			C.int(walkSteps), C.int(window), C.int(K), C.double(alpha), C.double(timeWindow),
			C.uint64_t(h.cfg.Seed), ord, C.int(h.cfg.Mode), 0, h.mean())
	}, progress)
}

// ---- UpdatePairs on the GPU (optimizer.go:8-18; smore_train_pairs) -----------

func init() { hipUpdatePairs = updatePairsHIP }

// one single-GPU context per *ProNet, made on the first UpdatePairs; the
// library context is not thread-safe, so batches from concurrent goroutines
// run one after another (each sees the tables the previous one wrote back)
type pairSession struct {
	once sync.Once // the context is made exactly once, before any caller uses it
	mu   sync.Mutex // guards the tables' (re)allocation only; training calls combine in the library
	h    *HIP
	err  error
}

var pairSessions sync.Map // *ProNet -> *pairSession

// pairSession returns pn's session with its context made: every goroutine,
// including ones that lost the LoadOrStore race, waits in once.Do until the
// winner's NewHIP returned, so none can see an unset h (ADVICE r4).
func (pn *ProNet) pairSession() *pairSession {
	v, _ := pairSessions.LoadOrStore(pn, &pairSession{})
	s := v.(*pairSession)
	s.once.Do(func() {
		cfg := HIPConfigFromEnv(1)
		cfg.GPUs = 1
		s.h, s.err = pn.NewHIP(cfg)
	})
	return s
}

// updatePairsHIP is (*ProNet).UpdatePairs under -tags smore_hip.  Only the
// rows the batch touches move (round 4 moved both whole tables per call, O(MaxVid
// x dim), ~180 ms per call at config 5's size): the library lists them
// (smore_pairs_rows: the vertices, the contexts and the negatives this call
// will draw, on the host), they go up fp64 -> fp32, the library runs Go
// UpdatePair for each pair in order (negatives from the rng's next word as the
// Philox unit, duplicates of the context skipped, the context's gradient
// deferred), and the same rows come back (smore_train_pairs_rows, one
// synchronisation) -- O(pairs x dim) per call.  The session's device tables
// are allocated once; rows a call does not touch are never read.  Concurrent
// goroutines do NOT take turns on a lock: each calls
// smore_train_pairs_rows_mt, which combines every batch queued while the
// device is busy into one call (the union of their rows up once, the batches
// in queue order, the union back; capi.cpp PairCombiner), so the reference's
// `workers` goroutines share one synchronisation instead of paying one each.
// UpdatePairs has no error path (the reference panics on a bad index):
// failures panic.
func updatePairsHIP(pn *ProNet, wVertex, wContext [][]float64, vertices, contexts []int64, dim,
	negativeSamples int, alpha float64, rng *rand.Rand) {
	if len(vertices) == 0 {
		return
	}
	s := pn.pairSession()
	if s.err != nil {
		panic(s.err)
	}
	s.mu.Lock()
	err := s.h.alloc(dim, 2)
	s.mu.Unlock()
	if err != nil {
		panic(err)
	}
	if err := s.h.pairsRows(wVertex, wContext, vertices, contexts, negativeSamples, alpha, rng.Uint64(),
		true); err != nil {
		panic(err)
	}
}

// PairsRows runs UpdatePair over (vertices[i], contexts[i]) in order against
// the caller's tables w (vertex) and c (context), moving only the rows the
// batch touches (smore_pairs_rows + smore_train_pairs_rows).
func (h *HIP) PairsRows(w, c [][]float64, vertices, contexts []int64, negativeSamples int, alpha float64,
	unit uint64) error {
	return h.pairsRows(w, c, vertices, contexts, negativeSamples, alpha, unit, false)
}

// pairsRows: PairsRows; concurrent = true goes through the combining entry
// point (smore_train_pairs_rows_mt), safe from several goroutines at once.
func (h *HIP) pairsRows(w, c [][]float64, vertices, contexts []int64, negativeSamples int, alpha float64,
	unit uint64, concurrent bool) error {
	n := len(vertices)
	if n != len(contexts) {
		return fmt.Errorf("PairsRows: %d vertices, %d contexts", n, len(contexts))
	}
	if n == 0 {
		return nil
	}
	K := negativeSamples
	v := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	cc := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	wi := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	ci := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n * (K + 1))))[: n*(K+1) : n*(K+1)]
	defer C.free(unsafe.Pointer(&v[0]))
	defer C.free(unsafe.Pointer(&cc[0]))
	defer C.free(unsafe.Pointer(&wi[0]))
	defer C.free(unsafe.Pointer(&ci[0]))
	for i := 0; i < n; i++ {
		// range-check before narrowing: an id >= 2^31 must not wrap to a small valid one
		if vertices[i] < 0 || vertices[i] >= h.maxVid || contexts[i] < 0 || contexts[i] >= h.maxVid {
			return fmt.Errorf("PairsRows: pair %d (%d, %d) out of range [0, %d)", i, vertices[i], contexts[i], h.maxVid)
		}
		v[i], cc[i] = C.int32_t(vertices[i]), C.int32_t(contexts[i])
	}
	var nw, nc C.int64_t
	if rc := C.smore_pairs_rows(h.ctx, &v[0], &cc[0], C.int64_t(n), C.int(K), C.uint64_t(h.cfg.Seed), C.uint64_t(unit),
		&wi[0], &nw, &ci[0], &nc); rc != C.SMORE_OK {
		return h.err("smore_pairs_rows")
	}
	d := h.dim
	wr := (*[1 << 40]C.float)(C.malloc(C.size_t(4 * int(nw) * d)))[: int(nw)*d : int(nw)*d]
	cr := (*[1 << 40]C.float)(C.malloc(C.size_t(4 * int(nc) * d)))[: int(nc)*d : int(nc)*d]
	defer C.free(unsafe.Pointer(&wr[0]))
	defer C.free(unsafe.Pointer(&cr[0]))
	gather := func(t [][]float64, ids []C.int32_t, buf []C.float) {
		for i, id := range ids {
			row := t[id]
			for k := 0; k < d; k++ {
				buf[i*d+k] = C.float(row[k])
			}
		}
	}
	scatter := func(t [][]float64, ids []C.int32_t, buf []C.float) {
		for i, id := range ids {
			row := t[id]
			for k := 0; k < d; k++ {
				row[k] = float64(buf[i*d+k])
			}
		}
	}
	gather(w, wi[:nw], wr)
	gather(c, ci[:nc], cr)
	var rc C.int
	if concurrent { // cgo calls a C function only by name: two call sites
		rc = C.smore_train_pairs_rows_mt(h.ctx, &v[0], &cc[0], C.int64_t(n), C.int(K), C.double(alpha),
			C.uint64_t(h.cfg.Seed), C.uint64_t(unit), C.int(h.cfg.Mode), &wi[0], nw, &wr[0], &ci[0], nc, &cr[0])
	} else {
		rc = C.smore_train_pairs_rows(h.ctx, &v[0], &cc[0], C.int64_t(n), C.int(K), C.double(alpha),
			C.uint64_t(h.cfg.Seed), C.uint64_t(unit), C.int(h.cfg.Mode), &wi[0], nw, &wr[0], &ci[0], nc, &cr[0])
	}
	if rc != C.SMORE_OK {
		return h.err("smore_train_pairs_rows")
	}
	scatter(w, wi[:nw], wr)
	scatter(c, ci[:nc], cr)
	return nil
}

// BeginPairs puts w (vertex) and c (context) on the GPU for Pairs calls.
func (h *HIP) BeginPairs(w, c [][]float64, dim int) error {
	if err := h.alloc(dim, 2); err != nil {
		return err
	}
	return h.transfer([][][]float64{w, c}, true)
}

// Pairs runs UpdatePair over (vertices[i], contexts[i]) in order on the
// resident tables with negativeSamples <= 10 negatives per pair from Philox
// unit `unit` (smore_train_pairs; pair i uses unit + i/2^20).
func (h *HIP) Pairs(vertices, contexts []int64, negativeSamples int, alpha float64, unit uint64) error {
	n := len(vertices)
	if n != len(contexts) {
		return fmt.Errorf("Pairs: %d vertices, %d contexts", n, len(contexts))
	}
	if n == 0 {
		return nil
	}
	v := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	c := (*[1 << 40]C.int32_t)(C.malloc(C.size_t(4 * n)))[:n:n]
	defer C.free(unsafe.Pointer(&v[0]))
	defer C.free(unsafe.Pointer(&c[0]))
	for i := 0; i < n; i++ {
		// range-check before narrowing: an id >= 2^31 must not wrap to a small valid one
		if vertices[i] < 0 || vertices[i] >= h.maxVid || contexts[i] < 0 || contexts[i] >= h.maxVid {
			return fmt.Errorf("Pairs: pair %d (%d, %d) out of range [0, %d)", i, vertices[i], contexts[i], h.maxVid)
		}
		v[i], c[i] = C.int32_t(vertices[i]), C.int32_t(contexts[i])
	}
	if rc := C.smore_train_pairs(h.ctx, &v[0], &c[0], C.int64_t(n), C.int(negativeSamples), C.double(alpha),
		C.uint64_t(h.cfg.Seed), C.uint64_t(unit), C.int(h.cfg.Mode)); rc != C.SMORE_OK {
		return h.err("smore_train_pairs")
	}
	return nil
}

// EndPairs copies the trained tables back into w and c.
func (h *HIP) EndPairs(w, c [][]float64) error {
	return h.transfer([][][]float64{w, c}, false)
}
