// go_walks.h -- Go CTDNE's temporal walk (internal/models/ctdne/ctdne.go,
// pkg/temporal/temporal_graph.go): device arrays and launchers shared by the
// C ABI (capi.cpp) and train_go.hip.
#pragma once
#include "train_kernels.h"

namespace smore {

struct TemporalArgs {
    const int64_t* off;       // V + 1: per-source ranges of the time-sorted out-edges (OutEdges)
    const int32_t* tgt;       // E: targets, per source in timestamp order (stable)
    const double* ts;         // E: their timestamps
    const double* tmin;       // V: GetActiveTimeRange over out- and in-edges ({0, 0}: no edges)
    const double* tmax;       // V
    double max_time;          // tg.MaxTime
    double window;            // timeWindow
};

// walk kernel: walks of [w.walk_begin, + w.nwalks) into w.walks / w.lens
hipError_t launch_go_ctdne_walk(const TemporalArgs& t, const WalkArgs& w, uint64_t seed, hipStream_t st);
// Go SkipGrams of the walks in w.walks / w.lens as pair records (train_go.hip):
// per-walk pair counts (fixed window: a function of the length), then, at the
// exclusive-scanned offsets, the records
hipError_t launch_go_pair_count(const WalkArgs& w, uint32_t* count, hipStream_t st);
// tagged: the context and negative ids carry the C hot map's bit 30 (hybrid)
hipError_t launch_go_pair_emit(const DevGraph& g, const WalkArgs& w, uint64_t seed, int K, double alpha0,
                               const uint64_t* off, int32_t* rec, int tagged, hipStream_t st);
// Go UpdatePair over pair records (go_rec.h go_pair_kernel; train_go_rec_*.hip):
// mode 2 serial (the Go loop's order), 1 atomic, 0 plain stores, 3 hybrid
hipError_t launch_go_pair_s(const EdgeArgs& a, int grid, hipStream_t st);
hipError_t launch_go_pair_a(const EdgeArgs& a, int grid, hipStream_t st);
hipError_t launch_go_pair_h(const EdgeArgs& a, int grid, hipStream_t st);
const void* go_pair_symbol_s(const EdgeArgs& a);
const void* go_pair_symbol_a(const EdgeArgs& a);
const void* go_pair_symbol_h(const EdgeArgs& a);

}  // namespace smore
