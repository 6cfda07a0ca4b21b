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
// Go SkipGrams + UpdatePair over walks already in w.walks / w.lens
hipError_t launch_go_pairs(const EdgeArgs& a, const WalkArgs& w, int grid, hipStream_t st);

}  // namespace smore
