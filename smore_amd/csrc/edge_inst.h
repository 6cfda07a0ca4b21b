// edge_inst.h -- instantiation helper for edge_train_kernel: one translation
// unit per (scatter MODE, KMAX) (train_edge_<mode>_k<KMAX>.hip) so the build
// compiles them in parallel.  Dispatch over (G, M) and the rule (SH = 0:
// LINE-2's two tables, 1: one shared table, LINE-1 / MF, 2: BPR, KMAX 5 only).
#pragma once
#include "edge_kernels.h"

namespace smore {

template <int KMAX, int MODE>
struct EdgeInst {
    template <int G, int M, int SH>
    static hipError_t go(const EdgeArgs& a, int grid, hipStream_t st) {
        const size_t lds = MODE == MODE_HYBRID ? sh_lds_bytes(a.sh_rows, a.dpad) : 0;
        hipLaunchKernelGGL((edge_train_kernel<G, M, KMAX, MODE, SH>), dim3(grid), dim3(256), lds, st, a);
        return hipGetLastError();
    }
    static hipError_t launch(const EdgeArgs& a, int grid, hipStream_t st) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m)                                                                           \
    if (G == g && M == m) {                                                               \
        if (a.model == 3) {                                                               \
            if constexpr (KMAX == 5) return go<g, m, 2>(a, grid, st);                     \
            else return hipErrorInvalidValue;                                             \
        }                                                                                 \
        return a.model == 0 ? go<g, m, 0>(a, grid, st) : go<g, m, 1>(a, grid, st);        \
    }
        SMORE_FOR_EACH_GM(X)
#undef X
        return hipErrorInvalidValue;
    }
    static const void* symbol(const EdgeArgs& a) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m)                                                                          \
    if (G == g && M == m) {                                                              \
        if (a.model == 3) {                                                              \
            if constexpr (KMAX == 5) return (const void*)edge_train_kernel<g, m, 5, MODE, 2>; \
            else return nullptr;                                                         \
        }                                                                                \
        return a.model == 0 ? (const void*)edge_train_kernel<g, m, KMAX, MODE, 0>        \
                            : (const void*)edge_train_kernel<g, m, KMAX, MODE, 1>;       \
    }
        SMORE_FOR_EACH_GM(X)
#undef X
        return nullptr;
    }
};

// DeepWalk pair records in the Hogwild modes (pair_train_kernel)
template <int KMAX, int MODE>
struct PairInst {
    static hipError_t launch(const EdgeArgs& a, int grid, hipStream_t st) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
        const size_t lds = MODE == MODE_HYBRID ? sh_lds_bytes(a.sh_rows, a.dpad) : 0;
#define X(g, m)                                                                                      \
    if (G == g && M == m) {                                                                          \
        hipLaunchKernelGGL((pair_train_kernel<g, m, KMAX, MODE>), dim3(grid), dim3(256), lds, st, a); \
        return hipGetLastError();                                                                    \
    }
        SMORE_FOR_EACH_GM(X)
#undef X
        return hipErrorInvalidValue;
    }
    static const void* symbol(const EdgeArgs& a) {
        const int G = lanes_of(a.dpad), M = regs_of(a.dpad);
#define X(g, m) \
    if (G == g && M == m) return (const void*)pair_train_kernel<g, m, KMAX, MODE>;
        SMORE_FOR_EACH_GM(X)
#undef X
        return nullptr;
    }
};

}  // namespace smore

// defines launch_pair_<name>(a, grid, st) and pair_symbol_<name>(a)
#define SMORE_PAIR_INST(name, KMAX, MODE)                                                  \
    namespace smore {                                                                      \
    hipError_t launch_pair_##name(const EdgeArgs& a, int grid, hipStream_t st) {           \
        return PairInst<KMAX, MODE>::launch(a, grid, st);                                  \
    }                                                                                      \
    const void* pair_symbol_##name(const EdgeArgs& a) { return PairInst<KMAX, MODE>::symbol(a); } \
    }

// defines launch_edge_<name>(a, grid, st) and edge_symbol_<name>(a)
#define SMORE_EDGE_INST(name, KMAX, MODE)                                                  \
    namespace smore {                                                                      \
    hipError_t launch_edge_##name(const EdgeArgs& a, int grid, hipStream_t st) {           \
        return EdgeInst<KMAX, MODE>::launch(a, grid, st);                                  \
    }                                                                                      \
    const void* edge_symbol_##name(const EdgeArgs& a) { return EdgeInst<KMAX, MODE>::symbol(a); } \
    }
