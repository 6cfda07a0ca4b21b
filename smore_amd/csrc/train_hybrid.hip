// train_hybrid.hip -- instantiations of edge_train_kernel with MODE_HYBRID
// scatter (split per mode so the build compiles them in parallel).
#include "edge_kernels.h"

namespace smore {

template <int G, int M>
static hipError_t go(const EdgeArgs& a, int grid, hipStream_t st) {
    const size_t lds = sh_lds_bytes(a.sh_rows, a.dpad);
    if (a.K <= 5) hipLaunchKernelGGL((edge_train_kernel<G, M, 5, MODE_HYBRID>), dim3(grid), dim3(256), lds, st, a);
    else if (a.K <= 10)
        hipLaunchKernelGGL((edge_train_kernel<G, M, 10, MODE_HYBRID>), dim3(grid), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((edge_train_kernel<G, M, 20, MODE_HYBRID>), dim3(grid), dim3(256), lds, st, a);
    return hipGetLastError();
}

template <int G, int M>
static const void* sym(const EdgeArgs& a) {
    if (a.K <= 5) return (const void*)edge_train_kernel<G, M, 5, MODE_HYBRID>;
    if (a.K <= 10) return (const void*)edge_train_kernel<G, M, 10, MODE_HYBRID>;
    return (const void*)edge_train_kernel<G, M, 20, MODE_HYBRID>;
}

hipError_t launch_edge_hybrid(const EdgeArgs& a, int grid, hipStream_t st) {
    const int G = lanes_of(a.dpad), M = (a.dpad + G - 1) / G;
#define X(g, m) if (G == g && M == m) return go<g, m>(a, grid, st);
    SMORE_FOR_EACH_GM(X)
#undef X
    return hipErrorInvalidValue;
}

const void* edge_symbol_hybrid(const EdgeArgs& a) {
    const int G = lanes_of(a.dpad), M = (a.dpad + G - 1) / G;
#define X(g, m) if (G == g && M == m) return sym<g, m>(a);
    SMORE_FOR_EACH_GM(X)
#undef X
    return nullptr;
}

}  // namespace smore
