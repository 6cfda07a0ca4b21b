// train_bpr.hip -- instantiations of bpr_train_kernel (both scatter modes).
#include "edge_kernels.h"

namespace smore {

hipError_t launch_bpr(const EdgeArgs& a, int grid, hipStream_t st) {
    const int G = lanes_of(a.dpad), M = (a.dpad + G - 1) / G;
#define X(g, m)                                                                                        \
    if (G == g && M == m) {                                                                            \
        if (a.mode == 1) hipLaunchKernelGGL((bpr_train_kernel<g, m, MODE_ATOMIC>), dim3(grid), dim3(256), 0, st, a); \
        else if (a.mode == 3) hipLaunchKernelGGL((bpr_train_kernel<g, m, MODE_HYBRID>), dim3(grid), dim3(256), 0, st, a); \
        else hipLaunchKernelGGL((bpr_train_kernel<g, m, MODE_STORE>), dim3(grid), dim3(256), 0, st, a);  \
        return hipGetLastError();                                                                      \
    }
    SMORE_FOR_EACH_GM(X)
#undef X
    return hipErrorInvalidValue;
}

const void* bpr_symbol(const EdgeArgs& a) {
    const int G = lanes_of(a.dpad), M = (a.dpad + G - 1) / G;
#define X(g, m)                                                                            \
    if (G == g && M == m)                                                                  \
        return a.mode == 1 ? (const void*)bpr_train_kernel<g, m, MODE_ATOMIC>              \
             : a.mode == 3 ? (const void*)bpr_train_kernel<g, m, MODE_HYBRID>              \
                           : (const void*)bpr_train_kernel<g, m, MODE_STORE>;
    SMORE_FOR_EACH_GM(X)
#undef X
    return nullptr;
}

}  // namespace smore
