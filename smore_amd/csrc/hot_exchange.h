// hot_exchange.h -- the hub-row exchange of the multi-GPU replicas (DESIGN.md
// 10): between two training launches the n rows idx[] of a table are synced
// synchronously,
//   pack   (compute stream):  P = T[idx] - S[idx];  R = P
//   all-reduce R (SUM) over RCCL on the compute stream
//   unpack (compute stream):  T[idx] += R - P;  S[idx] += R
// composing with the one-late full exchange (replica_sync.hip): the next
// begin sees only the hub rows' changes since the last unpack.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smore {
hipError_t launch_hot_pack(const float* T, const float* S, const int32_t* idx, uint64_t n, int dpad, float* P,
                           float* R, int cus, hipStream_t st);
// the delta end / cycle passes with a per-row scale (adaptive exchange):
// row i of `rows` (dpad floats each) uses scale[i]
hipError_t launch_delta_end_rows(float* T, float* S, const float* D, const float* R, const float* scale,
                                 uint64_t rows, int dpad, int cus, hipStream_t st);
hipError_t launch_delta_cycle_rows(float* T, float* S, float* D, float* R, const float* scale, uint64_t rows,
                                   int dpad, int cus, hipStream_t st);
hipError_t launch_hot_unpack(float* T, float* S, const int32_t* idx, uint64_t n, int dpad, const float* P,
                             const float* R, int cus, hipStream_t st);
// the all-reduce of a group whose replicas share one device (exchange.cpp
// local collectives): every bufs[r] (n floats, n % 4 == 0, 16-B aligned)
// becomes sum_r bufs[r], added in replica order; nrep <= LOCAL_MAX
constexpr int LOCAL_MAX = 64;
hipError_t launch_local_sum(float* const* bufs, int nrep, uint64_t n, int cus, hipStream_t st);
}  // namespace smore
