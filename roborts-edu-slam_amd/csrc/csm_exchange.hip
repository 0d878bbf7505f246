// csm_exchange.hip — the selections between the loop-closure exchange's
// collectives (csm_loop_closure.cpp): each runs as one thread
// on its device's stream, after the collective it depends on, so the host
// enqueues the whole exchange and waits once.
#include <hip/hip_runtime.h>

#include "csm_exchange.hpp"

namespace csm {
namespace {

// stage 2 input: this device's index if it holds the maximum score
__global__ void lc_pick_kernel(LcExchange* x) {
  x->idx = (x->local_idx >= 0 && x->local_score == x->score_max) ? x->local_idx : INT64_MAX;
}

// stage 3 input: the winner's (submap, x, y, angle) row, zeros elsewhere
__global__ void lc_row_kernel(LcExchange* x) {
  const bool win = x->local_idx >= 0 && x->local_idx == x->idx_min;
  for (int i = 0; i < 4; ++i) x->row[i] = win ? x->local_row[i] : 0.0;
}

}  // namespace

hipError_t launch_lc_pick(LcExchange* x, hipStream_t stream) {
  hipLaunchKernelGGL(lc_pick_kernel, dim3(1), dim3(1), 0, stream, x);
  return hipGetLastError();
}

hipError_t launch_lc_row(LcExchange* x, hipStream_t stream) {
  hipLaunchKernelGGL(lc_row_kernel, dim3(1), dim3(1), 0, stream, x);
  return hipGetLastError();
}

}  // namespace csm
