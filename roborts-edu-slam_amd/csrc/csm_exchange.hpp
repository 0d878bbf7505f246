// csm_exchange.hpp — device state of the loop-closure exchange (one per
// device, csm_loop_closure.cpp).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace csm {

struct LcExchange {
  // written by the host before the exchange (one copy)
  double local_score;   // this device's best (-DBL_MAX: no submap)
  int64_t local_idx;    // its global index (-1: none)
  double local_row[4];  // submap, x, y, angle
  double score;         // = local_score: the MAX all-reduce's input
  // collective outputs and the selections between them
  double score_max;
  int64_t idx;          // MIN all-reduce input
  int64_t idx_min;
  double row[4];        // SUM all-reduce input
  double row_sum[4];
};

hipError_t launch_lc_pick(LcExchange* x, hipStream_t stream);
hipError_t launch_lc_row(LcExchange* x, hipStream_t stream);

}  // namespace csm
