// csm_gridmap_internal.hpp — types shared by the occupancy-map kernels
// (csm_gridmap.hip) and their host side (csm_gridmap.cpp). Not installed;
// include/csm_gridmap.h is the public boundary.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace csm {

// Capacity to allocate for a buffer that must hold `bytes` and holds `cap`
// now: at least 64 KiB, and half as much again as before (at most 256 MiB
// more than asked), so per-scan sizes that creep up (a scan's points and
// endpoints) do not reallocate scan after scan — hipFree / hipHostFree
// synchronise the device, a few hundred microseconds in the online path.
inline size_t grow_bytes(size_t bytes, size_t cap) {
  size_t want = bytes < ((size_t)64 << 10) ? ((size_t)64 << 10) : bytes;
  if (cap) {
    size_t more = cap + cap / 2, lim = bytes + ((size_t)256 << 20);
    if (more > lim) more = lim;
    if (more > want) want = more;
  }
  return want;
}

enum { kGmProbability = 0, kGmCount = 1 };

// Device cell arrays of one map (pass/hit null for ProbabilityCell).
struct GmCells {
  float* prob;
  float* pass;
  float* hit;
  int32_t* uidx;
  uint8_t* touched;  // map_update_point_ as a set of linear indices
  int32_t row;       // size_x_ (row length of GetCell)
  int32_t size_x, size_y;
  // Fixed-point mirror of prob the scan matcher reads (nullable): cell (x, y)
  // at fpm[y * fpm_pitch + x] holds (prob - fpm_outside) * fpm_scale, exact
  // (csm_internal.hpp gridi layout). Kernels that write prob keep it equal.
  int32_t* fpm;
  int32_t fpm_pitch;
  float fpm_outside;
  double fpm_scale;
};

// Cell-function parameters (grid_map_cell.h).
struct GmOps {
  int32_t kind;
  float occu_factor, free_factor;
  float occu_threshold, min_pass;  // CountCell states
};

// One endpoint to draw: its cell and the scan's update indices
// (cur_mark_free_index / cur_mark_occu_index, occu_grid_map.h:272-273).
struct GmEnd {
  int32_t x, y;
  int32_t free_idx, occu_idx;
};

hipError_t gm_launch_fresh(const GmCells& C, int64_t n, float first, hipStream_t s);
hipError_t gm_launch_reset(const GmCells& C, int64_t n, float v, bool only_touched, bool clear_touched,
                           hipStream_t s);
hipError_t gm_launch_extend_copy(const GmCells& O, const GmCells& N, int gx, int gy, hipStream_t s);
hipError_t gm_launch_blur(const GmEnd* ends, int n, const GmCells& C, int hk, const float* ktab, int tol,
                          hipStream_t s);
hipError_t gm_launch_occupied(const GmEnd* ends, int n, const GmCells& C, const GmOps& P, int tol, hipStream_t s);
hipError_t gm_launch_lines(const GmEnd* ends, int n, int sx, int sy, const GmCells& C, const GmOps& P,
                           uint64_t* fkey, uint32_t* oseq, uint32_t seq, int tol, hipStream_t s);
hipError_t gm_launch_feedback(const GmEnd* ends, int n, int sx, int sy, const GmCells& C, const GmOps& P,
                              int use_blur, double occu_offset, int64_t min_d2, int* count, hipStream_t s);

// The map's fixed-point mirror for a matcher whose off-grid value is
// `outside` (gridmap_fixed_point): ok = false when the map's values are not
// known to be exactly summable in fixed point (a line or occupied update on
// the device wrote values the host cannot bound), and the matcher converts
// the grid itself.
struct GridMapFixed {
  bool ok;
  const int32_t* fpm;
  int32_t pitch;
  int32_t exp;        // E: values are multiples of 2^-E
  double max_abs;     // max |value| (and |outside|) the map can hold
  float outside;
};

// What the scan matcher needs to borrow a map's probabilities.
struct GridMapView {
  const float* prob;
  int32_t size_x, size_y;
  double resolution, offset_x, offset_y;
  int32_t map_update_index;
  hipEvent_t ready;  // recorded after the map's last update
  int device;
};
}  // namespace csm

struct csm_gridmap;
namespace csm {
int gridmap_view(csm_gridmap* m, GridMapView* v);
// Builds (or keeps) the mirror for `outside`; the map's `ready` event covers it.
int gridmap_fixed_point(csm_gridmap* m, float outside, GridMapFixed* f);
// A matcher stream reads the map: the map's next updates wait for the work
// enqueued on it so far. drop_reader: the stream is going away.
void gridmap_add_reader(csm_gridmap* m, hipStream_t s);
// The stream stops reading the map (its context moved to another grid): the
// reads enqueued so far become a one-shot fence the next update waits for.
void gridmap_release_reader(csm_gridmap* m, hipStream_t s);
// A one-shot fence: the reads enqueued on s so far (a device-to-device copy).
void gridmap_add_read_fence(csm_gridmap* m, hipStream_t s);
// The stream goes away: every map it reads keeps a fence of its reads.
void gridmap_drop_reader(hipStream_t s);

}  // namespace csm
