// csm_gridmap_internal.hpp — types shared by the occupancy-map kernels
// (csm_gridmap.hip) and their host side (csm_gridmap.cpp). Not installed;
// include/csm_gridmap.h is the public boundary.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace csm {

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
// A matcher stream reads the map: the map's next updates wait for the work
// enqueued on it so far. drop_reader: the stream is going away.
void gridmap_add_reader(csm_gridmap* m, hipStream_t s);
void gridmap_drop_reader(hipStream_t s);

}  // namespace csm
