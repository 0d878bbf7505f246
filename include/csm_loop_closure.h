/*
 * csm_loop_closure.h — C-ABI of the sharded loop-closure search (SURVEY.md 8e,
 * BASELINE config 3): one query scan against many submaps, the submaps
 * sharded over the GPUs of ONE process, the best candidate agreed over RCCL.
 *
 * Reference: the pose-graph back end closes loops by matching a scan against
 * the map around older chain candidates, one ScanMatchInterface call at a
 * time (pose_graph/range_scan_pose_graph.cpp:299-355 TryCloseLoop, :120-167
 * LinkNearChains -> slam/slam_processor.cpp:301 -> ScanMatchers::ScanMatch).
 * This entry point is what TryCloseLoop can call from C++ instead: every
 * submap window in one search per device, no Python, no torch.
 *
 *   devices            submaps [r*S/G, (r+1)*S/G) resident on device r only
 *                      (csm_set_grid_stack of that device's context)
 *   search             per device: csm_search_windows (admissible multi-
 *                      resolution branch and bound) or the exhaustive
 *                      csm_best_windows, run concurrently from host threads
 *   exchange           three ncclAllReduce over one communicator per device
 *                      (ncclCommInitAll, in-process): MAX of the 8-byte score,
 *                      MIN of the 8-byte global index among devices holding
 *                      that score, SUM of the winner's one-hot (submap, x, y,
 *                      angle) row; the selections between them run as tiny
 *                      device kernels, so the host waits once, at the end
 *
 * global index = submap * n_cand + flat index (reference enumeration order);
 * the result is what one device holding every submap returns (max score,
 * lowest global index), whatever the device count.
 *
 * RCCL is loaded at csm_loop_closure_create (dlopen of librccl.so.1, private
 * symbols), so the matcher library itself does not depend on it.
 */
#ifndef ROBORTS_CSM_LOOP_CLOSURE_H
#define ROBORTS_CSM_LOOP_CLOSURE_H

#include <stdint.h>

#include "csm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct csm_loop_closure csm_loop_closure;

typedef struct csm_loop_closure_result {
  double score;           /* best response (-DBL_MAX: no submap)                  */
  int64_t global_index;   /* submap * n_cand + flat index; -1: nothing scored     */
  int32_t submap;
  int32_t n_devices;
  double x, y, angle;     /* candidate pose in the submap's map cells / rad       */
  double pose_world[3];   /* the same pose in world coordinates (GetWorldCoordsPose,
                             grid_map_base.h:83-87, with the submap's offset)      */
  double search_ms;       /* host wall time of the concurrent per-device searches */
  double exchange_ms;     /* host wall time of the exchange: staging up, the three
                             all-reduces and two selections, result down, every
                             stream drained                                         */
} csm_loop_closure_result;

enum csm_loop_closure_search { CSM_LC_PYRAMID = 0, CSM_LC_EXHAUSTIVE = 1 };

/* n_devices HIP devices (devices == NULL: 0 .. n_devices-1), one matcher
 * context and one RCCL communicator each. */
int csm_loop_closure_create(int32_t n_devices, const int32_t* devices, csm_loop_closure** out);
int csm_loop_closure_destroy(csm_loop_closure* lc);
const char* csm_loop_closure_last_error(const csm_loop_closure* lc);

/* The submaps: n_submaps packed fp32 grids of one size (host memory,
 * n_submaps * size_y * size_x floats, kept alive by the caller while
 * resident), info->resolution their cell length, offsets[2i..2i+1] submap
 * i's map_offset_ (m). version as csm_set_grid_stack (unchanged: no upload). */
int csm_loop_closure_set_submaps(csm_loop_closure* lc, const float* cells, int32_t n_submaps,
                                 const csm_map_info* info, const double* offsets, int64_t version);

/* One query: points_xy in map cells (sensor frame, as csm_scan_match), the
 * window param (e.g. +-8 m / +-pi at one-cell steps), pose_world the centre
 * of every submap's window. search: enum csm_loop_closure_search. */
int csm_loop_closure_match(csm_loop_closure* lc, const double* points_xy, int32_t n_points,
                           const csm_param* param, const double pose_world[3], int32_t search,
                           csm_loop_closure_result* result);

#ifdef __cplusplus
}
#endif

#endif /* ROBORTS_CSM_LOOP_CLOSURE_H */
