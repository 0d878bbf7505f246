/*
 * csm_gridmap.h — C-ABI of the device-resident occupancy-grid maps that the
 * correlative scan matcher reads (map building; row f4:
 * the post-match map check).
 *
 * A csm_gridmap is one OccuGridMap<ProbabilityCell> (the reference's
 * ScanMatchMap) or OccuGridMap<CountCell> (its PubMap) whose cells live in
 * HBM as separate arrays (prob, pass, hit, update_index). Geometry, bound box
 * and update counters are mirrored on the host, where the reference's
 * per-scan bookkeeping runs; every per-cell update is a HIP kernel.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository root):
 *
 *   csm_gridmap_create        OccuGridMap(resolution, size, offset, deviation,
 *                             default_cell_prob)        map/occu_grid_map.h:201-217
 *                             (GaussianBlur kernel :38-115, AllocateGridCell
 *                             map/grid_map_base.h:152-166)
 *   csm_gridmap_set_options   set_use_auto_map_resize / set_just_update_occu /
 *                             set_cell_occu_prob_offset  occu_grid_map.h:429-439,
 *                             set_extend_factor          grid_map_base.h:175-179
 *   csm_gridmap_set_cell_params  SetUpdateFreeFactor / SetUpdateOccupiedFactor /
 *                             SetOccuThreshold / SetMinPassThrough  occu_grid_map.h:413-427
 *   csm_gridmap_set_map_offset   GridMapBase::set_map_offset  grid_map_base.h:275-279
 *   csm_gridmap_reset         GridMapBase::Reset               grid_map_base.h:95-103
 *   csm_gridmap_update_bound  GridMapBase::UpdateBound (may ExtendSize)  grid_map_base.h:247-264
 *                             (called by ScanMatchers::MapSizeCheck, scan_matchers.h:365-390)
 *   csm_gridmap_update_by_range  OccuGridMap::UpdateMapByRange occu_grid_map.h:258-329
 *   csm_gridmap_init_with_range_vec  OccuGridMap::InitMapWithRangeVec  occu_grid_map.h:222-255
 *                             (with use_reset_speedup: ResetValueSpeedup grid_map_base.h:112-117)
 *   csm_gridmap_feedback_penalty OccuGridMap::MapFeedbackResponsePenalty occu_grid_map.h:331-392
 *   csm_gridmap_info / csm_gridmap_download   GridMapBase getters and GetCell reads
 *   csm_set_grid_gridmap      the scan matcher reads this map's probabilities
 *                             (ScanMatchers::ScanMatch on fine_map, scan_matchers.h:238-256)
 *
 * Points are RangeDataContainer contents after CreateFrom(raw, 1/resolution)
 * (slam/sensor_data_manager.h:99-115): map-cell units, sensor frame. Poses are
 * world (x, y, theta) in metres / radians.
 *
 * Update modes (as the reference uses them):
 *   just_update_occu + blur    ScanMatchMaps (slam_processor.cpp:493-510,458): each
 *                              endpoint raises its blur kernel's cells (max);
 *   just_update_occu, no blur  each hit cell is set occupied once per scan;
 *   full (lines), no blur      PubMap: Bresenham free marking + occupied endpoints.
 *   full + blur is order-dependent in the reference and never used by it; it
 *   returns CSM_ERR_UNSUPPORTED. ProbabilityCell supports all three modes,
 *   CountCell the two without blur.
 *
 * Every result (cells, update indices, touched-cell set, bound box, offset,
 * size after growth) equals the reference's sequential code bit for bit.
 * Calls are ordered on the map's own HIP stream; csm_set_grid_gridmap makes
 * the matcher's stream wait for the map's last update.
 */
#ifndef ROBORTS_CSM_GRIDMAP_H
#define ROBORTS_CSM_GRIDMAP_H

#include <stdint.h>

#include "csm.h"

#ifdef __cplusplus
extern "C" {
#endif

enum csm_cell_kind {
  CSM_PROBABILITY_CELL = 0, /* ProbabilityCell (grid_map_cell.h:301-388): ScanMatchMap */
  CSM_COUNT_CELL = 1        /* CountCell (grid_map_cell.h:42-161): PubMap */
};

typedef struct csm_gridmap csm_gridmap;

/* Geometry and counters of a map. */
typedef struct csm_gridmap_state {
  double resolution;        /* GetCellLength()                                   */
  double offset_x, offset_y;/* map_offset_                                       */
  double bound_min_x, bound_min_y, bound_max_x, bound_max_y; /* bound_box_       */
  int32_t size_x, size_y;
  int32_t map_update_index; /* map_update_index_ (IsMapInit: >= 0)               */
  int32_t cur_update_index; /* OccuGridMap::cur_update_index                      */
  int32_t half_kernel;      /* GaussianBlur half kernel (0: blur invalid)         */
  int32_t blur_states;
  int32_t kind;             /* enum csm_cell_kind                                */
  int32_t reserved;
  double scale_factor;      /* scale_factor_ = 1/resolution as constructed         */
} csm_gridmap_state;

int csm_gridmap_create(int device, int32_t kind, double resolution, int32_t size_x, int32_t size_y,
                       double offset_x, double offset_y, double deviation, float default_cell_prob,
                       csm_gridmap** out);
int csm_gridmap_destroy(csm_gridmap* map);
const char* csm_gridmap_last_error(const csm_gridmap* map);

int csm_gridmap_set_options(csm_gridmap* map, int32_t use_auto_map_resize, int32_t just_update_occu,
                            double cell_occu_prob_offset, double extend_factor);
/* occu_threshold and min_pass apply to CountCell only (ProbabilityCell's setters are no-ops). */
int csm_gridmap_set_cell_params(csm_gridmap* map, float update_free_factor, float update_occu_factor,
                                float occu_threshold, float min_pass);
int csm_gridmap_set_map_offset(csm_gridmap* map, double offset_x, double offset_y);
int csm_gridmap_reset(csm_gridmap* map);
/* *inside = UpdateBound's return value (0: the map grew to hold the box). */
int csm_gridmap_update_bound(csm_gridmap* map, double min_x, double min_y, double max_x, double max_y,
                             int32_t* inside);

/* *updated = UpdateMapByRange's return value (0 when the scan made the map grow). */
int csm_gridmap_update_by_range(csm_gridmap* map, const double* points_xy, int32_t n_points,
                                const double origin[2], const double sensor_pose[3], int32_t use_blur,
                                int32_t* updated);
/* scans: point_offsets has n_scans+1 prefix offsets into points_xy; origins
 * n_scans*2 (null: all zero, as roborts_slam_node.cpp:293 sets), poses n_scans*3. */
int csm_gridmap_init_with_range_vec(csm_gridmap* map, int32_t n_scans, const double* points_xy,
                                    const int64_t* point_offsets, const double* origins,
                                    const double* sensor_poses, int32_t use_blur, int32_t use_reset_speedup);
int csm_gridmap_feedback_penalty(csm_gridmap* map, const double* points_xy, int32_t n_points,
                                 const double origin[2], const double best_pose[3], int32_t check_point_num,
                                 double bound_tolerance, double penalty_gain, int32_t use_blur,
                                 double* response_coeff);

int csm_gridmap_get_state(csm_gridmap* map, csm_gridmap_state* out);
/* Copy cells to the host (size_y*size_x each; any pointer may be null).
 * touched: 1 where map_update_point_ holds the linear index. */
int csm_gridmap_download(csm_gridmap* map, float* prob, float* pass_count, float* hit_count,
                         int32_t* update_index, uint8_t* touched);
/* Device pointer of the probability array (row-major y*size_x + x). Valid
 * until the next call that grows or destroys the map. */
int csm_gridmap_device_prob(csm_gridmap* map, const float** device_prob);

/* Point the scan matcher at this map (borrowed, like csm_set_grid_device):
 * size, resolution, offset and update index come from the map.
 * Ordering, both ways: the matcher's work runs after the map's last update,
 * and the map's later updates (update_by_range, reset, init, update_bound)
 * wait for every match or copy already enqueued on that matcher context, so
 * a map may be updated right after set_grid returns, from any thread. */
int csm_set_grid_gridmap(csm_ctx* ctx, csm_gridmap* map);

/* Make n maps of one size, resolution and offset resident as a grid stack
 * (device-to-device copies ordered after each map's last update); scans then
 * name their map with csm_scan_matchers_batch_grids. Replaces the grid. */
int csm_set_grid_stack_gridmaps(csm_ctx* ctx, csm_gridmap* const* maps, int32_t n_maps);

#ifdef __cplusplus
}
#endif

#endif /* ROBORTS_CSM_GRIDMAP_H */
