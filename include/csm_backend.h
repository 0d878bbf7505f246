/*
 * csm_backend.h — C-ABI of the back-end's scan-match service (SURVEY.md 8f
 * row f2): SlamProcessor::ScanMatchInterface (slam/slam_processor.cpp:250-326),
 * the callback RangeScanPoseGraph calls for near-chain links
 * (pose_graph/range_scan_pose_graph.cpp:120-167, via ScanMatchFunc
 * range_scan_pose_graph.h:30-35) and for loop closure (:299-355), issued as a
 * batch of independent jobs on the GPU.
 *
 * One job = one ScanMatchInterface call:
 *   - the back-end coarse and fine ScanMatchMaps are rebuilt from the chain's
 *     kept scans (ResetScanMatchMapWithRangeVec :448-462: offset centred on
 *     the current sensor pose, no auto resize, just_update_occu,
 *     InitMapWithRangeVec with the reset speed-up);
 *   - ScanMatchers::ScanMatch on them (scan_matchers.h:179-289; MapSizeCheck,
 *     optional Gauss-Newton on the coarse map, correlative levels on the fine
 *     map);
 *   - MapCheckPenalize with the logistic (:573-595) on the caller's PubMap;
 *     score *= penalty, clamped to 1.
 * The maps and the matcher stay in HBM. Job j of a call rebuilds and reads
 * map pair j of the service (created at the reference's back-end map size,
 * CreateScanMatchMapWithRangeVec :428-446), so a one-job call is exactly the
 * reference's call on its single pair of back-end maps, and a J-job call
 * equals J such calls as long as no MapSizeCheck grows a map (then that pair
 * keeps its growth, as the reference's pair would). When every job's fine map
 * has the same geometry and the Gauss-Newton matcher is off (both reference
 * YAMLs), the correlative levels of all jobs run as one batch over a stack of
 * the fine maps (csm_scan_matchers_batch_grids).
 *
 * Kept scans mirror SensorDataManager (slam/sensor_data_manager.h:366-592):
 * csm_backend_add_scan keeps the endpoints in metres with their sensor pose
 * and the coarse / fine copies CreateFrom(raw, 1/resolution) makes;
 * csm_backend_set_scan_pose is UpdateRangeData (slam_processor.cpp:597-603).
 *
 * Results equal the oracle's restatement of the same calls bit for bit.
 * Threading: one caller at a time (the reference's back-end thread).
 */
#ifndef ROBORTS_CSM_BACKEND_H
#define ROBORTS_CSM_BACKEND_H

#include <stdint.h>

#include "csm.h"
#include "csm_gridmap.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The ParamConfig fields ScanMatchInterface reads (param_config.h:40-118). */
typedef struct csm_backend_param {
  double range_max;                 /* back-end map size (range_max + 2 m) * 2      */
  double gaussian_blur_offset;
  double map_resolution;            /* PubMap: the map check's range data           */
  double coarse_map_resolution, coarse_map_deviation;
  double fine_map_resolution, fine_map_deviation;
  int32_t coarse_map_use_blur, fine_map_use_blur;
  int32_t use_map_check_feedback, map_check_point_num;
  double map_check_bound_tolerance, map_check_penalty_gain;
  csm_param levels[3];              /* the ScanMatchParam set installed for the call */
  int32_t use_optimize_scan_match;
  int32_t reserved;
  double optimize_failed_cost;
  csm_optimize_param optimize;
} csm_backend_param;

/* One ScanMatchInterface call. */
typedef struct csm_backend_job {
  const double* points_m;    /* the query range data: metres, sensor frame     */
  int32_t n_points;
  int32_t n_chain;           /* range_id: kept-scan ids the maps are built from */
  const int32_t* chain_ids;
  int32_t use_fine_scan_match;
  int32_t reserved;
  double pose[3];            /* best_pose in/out (world)                        */
  double cov[9];             /* cov_matrix out (row-major)                      */
  double score;              /* the return value                                */
  double map_penalty;        /* MapCheckPenalize (with the logistic), 1 if off  */
  double optimize_cost;      /* Gauss-Newton cost, 0 when not run               */
} csm_backend_job;

typedef struct csm_backend csm_backend;

int csm_backend_create(int device, const csm_backend_param* param, csm_backend** out);
int csm_backend_destroy(csm_backend* be);
const char* csm_backend_last_error(const csm_backend* be);
/* Keep a scan (AddSensorData + AddMultiresolutionRangeData); *id = 0, 1, ... */
int csm_backend_add_scan(csm_backend* be, const double* points_m, int32_t n_points, const double sensor_pose[3],
                         int32_t* id);
int csm_backend_set_scan_pose(csm_backend* be, int32_t id, const double sensor_pose[3]);
/* n_jobs ScanMatchInterface calls. current_pose = current_sensor_pose_ (the
 * back-end maps are centred on it); pub_map = the PubMap of the map check
 * (CountCell; null skips the check, penalty 1). */
int csm_backend_scan_match(csm_backend* be, csm_gridmap* pub_map, const double current_pose[3],
                           csm_backend_job* jobs, int32_t n_jobs);
/* Borrow map pair `slot` (which: 0 coarse, 1 fine); null before first use. */
int csm_backend_map(csm_backend* be, int32_t slot, int32_t which, csm_gridmap** map);

#ifdef __cplusplus
}
#endif

#endif /* ROBORTS_CSM_BACKEND_H */
