/*
 * csm_frontend.h — C-ABI of the device-resident SLAM front-end: one call per
 * laser scan runs the reference's SlamProcessor::process front-end
 * (slam/slam_processor.cpp:66-258) with every map and the scan matcher on the
 * GPU. It is what BASELINE config 5 ("online mode: scan stream against a
 * growing map") measures; the pose-graph back-end is out of scope (SURVEY.md
 * 8f); its result, the corrected poses, comes back through
 * csm_frontend_correct_pose_and_map (SlamProcessor::CorrectPoseAndMap).
 *
 * Per scan (reference lines):
 *   - first scan: CreateAllMap (slam_processor.cpp:466-524) makes the PubMap
 *     (CountCell) and the coarse and fine ScanMatchMaps; the pose starts at 0;
 *   - later scans: the odometry prediction (PredictPoseByOdom :606-621),
 *     ScanMatchers::ScanMatch (scan_matchers.h:179-289): MapSizeCheck on both
 *     maps, optionally the Gauss-Newton matcher on the coarse map
 *     (use_optimize_scan_match; both reference YAMLs set it false, ParamConfig
 *     defaults it true) with the correlative coarse level as its fallback,
 *     then fine and super-fine on the fine map; the map check on the PubMap
 *     (MapCheckPenalize :569-593 -> MapFeedbackResponsePenalty) and the
 *     score gate on the pose (:166-186);
 *   - every scan: UpdateMap (:527-567) draws the scan into the three maps when
 *     the score passes (always for the first scan).
 * Results equal the reference's sequential code bit for bit (tested against
 * the oracle's restatement of the same loop).
 *
 * Threading: one caller at a time per front-end (the reference serialises the
 * front-end in its ROS callback).
 */
#ifndef ROBORTS_CSM_FRONTEND_H
#define ROBORTS_CSM_FRONTEND_H

#include <stdint.h>

#include "csm.h"
#include "csm_gridmap.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The ParamConfig fields the front-end reads (param_config.h:40-118); the
 * default values of config/simulatin_param.yaml are in roborts_csm.frontend. */
typedef struct csm_frontend_param {
  double range_max;                /* laser range_max (m): map sizes, MapSizeCheck  */
  double init_map_size;            /* x range_max (kMinMapSize = 3 floor)           */
  double map_offset_x, map_offset_y;
  double map_extend_factor;
  double gaussian_blur_offset;
  double map_resolution;           /* PubMap                                        */
  double map_update_free_factor, map_update_occu_factor;
  double map_occu_threshold, map_min_passthrough;
  double coarse_map_resolution, coarse_map_deviation;
  double fine_map_resolution, fine_map_deviation;
  int32_t coarse_map_use_blur, fine_map_use_blur;
  int32_t use_odometry;
  int32_t use_map_check_feedback;
  int32_t map_check_point_num;
  int32_t use_map_update_move_check;
  double map_check_bound_tolerance, map_check_penalty_gain;
  double map_update_score_threshold, map_update_distance_threshold, map_update_angle_threshold;
  csm_param levels[3];             /* coarse, fine, super-fine correlative windows  */
  int32_t use_optimize_scan_match; /* Gauss-Newton first, on the coarse map          */
  int32_t reserved;
  double optimize_failed_cost;     /* cost above which the correlative coarse runs   */
  csm_optimize_param optimize;
} csm_frontend_param;

/* What one processed scan produced. */
typedef struct csm_frontend_result {
  double pose[3];         /* current_sensor_pose_ after the scan (world)            */
  double match_pose[3];   /* the matcher's pose (before the score gate)              */
  double cov[9];          /* process_cov_matrix                                      */
  double score;           /* scan_match_score_ after the map check                   */
  double map_penalty;     /* MapCheckPenalize result (1 when not run)                */
  double optimize_cost;   /* BasedOptimizeScanMatch cost (0 when not run)            */
  int32_t data_index;     /* current_data_index_ of the scan                          */
  int32_t matched;        /* 0 for the first scan                                     */
  int32_t map_updated;    /* UpdateMap drew the scan (it is kept)                     */
  int32_t pose_accepted;  /* the score gate took the matched pose                     */
} csm_frontend_result;

enum csm_frontend_map { CSM_PUB_MAP = 0, CSM_COARSE_MAP = 1, CSM_FINE_MAP = 2 };

typedef struct csm_frontend csm_frontend;

int csm_frontend_create(int device, const csm_frontend_param* param, csm_frontend** out);
int csm_frontend_destroy(csm_frontend* fe);
const char* csm_frontend_last_error(const csm_frontend* fe);
/* One scan: points_xy are the sensor-frame endpoints in metres
 * (RangeDataContainer before CreateFrom); odom_pose the odometry pose read
 * with the scan (used when use_odometry). */
int csm_frontend_process(csm_frontend* fe, const double* points_xy, int32_t n_points, const double odom_pose[3],
                         csm_frontend_result* result);
/* Borrow one of the front-end's maps (owned by the front-end; null before the
 * first scan). */
int csm_frontend_map(csm_frontend* fe, int32_t which, csm_gridmap** map);
/* The front end's scan-matcher context (borrowed; owned and destroyed by the
 * front end): for profiling and kernel statistics (csm_set_profiling,
 * csm_kernel_stats) of the matches csm_frontend_process runs. */
int csm_frontend_matcher(csm_frontend* fe, csm_ctx** ctx);

/* SlamProcessor::CorrectPoseAndMap (slam/slam_processor.cpp:329-370): the
 * pose-graph back end's corrected world poses for kept scans ids[0..n)
 * (0 = the first kept scan; UpdateRangeData :597-602) replace their poses,
 * then all three maps are rebuilt on the device from every kept scan
 * (InitMapWithRangeVec, occu_grid_map.h:222-255): the PubMap from ids
 * 0..last plus map_min_passthrough_ more copies of scan 0, the coarse and fine
 * ScanMatchMaps with their blur settings. An id beyond the kept scans is
 * CSM_ERR_INVALID_ARG (the reference's CHECK_LE aborts). */
int csm_frontend_correct_pose_and_map(csm_frontend* fe, int32_t n, const int32_t* ids, const double* poses);
/* Kept scans so far (*n in: capacity of poses, out: count) and their poses. */
int csm_frontend_kept_scans(csm_frontend* fe, int32_t* n, double* poses);
/* Host wall time (ms) of the last csm_frontend_process call's phases:
 * [0] points scaled to the three resolutions, [1] the 3-level match
 * (ScanMatchers::ScanMatch), [2] the map check (MapCheckPenalize), [3] the
 * three map updates (UpdateMap; 0 when the scan was not kept), and of those
 * [4] the PubMap's, [5] the coarse map's, [6] the fine map's. Diagnostics of
 * the latency tail (no reference counterpart). */
int csm_frontend_last_phases(const csm_frontend* fe, double ms[7]);

#ifdef __cplusplus
}
#endif

#endif /* ROBORTS_CSM_FRONTEND_H */
