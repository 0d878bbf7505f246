// csm_frontend.cpp — device-resident SLAM front-end (include/csm_frontend.h):
// the reference's SlamProcessor::process front-end loop
// (slam/slam_processor.cpp:65-248) over the GPU scan matcher (csm.h) and the
// GPU occupancy maps (csm_gridmap.h). The host runs the reference's per-scan
// control flow and pose arithmetic (g++ -O2 -ffp-contract=off); the maps and
// the matcher stay resident in HBM between scans.
//
// Paths cited are relative to the reference root.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "csm.h"
#include "csm_frontend.h"
#include "csm_gridmap.h"
#include "csm_matchers.hpp"
#include "host_math.hpp"

namespace {

constexpr double kMinMapSize = 3;             // slam_processor.h:262
constexpr float kMapUnknownCellProb = 0.3f;   // slam_processor.h:264
constexpr float kDefaultCellProb = 0.5f;      // map/grid_map_cell.h:30

// util::NormalizeAngle / PoseChangeEnough (util/slam_util.h:103-126)
double normalize_angle(double a) {
  double n = std::fmod(std::fmod(a, 2.0 * M_PI) + 2.0 * M_PI, 2.0 * M_PI);
  if (n > M_PI) n -= 2.0 * M_PI;
  return n;
}
bool pose_change_enough(const double* p1, const double* p2, double dist, double ang) {
  const double dx = p1[0] - p2[0], dy = p1[1] - p2[1];
  if (std::sqrt(dx * dx + dy * dy) >= dist) return true;
  return std::fabs(normalize_angle(p1[2] - p2[2])) >= ang;
}

// PredictPoseByOdom (slam_processor.cpp:618-635), Eigen's 2x2 products.
void predict_by_odom(const double* last_pose, const double* last_odom, const double* cur_odom, double* out) {
  const double a = last_pose[2] - last_odom[2];
  double c, s;
  csm::host_sincos(a, &s, &c);
  const double tx = last_pose[0] - (c * last_odom[0] + (-s) * last_odom[1]);
  const double ty = last_pose[1] - (s * last_odom[0] + c * last_odom[1]);
  out[0] = (c * cur_odom[0] + (-s) * cur_odom[1]) + tx;
  out[1] = (s * cur_odom[0] + c * cur_odom[1]) + ty;
  out[2] = a + cur_odom[2];
}

// RangeDataContainer::CreateFrom(raw, factor) (sensor_data_manager.h:99-115)
void scale_points(const double* pts, int n, double factor, std::vector<double>& out) {
  out.resize((size_t)2 * n);
  for (int i = 0; i < 2 * n; ++i) out[(size_t)i] = pts[i] * factor;
}

}  // namespace

struct csm_frontend {
  int device = 0;
  csm_frontend_param p{};
  std::string err;
  csm_ctx* ctx = nullptr;         // matcher on the fine map
  csm_ctx* ctx_coarse = nullptr;  // Gauss-Newton matcher on the coarse map (use_optimize_scan_match)
  csm_gridmap* maps[3] = {nullptr, nullptr, nullptr};
  int32_t data_index = 0;  // scans kept so far (SensorDataManager::current_data_index_ + 1)
  double current_pose[3] = {0, 0, 0};
  double last_odom[3] = {0, 0, 0};
  double last_map_update_pose[3] = {0, 0, 0};
  double scan_match_score = 0.0;
  int map_penalize_times = 0;
  std::vector<double> pub_pts, coarse_pts, fine_pts;
  // the kept scans (SensorDataManager's multiresolution range data,
  // slam_processor.cpp:216-221): sensor-frame points (m), the pose each was
  // drawn at (:196-205); CorrectPoseAndMap rebuilds the maps from them
  std::vector<double> kept_pts;
  std::vector<int64_t> kept_off{0};
  std::vector<double> kept_pose;
  // CSM_FE_TIMING=1: host wall time per phase, printed at destroy
  bool timing = false;
  double t_phase[6] = {0, 0, 0, 0, 0, 0};
  int64_t n_timed = 0;
  double last_phase[6] = {0, 0, 0, 0, 0, 0};  // the last call's (csm_frontend_last_phases)
  double last_update[3] = {0, 0, 0};          // ... its three map updates: pub, coarse, fine

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int check(int st, const char* what) {
    if (st == CSM_OK) return CSM_OK;
    err = what;
    return st;
  }
};

namespace {

// CreateAllMap (slam_processor.cpp:464-527) without the back-end maps.
int create_all_maps(csm_frontend* f) {
  const csm_frontend_param& p = f->p;
  const double range_max = p.range_max;
  const double init_map_size = (p.init_map_size < kMinMapSize) ? (kMinMapSize * range_max)
                                                                : (p.init_map_size * range_max);
  const double ox = init_map_size * p.map_offset_x, oy = init_map_size * p.map_offset_y;
  const double res[3] = {p.map_resolution, p.coarse_map_resolution, p.fine_map_resolution};
  const double dev[3] = {0.0, p.coarse_map_deviation, p.fine_map_deviation};
  const float dflt[3] = {kDefaultCellProb, kMapUnknownCellProb, kMapUnknownCellProb};
  const int32_t kind[3] = {CSM_COUNT_CELL, CSM_PROBABILITY_CELL, CSM_PROBABILITY_CELL};
  for (int k = 0; k < 3; ++k) {
    const int32_t sz = static_cast<int>(init_map_size / res[k]);
    int st = csm_gridmap_create(f->device, kind[k], res[k], sz, sz, ox, oy, dev[k], dflt[k], &f->maps[k]);
    if (st != CSM_OK) return f->fail(st, "csm_gridmap_create failed");
    // PubMap: extend factor + auto resize (:477-478); ScanMatchMaps: also the
    // blur offset and just_update_occu (:492-495, :507-510)
    const bool pub = k == CSM_PUB_MAP;
    st = csm_gridmap_set_options(f->maps[k], 1, pub ? 0 : 1, pub ? 0.72 : p.gaussian_blur_offset,
                                 p.map_extend_factor);
    if (st != CSM_OK) return f->fail(st, "csm_gridmap_set_options failed");
  }
  return CSM_OK;
}

}  // namespace

extern "C" {

int csm_frontend_create(int device, const csm_frontend_param* param, csm_frontend** out) {
  if (!param || !out) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  auto* f = new csm_frontend();
  f->device = device;
  f->p = *param;
#ifdef CSM_FE_TIMING  // diagnostic builds: per-phase host timings of every call
  f->timing = true;
#endif
  int st = csm_create(device, &f->ctx);
  if (st == CSM_OK && param->use_optimize_scan_match) st = csm_create(device, &f->ctx_coarse);
  if (st != CSM_OK) {
    if (f->ctx) csm_destroy(f->ctx);
    delete f;
    return st;
  }
  *out = f;
  return CSM_OK;
}

int csm_frontend_destroy(csm_frontend* f) {
  if (!f) return CSM_OK;
  if (f->timing && f->n_timed > 0) {
    static const char* names[6] = {"prepare", "-", "-", "scan_matchers", "map_check", "update_map"};
    std::fprintf(stderr, "csm_frontend timing over %lld scans (ms/scan):", (long long)f->n_timed);
    for (int i = 0; i < 6; ++i) std::fprintf(stderr, " %s %.4f", names[i], f->t_phase[i] / f->n_timed);
    std::fprintf(stderr, "\n");
  }
  for (auto*& m : f->maps)
    if (m) csm_gridmap_destroy(m);
  if (f->ctx) csm_destroy(f->ctx);
  if (f->ctx_coarse) csm_destroy(f->ctx_coarse);
  delete f;
  return CSM_OK;
}

const char* csm_frontend_last_error(const csm_frontend* f) { return f ? f->err.c_str() : "null front-end"; }

int csm_frontend_map(csm_frontend* f, int32_t which, csm_gridmap** m) {
  if (!f || !m || which < 0 || which > 2) return CSM_ERR_INVALID_ARG;
  *m = f->maps[which];
  return CSM_OK;
}

int csm_frontend_process(csm_frontend* f, const double* pts, int32_t n, const double odom[3],
                         csm_frontend_result* r) {
  if (!f || !r || !odom || n < 0 || (n > 0 && !pts)) return CSM_ERR_INVALID_ARG;
  const csm_frontend_param& p = f->p;
  std::memset(r, 0, sizeof(*r));
  int st;
  using clk = std::chrono::steady_clock;
  auto tp = clk::now();
  for (double& t : f->last_phase) t = 0.0;
  for (double& t : f->last_update) t = 0.0;
  auto lap = [&](int k) {
    const auto now = clk::now();
    const double ms = std::chrono::duration<double, std::milli>(now - tp).count();
    f->last_phase[k] += ms;
    if (f->timing) f->t_phase[k] += ms;
    tp = now;
  };
  const bool first = f->data_index == 0;  // IsFirstRangeData
  if (first) {
    if ((st = create_all_maps(f)) != CSM_OK) return st;
    f->current_pose[0] = f->current_pose[1] = f->current_pose[2] = 0.0;
  }
  double predict[3] = {f->current_pose[0], f->current_pose[1], f->current_pose[2]};
  // range data at each map's resolution (:104-111)
  scale_points(pts, n, 1 / p.map_resolution, f->pub_pts);
  scale_points(pts, n, 1 / p.coarse_map_resolution, f->coarse_pts);
  scale_points(pts, n, 1 / p.fine_map_resolution, f->fine_pts);
  double cov[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  r->map_penalty = 1.0;
  lap(0);
  if (!first) {
    if (p.use_odometry) predict_by_odom(f->current_pose, f->last_odom, odom, predict);
    double pose[3] = {predict[0], predict[1], predict[2]};
    // ScanMatchers::ScanMatch (scan_matchers.h:179-289) on the fine / coarse maps
    csm::MatchersConfig cfg{p.levels, p.use_optimize_scan_match, p.optimize_failed_cost, p.optimize, p.range_max};
    double score = 0.0;
    std::string why;
    if ((st = csm::scan_matchers_on_maps(f->ctx, f->ctx_coarse, f->maps[CSM_COARSE_MAP], f->maps[CSM_FINE_MAP],
                                         f->coarse_pts.data(), f->fine_pts.data(), n, cfg, 1, pose, cov, &score,
                                         &r->optimize_cost, &why)) != CSM_OK)
      return f->fail(st, why);
    std::memcpy(r->match_pose, pose, sizeof(pose));
    lap(3);
    // MapCheckPenalize (:573-595), use_logistic = false
    double penalty = 1.0;
    if (p.use_map_check_feedback) {
      if ((st = csm_gridmap_feedback_penalty(f->maps[CSM_PUB_MAP], f->pub_pts.data(), n, nullptr, pose,
                                             p.map_check_point_num, p.map_check_bound_tolerance,
                                             p.map_check_penalty_gain, 0, &penalty)) != CSM_OK)
        return f->check(st, "MapFeedbackResponsePenalty");
    }
    r->map_penalty = penalty;
    lap(4);
    if (f->map_penalize_times < 5) {  // :158-170
      score *= penalty;
      score = (score > 1.0) ? (1.0) : (score);
      if (penalty < 0.7)
        f->map_penalize_times++;
      else
        f->map_penalize_times = 0;
    } else {
      f->map_penalize_times = 0;
    }
    if (score > std::max(0.5, p.map_update_score_threshold)) {  // :174-177
      std::memcpy(f->current_pose, pose, sizeof(pose));
      r->pose_accepted = 1;
    }
    f->scan_match_score = score;
    r->matched = 1;
  }
  // UpdateMap (:529-571)
  bool updated = false;
  if ((f->scan_match_score > p.map_update_score_threshold &&
       (pose_change_enough(f->current_pose, f->last_map_update_pose, p.map_update_distance_threshold,
                           p.map_update_angle_threshold) ||
        !p.use_map_update_move_check)) ||
      f->data_index < 1) {
    csm_gridmap* pub = f->maps[CSM_PUB_MAP];
    if (first)  // :537-542
      st = csm_gridmap_set_cell_params(pub, (float)p.map_min_passthrough, (float)(p.map_min_passthrough * 2), 0.5f,
                                       1.0f);
    else  // :543-548
      st = csm_gridmap_set_cell_params(pub, (float)p.map_update_free_factor, (float)p.map_update_occu_factor,
                                       (float)p.map_occu_threshold, (float)p.map_min_passthrough);
    if (st != CSM_OK) return f->check(st, "pub map cell params");
    int32_t up = 0;
    const double* pose = f->current_pose;
    const auto tu0 = clk::now();
    if ((st = csm_gridmap_update_by_range(pub, f->pub_pts.data(), n, nullptr, pose, 0, &up)) != CSM_OK)
      return f->check(st, "UpdateMapByRange(pub)");
    const auto tu1 = clk::now();
    if ((st = csm_gridmap_update_by_range(f->maps[CSM_COARSE_MAP], f->coarse_pts.data(), n, nullptr, pose,
                                          p.coarse_map_use_blur, &up)) != CSM_OK)
      return f->check(st, "UpdateMapByRange(coarse)");
    const auto tu2 = clk::now();
    if ((st = csm_gridmap_update_by_range(f->maps[CSM_FINE_MAP], f->fine_pts.data(), n, nullptr, pose,
                                          p.fine_map_use_blur, &up)) != CSM_OK)
      return f->check(st, "UpdateMapByRange(fine)");
    f->last_update[0] = std::chrono::duration<double, std::milli>(tu1 - tu0).count();
    f->last_update[1] = std::chrono::duration<double, std::milli>(tu2 - tu1).count();
    f->last_update[2] = std::chrono::duration<double, std::milli>(clk::now() - tu2).count();
    std::memcpy(f->last_map_update_pose, f->current_pose, sizeof(f->current_pose));
    updated = true;
  }
  lap(5);
  if (f->timing && !first) f->n_timed++;
  r->data_index = f->data_index;
  if (updated) {  // the scan is kept (AddMultiresolutionRangeData); else ClearCurrentData
    f->data_index++;
    std::memcpy(f->last_odom, odom, sizeof(f->last_odom));
    f->kept_pts.insert(f->kept_pts.end(), pts, pts + 2 * (size_t)n);
    f->kept_off.push_back((int64_t)(f->kept_pts.size() / 2));
    f->kept_pose.insert(f->kept_pose.end(), f->current_pose, f->current_pose + 3);
  }
  std::memcpy(r->pose, f->current_pose, sizeof(r->pose));
  std::memcpy(r->cov, cov, sizeof(cov));
  r->score = f->scan_match_score;
  r->map_updated = updated ? 1 : 0;
  return CSM_OK;
}

int csm_frontend_matcher(csm_frontend* f, csm_ctx** ctx) {
  if (!f || !ctx) return CSM_ERR_INVALID_ARG;
  *ctx = f->ctx;
  return CSM_OK;
}

int csm_frontend_correct_pose_and_map(csm_frontend* f, int32_t n, const int32_t* ids, const double* poses) {
  if (!f || n < 0 || (n > 0 && (!ids || !poses))) return CSM_ERR_INVALID_ARG;
  const csm_frontend_param& p = f->p;
  const int kept = (int)f->kept_off.size() - 1;
  for (int i = 0; i < n; ++i)  // CHECK_LE(id, current_data_index_) (:341)
    if (ids[i] < 0 || ids[i] >= kept) return f->fail(CSM_ERR_INVALID_ARG, "corrected id beyond the kept scans");
  if (kept == 0) return CSM_OK;
  for (int i = 0; i < n; ++i)  // UpdateRangeData (:597-602)
    std::memcpy(&f->kept_pose[3 * (size_t)ids[i]], poses + 3 * i, 3 * sizeof(double));
  // the PubMap's scans: every kept id, then map_min_passthrough_ more copies of
  // scan 0 (:349-355); the scan-match maps: every kept scan (:357-366)
  std::vector<int> pub_ids;
  for (int i = 0; i < kept; ++i) pub_ids.push_back(i);
  for (int i = 0; i < p.map_min_passthrough; ++i) pub_ids.push_back(0);
  const double res[3] = {p.map_resolution, p.coarse_map_resolution, p.fine_map_resolution};
  const int32_t blur[3] = {0, p.coarse_map_use_blur, p.fine_map_use_blur};
  std::vector<double> pts, ps;
  std::vector<int64_t> off;
  for (int k = 0; k < 3; ++k) {
    const size_t use = k == 0 ? pub_ids.size() : (size_t)kept;
    const double factor = 1 / res[k];  // CreateFrom (sensor_data_manager.h:99-115)
    pts.clear();
    ps.clear();
    off.assign(1, 0);
    for (size_t u = 0; u < use; ++u) {
      const int id = pub_ids[u];
      for (int64_t j = 2 * f->kept_off[(size_t)id]; j < 2 * f->kept_off[(size_t)id + 1]; ++j)
        pts.push_back(f->kept_pts[(size_t)j] * factor);
      off.push_back((int64_t)(pts.size() / 2));
      ps.insert(ps.end(), &f->kept_pose[3 * (size_t)id], &f->kept_pose[3 * (size_t)id] + 3);
    }
    // InitMapWithRangeVec (occu_grid_map.h:222-255) on the device map: the
    // scan-match maps' blur splats of every scan go down in one launch
    const int st = csm_gridmap_init_with_range_vec(f->maps[k], (int32_t)use, pts.data(), off.data(), nullptr,
                                                   ps.data(), blur[k], 0);
    if (st != CSM_OK) return f->fail(st, std::string("InitMapWithRangeVec: ") + csm_gridmap_last_error(f->maps[k]));
  }
  return CSM_OK;
}

int csm_frontend_last_phases(const csm_frontend* f, double ms[7]) {
  if (!f || !ms) return CSM_ERR_INVALID_ARG;
  ms[0] = f->last_phase[0];
  ms[1] = f->last_phase[3];
  ms[2] = f->last_phase[4];
  ms[3] = f->last_phase[5];
  ms[4] = f->last_update[0];
  ms[5] = f->last_update[1];
  ms[6] = f->last_update[2];
  return CSM_OK;
}

int csm_frontend_kept_scans(csm_frontend* f, int32_t* n, double* poses) {
  if (!f || !n) return CSM_ERR_INVALID_ARG;
  const int kept = (int)f->kept_off.size() - 1;
  if (poses && *n >= kept) std::memcpy(poses, f->kept_pose.data(), 3 * (size_t)kept * sizeof(double));
  *n = kept;
  return CSM_OK;
}

}  // extern "C"
