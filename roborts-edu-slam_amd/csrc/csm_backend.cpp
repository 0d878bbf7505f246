// csm_backend.cpp — the back-end's scan-match service (include/csm_backend.h):
// SlamProcessor::ScanMatchInterface (slam/slam_processor.cpp:250-326) for a
// batch of pose-graph jobs, over device-resident maps and the GPU matcher.
// Host control flow and pose arithmetic only (g++ -O2 -ffp-contract=off);
// every map update and every scoring runs on the device.
//
// Paths cited are relative to the reference root.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "csm.h"
#include "csm_backend.h"
#include "csm_gridmap.h"
#include "csm_matchers.hpp"

namespace {

constexpr double kMinScanMatchMapBound = 2.0;  // slam_processor.h:263
constexpr float kMapUnknownCellProb = 0.3f;    // slam_processor.h:264

struct KeptScan {  // RangeDataContainer copies (sensor_data_manager.h:99-115)
  std::vector<double> raw, coarse, fine;
  double pose[3];
};

struct MapPair {
  csm_gridmap* map[2] = {nullptr, nullptr};  // coarse, fine
};

void scale_points(const double* pts, int n, double factor, std::vector<double>& out) {
  out.resize((size_t)2 * n);
  for (int i = 0; i < 2 * n; ++i) out[(size_t)i] = pts[i] * factor;
}

}  // namespace

struct csm_backend {
  int device = 0;
  csm_backend_param p{};
  std::string err;
  csm_ctx* ctx = nullptr;         // correlative levels, one job at a time
  csm_ctx* ctx_coarse = nullptr;  // Gauss-Newton on a coarse map
  csm_ctx* ctx_stack = nullptr;   // correlative levels of all jobs over a stack of fine maps
  std::vector<KeptScan> scans;
  std::vector<MapPair> pairs;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
};

namespace {

// The back-end ScanMatchMaps (CreateScanMatchMapWithRangeVec,
// slam_processor.cpp:428-446): (range_max + 2 m) * 2 square at each
// resolution. Their first contents are wiped by the first reset, so they
// start empty here.
int ensure_pair(csm_backend* b, int32_t slot) {
  while ((int32_t)b->pairs.size() <= slot) b->pairs.emplace_back();
  MapPair& mp = b->pairs[(size_t)slot];
  const csm_backend_param& p = b->p;
  const double init_map_size = (p.range_max + kMinScanMatchMapBound) * 2;
  const double res[2] = {p.coarse_map_resolution, p.fine_map_resolution};
  const double dev[2] = {p.coarse_map_deviation, p.fine_map_deviation};
  for (int k = 0; k < 2; ++k) {
    if (mp.map[k]) continue;
    const int32_t sz = static_cast<int>(init_map_size / res[k]);
    int st = csm_gridmap_create(b->device, CSM_PROBABILITY_CELL, res[k], sz, sz, 0.0, 0.0, dev[k], kMapUnknownCellProb,
                                &mp.map[k]);
    if (st != CSM_OK) return b->fail(st, "csm_gridmap_create(back-end map)");
  }
  return CSM_OK;
}

// ResetScanMatchMapWithRangeVec (slam_processor.cpp:448-462) with the chain's
// multi-resolution range data (GetMultiresolutionRangeDataVecWithId).
int reset_map(csm_backend* b, csm_gridmap* m, int which, const csm_backend_job& job, const double cur[3]) {
  csm_gridmap_state s{};
  int st = csm_gridmap_get_state(m, &s);
  if (st != CSM_OK) return st;
  const double resolution = s.resolution;  // GetCellLength()
  const double ox = -(cur[0] - 0.5 * s.size_x * resolution);
  const double oy = -(cur[1] - 0.5 * s.size_y * resolution);
  if ((st = csm_gridmap_set_map_offset(m, ox, oy)) != CSM_OK) return st;
  if ((st = csm_gridmap_set_options(m, 0, 1, b->p.gaussian_blur_offset, 0.0)) != CSM_OK) return st;
  std::vector<double> pts, poses;
  std::vector<int64_t> off(1, 0);
  for (int32_t k = 0; k < job.n_chain; ++k) {
    const KeptScan& ks = b->scans[(size_t)job.chain_ids[k]];
    const std::vector<double>& v = which ? ks.fine : ks.coarse;
    pts.insert(pts.end(), v.begin(), v.end());
    off.push_back(off.back() + (int64_t)(v.size() / 2));
    poses.insert(poses.end(), ks.pose, ks.pose + 3);
  }
  const int32_t use_blur = which ? b->p.fine_map_use_blur : b->p.coarse_map_use_blur;
  return csm_gridmap_init_with_range_vec(m, job.n_chain, pts.data(), off.data(), nullptr, poses.data(), use_blur, 1);
}

bool same_geometry(const csm_gridmap_state& a, const csm_gridmap_state& b) {
  return a.size_x == b.size_x && a.size_y == b.size_y && a.resolution == b.resolution && a.offset_x == b.offset_x &&
         a.offset_y == b.offset_y;
}

}  // namespace

extern "C" {

int csm_backend_create(int device, const csm_backend_param* param, csm_backend** out) {
  if (!param || !out) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  if (!(param->coarse_map_resolution > 0.0) || !(param->fine_map_resolution > 0.0) || !(param->map_resolution > 0.0))
    return CSM_ERR_INVALID_ARG;
  auto* b = new csm_backend();
  b->device = device;
  b->p = *param;
  int st = csm_create(device, &b->ctx);
  if (st == CSM_OK) st = csm_create(device, &b->ctx_stack);
  if (st == CSM_OK && param->use_optimize_scan_match) st = csm_create(device, &b->ctx_coarse);
  if (st != CSM_OK) {
    csm_backend_destroy(b);
    return st;
  }
  *out = b;
  return CSM_OK;
}

int csm_backend_destroy(csm_backend* b) {
  if (!b) return CSM_OK;
  for (auto& mp : b->pairs)
    for (auto*& m : mp.map)
      if (m) csm_gridmap_destroy(m);
  for (csm_ctx* c : {b->ctx, b->ctx_coarse, b->ctx_stack})
    if (c) csm_destroy(c);
  delete b;
  return CSM_OK;
}

const char* csm_backend_last_error(const csm_backend* b) { return b ? b->err.c_str() : "null back-end"; }

int csm_backend_add_scan(csm_backend* b, const double* pts, int32_t n, const double pose[3], int32_t* id) {
  if (!b || !pose || !id || n < 0 || (n > 0 && !pts)) return CSM_ERR_INVALID_ARG;
  KeptScan ks;
  ks.raw.assign(pts, pts + 2 * (size_t)n);
  scale_points(pts, n, 1 / b->p.coarse_map_resolution, ks.coarse);  // CreateFrom (:99-115)
  scale_points(pts, n, 1 / b->p.fine_map_resolution, ks.fine);
  std::memcpy(ks.pose, pose, sizeof(ks.pose));
  b->scans.push_back(std::move(ks));
  *id = (int32_t)b->scans.size() - 1;
  return CSM_OK;
}

int csm_backend_set_scan_pose(csm_backend* b, int32_t id, const double pose[3]) {
  if (!b || !pose || id < 0 || id >= (int32_t)b->scans.size()) return CSM_ERR_INVALID_ARG;
  std::memcpy(b->scans[(size_t)id].pose, pose, sizeof(double) * 3);
  return CSM_OK;
}

int csm_backend_map(csm_backend* b, int32_t slot, int32_t which, csm_gridmap** m) {
  if (!b || !m || slot < 0 || which < 0 || which > 1) return CSM_ERR_INVALID_ARG;
  *m = slot < (int32_t)b->pairs.size() ? b->pairs[(size_t)slot].map[which] : nullptr;
  return CSM_OK;
}

int csm_backend_scan_match(csm_backend* b, csm_gridmap* pub, const double cur[3], csm_backend_job* jobs,
                           int32_t n_jobs) {
  if (!b || !cur || n_jobs < 0 || (n_jobs > 0 && !jobs)) return CSM_ERR_INVALID_ARG;
  const csm_backend_param& p = b->p;
  for (int32_t j = 0; j < n_jobs; ++j) {
    const csm_backend_job& jb = jobs[j];
    if (jb.n_points < 0 || (jb.n_points > 0 && !jb.points_m) || jb.n_chain < 0 || (jb.n_chain > 0 && !jb.chain_ids))
      return b->fail(CSM_ERR_INVALID_ARG, "bad job");
    for (int32_t k = 0; k < jb.n_chain; ++k)
      if (jb.chain_ids[k] < 0 || jb.chain_ids[k] >= (int32_t)b->scans.size())
        return b->fail(CSM_ERR_INVALID_ARG, "chain id of no kept scan");
  }
  int st;
  // per job: range data at each resolution, the rebuilt map pair, MapSizeCheck
  std::vector<std::vector<double>> cpts((size_t)n_jobs), fpts((size_t)n_jobs);
  std::vector<csm_gridmap_state> fst((size_t)n_jobs);
  for (int32_t j = 0; j < n_jobs; ++j) {
    csm_backend_job& jb = jobs[j];
    scale_points(jb.points_m, jb.n_points, 1 / p.coarse_map_resolution, cpts[(size_t)j]);  // :268-272
    scale_points(jb.points_m, jb.n_points, 1 / p.fine_map_resolution, fpts[(size_t)j]);
    if ((st = ensure_pair(b, j)) != CSM_OK) return st;
    MapPair& mp = b->pairs[(size_t)j];
    for (int k = 0; k < 2; ++k)
      if ((st = reset_map(b, mp.map[k], k, jb, cur)) != CSM_OK) return b->fail(st, "ResetScanMatchMapWithRangeVec");
    for (int k = 0; k < 2; ++k)  // ScanMatchers::MapSizeCheck (scan_matchers.h:195-199)
      if ((st = csm::map_size_check(mp.map[k], jb.pose, p.range_max, p.levels[0].search_space_size)) != CSM_OK)
        return b->fail(st, "MapSizeCheck");
    if ((st = csm_gridmap_get_state(mp.map[1], &fst[(size_t)j])) != CSM_OK) return st;
    std::memcpy(jb.cov, (const double[9]){1, 0, 0, 0, 1, 0, 0, 0, 1}, sizeof(jb.cov));
    jb.score = 0.0;
    jb.optimize_cost = 0.0;
    jb.map_penalty = 1.0;
  }
  // correlative levels: all jobs in one batch over a stack of the fine maps
  // when they share one geometry, else job by job
  bool batch = n_jobs > 1 && !p.use_optimize_scan_match;
  for (int32_t j = 1; batch && j < n_jobs; ++j)
    batch = same_geometry(fst[0], fst[(size_t)j]) && jobs[j].use_fine_scan_match == jobs[0].use_fine_scan_match;
  if (batch) {
    std::vector<csm_gridmap*> fine((size_t)n_jobs);
    std::vector<double> pts, poses((size_t)n_jobs * 3), covs((size_t)n_jobs * 9), scores((size_t)n_jobs);
    std::vector<int64_t> off(1, 0);
    std::vector<int32_t> gidx((size_t)n_jobs);
    for (int32_t j = 0; j < n_jobs; ++j) {
      fine[(size_t)j] = b->pairs[(size_t)j].map[1];
      pts.insert(pts.end(), fpts[(size_t)j].begin(), fpts[(size_t)j].end());
      off.push_back(off.back() + jobs[j].n_points);
      gidx[(size_t)j] = j;
      std::memcpy(&poses[(size_t)3 * j], jobs[j].pose, sizeof(double) * 3);
      std::memcpy(&covs[(size_t)9 * j], jobs[j].cov, sizeof(double) * 9);
    }
    if ((st = csm_set_grid_stack_gridmaps(b->ctx_stack, fine.data(), n_jobs)) != CSM_OK ||
        (st = csm_scan_matchers_batch_grids(b->ctx_stack, n_jobs, pts.data(), off.data(), gidx.data(), p.levels,
                                            jobs[0].use_fine_scan_match, poses.data(), covs.data(),
                                            scores.data())) != CSM_OK)
      return b->fail(st, std::string("batched ScanMatchers: ") + csm_last_error(b->ctx_stack));
    for (int32_t j = 0; j < n_jobs; ++j) {
      std::memcpy(jobs[j].pose, &poses[(size_t)3 * j], sizeof(double) * 3);
      std::memcpy(jobs[j].cov, &covs[(size_t)9 * j], sizeof(double) * 9);
      jobs[j].score = scores[(size_t)j];
    }
  } else {
    const csm::MatchersConfig cfg{p.levels, p.use_optimize_scan_match, p.optimize_failed_cost, p.optimize,
                                  p.range_max};
    for (int32_t j = 0; j < n_jobs; ++j) {
      csm_backend_job& jb = jobs[j];
      MapPair& mp = b->pairs[(size_t)j];
      std::string why;
      if ((st = csm::scan_matchers_on_maps(b->ctx, b->ctx_coarse, mp.map[0], mp.map[1], cpts[(size_t)j].data(),
                                           fpts[(size_t)j].data(), jb.n_points, cfg, jb.use_fine_scan_match, jb.pose,
                                           jb.cov, &jb.score, &jb.optimize_cost, &why)) != CSM_OK)
        return b->fail(st, why);
    }
  }
  // MapCheckPenalize(pub range data, best_pose, use_logistic = true) (:315-317, :573-595)
  for (int32_t j = 0; j < n_jobs && pub && p.use_map_check_feedback; ++j) {
    csm_backend_job& jb = jobs[j];
    std::vector<double> pp;
    scale_points(jb.points_m, jb.n_points, 1 / p.map_resolution, pp);
    double penalty = 1.0;
    if ((st = csm_gridmap_feedback_penalty(pub, pp.data(), jb.n_points, nullptr, jb.pose, p.map_check_point_num,
                                           p.map_check_bound_tolerance, p.map_check_penalty_gain, 0, &penalty)) !=
        CSM_OK)
      return b->fail(st, "MapFeedbackResponsePenalty");
    jb.map_penalty = (1 / (1 + std::exp(-10 * (penalty - 0.4))));
  }
  for (int32_t j = 0; j < n_jobs; ++j) {
    jobs[j].score *= jobs[j].map_penalty;  // :318-319
    jobs[j].score = (jobs[j].score > 1.0) ? (1.0) : (jobs[j].score);
  }
  return CSM_OK;
}

}  // extern "C"
