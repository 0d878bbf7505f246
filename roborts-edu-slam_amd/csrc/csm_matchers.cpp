// csm_matchers.cpp — ScanMatchers::ScanMatch over device-resident maps
// (csm_matchers.hpp). Host control flow of scan_matchers.h:179-289 over the
// public C-ABI: every map and every matcher stays on the GPU.
#include "csm_matchers.hpp"

#include <cstring>

namespace csm {

int map_size_check(csm_gridmap* m, const double pose[3], double range_max, double offset) {
  csm_gridmap_state s{};
  int st = csm_gridmap_get_state(m, &s);
  if (st != CSM_OK) return st;
  // GetMapCoordsPose (scale_factor_ * w + scale_factor_ * offset) and GetCellLength
  const double sc = s.scale_factor;
  const double cx = sc * pose[0] + sc * s.offset_x, cy = sc * pose[1] + sc * s.offset_y;
  const double max_size = (range_max + offset) / s.resolution;
  int32_t inside = 0;
  return csm_gridmap_update_bound(m, cx - max_size, cy - max_size, cx + max_size, cy + max_size, &inside);
}

int scan_matchers_on_maps(csm_ctx* fine_ctx, csm_ctx* coarse_ctx, csm_gridmap* coarse_map, csm_gridmap* fine_map,
                          const double* coarse_pts, const double* fine_pts, int32_t n, const MatchersConfig& cfg,
                          int use_fine, double pose[3], double cov[9], double* score, double* opt_cost,
                          std::string* err) {
  auto fail = [&](int st, const char* what, csm_ctx* c) {
    if (err) *err = std::string(what) + (c ? std::string(": ") + csm_last_error(c) : std::string());
    return st;
  };
  int st;
  *opt_cost = 0.0;
  const double margin = cfg.levels[0].search_space_size;  // coarse window for both maps (:195-199)
  if ((st = map_size_check(coarse_map, pose, cfg.range_max, margin)) != CSM_OK)
    return fail(st, "MapSizeCheck(coarse)", nullptr);
  if ((st = map_size_check(fine_map, pose, cfg.range_max, margin)) != CSM_OK)
    return fail(st, "MapSizeCheck(fine)", nullptr);
  if ((st = csm_set_grid_gridmap(fine_ctx, fine_map)) != CSM_OK) return fail(st, "csm_set_grid_gridmap", fine_ctx);
  if (!cfg.use_optimize_scan_match) {  // the correlative levels in one call
    if ((st = csm_scan_matchers(fine_ctx, fine_pts, n, cfg.levels, use_fine, pose, cov, score)) != CSM_OK)
      return fail(st, "csm_scan_matchers", fine_ctx);
    return CSM_OK;
  }
  if (!coarse_ctx) return fail(CSM_ERR_INVALID_ARG, "Gauss-Newton matcher without a coarse context", nullptr);
  double sum = 0.0, process[3] = {pose[0], pose[1], pose[2]}, cost = 0.0, resp = 0.0;
  int times = 0;
  if ((st = csm_set_grid_gridmap(coarse_ctx, coarse_map)) != CSM_OK ||
      (st = csm_optimize_scan_match(coarse_ctx, coarse_pts, n, &cfg.optimize, process, &cost)) != CSM_OK)
    return fail(st, "csm_optimize_scan_match", coarse_ctx);
  *opt_cost = cost;
  sum = cfg.optimize_failed_cost / (cost + cfg.optimize_failed_cost);  // :211
  times++;
  if (!use_fine || cost > cfg.optimize_failed_cost) {  // :224-242
    sum = 0.0;
    times--;
    std::memcpy(process, pose, sizeof(process));
    if ((st = csm_scan_match(fine_ctx, fine_pts, n, &cfg.levels[0], process, cov, &resp, nullptr)) != CSM_OK)
      return fail(st, "csm_scan_match(coarse)", fine_ctx);
    sum += resp;
    times++;
  }
  if (use_fine) {
    for (int k = 1; k <= 2; ++k) {  // fine, super-fine (:247-261)
      if ((st = csm_scan_match(fine_ctx, fine_pts, n, &cfg.levels[k], process, cov, &resp, nullptr)) != CSM_OK)
        return fail(st, "csm_scan_match", fine_ctx);
      sum += resp;
      times++;
    }
  }
  std::memcpy(pose, process, sizeof(process));
  *score = sum / times;  // :281
  return CSM_OK;
}

}  // namespace csm
