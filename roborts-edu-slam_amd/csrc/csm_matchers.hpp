// csm_matchers.hpp — ScanMatchers::ScanMatch over device-resident maps, the
// composition the front-end (csm_frontend.cpp) and the back-end
// (csm_backend.cpp) share. Built from the public C-ABI only. Not installed.
#pragma once

#include <string>

#include "csm.h"
#include "csm_gridmap.h"

namespace csm {

// What ScanMatchers reads besides the maps (scan_matchers.h:160-416,
// ScanMatchParamInit :307-355).
struct MatchersConfig {
  const csm_param* levels;         // coarse, fine, super-fine
  int use_optimize_scan_match;
  double optimize_failed_cost;
  csm_optimize_param optimize;
  double range_max;                // MapSizeCheck margin (scan_matchers.h:365-390)
};

// ScanMatchers::ScanMatch (scan_matchers.h:179-289): MapSizeCheck on both
// maps, the optional Gauss-Newton matcher on coarse_map (coarse_ctx), the
// correlative coarse level when it is off, failed or !use_fine, then fine and
// super-fine; every correlative level on fine_map (fine_ctx). coarse_pts /
// fine_pts are the scan in each map's cells. pose, cov in/out; *score = the
// mean response (:281); *opt_cost = the optimiser's cost (0 when not run).
// coarse_ctx may be null when use_optimize_scan_match is off.
int scan_matchers_on_maps(csm_ctx* fine_ctx, csm_ctx* coarse_ctx, csm_gridmap* coarse_map, csm_gridmap* fine_map,
                          const double* coarse_pts, const double* fine_pts, int32_t n, const MatchersConfig& cfg,
                          int use_fine, double pose[3], double cov[9], double* score, double* opt_cost,
                          std::string* err);

// ScanMatchers::MapSizeCheck (scan_matchers.h:365-390) for one map.
int map_size_check(csm_gridmap* m, const double pose[3], double range_max, double offset);

}  // namespace csm
