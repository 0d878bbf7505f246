// csm_optimize_host.cpp — the Gauss-Newton matcher's host loop
// (BasedOptimizeScanMatch, optimize_scan_matcher.h:60-237): per-iteration
// control flow, glibc sincos, Eigen's 3x3 LDLT solve and UpdatePose around
// optimize_cost_kernel (csm_optimize.hip).
#include "csm_host.hpp"

namespace csmh {

// ---- Gauss-Newton scan matcher ------------------------------------------------
// BasedOptimizeScanMatch (optimize_scan_matcher.h:60-237; SURVEY.md 8f row
// f3). The device evaluates UpdateCost for every active scan per launch
// (csm_optimize.hip); the host keeps the reference's per-iteration control
// flow, glibc cos/sin, the 3x3 LDLT solve and UpdatePose.


// util::MaxAbxLimit (util/slam_util.h:79-86)
double max_abs_limit(double value, double limit) {
  if (value > std::fabs(limit))
    value = std::fabs(limit);
  else if (value < -std::fabs(limit))
    value = -std::fabs(limit);
  return value;
}

// util::NormalizeAngle (util/slam_util.h:103-111)
double normalize_angle(double a) {
  double n = std::fmod(std::fmod(a, 2.0 * M_PI) + 2.0 * M_PI, 2.0 * M_PI);
  if (n > M_PI) n -= 2.0 * M_PI;
  return n;
}

// H_.ldlt().solve(b_) (optimize_scan_matcher.h:136-142): Eigen 3.3
// LDLT<Matrix3d, Lower>. Factor: diagonal pivoting on the trailing corner
// (first maximum wins), symmetric swaps through the lower triangle, then
// a_kk -= a_k. . (D a_k.)^T and the column below scaled by the pivot.
// Solve: P, unit-lower rows, D pseudo-inverse (|d| > DBL_MIN), unit-upper
// rows from the bottom, P^T. s = lower triangle of the symmetric H as
// {H00, H10, H11, H20, H21, H22}.
void ldlt_solve3(const double s[6], const double rhs[3], double out[3]) {
  double a[3][3] = {{s[0], s[1], s[3]}, {s[1], s[2], s[4]}, {s[3], s[4], s[5]}};
  int tr[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) {
    int big = k;
    double bv = std::fabs(a[k][k]);
    for (int i = k + 1; i < 3; ++i)
      if (std::fabs(a[i][i]) > bv) {
        bv = std::fabs(a[i][i]);
        big = i;
      }
    tr[k] = big;
    if (big != k) {
      for (int j = 0; j < k; ++j) std::swap(a[k][j], a[big][j]);
      for (int i = big + 1; i < 3; ++i) std::swap(a[i][k], a[i][big]);
      std::swap(a[k][k], a[big][big]);
      for (int i = k + 1; i < big; ++i) {
        const double t = a[i][k];
        a[i][k] = a[big][i];
        a[big][i] = t;
      }
    }
    if (k > 0) {
      double t[2];
      for (int i = 0; i < k; ++i) t[i] = a[i][i] * a[k][i];
      a[k][k] -= (k == 1) ? (a[k][0] * t[0]) : (a[k][0] * t[0] + a[k][1] * t[1]);
      if (k == 1) a[2][1] -= a[2][0] * t[0];
    }
    const double akk = a[k][k];
    const bool valid = std::fabs(akk) > 0.0;
    if (k == 0 && !valid) {
      tr[0] = 0;
      tr[1] = 1;
      tr[2] = 2;
      break;
    }
    if (k < 2 && valid)
      for (int r = k + 1; r < 3; ++r) a[r][k] /= akk;
  }
  double d[3] = {rhs[0], rhs[1], rhs[2]};
  for (int k = 0; k < 3; ++k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  d[1] -= a[1][0] * d[0];
  d[2] -= (a[2][0] * d[0] + a[2][1] * d[1]);
  for (int i = 0; i < 3; ++i) d[i] = (std::fabs(a[i][i]) > DBL_MIN) ? d[i] / a[i][i] : 0.0;
  d[1] -= a[2][1] * d[2];
  d[0] -= (a[1][0] * d[1] + a[2][0] * d[2]);
  for (int k = 2; k >= 0; --k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  out[0] = d[0];
  out[1] = d[1];
  out[2] = d[2];
}

// n_scans scans whose points are resident in c->pts at offsets off (n+1,
// relative). poses world in/out, costs out; iters (nullable) = UpdateCost
// evaluations per scan.
int optimize_batch(csm_ctx* c, int32_t n_scans, const int64_t* off, const csm_optimize_param& P, double* poses,
                   double* costs, int32_t* iters) {
  const Geometry geo(c->info);
  const bool ready = map_ready(c);
  // per scan: kSkip = invalid input (pose untouched, kMaxCost), kRun =
  // iterating, kDone = converged or out of iterations, kNan = NaN step
  enum : uint8_t { kSkip = 0, kRun = 1, kDone = 2, kNan = 3 };
  std::vector<double> est((size_t)n_scans * 3), cost((size_t)n_scans, 0.0), last((size_t)n_scans, 0.0);
  std::vector<uint8_t> state((size_t)n_scans, kSkip);
  int n_active = 0;
  for (int32_t s = 0; s < n_scans; ++s) {
    if (iters) iters[s] = 0;
    if (!ready || off[s + 1] == off[s]) continue;  // :73-76
    geo.to_map(poses + 3 * s, &est[(size_t)3 * s]);  // GetMapCoordsPose (:79-80)
    // cost_ starts at 0.0 here; the reference returns its stale member when
    // iterate_max_times <= 0 (no iteration) — defined as 0.0
    state[(size_t)s] = (P.iterate_max_times > 0) ? kRun : kDone;
    n_active += state[(size_t)s] == kRun;
  }
  std::vector<uint8_t> active(state);
  for (auto& a : active) a = (a == kRun);
  hipError_t e;
  if ((e = c->opt_off.ensure(sizeof(int64_t) * (size_t)(n_scans + 1))) != hipSuccess ||
      (e = c->opt_scans.ensure(sizeof(csm::OptScan) * (size_t)n_scans)) != hipSuccess ||
      (e = c->opt_sums.ensure(sizeof(csm::OptSums) * (size_t)n_scans)) != hipSuccess ||
      (e = c->h_opt_scans.ensure(sizeof(csm::OptScan) * (size_t)n_scans)) != hipSuccess ||
      (e = c->h_opt_sums.ensure(sizeof(csm::OptSums) * (size_t)n_scans)) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(optimize)");
  if ((e = hipMemcpyAsync(c->opt_off.p, off, sizeof(int64_t) * (size_t)(n_scans + 1), hipMemcpyHostToDevice,
                          c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(optimize offsets)");
  csm::OptArgs A{};
  A.grid = c->d_grid;
  A.size_x = c->info.size_x;
  A.size_y = c->info.size_y;
  A.outside = c->outside;
  A.pts = (const double*)c->pts.p;
  A.offsets = (const int64_t*)c->opt_off.p;
  A.scans = (const csm::OptScan*)c->opt_scans.p;
  A.out = (csm::OptSums*)c->opt_sums.p;
  auto* hs = (csm::OptScan*)c->h_opt_scans.p;
  auto* hr = (const csm::OptSums*)c->h_opt_sums.p;
  const double mres = geo.mres;  // map_resolution_ = GetCellLength() (:82)
  for (int iter = 0; iter < P.iterate_max_times && n_active > 0; ++iter) {
    for (int32_t s = 0; s < n_scans; ++s) {
      csm::OptScan& o = hs[s];
      o.active = active[(size_t)s];
      if (!o.active) continue;
      const double* m = &est[(size_t)3 * s];
      csm::host_sincos(m[2], &o.s, &o.c);  // rotation (:96-97), de_s (:200-201)
      o.tx = m[0];
      o.ty = m[1];
    }
    if ((e = hipMemcpyAsync(c->opt_scans.p, hs, sizeof(csm::OptScan) * (size_t)n_scans, hipMemcpyHostToDevice,
                            c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(optimize state)");
    if (c->profiling && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = csm::launch_optimize_cost(A, n_scans, c->stream)) != hipSuccess)
      return c->hip_fail(e, "optimize_cost_kernel");
    if (c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = hipMemcpyAsync(c->h_opt_sums.p, c->opt_sums.p, sizeof(csm::OptSums) * (size_t)n_scans,
                            hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(optimize sums)");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(optimize)");
    if (c->profiling) {
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
      double in_map = 0.0;
      for (int32_t s = 0; s < n_scans; ++s)
        if (active[(size_t)s]) in_map += hr[s].valid;
      c->account("optimize_cost_kernel", ms, 16.0 * in_map, 0.0);  // 4 fp32 corners per point in the map
    }
    for (int32_t s = 0; s < n_scans; ++s) {
      if (!active[(size_t)s]) continue;
      const csm::OptSums& r = hr[s];
      last[(size_t)s] = cost[(size_t)s];  // :88
      const int valid_point = 1 + r.valid;
      cost[(size_t)s] = r.v[0] * (kOptCostPointSize / valid_point);  // :220
      if (iters) iters[s] = iter + 1;
      double det[3];
      ldlt_solve3(&r.v[1], &r.v[7], det);  // CalculateDet (:101, :136-142)
      double* m = &est[(size_t)3 * s];
      const bool nan = std::isnan(det[0]) || std::isnan(det[1]) || std::isnan(det[2]);  // :103-106
      if (nan || (iter > 0 && (last[(size_t)s] - cost[(size_t)s] < P.cost_decrease_threshold ||
                               cost[(size_t)s] < P.cost_min_threshold))) {  // :112-118
        state[(size_t)s] = nan ? kNan : kDone;
        active[(size_t)s] = 0;
        --n_active;
        continue;
      }
      m[0] += max_abs_limit(det[0], P.max_update_distance / mres);  // UpdatePose (:144-152)
      m[1] += max_abs_limit(det[1], P.max_update_distance / mres);
      m[2] += max_abs_limit(det[2], P.max_update_angle);
    }
  }
  for (int32_t s = 0; s < n_scans; ++s) {
    if (state[(size_t)s] == kSkip || state[(size_t)s] == kNan) {
      costs[s] = kOptMaxCost;  // pose untouched
      continue;
    }
    double* m = &est[(size_t)3 * s];
    m[2] = normalize_angle(m[2]);    // :126
    geo.to_world(m, poses + 3 * s);  // GetWorldCoordsPose (:128)
    costs[s] = cost[(size_t)s];
  }
  return CSM_OK;
}

}  // namespace csmh

using namespace csmh;

extern "C" {

int csm_optimize_scan_match_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                                  const csm_optimize_param* param, double* poses, double* costs,
                                  int32_t* iterations) {
  if (!c || !param || (n_scans > 0 && (!poses || !costs))) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
  int st;
  if ((st = check_offsets(c, n_scans, offsets)) != CSM_OK) return st;
  if (n_scans == 0) return CSM_OK;
  const int64_t n_total = offsets[n_scans] - offsets[0];
  if ((st = check_points(c, pts, n_total)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  std::vector<int64_t> off(offsets, offsets + n_scans + 1);
  for (auto& o : off) o -= offsets[0];
  if ((st = upload_points(c, pts + 2 * offsets[0], n_total)) != CSM_OK) return st;
  return optimize_batch(c, n_scans, off.data(), *param, poses, costs, iterations);
}

int csm_optimize_scan_match(csm_ctx* c, const double* pts, int32_t n_points, const csm_optimize_param* param,
                            double pose[3], double* cost) {
  if (!c || !cost || !pose) return CSM_ERR_INVALID_ARG;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  const int64_t off[2] = {0, n_points};
  return csm_optimize_scan_match_batch(c, 1, pts, off, param, pose, cost, nullptr);
}

int csm_optimize_update_cost(csm_ctx* c, const double* pts, int32_t n_points, const double est_map[3],
                             double* cost, double H[9], double b[3]) {
  if (!c || !est_map || !cost || !H || !b) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
  int st;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  if ((st = upload_points(c, pts, n_points)) != CSM_OK) return st;
  const int64_t off[2] = {0, n_points};
  hipError_t e;
  if ((e = c->opt_off.ensure(sizeof(off))) != hipSuccess || (e = c->opt_scans.ensure(sizeof(csm::OptScan))) != hipSuccess ||
      (e = c->opt_sums.ensure(sizeof(csm::OptSums))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(optimize)");
  csm::OptScan o{};
  csm::host_sincos(est_map[2], &o.s, &o.c);
  o.tx = est_map[0];
  o.ty = est_map[1];
  o.active = 1;
  csm::OptArgs A{};
  A.grid = c->d_grid;
  A.size_x = c->info.size_x;
  A.size_y = c->info.size_y;
  A.outside = c->outside;
  A.pts = (const double*)c->pts.p;
  A.offsets = (const int64_t*)c->opt_off.p;
  A.scans = (const csm::OptScan*)c->opt_scans.p;
  A.out = (csm::OptSums*)c->opt_sums.p;
  csm::OptSums r{};
  if ((e = hipMemcpyAsync(c->opt_off.p, off, sizeof(off), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(c->opt_scans.p, &o, sizeof(o), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = csm::launch_optimize_cost(A, 1, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(&r, c->opt_sums.p, sizeof(r), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return c->hip_fail(e, "optimize_cost_kernel");
  *cost = r.v[0] * (kOptCostPointSize / (1 + r.valid));
  const double h[9] = {r.v[1], r.v[2], r.v[4], r.v[2], r.v[3], r.v[5], r.v[4], r.v[5], r.v[6]};
  std::memcpy(H, h, sizeof(h));
  b[0] = r.v[7];
  b[1] = r.v[8];
  b[2] = r.v[9];
  return CSM_OK;
}

}  // extern "C"
