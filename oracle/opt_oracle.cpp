// opt_oracle.cpp — CPU restatement of RoboRTS-Edu-SLAM's Gauss-Newton scan
// matcher (src/scan_match/optimize_scan_matcher.h), used ONLY as test
// infrastructure.
//
// *** TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT. ***
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// this library (liboracle.so), as the checker / CPU baseline.
//
// PARITY UNPINNED by the reference (no tests, unbuildable: Eigen absent). The
// per-point arithmetic follows optimize_scan_matcher.h expression by
// expression; the 3x3 solve restates Eigen 3.3's LDLT<Matrix3d, Lower>
// (ldlt_inplace<Lower>::unblocked with diagonal pivoting, then
// _solve_impl: P, unit-lower solve unrolled row-wise for a fixed 3-vector,
// D pseudo-inverse with tolerance DBL_MIN, unit-upper solve, P^T). Eigen's
// source is not in this image, so that part is pinned only by this
// restatement and by tests/test_optimize.py's algebraic checks.
//
// Defined behaviour where the reference has none: a bilinear corner read at
// ceil(x) == size_x or ceil(y) == size_y (PointInMap admits
// 0 < x < size_x) goes through GetCell's flat index y*size_x + x exactly as
// the reference (grid_map_base.h:352-354); a flat index past the last cell
// reads outside_value (the reference reads past its array: UB).
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>

#include "oracle_math.hpp"

extern "C" {
struct oracle_map_c {  // csm_oracle.cpp
  const float* cells;
  int64_t stride_floats;
  int32_t size_x, size_y;
  double resolution;
  double offset_x, offset_y;
  int32_t update_index;
  float outside_value;
};
}

namespace {

// OptimizeScanMatchParam (optimize_scan_matcher.h:33-58) = csm_optimize_param.
struct OptParam {
  int32_t iterate_max_times;
  int32_t reserved;
  double cost_decrease_threshold;
  double cost_min_threshold;
  double max_update_distance;
  double max_update_angle;
};

constexpr double kCostPointSize = 1000;             // optimize_scan_matcher.h:234
constexpr double kMaxCost = 1.0 * kCostPointSize;   // :235

double cell(const oracle_map_c& m, int x, int y) {  // GetGridProbValue (occu_grid_map.h:395-397)
  const int64_t idx = (int64_t)y * m.size_x + x;
  if (idx < 0 || idx >= (int64_t)m.size_x * m.size_y) return (double)m.outside_value;
  return (double)m.cells[idx * m.stride_floats];
}

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

// H_.ldlt().solve(b_) (optimize_scan_matcher.h:136-142), Eigen 3.3 LDLT.
// H row-major 3x3; only its lower triangle is read.
void ldlt_solve(const double Hin[9], const double b[3], double x[3]) {
  double a[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) a[i][j] = Hin[3 * i + j];
  int tr[3];
  double temp[3];
  const int n = 3;
  for (int k = 0; k < n; ++k) {
    // largest diagonal element of the trailing corner (first one on ties)
    int big = k;
    double bv = std::fabs(a[k][k]);
    for (int i = k + 1; i < n; ++i)
      if (std::fabs(a[i][i]) > bv) {
        bv = std::fabs(a[i][i]);
        big = i;
      }
    tr[k] = big;
    if (k != big) {  // symmetric swap through the lower triangle
      for (int j = 0; j < k; ++j) std::swap(a[k][j], a[big][j]);
      for (int i = big + 1; i < n; ++i) std::swap(a[i][k], a[i][big]);
      std::swap(a[k][k], a[big][big]);
      for (int i = k + 1; i < big; ++i) {
        const double t = a[i][k];
        a[i][k] = a[big][i];
        a[big][i] = t;
      }
    }
    const int rs = n - k - 1;
    if (k > 0) {
      for (int i = 0; i < k; ++i) temp[i] = a[i][i] * a[k][i];
      double dot = a[k][0] * temp[0];
      for (int i = 1; i < k; ++i) dot = dot + a[k][i] * temp[i];
      a[k][k] -= dot;
      for (int r = k + 1; r < n; ++r) {
        double d = a[r][0] * temp[0];
        for (int i = 1; i < k; ++i) d = d + a[r][i] * temp[i];
        a[r][k] -= d;
      }
    }
    const double akk = a[k][k];
    const bool valid = std::fabs(akk) > 0.0;
    if (k == 0 && !valid) {  // the whole diagonal is zero
      for (int j = 0; j < n; ++j) tr[j] = j;
      break;
    }
    if (rs > 0 && valid)
      for (int r = k + 1; r < n; ++r) a[r][k] /= akk;
  }
  // dst = P b
  double d[3] = {b[0], b[1], b[2]};
  for (int k = 0; k < n; ++k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  // L^-1 (unit lower, unrolled: row dot products)
  d[1] -= a[1][0] * d[0];
  d[2] -= (a[2][0] * d[0] + a[2][1] * d[1]);
  // D^+ (tolerance numeric_limits<double>::min())
  for (int i = 0; i < n; ++i) {
    if (std::fabs(a[i][i]) > DBL_MIN)
      d[i] /= a[i][i];
    else
      d[i] = 0.0;
  }
  // L^-T (unit upper, unrolled from the bottom)
  d[1] -= a[2][1] * d[2];
  d[0] -= (a[1][0] * d[1] + a[2][0] * d[2]);
  // P^T
  for (int k = n - 1; k >= 0; --k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  x[0] = d[0];
  x[1] = d[1];
  x[2] = d[2];
}

// BasedOptimizeScanMatch::UpdateCost (optimize_scan_matcher.h:154-221).
// est: map-cell pose; H row-major, all 9 entries accumulated.
double update_cost(const oracle_map_c& m, const double* pts, int n, const double est[3], double H[9],
                   double b[3]) {
  double s, c;  // one sincos per evaluation: rotation (:96-97) and de_s (:200-201)
  ref_sincos(est[2], &s, &c);
  const double r00 = c, r01 = -s, r10 = s, r11 = c;
  double cost = 0.0;
  int valid_point = 1;
  for (int p = 0; p < n; ++p) {
    const double lx = pts[2 * p], ly = pts[2 * p + 1];
    const double x = (r00 * lx + r01 * ly) + est[0];  // rotation * local_point + translation (:167)
    const double y = (r10 * lx + r11 * ly) + est[1];
    if (!(x > 0 && x < m.size_x && y > 0 && y < m.size_y)) continue;  // PointInMap (grid_map_base.h:330-337)
    const double x0 = std::floor(x), y0 = std::floor(y);
    const double x1 = std::ceil(x), y1 = std::ceil(y);
    const double p00 = cell(m, (int)x0, (int)y0);
    const double p01 = cell(m, (int)x0, (int)y1);
    const double p10 = cell(m, (int)x1, (int)y0);
    const double p11 = cell(m, (int)x1, (int)y1);
    double r = ((y - y0) * (p11 * (x - x0) + p01 * (x1 - x)) + (y1 - y) * (p10 * (x - x0) + p00 * (x1 - x)));
    r = (r >= 0) ? ((r <= 1) ? (r) : (1)) : (0);
    const double error = 1 - r;
    cost += (error * error);
    const double ds02 = (-s * lx - c * ly);
    const double ds12 = (c * lx - s * ly);
    const double dm0 = (((y - y0)) * (p11 - p01) + ((y1 - y)) * (p10 - p00));
    const double dm1 = (((x - x0)) * (p11 - p10) + ((x1 - x)) * (p01 - p00));
    // J = -de_m * de_s with de_s = [1 0 ds02; 0 1 ds12]
    const double n0 = -dm0, n1 = -dm1;
    const double J[3] = {n0 * 1.0 + n1 * 0.0, n0 * 0.0 + n1 * 1.0, n0 * ds02 + n1 * ds12};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) H[3 * i + j] += J[i] * J[j];
    for (int i = 0; i < 3; ++i) b[i] += (-J[i]) * error;
    valid_point++;
  }
  cost *= (kCostPointSize / valid_point);
  return cost;
}

}  // namespace

extern "C" {

int oracle_optimize_param_size(void) { return (int)sizeof(OptParam); }

// BasedOptimizeScanMatch::ScanMatch (optimize_scan_matcher.h:68-132): pose
// (world) in/out; returns the cost (kMaxCost on invalid input or a NaN step,
// pose untouched then). iterations (nullable): UpdateCost evaluations.
double oracle_optimize_scan_match(const oracle_map_c* mc, const double* pts, int n, const void* param,
                                  double pose[3], int* iterations) {
  OptParam P;
  std::memcpy(&P, param, sizeof(P));
  if (iterations) *iterations = 0;
  if (mc->update_index < 0 || n == 0) return kMaxCost;  // :73-76
  const double sf = 1.0 / mc->resolution;               // scale_factor_ (grid_map_base.h:50)
  double est[3] = {sf * pose[0] + sf * mc->offset_x, sf * pose[1] + sf * mc->offset_y, pose[2]};  // :80
  const double map_resolution = 1 / sf;                  // GetCellLength (:82)
  double cost = 0.0, last_cost = 0.0;
  for (int iter = 0; iter < P.iterate_max_times; ++iter) {
    last_cost = cost;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
    cost = update_cost(*mc, pts, n, est, H, b);
    if (iterations) *iterations = iter + 1;
    double det[3];
    ldlt_solve(H, b, det);
    if (std::isnan(det[0]) || std::isnan(det[1]) || std::isnan(det[2])) return kMaxCost;  // :103-106
    if (iter > 0 && (last_cost - cost < P.cost_decrease_threshold || cost < P.cost_min_threshold)) break;
    est[0] += max_abs_limit(det[0], P.max_update_distance / map_resolution);  // UpdatePose :144-152
    est[1] += max_abs_limit(det[1], P.max_update_distance / map_resolution);
    est[2] += max_abs_limit(det[2], P.max_update_angle);
  }
  est[2] = normalize_angle(est[2]);  // :126
  // GetWorldCoordsPose through Eigen's affine inverse (grid_map_base.h:83-87)
  const double tx = sf * mc->offset_x, ty = sf * mc->offset_y;
  const double det = sf * sf - 0.0 * 0.0;
  const double a = sf * (1.0 / det);
  pose[0] = a * est[0] + (-(a * tx));
  pose[1] = a * est[1] + (-(a * ty));
  pose[2] = est[2];
  return cost;
}

// One UpdateCost evaluation at a map-cell pose (test hook).
double oracle_optimize_update_cost(const oracle_map_c* mc, const double* pts, int n, const double est[3],
                                   double H[9], double b[3]) {
  for (int i = 0; i < 9; ++i) H[i] = 0.0;
  for (int i = 0; i < 3; ++i) b[i] = 0.0;
  return update_cost(*mc, pts, n, est, H, b);
}

void oracle_ldlt_solve(const double H[9], const double b[3], double x[3]) { ldlt_solve(H, b, x); }

}  // extern "C"
