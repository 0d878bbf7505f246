// csm_oracle.cpp — CPU restatement of RoboRTS-Edu-SLAM's correlative scan
// matcher, used ONLY as test infrastructure.
//
// *** TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT. ***
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker / CPU baseline. The product
// (libroborts_csm.so) never links, loads or calls it.
//
// PARITY UNPINNED: the reference ships no golden vectors or known-answer tests
// for this path (its only test, src/test/util_test.cpp:21-66, prints and asserts
// nothing), and it cannot be compiled here (Eigen3, glog, boost and ROS headers
// are absent). This file restates the reference's arithmetic
// expression by expression instead; every function cites the reference lines
// (paths relative to the reference root) it follows. Built with
// -O2 -ffp-contract=off and no -march, like the reference's x86-64 Release build
// (CMakeLists.txt:5): SSE2 doubles, no FMA contraction.
//
// Differences from the reference that are definitions, not changes:
//  * An endpoint outside the grid reads `outside_value` (default 0.3f,
//    kMapUnknownCellProb, slam/slam_processor.h:264). The reference reads out of
//    bounds (UB, map/grid_map_base.h:352-354) and avoids it by pre-extending the
//    map (scan_matchers.h:195-199). Parity fixtures stay in bounds.
//  * pow(x, 2) is written x*x: GCC expands pow with an integer exponent in
//    [-1, 2] into multiplications at -O2 without -ffast-math, so that is what the
//    reference binary computes.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle_math.hpp"

namespace {

int g_threads = 1;  // oracle_set_threads: 1 = single-threaded like the reference

// Geometry + cells of one ScanMatchMap (map/grid_map_base.h:47-71,352-354).
struct OracleMap {
  const float* cells;      // &cell[0].prob_value_
  int64_t stride_floats;   // 2 for the AoS ProbabilityCell, 1 for packed floats
  int32_t size_x, size_y;
  double scale_factor;     // 1.0 / resolution (grid_map_base.h:50)
  double offset_x, offset_y;
  int32_t update_index;    // map_update_index_ (grid_map_base.h:371-378)
  float outside_value;
};

// CorrelationScanMatchParam (correlate_scan_matcher.h:41-86).
struct OracleParam {
  double search_space_size;
  double search_space_resolution;
  double search_angle_offset;
  double search_angle_resolution;
  double response_threshold;
  int32_t use_point_size;
  int32_t max_depth;
  int32_t use_center_penalty;
  int32_t type;
};

enum { kCoarse = 0, kFine = 1, kSuper = 2, kFast = 3 };

const double kMaxVariance = 500.0;      // util/slam_util.h:57
const double kDoubleTolerance = 1e-06;  // util/slam_util.h:59

// util::DoubleEqual (util/slam_util.h:70-73)
inline bool double_equal(double a, double b, double tol = kDoubleTolerance) {
  double delta = a - b;
  if (delta < 0.0) return delta >= -std::fabs(tol);
  return delta <= std::fabs(tol);
}

// util::Round, half away from zero (util/slam_util.h:75-77)
inline double round_half_away(double v) {
  return v >= 0.0 ? std::floor(v + 0.5) : std::ceil(v - 0.5);
}

// GridMapBase::GetCellLength (grid_map_base.h:307-309)
inline double cell_length(const OracleMap& m) { return 1 / m.scale_factor; }

// GetMapCoordsPose (grid_map_base.h:89-93). world_to_map_ =
// AlignedScaling2d(s,s) * Translation2d(o) (:69): linear diag(s,s), translation
// (s*ox, s*oy); applying it is linear*v + t, the zero off-diagonal terms add +-0.
inline void world_to_map(const OracleMap& m, const double w[3], double out[3]) {
  const double s = m.scale_factor;
  const double tx = s * m.offset_x, ty = s * m.offset_y;
  out[0] = s * w[0] + tx;
  out[1] = s * w[1] + ty;
  out[2] = w[2];
}

// GetWorldCoordsPose (grid_map_base.h:83-87) through map_to_world_ =
// world_to_map_.inverse() (:70): Eigen's Affine inverse takes the 2x2 inverse
// (invdet = 1/det, a00 = m11*invdet) and translation -(A^-1 * t).
inline void map_to_world(const OracleMap& m, const double p[3], double out[3]) {
  const double s = m.scale_factor;
  const double tx = s * m.offset_x, ty = s * m.offset_y;
  const double det = s * s - 0.0 * 0.0;
  const double invdet = 1.0 / det;
  const double a = s * invdet;
  const double ntx = -(a * tx), nty = -(a * ty);
  out[0] = a * p[0] + ntx;
  out[1] = a * p[1] + nty;
  out[2] = p[2];
}

// OccuGridMap::GetGridProbValue -> GetCell (occu_grid_map.h:395-397,
// grid_map_cell.h:357-359, grid_map_base.h:352-354); float widened to double.
inline double grid_value(const OracleMap& m, int gx, int gy) {
  if (gx < 0 || gy < 0 || gx >= m.size_x || gy >= m.size_y)
    return (double)m.outside_value;
  return (double)m.cells[((int64_t)gy * m.size_x + gx) * m.stride_floats];
}

// Candidate2D (correlate_scan_matcher.h:227-268) plus the candidate's flat
// enumeration index for reporting (not used by any comparison).
struct Cand {
  double x = 0., y = 0., angle = 0.;
  int angle_index = 0;
  double score = 0.0;
  int64_t flat = 0;
};
struct CandGreater {
  bool operator()(const Cand& a, const Cand& b) const { return a.score > b.score; }
};

// AngleSearchLookUpTable::UpdateLookUpTable (correlate_scan_matcher.h:150-186).
struct AngleLut {
  std::vector<double> angles;
  std::vector<std::vector<std::pair<double, double>>> rows;
  void update(const double* pts, int n, double base_angle, double angle_offset,
              double angle_resolution) {
    int n_angles = (int)(std::floor(angle_offset * 2 / angle_resolution) + 1);
    angles.assign(n_angles, 0.0);
    rows.assign(n_angles, {});
    double start_angle = base_angle - angle_offset;
    for (int a = 0; a < n_angles; ++a) {
      double angle = start_angle + a * angle_resolution;
      angles[a] = angle;
      double cs, sn;
      ref_sincos(angle, &sn, &cs);
      rows[a].resize(n);
      for (int p = 0; p < n; ++p) {
        double px = pts[2 * p], py = pts[2 * p + 1];
        rows[a][p].first = cs * px - sn * py;
        rows[a][p].second = sn * px + cs * py;
      }
    }
  }
};

// Beam subsampling rule (correlate_scan_matcher.h:561-566): returns the step,
// updates the divisor `use` in place exactly as the reference loop does.
inline int beam_step(int point_size, int& use) {
  if (point_size < 2 * use) {
    use = point_size;
    return 1;
  }
  return point_size / (use - 1);
}

// GetResponse (correlate_scan_matcher.h:637-662).
inline double response_at(const OracleMap& m, double x, double y,
                          const std::pair<double, double>* lut, int n, int step, int use) {
  double r = 0.0;
  for (int p = 0; p < n; p += step) {
    int gx = (int)(lut[p].first + x + 0.5);
    int gy = (int)(lut[p].second + y + 0.5);
    r += grid_value(m, gx, gy);
  }
  r /= (use - 0);
  return r;
}

// PenalizeResponse (correlate_scan_matcher.h:718-745), gains :759-761.
void penalize(const double center[3], std::vector<Cand>& cands, double scale,
              double max_bound, double dist_gain, double ang_gain) {
  for (Cand& c : cands) {
    if (double_equal(c.score, 0.0)) continue;
    double dx = c.x - center[0], dy = c.y - center[1];
    double d2 = dx * dx + dy * dy;
    d2 *= (scale * scale);
    double dp = 1.0 - (dist_gain * d2 / (max_bound / 2));
    dp = std::max(dp, 0.5);
    double da = c.angle - center[2];
    da = da * da;
    double ap = 1.0 - (ang_gain * da / 0.349);
    ap = std::max(ap, 0.9);
    c.score = c.score * (dp * ap);
  }
}

// FindBestCandidate (correlate_scan_matcher.h:670-710), tolerance 1e-2 (:763).
Cand find_best(const std::vector<Cand>& sorted, double tol) {
  Cand best = sorted.front();
  double ax = 0.0, ay = 0.0, tx = 0.0, ty = 0.0, ssum = 0.0;
  int count = 0;
  for (const Cand& c : sorted) {
    double sc = c.score;
    if (!double_equal(sc, best.score, tol)) break;
    ax += c.x * sc;
    ay += c.y * sc;
    double sa, ca;
    ref_sincos(c.angle, &sa, &ca);
    tx += ca * sc;
    ty += sa * sc;
    ssum += sc;
    count++;
  }
  if (count > 1) {
    ax /= ssum;
    ay /= ssum;
    tx /= ssum;
    ty /= ssum;
    best.x = ax;
    best.y = ay;
    best.angle = std::atan2(ty, tx);
  }
  return best;
}

// MultiResolutionCorrelateScanMatcher::ScanMatch (correlate_scan_matcher.h:516-614)
// up to (and including) the penalty; candidates stay in enumeration order.
void enumerate_scores(const OracleMap& m, const double* pts, int n, const OracleParam& prm,
                      const double center[3], AngleLut& lut, std::vector<Cand>& cands) {
  double sres = prm.search_space_resolution;
  double ares = prm.search_angle_resolution;
  double ssize = prm.search_space_size;
  double asize = prm.search_angle_offset * 2;
  double mres = cell_length(m);
  lut.update(pts, n, center[2], asize / 2, ares);
  int n_space = (int)(round_half_away(ssize / sres) + 1);
  int n_ang = (int)lut.angles.size();
  int use = prm.use_point_size;
  int step = 1;
  double sx0 = center[0] - (ssize / mres) * 0.5;
  double sy0 = center[1] - (ssize / mres) * 0.5;
  double f = sres / mres;
  // The reference re-runs the beam rule inside the angle loop (:561-566); it is
  // idempotent after the first angle, so it is evaluated once here.
  step = beam_step(n, use);
  const int64_t per_angle = (int64_t)n_space * n_space;
  cands.assign((size_t)(n_ang * per_angle), Cand());
  // g_threads > 1: the all-cores CPU baseline (OpenMP over theta, the loop the
  // reference's commented-out OpenMP pragma sat on, grid_map_base.h:98). Each
  // candidate is computed by the same expressions, so results are identical.
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_threads) if (g_threads > 1)
  for (int a = 0; a < n_ang; ++a) {
    Cand cur;
    cur.angle_index = a;
    cur.angle = lut.angles[a];
    int64_t flat = a * per_angle;
    for (int xi = 0; xi < n_space; ++xi) {
      cur.x = sx0 + xi * f;
      for (int yi = 0; yi < n_space; ++yi) {
        cur.y = sy0 + yi * f;
        cur.score = response_at(m, cur.x, cur.y, lut.rows[a].data(), n, step, use);
        cur.flat = flat;
        cands[(size_t)flat++] = cur;
      }
    }
  }
  if (prm.use_center_penalty) {
    double g = (prm.type == kCoarse) ? 0.4 : 0.2;
    penalize(center, cands, mres, ssize, g, 0.25);
  }
}

// ComputePositionalCovariance (correlate_scan_matcher.h:887-956).
void positional_cov(const std::vector<Cand>& cands, const Cand& best, double mres,
                    double sres, double max_ang_var, double cov[9]) {
  for (int i = 0; i < 9; ++i) cov[i] = (i % 4 == 0) ? 1.0 : 0.0;
  double bs = best.score;
  if (bs < kDoubleTolerance) {
    cov[0] = kMaxVariance;
    cov[4] = kMaxVariance;
    cov[8] = max_ang_var;
    return;
  }
  double vxx = 0.0, vxy = 0.0, vyy = 0.0, norm = 0.0;
  double bound = std::min(bs - 0.1, 0.5);
  int counter = 0;
  for (const Cand& c : cands) {
    double sc = c.score;
    if (!(sc > bound && counter < 20)) break;
    norm += sc;
    double dx = c.x - best.x, dy = c.y - best.y;
    vxx += (dx * dx * sc);
    vxy += (dx * dy * sc);
    vyy += (dy * dy * sc);
    counter++;
  }
  if (norm > kDoubleTolerance) {
    double xx = vxx / norm, xy = vxy / norm, yy = vyy / norm;
    double r = sres / mres;
    double minv = 0.1 * (r * r);
    xx = std::max<double>(xx, minv);
    yy = std::max<double>(yy, minv);
    double m2 = mres * mres;
    cov[0] = (xx * m2) / bs;
    cov[1] = (xy * m2) / bs;
    cov[3] = (xy * m2) / bs;
    cov[4] = (yy * m2) / bs;
    cov[8] = max_ang_var;
  }
  if (double_equal(cov[0], 0.0)) cov[0] = kMaxVariance;
  if (double_equal(cov[4], 0.0)) cov[4] = kMaxVariance;
}

// ComputeAngularCovariance (correlate_scan_matcher.h:965-1019).
void angular_cov(const std::vector<Cand>& cands, const Cand& best, double lin_tol,
                 double max_ang_var, double cov[9]) {
  double bs = best.score;
  if (bs < kDoubleTolerance) {
    cov[8] = max_ang_var;
    return;
  }
  double norm = 0.0, acc = 0.0;
  double bound = std::min(bs - 0.1, 0.5);
  int counter = 0;
  for (const Cand& c : cands) {
    double sc = c.score;
    if (sc >= bound && counter < 20) {
      if (double_equal(c.x, best.x, lin_tol) && double_equal(c.y, best.y, lin_tol)) {
        double d = c.angle - best.angle;
        norm += sc;
        acc += (d * d * sc);
        counter++;
      }
    }
  }
  double var = max_ang_var;
  if (norm > kDoubleTolerance) {
    // :1008-1010 assigns max_ang_var/4 when acc is tiny, then :1012 overwrites it.
    var = acc / norm;
  } else {
    var = 200 * max_ang_var;
  }
  cov[8] = var;
}

// BranchAndBoundCorrelateScanMatcher (correlate_scan_matcher.h:271-502).
struct Bnb {
  const OracleMap* m;
  AngleLut* lut;
  double sres, ssize, mres;
  int use_point_size;
  int64_t scored = 0;

  // ScoreCandidates (:398-431): the `use` divisor persists across candidates.
  void score_and_sort(std::vector<Cand>& cands) {
    int step = 1;
    int use = use_point_size;
    for (Cand& c : cands) {
      const auto& row = lut->rows[c.angle_index];
      int n = (int)row.size();
      if (n <= 0) continue;
      step = beam_step(n, use);
      double r = 0.0;
      for (int p = 0; p < n; p += step) {
        int gx = (int)(row[p].first + c.x + 0.5);
        int gy = (int)(row[p].second + c.y + 0.5);
        r += grid_value(*m, gx, gy);
      }
      r /= use;
      c.score = r;
      scored++;
    }
    std::sort(cands.begin(), cands.end(), CandGreater());
  }

  // BranchAndBound (:434-476).
  Cand search(const std::vector<Cand>& cands, int depth, double min_score) {
    if (depth == 0) return cands.front();
    Cand best;
    best.x = 0;
    best.y = 0.0;
    best.angle = 0.0;
    best.angle_index = 0;
    best.score = min_score;
    for (const Cand& c : cands) {
      if (c.score <= min_score) break;
      std::vector<Cand> kids;
      double half_res = (1 << (depth - 1)) * sres;
      double hw = half_res / mres;
      const double offs[2] = {0.0, hw};
      for (double ox : offs)
        for (double oy : offs) {
          Cand k;
          k.x = c.x + ox;
          k.y = c.y + oy;
          k.angle = lut->angles[c.angle_index];
          k.angle_index = c.angle_index;
          kids.push_back(k);
        }
      score_and_sort(kids);
      Cand sub = search(kids, depth - 1, best.score);
      // std::max(best, sub) returns `best` unless best < sub (by score).
      if (best.score < sub.score) best = sub;
    }
    return best;
  }
};

struct Matcher {
  AngleLut lut;
  std::vector<Cand> cands;
};

// BasedCorrelationScanMatch::ScanMatch (correlate_scan_matcher.h:784-875).
double scan_match(Matcher& mt, const OracleMap& m, const double* pts, int n,
                  const OracleParam& prm, double pose[3], double cov[9],
                  int64_t* argmax_flat, int64_t* n_scored) {
  double response = 0.0;  // kMinResponse (:1034)
  if (m.update_index < 0 || n == 0) return response;
  double sres = prm.search_space_resolution;
  double ares = prm.search_angle_resolution;
  double max_ang_var = 4 * (ares * ares);
  double mres = cell_length(m);
  double center[3];
  world_to_map(m, pose, center);
  Cand best;
  if (prm.type == kFast) {
    // BranchAndBoundCorrelateScanMatcher::ScanMatch (:274-331).
    Bnb b;
    b.m = &m;
    b.lut = &mt.lut;
    b.sres = sres;
    b.ssize = prm.search_space_size;
    b.mres = mres;
    b.use_point_size = prm.use_point_size;
    double asize = prm.search_angle_offset * 2;
    mt.lut.update(pts, n, center[2], asize / 2, ares);
    int depth = prm.max_depth;
    double lowest = (1 << depth) * sres;
    // ComputeLowestResolutionCandidates (:333-393).
    int n_space = (int)(round_half_away(b.ssize / lowest) + 1);
    int n_ang = (int)mt.lut.angles.size();
    int step = 1, use = b.use_point_size;
    double sx0 = center[0] - (b.ssize / mres) * 0.5;
    double sy0 = center[1] - (b.ssize / mres) * 0.5;
    double f = lowest / mres;
    std::vector<Cand> low;
    low.reserve((size_t)n_ang * n_space * n_space);
    int64_t flat = 0;
    for (int a = 0; a < n_ang; ++a) {
      double angle = mt.lut.angles[a];
      const auto& row = mt.lut.rows[a];
      int np = (int)row.size();
      if (np <= 0) continue;
      step = beam_step(np, use);
      for (int xi = 0; xi < n_space; ++xi) {
        double x = sx0 + xi * f;
        for (int yi = 0; yi < n_space; ++yi) {
          double y = sy0 + yi * f;
          double r = 0.0;
          for (int p = 0; p < np; p += step) {
            int gx = (int)(row[p].first + x + 0.5);
            int gy = (int)(row[p].second + y + 0.5);
            r += grid_value(m, gx, gy);
          }
          r /= use;
          Cand c;
          c.x = x;
          c.y = y;
          c.angle = angle;
          c.angle_index = a;
          c.score = r;
          c.flat = flat++;
          low.push_back(c);
          b.scored++;
        }
      }
    }
    std::sort(low.begin(), low.end(), CandGreater());
    mt.cands = low;
    best = b.search(low, depth, low.front().score - 0.1);
    if (n_scored) *n_scored = b.scored;
    if (argmax_flat) *argmax_flat = -1;
  } else {
    enumerate_scores(m, pts, n, prm, center, mt.lut, mt.cands);
    std::sort(mt.cands.begin(), mt.cands.end(), CandGreater());
    best = find_best(mt.cands, 1e-2);
    if (argmax_flat) *argmax_flat = mt.cands.front().flat;
    if (n_scored) *n_scored = (int64_t)mt.cands.size();
  }
  switch (prm.type) {
    case kFast:
    case kCoarse:
      positional_cov(mt.cands, best, mres, sres, max_ang_var, cov);
      angular_cov(mt.cands, best, sres / mres, max_ang_var, cov);
      break;
    case kFine:
      positional_cov(mt.cands, best, mres, sres, max_ang_var, cov);
      break;
    case kSuper:
      angular_cov(mt.cands, best, sres / mres, max_ang_var, cov);
      break;
    default:
      break;
  }
  double bs = best.score;
  bs = (bs > 1.0) ? 1.0 : bs;
  response = bs;
  if (response > prm.response_threshold) {
    double bp[3] = {best.x, best.y, best.angle};
    map_to_world(m, bp, pose);
  }
  return response;
}

}  // namespace

extern "C" {

struct oracle_map_c {
  const float* cells;
  int64_t stride_floats;
  int32_t size_x, size_y;
  double resolution;
  double offset_x, offset_y;
  int32_t update_index;
  float outside_value;
};

static OracleMap to_map(const oracle_map_c* c) {
  OracleMap m;
  m.cells = c->cells;
  m.stride_floats = c->stride_floats;
  m.size_x = c->size_x;
  m.size_y = c->size_y;
  m.scale_factor = 1.0 / c->resolution;
  m.offset_x = c->offset_x;
  m.offset_y = c->offset_y;
  m.update_index = c->update_index;
  m.outside_value = c->outside_value;
  return m;
}

static OracleParam to_param(const void* p) {
  OracleParam q;
  std::memcpy(&q, p, sizeof(OracleParam));
  return q;
}

int oracle_param_size(void) { return (int)sizeof(OracleParam); }
// Threads for the candidate enumeration (CPU baseline's all-cores variant).
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int oracle_map_size(void) { return (int)sizeof(oracle_map_c); }

// All candidate scores (after penalty) in enumeration order (theta, x, y).
int oracle_score_window(const oracle_map_c* mc, const double* pts, int n, const void* param,
                        const double center[3], double* scores, int64_t n_out) {
  OracleMap m = to_map(mc);
  OracleParam prm = to_param(param);
  AngleLut lut;
  std::vector<Cand> cands;
  enumerate_scores(m, pts, n, prm, center, lut, cands);
  if ((int64_t)cands.size() != n_out) return 1;
  for (size_t i = 0; i < cands.size(); ++i) scores[i] = cands[i].score;
  return 0;
}

// Sorted order (flat indices after std::sort(greater)) of one window.
int oracle_sorted_order(const oracle_map_c* mc, const double* pts, int n, const void* param,
                        const double center[3], int64_t* order, int64_t n_out) {
  OracleMap m = to_map(mc);
  OracleParam prm = to_param(param);
  AngleLut lut;
  std::vector<Cand> cands;
  enumerate_scores(m, pts, n, prm, center, lut, cands);
  if ((int64_t)cands.size() != n_out) return 1;
  std::sort(cands.begin(), cands.end(), CandGreater());
  for (size_t i = 0; i < cands.size(); ++i) order[i] = cands[i].flat;
  return 0;
}

// BasedCorrelationScanMatch::ScanMatch. Returns the response.
double oracle_scan_match(const oracle_map_c* mc, const double* pts, int n, const void* param,
                         double pose[3], double cov[9], int64_t* argmax_flat,
                         int64_t* n_scored) {
  OracleMap m = to_map(mc);
  OracleParam prm = to_param(param);
  Matcher mt;
  return scan_match(mt, m, pts, n, prm, pose, cov, argmax_flat, n_scored);
}

// ScanMatchers::ScanMatch (scan_matchers.h:179-289) with
// use_optimize_scan_match_ = false and MapSizeCheck left to the caller.
double oracle_scan_matchers(const oracle_map_c* mc, const double* pts, int n,
                            const void* levels3, int use_fine, double pose[3], double cov[9]) {
  OracleMap m = to_map(mc);
  const OracleParam* lv = (const OracleParam*)levels3;
  OracleParam p0 = to_param(&lv[0]), p1 = to_param(&lv[1]), p2 = to_param(&lv[2]);
  Matcher mt;  // one BasedCorrelationScanMatch shared by the three levels
  double score = 0.0;
  int times = 0;
  double proc[3] = {pose[0], pose[1], pose[2]};
  score += scan_match(mt, m, pts, n, p0, proc, cov, nullptr, nullptr);
  times++;
  pose[0] = proc[0];
  pose[1] = proc[1];
  pose[2] = proc[2];
  if (use_fine) {
    score += scan_match(mt, m, pts, n, p1, proc, cov, nullptr, nullptr);
    times++;
    score += scan_match(mt, m, pts, n, p2, proc, cov, nullptr, nullptr);
    times++;
  }
  pose[0] = proc[0];
  pose[1] = proc[1];
  pose[2] = proc[2];
  score /= times;
  return score;
}

// Batched 3-level matching over independent scans (CPU baseline leg).
// n_threads <= 1 runs single-threaded like the reference.
void oracle_scan_matchers_batch(const oracle_map_c* mc, int n_scans, const double* pts,
                                const int64_t* offsets, const void* levels3, int use_fine,
                                double* poses, double* covs, double* scores) {
  for (int s = 0; s < n_scans; ++s) {
    int64_t o = offsets[s];
    int n = (int)(offsets[s + 1] - o);
    scores[s] = oracle_scan_matchers(mc, pts + 2 * o, n, levels3, use_fine, poses + 3 * s,
                                     covs + 9 * s);
  }
}

// Map <-> world helpers (grid_map_base.h:83-93) for tests.
void oracle_world_to_map(const oracle_map_c* mc, const double w[3], double out[3]) {
  OracleMap m = to_map(mc);
  world_to_map(m, w, out);
}
void oracle_map_to_world(const oracle_map_c* mc, const double p[3], double out[3]) {
  OracleMap m = to_map(mc);
  map_to_world(m, p, out);
}

// Argmax over one window with ties broken by the lowest flat index (the
// definition the device reduction uses; no reference counterpart).
double oracle_best_window(const oracle_map_c* mc, const double* pts, int n, const void* param,
                          const double center[3], int64_t* flat) {
  OracleMap m = to_map(mc);
  OracleParam prm = to_param(param);
  AngleLut lut;
  std::vector<Cand> cands;
  enumerate_scores(m, pts, n, prm, center, lut, cands);
  double best = -1.0;
  int64_t bi = -1;
  for (const Cand& c : cands)
    if (bi < 0 || c.score > best) {
      best = c.score;
      bi = c.flat;
    }
  *flat = bi;
  return best;
}

}  // extern "C"

extern "C" {
// Permutation std::sort(greater-by-key) applies to keys[0..n) (tests of the
// tie-order model in tests/introsort_ref.py).
void oracle_std_sort_order(const double* keys, int64_t n, int64_t* order) {
  std::vector<Cand> v((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    v[(size_t)i].score = keys[i];
    v[(size_t)i].flat = i;
  }
  std::sort(v.begin(), v.end(), CandGreater());
  for (int64_t i = 0; i < n; ++i) order[i] = v[(size_t)i].flat;
}

// The host libm's sincos over x[0..n) (AngleSearchLookUpTable :171-172 as
// GCC compiles it): the checker of the device's angle rows (csm_sincos_device).
void oracle_sincos_batch(const double* x, int64_t n, double* s, double* c) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) ref_sincos(x[i], &s[i], &c[i]);
}
}
