// Runs include/csm_reference_adapter.hpp — the reference-side drop-in for
// BasedCorrelationScanMatch — on the GPU, the way ScanMatchers::ScanMatch
// calls it (scan_matchers.h:238,249,256: coarse, fine, super-fine on the fine
// map, the pose fed forward), with the map mutated between scans like
// OccuGridMap::UpdateMapByRange (occu_grid_map.h:258-329: cells rewritten and
// appended to map_update_point_), reset like InitMapWithRangeVec
// (ResetValueSpeedup, :226-237) and grown like ExtendSize (grid_map_base.h:186-254).
// Every level's response, pose and covariance are compared bit for bit with
// the CPU oracle (test infrastructure, oracle/liboracle.so) on the same map.
//
// The map / range / param types are this test's own stand-ins with the
// reference's member names and layouts (ProbabilityCell {float, int}); no
// reference source is used.
//
//   adapter_run check [scans]         parity run (exit 0 = bit-exact)
//   adapter_run bench [scans] [size]  per-scan latency of the 3-level match through
//                                     the adapter (incremental refresh vs whole-grid
//                                     upload) and of the oracle; one JSON line
//   adapter_run nodevice              error convention without a usable device
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "csm_reference_adapter.hpp"

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
double oracle_scan_match(const oracle_map_c* mc, const double* pts, int n, const void* param, double pose[3],
                         double cov[9], int64_t* argmax_flat, int64_t* n_scored);
}

namespace {

struct Vec2 {
  double a[2];
  double x() const { return a[0]; }
  double y() const { return a[1]; }
};
struct Vec3 {
  double a[3];
  double& operator[](int i) { return a[i]; }
  double operator[](int i) const { return a[i]; }
};
struct Mat3 {
  double a[9];
  double& operator()(int r, int c) { return a[3 * r + c]; }
};
struct ProbabilityCell {
  float prob_value_;
  int update_index_;
};

// OccuGridMap stand-in: AoS cells, map_update_index_, map_update_point_ and a
// reset counter (the two accessors INTEGRATION.md §2a adds).
struct Map {
  std::vector<ProbabilityCell> cells;
  int sx = 0, sy = 0;
  double res = 0.05, ox = 0.0, oy = 0.0;
  int index = 0;
  std::vector<int> update_points;
  int64_t resets = 0;
  int64_t generation = 0;  // bumped whenever the cell buffer is (re)allocated
  int GetSizeX() const { return sx; }
  int GetSizeY() const { return sy; }
  double GetCellLength() const { return res; }
  int map_update_index() const { return index; }
  const ProbabilityCell* GetCellData() const { return cells.data(); }
  const std::vector<int>& GetUpdatePoints() const { return update_points; }
  int64_t GetResetCount() const { return resets; }
  int64_t GetCellGeneration() const { return generation; }
  float& prob(int x, int y) { return cells[(size_t)y * sx + x].prob_value_; }
};
// The same map without the incremental-refresh accessors (whole-grid uploads).
struct PlainMap {
  Map* m;
  int GetSizeX() const { return m->sx; }
  int GetSizeY() const { return m->sy; }
  double GetCellLength() const { return m->res; }
  int map_update_index() const { return m->index; }
  const ProbabilityCell* GetCellData() const { return m->cells.data(); }
};
struct Range {
  std::vector<Vec2> pts;
  int GetSize() const { return (int)pts.size(); }
  const Vec2& GetDataPoint(int i) const { return pts[(size_t)i]; }
};
enum Type { COARSE = 0, FINE = 1, SUPER = 2 };
struct Param {
  double size, res, aoff, ares, thr;
  int use;
  bool penalty;
  Type type;
  double search_space_size() const { return size; }
  double search_space_resolution() const { return res; }
  double search_angle_offset() const { return aoff; }
  double search_angle_resolution() const { return ares; }
  double response_threshold() const { return thr; }
  int use_point_size() const { return use; }
  int max_depth() const { return 0; }
  bool use_center_penalty() const { return penalty; }
  Type correlation_scan_match_type() const { return type; }
};
struct OffsetOf {
  std::array<double, 2> operator()(const Map& m) const { return {m.ox, m.oy}; }
  std::array<double, 2> operator()(const PlainMap& m) const { return {m.m->ox, m.m->oy}; }
};

uint64_t rng_state = 20261016;
double urand() {  // xorshift64*
  rng_state ^= rng_state >> 12;
  rng_state ^= rng_state << 25;
  rng_state ^= rng_state >> 27;
  return (double)((rng_state * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}

// Values of the reference's scan-match maps: unknown 0.3, the blur splat
// (kernel * 0.88) and 1.0 (occu_grid_map.h:531-576), all exact in fp32.
const float kValues[] = {0.3f, 0.44f, 0.6f, 0.7392f, 0.88f, 1.0f};

void wall(Map& m, int x0, int y0, int x1, int y1) {
  const int n = std::max(std::abs(x1 - x0), std::abs(y1 - y0));
  for (int i = 0; i <= n; ++i) {
    const int x = x0 + (int)std::lround((double)(x1 - x0) * i / std::max(n, 1));
    const int y = y0 + (int)std::lround((double)(y1 - y0) * i / std::max(n, 1));
    for (int dy = -2; dy <= 2; ++dy)
      for (int dx = -2; dx <= 2; ++dx) {
        const int xx = x + dx, yy = y + dy;
        if (xx < 0 || yy < 0 || xx >= m.sx || yy >= m.sy) continue;
        const float v = (dx == 0 && dy == 0) ? 1.0f : kValues[4 - std::max(std::abs(dx), std::abs(dy))];
        float& c = m.prob(xx, yy);
        c = std::max(c, v);
      }
  }
}

Map make_map(int side, double res) {
  Map m;
  m.sx = m.sy = side;
  m.res = res;
  m.ox = side * res * 0.5;  // world (0, 0) at the map centre
  m.oy = side * res * 0.5;
  m.cells.assign((size_t)side * side, ProbabilityCell{0.3f, -1});
  for (int w = 0; w < side / 10; ++w) {
    const int x0 = (int)(urand() * side), y0 = (int)(urand() * side);
    const bool horiz = urand() < 0.5;
    const int len = 20 + (int)(urand() * side / 4);
    wall(m, x0, y0, horiz ? std::min(side - 1, x0 + len) : x0, horiz ? y0 : std::min(side - 1, y0 + len));
  }
  return m;
}

// 1081 beams (Hokuyo, -135.125 deg + 0.25 deg steps) ray-marched to the first
// cell >= 0.88; points in cells, sensor frame (RangeDataContainer::CreateFrom).
Range make_scan(Map& m, double wx, double wy, double wth) {
  Range r;
  const double s = 1.0 / m.res;
  double a = -135.125 * M_PI / 180.0;
  for (int b = 0; b < 1081; ++b, a += 0.25 * M_PI / 180.0) {
    double d = 0.1;
    for (; d < 10.0; d += m.res * 0.5) {
      const double x = (wx + m.ox) * s + std::cos(wth + a) * d * s, y = (wy + m.oy) * s + std::sin(wth + a) * d * s;
      const int ix = (int)x, iy = (int)y;
      if (ix < 0 || iy < 0 || ix >= m.sx || iy >= m.sy) break;
      if (m.prob(ix, iy) >= 0.88f) break;
    }
    r.pts.push_back(Vec2{{std::cos(a) * d * s, std::sin(a) * d * s}});
  }
  return r;
}

// UpdateMapByRange-like mutation: n cells rewritten and appended to the list.
void mutate(Map& m, int n) {
  for (int i = 0; i < n; ++i) {
    const int k = (int)(urand() * (double)m.cells.size());
    m.cells[(size_t)k].prob_value_ = kValues[(int)(urand() * 6) % 6];
    m.update_points.push_back(k);
  }
  m.index++;
}
// InitMapWithRangeVec with the reset speed-up: listed cells back to 0.3.
void reset(Map& m) {
  for (int k : m.update_points) m.cells[(size_t)k] = ProbabilityCell{0.3f, -1};
  m.update_points.clear();
  m.resets++;
}
// ExtendSize: a larger buffer, the old cells at an offset, the offset moved.
void extend(Map& m, int pad) {
  std::vector<ProbabilityCell> c((size_t)(m.sx + 2 * pad) * (m.sy + 2 * pad), ProbabilityCell{0.3f, -1});
  for (int y = 0; y < m.sy; ++y)
    std::memcpy(&c[(size_t)(y + pad) * (m.sx + 2 * pad) + pad], &m.cells[(size_t)y * m.sx],
                (size_t)m.sx * sizeof(ProbabilityCell));
  m.cells.swap(c);
  m.sx += 2 * pad;
  m.sy += 2 * pad;
  m.ox += pad * m.res;
  m.oy += pad * m.res;
  m.update_points.clear();
  m.generation++;
}
// A map freed and another allocated at the same address and size: fresh
// walls, an update list at least as long as the old map's, the same reset
// count -- only the generation tells them apart.
void reuse_buffer(Map& m) {
  const size_t listed = m.update_points.size();
  const ProbabilityCell* before = m.cells.data();
  Map fresh = make_map(m.sx, m.res);
  std::copy(fresh.cells.begin(), fresh.cells.end(), m.cells.begin());  // same buffer, new contents
  if (m.cells.data() != before) std::abort();
  m.update_points.clear();
  for (size_t i = 0; i < listed + 7; ++i) m.update_points.push_back((int)(urand() * (double)m.cells.size()));
  m.index = 0;
  m.generation++;
}

oracle_map_c omap(const Map& m) {
  return oracle_map_c{&m.cells[0].prob_value_, 2, m.sx, m.sy, m.res, m.ox, m.oy, m.index, 0.3f};
}

// simulatin_param.yaml levels (:51-70), every beam summed or U = 100.
std::array<Param, 3> levels(int use) {
  return {Param{0.6, 0.05, 0.523, 0.0349, 0.6, use, true, COARSE}, Param{0.2, 0.02, 0.175, 0.0349, 0.6, use, true, FINE},
          Param{0.02, 0.01, 0.0349, 0.00349, 0.6, use, true, SUPER}};
}

using Adapter = roborts_csm::BasedCorrelationScanMatchGpu<Map, Range, Param, Vec3, Mat3, OffsetOf>;
using PlainAdapter = roborts_csm::BasedCorrelationScanMatchGpu<PlainMap, Range, Param, Vec3, Mat3, OffsetOf>;

std::string g_log;
void capture(const char* m) { g_log += m; }

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int check(int n_scans) {
  auto dev = std::make_shared<roborts_csm::DeviceContext>(0);
  if (!dev->ok()) {
    std::printf("no device: %s\n", dev->last_error().c_str());
    return 2;
  }
  Adapter ad(dev, OffsetOf{}, capture);
  auto map = std::make_shared<Map>(make_map(700, 0.05));
  int incremental = 0, whole = 0, mismatches = 0;
  for (int s = 0; s < n_scans; ++s) {
    if (s % 5 == 4) reset(*map);
    if (s == 7) extend(*map, 40);
    if (s == 11 || s == 17) reuse_buffer(*map);
    if (s > 0) mutate(*map, 3000 + (int)(urand() * 20000));
    const double wx = (urand() - 0.5) * 20.0, wy = (urand() - 0.5) * 20.0, wth = (urand() - 0.5) * 6.0;
    auto range = std::make_shared<Range>(make_scan(*map, wx, wy, wth));
    Vec3 pose{{wx + 0.12, wy - 0.07, wth + 0.07}};
    double opose[3] = {pose[0], pose[1], pose[2]};
    Mat3 cov{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    double ocov[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const auto lv = levels(s % 2 ? 100 : 1081);
    std::vector<double> pts(range->pts.size() * 2);
    for (size_t i = 0; i < range->pts.size(); ++i) {
      pts[2 * i] = range->pts[i].a[0];
      pts[2 * i + 1] = range->pts[i].a[1];
    }
    for (int l = 0; l < 3; ++l) {
      auto prm = std::make_shared<Param>(lv[(size_t)l]);
      const double r = ad.ScanMatch(map, range, prm, pose, cov);
      const int64_t refreshed = ad.last_refresh_cells();
      if (l == 0) (refreshed < 0 ? whole : incremental) += 1;
      const csm_param cp = roborts_csm::to_csm_param(*prm);
      const oracle_map_c om = omap(*map);
      const double ro = oracle_scan_match(&om, pts.data(), (int)range->pts.size(), &cp, opose, ocov, nullptr, nullptr);
      bool same = r == ro && std::memcmp(pose.a, opose, sizeof(opose)) == 0 && std::memcmp(cov.a, ocov, sizeof(ocov)) == 0;
      if (!same) {
        mismatches++;
        std::printf("scan %d level %d: response %.17g vs %.17g pose %.17g %.17g %.17g vs %.17g %.17g %.17g\n", s, l,
                    r, ro, pose[0], pose[1], pose[2], opose[0], opose[1], opose[2]);
      }
    }
  }
  std::printf("{\"scans\": %d, \"levels\": %d, \"mismatches\": %d, \"incremental_refreshes\": %d, "
              "\"whole_uploads\": %d, \"log\": \"%s\"}\n",
              n_scans, 3 * n_scans, mismatches, incremental, whole, g_log.c_str());
  return (mismatches == 0 && incremental > 0 && whole > 1 && g_log.empty()) ? 0 : 1;
}

int nodevice() {
  // a device index that cannot exist: csm_create fails; the adapter must log
  // and return 0.0 with the pose and covariance untouched (no exception)
  auto dev = std::make_shared<roborts_csm::DeviceContext>(1 << 20);
  Adapter ad(dev, OffsetOf{}, capture);
  auto map = std::make_shared<Map>(make_map(200, 0.05));
  auto range = std::make_shared<Range>(make_scan(*map, 0.0, 0.0, 0.0));
  auto prm = std::make_shared<Param>(levels(100)[0]);
  Vec3 pose{{0.5, -0.25, 0.125}};
  Mat3 cov{{2, 0, 0, 0, 3, 0, 0, 0, 4}};
  const double r = ad.ScanMatch(map, range, prm, pose, cov);
  const bool ok = !dev->ok() && r == 0.0 && pose[0] == 0.5 && pose[1] == -0.25 && pose[2] == 0.125 && cov(0, 0) == 2 &&
                  cov(2, 2) == 4 && !g_log.empty();
  std::printf("{\"response\": %g, \"logged\": %d, \"ok\": %d}\n", r, (int)!g_log.empty(), (int)ok);
  return ok ? 0 : 1;
}

int bench(int n_scans, int side) {
  auto dev = std::make_shared<roborts_csm::DeviceContext>(0);
  if (!dev->ok()) {
    std::printf("no device: %s\n", dev->last_error().c_str());
    return 2;
  }
  // config 5 shape: the front end's 1 cm fine map (slam_processor.cpp:469,499-500),
  // a drive through it, ~1e5 cells rewritten per scan (1081 rays at 1 cm), U = 100
  auto map = std::make_shared<Map>(make_map(side, 0.01));
  PlainMap plain{map.get()};
  auto pmap = std::make_shared<PlainMap>(plain);
  Adapter inc(dev, OffsetOf{}, capture);
  PlainAdapter full(dev, OffsetOf{}, capture);
  const auto lv = levels(100);
  std::vector<double> t_inc, t_full, t_cpu, t_mut, t_inc_l0;
  for (int s = 0; s < n_scans; ++s) {
    const double tm = now_ms();
    mutate(*map, 100000);
    t_mut.push_back(now_ms() - tm);
    const double wx = (urand() - 0.5) * side * 0.01 * 0.5, wy = (urand() - 0.5) * side * 0.01 * 0.5;
    auto range = std::make_shared<Range>(make_scan(*map, wx, wy, urand() * 6.0));
    std::vector<double> pts(range->pts.size() * 2);
    for (size_t i = 0; i < range->pts.size(); ++i) {
      pts[2 * i] = range->pts[i].a[0];
      pts[2 * i + 1] = range->pts[i].a[1];
    }
    for (int mode = 0; mode < 3; ++mode) {
      Vec3 pose{{wx + 0.05, wy - 0.03, 0.02}};
      Mat3 cov{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
      double op[3] = {pose[0], pose[1], pose[2]}, oc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      if (mode == 1) map->index++;  // the whole-grid path sees a changed map every scan too
      const double t0 = now_ms();
      for (int l = 0; l < 3; ++l) {
        auto prm = std::make_shared<Param>(lv[(size_t)l]);
        if (mode == 0) {
          inc.ScanMatch(map, range, prm, pose, cov);
          if (l == 0 && s > 0) t_inc_l0.push_back(now_ms() - t0);  // the level that refreshes the grid
        } else if (mode == 1) {
          full.ScanMatch(pmap, range, prm, pose, cov);
        } else {
          const csm_param cp = roborts_csm::to_csm_param(*prm);
          const oracle_map_c om = omap(*map);
          oracle_scan_match(&om, pts.data(), (int)range->pts.size(), &cp, op, oc, nullptr, nullptr);
        }
      }
      const double dt = now_ms() - t0;
      if (s > 0) (mode == 0 ? t_inc : mode == 1 ? t_full : t_cpu).push_back(dt);
    }
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  std::printf("{\"scans\": %d, \"map_cells\": %d, \"cells_per_update\": 100000, "
              "\"adapter_incremental_ms_p50\": %.4f, \"adapter_whole_upload_ms_p50\": %.4f, "
              "\"oracle_cpu_ms_p50\": %.4f, \"host_map_mutation_ms_p50\": %.4f, "
              "\"adapter_first_level_ms_p50\": %.4f, \"log\": \"%s\"}\n",
              n_scans, side * side, med(t_inc), med(t_full), med(t_cpu), med(t_mut), med(t_inc_l0), g_log.c_str());
  return g_log.empty() ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "check";
  if (mode == "check") return check(argc > 2 ? std::atoi(argv[2]) : 24);
  if (mode == "bench") return bench(argc > 2 ? std::atoi(argv[2]) : 40, argc > 3 ? std::atoi(argv[3]) : 3000);
  if (mode == "nodevice") return nodevice();
  std::fprintf(stderr, "usage: adapter_run check|bench|nodevice\n");
  return 2;
}
