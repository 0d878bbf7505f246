// Sanitizer run of the CPU oracle (test infrastructure; SURVEY §5's ASAN/UBSAN
// auxiliary). Built by `make -C oracle san` with -fsanitize=address,undefined
// from the oracle's own sources, it drives every matcher entry point the
// parity tests use on seeded inputs that reach the edge cases: beams off the
// grid on every side, the beam-subsampling rule at n = 0, 1, use, 2*use - 1,
// 2*use and far above it, all three sim-YAML levels (coarse / fine / super-fine
// windows, correlate_scan_matcher.h:561-745), the FAST branch and bound
// (:274-331), std::sort over keys with heavy ties, and the map oracle: both
// cell kinds, blur on/off, auto-resize past every edge, the batch rebuild,
// the map-check penalty and Bresenham. Any out-of-bounds read,
// overflow or undefined shift aborts the run (halt_on_error); the result
// checks below are only self-consistency (the parity tests compare values).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

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
struct oracle_param_c {  // OracleParam (csm_oracle.cpp:51-61)
  double search_space_size, search_space_resolution, search_angle_offset, search_angle_resolution,
      response_threshold;
  int32_t use_point_size, max_depth, use_center_penalty, type;
};
int oracle_param_size(void);
int oracle_map_size(void);
int oracle_score_window(const oracle_map_c*, const double*, int, const void*, const double*, double*, int64_t);
double oracle_scan_match(const oracle_map_c*, const double*, int, const void*, double*, double*, int64_t*,
                         int64_t*);
double oracle_scan_matchers(const oracle_map_c*, const double*, int, const void*, int, double*, double*);
double oracle_best_window(const oracle_map_c*, const double*, int, const void*, const double*, int64_t*);
void oracle_std_sort_order(const double*, int64_t, int64_t*);
void* oracle_gridmap_create(int, double, int, int, double, double, double, float);
void oracle_gridmap_destroy(void*);
void oracle_gridmap_set_options(void*, int, int, double, double);
int oracle_gridmap_update_by_range(void*, const double*, int, const double*, const double*, int);
void oracle_gridmap_init_with_range_vec(void*, const double*, const int64_t*, int, const double*, const double*, int,
                                        int);
double oracle_gridmap_feedback_penalty(void*, const double*, int, const double*, const double*, int, double, double,
                                       int);
void oracle_gridmap_info(void*, int32_t*, double*);
int oracle_bresenham(int, int, int, int, int32_t*, int);
}

namespace {

int failures = 0;
void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "san_driver: %s\n", what);
    ++failures;
  }
}

oracle_param_c level(double size, double res, double off, double ares, int use, int type) {
  return oracle_param_c{size, res, off, ares, 0.6, use, 0, 1, type};
}

}  // namespace

int main() {
  if (oracle_param_size() != (int)sizeof(oracle_param_c) || oracle_map_size() != (int)sizeof(oracle_map_c)) {
    std::fprintf(stderr, "san_driver: ABI sizes differ\n");
    return 2;
  }
  // a 300 x 240 map of 5 cm cells (AoS stride 2: prob + a second field), walls and blur
  const int sx = 300, sy = 240, stride = 2;
  std::vector<float> cells((size_t)sx * sy * stride, 0.3f);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  for (int x = 0; x < sx; ++x)
    for (int y = 0; y < sy; ++y) {
      const bool wall = x % 37 == 0 || y % 29 == 0 || (x - y) % 53 == 0;
      cells[((size_t)x * sy + y) * stride] = wall ? 0.9f : (float)(0.1 + 0.2 * u(rng));
    }
  oracle_map_c m{cells.data(), stride, sx, sy, 0.05, -2.0, -1.5, 0, 0.3f};

  const oracle_param_c levels[3] = {level(0.6, 0.05, 0.523, 0.0349, 100, 0),   // simulatin_param.yaml:51-70
                                    level(0.2, 0.02, 0.175, 0.0349, 100, 1),
                                    level(0.02, 0.01, 0.0349, 0.00349, 100, 2)};
  // beam counts around the subsampling rule (use = 100: n < 200 keeps every beam)
  const int counts[] = {0, 1, 2, 99, 100, 199, 200, 201, 1081};
  for (int n : counts) {
    std::vector<double> pts((size_t)2 * n);
    for (int i = 0; i < n; ++i) {  // beams in cells, some far off the grid on every side
      const double r = (i % 17 == 0) ? 900.0 : 5.0 + 80.0 * u(rng);
      const double a = 2.0 * M_PI * i / std::max(n, 1);
      pts[2 * (size_t)i] = r * std::cos(a);
      pts[2 * (size_t)i + 1] = r * std::sin(a);
    }
    for (int lv = 0; lv < 3; ++lv) {
      const double center[3] = {150.0 + lv, 120.0 - lv, 0.3 * lv};
      double flat_best = 0.0;
      int64_t flat = -1;
      flat_best = oracle_best_window(&m, pts.data(), n, &levels[lv], center, &flat);
      check(n == 0 || flat >= 0, "best window without an index");
      double pose[3] = {1.0, 0.5, 0.2}, cov[9] = {0};
      int64_t am = -1, scored = 0;
      const double resp = oracle_scan_match(&m, pts.data(), n, &levels[lv], pose, cov, &am, &scored);
      check(std::isfinite(resp), "non-finite response");
      (void)flat_best;
    }
    double pose[3] = {1.0, 0.5, 0.2}, cov[9] = {0};
    const double s = oracle_scan_matchers(&m, pts.data(), n, levels, 1, pose, cov);
    check(std::isfinite(s), "non-finite 3-level score");
    // the whole coarse window's scores (30 x 13^2 candidates)
    std::vector<double> sc(30 * 13 * 13);
    const double c0[3] = {150.0, 120.0, 0.0};
    check(oracle_score_window(&m, pts.data(), n, &levels[0], c0, sc.data(), (int64_t)sc.size()) == 0,
          "coarse window size");
  }
  // FAST (branch and bound, max_depth 4; params.py FAST_PARAM)
  {
    oracle_param_c fast{0.8, 0.01, 0.523, 0.00349, 0.5, 100, 4, 0, 3};
    std::vector<double> pts(2 * 360);
    for (int i = 0; i < 360; ++i) {
      pts[2 * (size_t)i] = 40.0 * std::cos(i * M_PI / 180.0);
      pts[2 * (size_t)i + 1] = 40.0 * std::sin(i * M_PI / 180.0);
    }
    double pose[3] = {1.0, 0.5, 0.0}, cov[9] = {0};
    int64_t am = -1, scored = 0;
    const double r = oracle_scan_match(&m, pts.data(), 360, &fast, pose, cov, &am, &scored);
    check(std::isfinite(r), "non-finite FAST response");
  }
  // std::sort over keys with heavy ties (introsort, heap fallback and insertion sort)
  for (int64_t n : {0, 1, 16, 17, 64, 257, 5070}) {
    std::vector<double> keys((size_t)n);
    for (int64_t i = 0; i < n; ++i) keys[(size_t)i] = (double)(rng() % 7) * 0.125;
    std::vector<int64_t> order((size_t)n, -1);
    oracle_std_sort_order(keys.data(), n, order.data());
    std::vector<char> seen((size_t)n, 0);
    for (int64_t i = 0; i < n; ++i) {
      check(order[(size_t)i] >= 0 && order[(size_t)i] < n && !seen[(size_t)order[(size_t)i]], "not a permutation");
      if (order[(size_t)i] >= 0 && order[(size_t)i] < n) seen[(size_t)order[(size_t)i]] = 1;
      if (i > 0) check(keys[(size_t)order[(size_t)i - 1]] >= keys[(size_t)order[(size_t)i]], "not descending");
    }
  }
  // map building (f1) and the map check (f4): both cell kinds, blur on and off,
  // auto-resize growing the map past every edge, the sped-up batch rebuild
  for (int kind = 0; kind < 2; ++kind)
    for (int blur = 0; blur < 2; ++blur) {
      void* g = oracle_gridmap_create(kind, 0.05, 120, 100, -3.0, -2.5, 0.05, 0.5f);
      oracle_gridmap_set_options(g, 1, 0, 0.0, 0.5);
      std::vector<double> scan(2 * 361);
      std::vector<double> poses, origins, all;
      std::vector<int64_t> offs{0};
      for (int k = 0; k < 6; ++k) {
        for (int i = 0; i < 361; ++i) {  // meters in the sensor frame; a few far beams force resizes
          const double r = (i % 45 == 0) ? 9.0 + 2.0 * k : 1.0 + 3.0 * u(rng);
          const double a = M_PI * i / 180.0;
          scan[2 * (size_t)i] = r * std::cos(a);
          scan[2 * (size_t)i + 1] = r * std::sin(a);
        }
        const double origin[2] = {0.1, 0.0}, pose[3] = {0.3 * k, -0.2 * k, 0.1 * k};
        oracle_gridmap_update_by_range(g, scan.data(), 361, origin, pose, blur);
        const double pen = oracle_gridmap_feedback_penalty(g, scan.data(), 361, origin, pose, 100, 0.3, 2.0, blur);
        check(std::isfinite(pen), "non-finite map penalty");
        all.insert(all.end(), scan.begin(), scan.end());
        offs.push_back(offs.back() + 361);
        origins.insert(origins.end(), origin, origin + 2);
        poses.insert(poses.end(), pose, pose + 3);
      }
      int32_t ints[8];
      double dbl[7];
      oracle_gridmap_info(g, ints, dbl);
      check(ints[0] >= 120 && ints[1] >= 100, "map shrank");
      oracle_gridmap_destroy(g);
      for (int speedup = 0; speedup < 2; ++speedup) {
        void* h = oracle_gridmap_create(kind, 0.05, 400, 400, -10.0, -10.0, 0.05, 0.5f);
        oracle_gridmap_init_with_range_vec(h, all.data(), offs.data(), 6, origins.data(), poses.data(), blur, speedup);
        oracle_gridmap_destroy(h);
      }
    }
  {
    std::vector<int32_t> line(2 * 512);
    const int n = oracle_bresenham(-7, 3, 250, -40, line.data(), 512);
    check(n == 258, "bresenham length");
  }
  if (failures) return 1;
  std::printf("san_driver ok\n");
  return 0;
}
