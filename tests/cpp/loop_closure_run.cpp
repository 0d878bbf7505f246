// A C++ caller of the sharded loop-closure C-ABI (include/csm_loop_closure.h)
// the way the reference's back end would call it from TryCloseLoop
// (pose_graph/range_scan_pose_graph.cpp:299-355): no Python, no torch.
// Synthetic submaps and one query scan; the answer (max score, lowest global
// index) is compared with the CPU oracle's per-submap argmax (test
// infrastructure, oracle/liboracle.so) reduced the same way.
//
//   loop_closure_run check [n_submaps] [devices]   exit 0 = identical to the oracle, both searches
//   loop_closure_run bench [n_submaps] [devices]   one JSON line: ms per query, both searches
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "csm_loop_closure.h"

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
double oracle_best_window(const oracle_map_c* mc, const double* pts, int n, const void* param, const double center[3],
                          int64_t* flat);
void oracle_set_threads(int n);
}

namespace {

uint64_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ULL + 1442695040888963407ULL;
  return s >> 33;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "check";
  const int n_sub = argc > 2 ? std::atoi(argv[2]) : 24;
  const int n_dev = argc > 3 ? std::atoi(argv[3]) : 1;
  const int sx = 240, sy = 200;
  const double res = 0.05;
  // submaps: rooms of walls (1.0) on free space (0.1), unknown (0.3) border;
  // every submap different, submap 7 holds the room the scan was taken in
  std::vector<float> cells((size_t)n_sub * sx * sy);
  std::vector<double> offsets(2 * (size_t)n_sub);
  uint64_t seed = 20261016;
  for (int g = 0; g < n_sub; ++g) {
    float* m = cells.data() + (size_t)g * sx * sy;
    const int x0 = 30 + (int)(lcg(seed) % 40), y0 = 25 + (int)(lcg(seed) % 40);
    const int x1 = x0 + 110 + (int)(lcg(seed) % 50), y1 = y0 + 90 + (int)(lcg(seed) % 40);
    for (int y = 0; y < sy; ++y)
      for (int x = 0; x < sx; ++x) {
        float v = 0.3f;
        if (x >= x0 && x <= x1 && y >= y0 && y <= y1) v = 0.1f;
        if (((x == x0 || x == x1) && y >= y0 && y <= y1) || ((y == y0 || y == y1) && x >= x0 && x <= x1)) v = 1.0f;
        m[(size_t)y * sx + x] = v;
      }
    offsets[2 * (size_t)g] = 0.5 * (double)(lcg(seed) % 8);
    offsets[2 * (size_t)g + 1] = -0.25 * (double)(lcg(seed) % 8);
  }
  // the query: 360 beams from the centre of submap 7's room (map cells,
  // sensor frame), the pose a little off
  std::vector<double> pts;
  {
    const float* m = cells.data() + (size_t)(7 % n_sub) * sx * sy;
    const double cx = sx / 2.0, cy = sy / 2.0;
    for (int k = 0; k < 360; ++k) {
      const double a = k * M_PI / 180.0;
      for (double r = 1.0; r < 150.0; r += 0.5) {
        const int x = (int)(cx + r * std::cos(a)), y = (int)(cy + r * std::sin(a));
        if (x < 0 || y < 0 || x >= sx || y >= sy) break;
        if (m[(size_t)y * sx + x] == 1.0f) {
          pts.push_back(r * std::cos(a));
          pts.push_back(r * std::sin(a));
          break;
        }
      }
    }
  }
  const int n_pts = (int)pts.size() / 2;
  const int g7 = 7 % n_sub;
  double pose_world[3] = {(sx / 2.0 + 3.0) * res - offsets[2 * (size_t)g7],
                          (sy / 2.0 - 2.0) * res - offsets[2 * (size_t)g7 + 1], 0.06};
  csm_param p{};
  p.search_space_size = 1.2;
  p.search_space_resolution = res;
  p.search_angle_offset = 0.35;
  p.search_angle_resolution = 0.0349;
  p.response_threshold = 0.5;
  p.use_point_size = 100;
  p.type = CSM_COARSE;
  csm_map_info info{};
  info.resolution = res;
  info.size_x = sx;
  info.size_y = sy;

  std::vector<int32_t> devs((size_t)n_dev);
  for (int i = 0; i < n_dev; ++i) devs[(size_t)i] = i;
  csm_loop_closure* lc = nullptr;
  int st = csm_loop_closure_create(n_dev, devs.data(), &lc);
  if (st != CSM_OK) {
    std::fprintf(stderr, "csm_loop_closure_create: %d %s\n", st, csm_loop_closure_last_error(lc));
    if (lc) csm_loop_closure_destroy(lc);
    return 2;
  }
  if ((st = csm_loop_closure_set_submaps(lc, cells.data(), n_sub, &info, offsets.data(), 1)) != CSM_OK) {
    std::fprintf(stderr, "set_submaps: %s\n", csm_loop_closure_last_error(lc));
    return 2;
  }
  csm_loop_closure_result r[2];
  double ms[2] = {0, 0};
  for (int s = 0; s < 2; ++s) {
    if ((st = csm_loop_closure_match(lc, pts.data(), n_pts, &p, pose_world, s, &r[s])) != CSM_OK) {  // warm
      std::fprintf(stderr, "match: %s\n", csm_loop_closure_last_error(lc));
      return 2;
    }
    const int reps = 5;
    const double t = now_ms();
    for (int k = 0; k < reps; ++k) csm_loop_closure_match(lc, pts.data(), n_pts, &p, pose_world, s, &r[s]);
    ms[s] = (now_ms() - t) / reps;
  }
  // the oracle: every submap's whole window, reduced to (max, lowest global index)
  int32_t na = (int32_t)std::floor(2 * p.search_angle_offset / p.search_angle_resolution) + 1;
  int32_t ns = (int32_t)std::floor(p.search_space_size / p.search_space_resolution + 0.5) + 1;
  csm_window_dims(&p, &na, &ns);
  const int64_t n_cand = (int64_t)na * ns * ns;
  oracle_set_threads(8);
  double bs = -1e300;
  int64_t bi = -1;
  const double sc = 1.0 / res;
  for (int g = 0; g < n_sub; ++g) {
    oracle_map_c mc{cells.data() + (size_t)g * sx * sy, 1, sx, sy, res, offsets[2 * (size_t)g],
                    offsets[2 * (size_t)g + 1], 0, 0.3f};
    const double c[3] = {sc * pose_world[0] + sc * offsets[2 * (size_t)g], sc * pose_world[1] + sc * offsets[2 * (size_t)g + 1],
                         pose_world[2]};
    int64_t flat = -1;
    const double s = oracle_best_window(&mc, pts.data(), n_pts, &p, c, &flat);
    const int64_t gi = (int64_t)g * n_cand + flat;
    if (s > bs || (s == bs && gi < bi)) {
      bs = s;
      bi = gi;
    }
  }
  const bool ok = r[0].score == bs && r[0].global_index == bi && r[1].score == bs && r[1].global_index == bi &&
                  r[0].x == r[1].x && r[0].y == r[1].y && r[0].angle == r[1].angle;
  std::printf("{\"mode\": \"%s\", \"devices\": %d, \"submaps\": %d, \"beams\": %d, \"candidates_per_submap\": %lld, "
              "\"pyramid_ms\": %.4f, \"exhaustive_ms\": %.4f, \"score\": %.17g, \"global_index\": %lld, "
              "\"submap\": %d, \"oracle_score\": %.17g, \"oracle_global_index\": %lld, \"identical\": %s}\n",
              mode, n_dev, n_sub, n_pts, (long long)n_cand, ms[0], ms[1], r[0].score, (long long)r[0].global_index,
              r[0].submap, bs, (long long)bi, ok ? "true" : "false");
  csm_loop_closure_destroy(lc);
  return (std::strcmp(mode, "check") == 0 && !ok) ? 1 : 0;
}
