// csm_bnb.hip — device scoring for the FAST (branch-and-bound) matcher.
//
// Reference: BranchAndBoundCorrelateScanMatcher (correlate_scan_matcher.h:271-502).
// The reference scores the lowest-resolution grid exhaustively (:333-393) and
// then walks a depth-first search whose children are re-scored on the fly
// (:398-476). Every node of that tree is a candidate at full resolution
// (ScoreCandidates reads the same grid with the same beam rule), so its score
// does not depend on the search order: this kernel scores EVERY node of the
// tree once, in parallel, and the host replays the reference's search over
// the table (csm_api.cpp, bnb_search) — same visiting order, same pruning,
// same std::sort calls, bit-identical result.
//
// Node (level l, i, j) of angle a: level max_depth is the lowest-resolution
// grid (n_low x n_low), level l has n_low << (max_depth - l) nodes per axis.
// Its x is the reference's own expression chain: the lowest candidate's
// search_space_start_x + i_low * space_step_factor (:363), then + half_width
// of every depth d > l on the path whose offset bit is set (:455-460; an
// offset of 0.0 leaves the double unchanged, so it is skipped).
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

__global__ __launch_bounds__(256) void score_tree_kernel(TreeWork T, const ScanWork* __restrict__ scans,
                                                         const double2* __restrict__ pts,
                                                         const AngleEntry* __restrict__ angles,
                                                         double* __restrict__ out) {
  const int64_t per_window = (int64_t)T.n_angles * T.nodes_per_angle;
  const int64_t total = per_window * T.n_windows;
  for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(gid / per_window);
    const int64_t rw = gid - (int64_t)w * per_window;
    const int a = (int)(rw / T.nodes_per_angle);
    int64_t t = rw - (int64_t)a * T.nodes_per_angle;
    // level: offsets grow from the lowest-resolution level downwards
    int level = T.depth;
    int64_t m = T.n_low;
    while (t >= m * m) {
      t -= m * m;
      m <<= 1;
      --level;
    }
    const int i = (int)(t / m), j = (int)(t - (t / m) * m);
    const int shift = T.depth - level;
    const ScanWork S = scans[w];
    double x = S.x0 + (i >> shift) * T.f_low;  // :363
    double y = S.y0 + (j >> shift) * T.f_low;  // :366
    for (int s = 0; s < shift; ++s) {
      const int d = T.depth - s;  // the half_width of depth d (:454-455)
      if ((i >> (shift - 1 - s)) & 1) x = x + T.hw[d];
      if ((j >> (shift - 1 - s)) & 1) y = y + T.hw[d];
    }
    const AngleEntry ae = angles[S.angle_off + a];
    const double2* P = pts + S.pts_off;
    double acc = 0.0;
    for (int b = 0; b < S.n_used; ++b) {  // :369-375 / :419-424, beam order
      const double2 p = P[(int64_t)b * S.step];
      const double lx = ae.cosine * p.x - ae.sine * p.y;
      const double ly = ae.sine * p.x + ae.cosine * p.y;
      const int gx = (int)((lx + x) + 0.5);
      const int gy = (int)((ly + y) + 0.5);
      const bool inb = ((unsigned)gx < (unsigned)T.size_x) & ((unsigned)gy < (unsigned)T.size_y);
      const float v = T.grid[inb ? (int64_t)gy * T.size_x + gx : 0];
      acc += (double)(inb ? v : T.outside);
    }
    out[gid] = acc / S.divisor;  // :377 / :426
  }
}

}  // namespace

hipError_t launch_score_tree(const TreeWork& T, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, hipStream_t stream) {
  const int64_t total = (int64_t)T.n_angles * T.nodes_per_angle * T.n_windows;
  if (total <= 0 || T.depth < 0 || T.depth > kTreeMaxDepth) return hipErrorInvalidValue;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(score_tree_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, T, d_scans,
                     reinterpret_cast<const double2*>(d_pts), d_angles, d_out);
  return hipGetLastError();
}

}  // namespace csm
