// csm_optimize.hip — per-point work of the Gauss-Newton scan matcher
// (BasedOptimizeScanMatch::UpdateCost, optimize_scan_matcher.h:154-221;
// SURVEY.md 8f row f3) for gfx950.
//
// One workgroup per scan and Gauss-Newton iteration. The 256 lanes project,
// gather and differentiate points in parallel (4 corner reads per point from
// the resident fp32 grid, no LDS staging: 16 B per point is nothing next to
// the launch latency), write each point's ten terms (cost, six lower-triangle
// entries of J^T J, three of -J^T e) to LDS, and ten lanes then add them up
// one accumulator each in point order. That order is the reference's loop
// order, so every sum is the reference's fp64 sum bit for bit; a tree
// reduction would not be. The host (csm_api.cpp) computes cos/sin with glibc,
// solves the 3x3 system and steps the pose between launches.
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

constexpr int kOptChunk = 512;  // points per LDS pass (10 x 4 KB of terms)

__device__ __forceinline__ double opt_cell(const float* g, int32_t sx, int64_t ncell, float outside, int x, int y) {
  // GetCell's flat index (grid_map_base.h:352-354); past the array: outside
  const int64_t idx = (int64_t)y * sx + x;
  return (idx >= 0 && idx < ncell) ? (double)g[idx] : (double)outside;
}

__global__ __launch_bounds__(kBlock) void optimize_cost_kernel(OptArgs A) {
  const int s = blockIdx.x;
  const OptScan sc = A.scans[s];
  if (!sc.active) return;  // uniform over the block
  const int64_t p0 = A.offsets[s];
  const int64_t n = A.offsets[s + 1] - p0;
  const int64_t ncell = (int64_t)A.size_x * A.size_y;
  const double fsx = (double)A.size_x, fsy = (double)A.size_y;
  __shared__ double terms[10][kOptChunk];
  __shared__ int32_t ok[kOptChunk];
  const int tid = threadIdx.x;
  double acc = 0.0;
  int32_t cnt = 0;
  for (int64_t base = 0; base < n; base += kOptChunk) {
    const int m = (int)((n - base < kOptChunk) ? (n - base) : kOptChunk);
    for (int i = tid; i < m; i += kBlock) {
      const double2 lp = reinterpret_cast<const double2*>(A.pts)[p0 + base + i];
      const double lx = lp.x, ly = lp.y;
      // rotation * local_point + translation (:94-97, :167)
      const double x = (sc.c * lx + (-sc.s) * ly) + sc.tx;
      const double y = (sc.s * lx + sc.c * ly) + sc.ty;
      const bool in = x > 0 && x < fsx && y > 0 && y < fsy;  // PointInMap (grid_map_base.h:330-337)
      ok[i] = in ? 1 : 0;
      if (!in) continue;
      const double x0 = floor(x), y0 = floor(y), x1 = ceil(x), y1 = ceil(y);
      const double p00 = opt_cell(A.grid, A.size_x, ncell, A.outside, (int)x0, (int)y0);
      const double p01 = opt_cell(A.grid, A.size_x, ncell, A.outside, (int)x0, (int)y1);
      const double p10 = opt_cell(A.grid, A.size_x, ncell, A.outside, (int)x1, (int)y0);
      const double p11 = opt_cell(A.grid, A.size_x, ncell, A.outside, (int)x1, (int)y1);
      double r = ((y - y0) * (p11 * (x - x0) + p01 * (x1 - x)) + (y1 - y) * (p10 * (x - x0) + p00 * (x1 - x)));
      r = (r >= 0) ? ((r <= 1) ? r : 1.0) : 0.0;
      const double e = 1 - r;
      const double ds02 = ((-sc.s) * lx - sc.c * ly);  // de_s (:200-201)
      const double ds12 = (sc.c * lx - sc.s * ly);
      const double dm0 = ((y - y0) * (p11 - p01) + (y1 - y) * (p10 - p00));  // de_m (:203-204)
      const double dm1 = ((x - x0) * (p11 - p10) + (x1 - x) * (p01 - p00));
      const double n0 = -dm0, n1 = -dm1;  // J = -de_m * de_s (:207)
      const double j0 = n0 * 1.0 + n1 * 0.0;
      const double j1 = n0 * 0.0 + n1 * 1.0;
      const double j2 = n0 * ds02 + n1 * ds12;
      terms[0][i] = e * e;
      terms[1][i] = j0 * j0;
      terms[2][i] = j1 * j0;
      terms[3][i] = j1 * j1;
      terms[4][i] = j2 * j0;
      terms[5][i] = j2 * j1;
      terms[6][i] = j2 * j2;
      terms[7][i] = (-j0) * e;
      terms[8][i] = (-j1) * e;
      terms[9][i] = (-j2) * e;
    }
    __syncthreads();
    if (tid < 10) {
      for (int i = 0; i < m; ++i)
        if (ok[i]) acc = acc + terms[tid][i];
    } else if (tid == 10) {
      for (int i = 0; i < m; ++i) cnt += ok[i];
    }
    __syncthreads();
  }
  if (tid < 10) A.out[s].v[tid] = acc;
  if (tid == 10) A.out[s].valid = cnt;
}

}  // namespace

hipError_t launch_optimize_cost(const OptArgs& A, int32_t n_scans, hipStream_t stream) {
  if (n_scans <= 0) return hipSuccess;
  hipLaunchKernelGGL(optimize_cost_kernel, dim3((unsigned)n_scans), dim3(kBlock), 0, stream, A);
  return hipGetLastError();
}

}  // namespace csm
