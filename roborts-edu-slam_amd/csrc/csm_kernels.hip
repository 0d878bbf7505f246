// csm_kernels.hip — CDNA4 (gfx950) kernels of the correlative scan matcher.
//
// Hot path replaced: the theta x X x Y x beam loops of
// MultiResolutionCorrelateScanMatcher::ScanMatch / GetResponse
// (correlate_scan_matcher.h:552-584, 637-662) plus PenalizeResponse (:718-745).
//
// Mapping (DESIGN.md "Kernel"): one lane per candidate pose, CPL candidates per
// lane, 256-thread workgroups, every workgroup inside one window (scan x level).
// Lanes are ordered x-fastest inside a row of the window so that, for a given
// beam, the 64 lanes of a wave gather from a few adjacent grid rows (the
// candidate window maps onto a small patch around each beam endpoint). The
// window's subsampled beams are staged in LDS 1024 at a time and broadcast to
// all lanes. Each lane accumulates its beams sequentially in fp64, in the
// reference's beam order, so the score is bit-identical to the reference's
// for ANY fp32 grid (not only for the exactly-summable values real maps hold).
//
// Exactness: every double expression is evaluated in the reference's order
// with contraction disabled (pragma below + -ffp-contract=off), the cast to
// int truncates toward zero (v_cvt_i32_f64), and cos/sin come from the host.
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {

namespace {

// XCD-aware, bijective block remap (cdna_hip_programming.md T1): blocks that
// share a logical neighbourhood (one window) land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

struct Lane {
  double x, y, c, s, acc;
  int64_t flat;  // reference enumeration index (theta, x, y)
  double angle;
  bool valid;
};

template <int CPL>
__device__ __forceinline__ void setup_lanes(const LevelWork& L, const ScanWork& S,
                                            const AngleEntry* __restrict__ angles,
                                            int blk, Lane (&ln)[CPL]) {
  const int64_t nss = (int64_t)L.n_space * L.n_space;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int64_t q = (int64_t)blk * (kBlock * CPL) + (int64_t)i * kBlock + threadIdx.x;
    const bool valid = q < L.n_cand;
    const int64_t qq = valid ? q : 0;
    const int64_t a = qq / nss;
    const int64_t r = qq - a * nss;
    const int k = (int)(r / L.n_space);     // y index (row)
    const int j = (int)(r - (int64_t)k * L.n_space);  // x index (fastest in lanes)
    const AngleEntry ae = angles[S.angle_off + a];
    ln[i].x = S.x0 + j * L.step_cells;      // :569
    ln[i].y = S.y0 + k * L.step_cells;      // :572
    ln[i].c = ae.cosine;
    ln[i].s = ae.sine;
    ln[i].angle = ae.angle;
    ln[i].acc = 0.0;
    ln[i].flat = (a * L.n_space + j) * L.n_space + k;  // order of :552-583
    ln[i].valid = valid;
  }
}

// Sum the window's beams for each of this lane's candidates (GetResponse
// :645-654). All threads of the block must call this (barriers inside).
template <int CPL>
__device__ __forceinline__ void accumulate(const LevelWork& L, const ScanWork& S,
                                           const double2* __restrict__ pts,
                                           const float* __restrict__ grid,
                                           double2* __restrict__ lds, Lane (&ln)[CPL]) {
  const int sx = L.size_x, sy = L.size_y;
  const float outside = L.outside;
  for (int base = 0; base < S.n_used; base += kChunk) {
    const int nb = min(kChunk, S.n_used - base);
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += kBlock)
      lds[b] = pts[S.pts_off + (int64_t)(base + b) * S.step];
    __syncthreads();
#pragma unroll 4
    for (int b = 0; b < nb; ++b) {
      const double2 p = lds[b];
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        // LUT entry of :179-180, then the endpoint cell of :647-648.
        const double lx = ln[i].c * p.x - ln[i].s * p.y;
        const double ly = ln[i].s * p.x + ln[i].c * p.y;
        const int gx = (int)((lx + ln[i].x) + 0.5);
        const int gy = (int)((ly + ln[i].y) + 0.5);
        const bool inb = ((unsigned)gx < (unsigned)sx) & ((unsigned)gy < (unsigned)sy);
        const int idx = inb ? gy * sx + gx : 0;
        float v = grid[idx];
        v = inb ? v : outside;
        ln[i].acc += (double)v;
      }
    }
  }
}

// Divisor (:659) and centre penalty (:718-745) of one candidate.
__device__ __forceinline__ double finish_score(const LevelWork& L, const ScanWork& S,
                                              const Lane& ln) {
  double score = ln.acc / S.divisor;
  if (L.use_penalty) {
    // util::DoubleEqual(score, 0.0) with kDoubleTolerance = 1e-6.
    const bool is_zero = (score < 0.0) ? (score >= -1e-06) : (score <= 1e-06);
    if (!is_zero) {
      const double dx = ln.x - S.cx, dy = ln.y - S.cy;
      double d2 = dx * dx + dy * dy;
      d2 *= (L.mres * L.mres);
      double dp = 1.0 - (L.dist_gain * d2 / (L.size / 2));
      dp = dp < 0.5 ? 0.5 : dp;  // std::max(dp, 0.5)
      double da = ln.angle - S.ct;
      da = da * da;
      double ap = 1.0 - (0.25 * da / 0.349);
      ap = ap < 0.9 ? 0.9 : ap;
      score = score * (dp * ap);
    }
  }
  return score;
}

template <int CPL>
__global__ __launch_bounds__(kBlock) void score_all_kernel(
    LevelWork L, const ScanWork* __restrict__ scans, const double2* __restrict__ pts,
    const AngleEntry* __restrict__ angles, double* __restrict__ out) {
  __shared__ double2 lds[kChunk];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int scan = bid / L.blocks_per_scan;
  const int blk = bid - scan * L.blocks_per_scan;
  const ScanWork S = scans[scan];
  const float* grid = L.grid + (int64_t)S.grid_index * L.grid_stride;
  Lane ln[CPL];
  setup_lanes<CPL>(L, S, angles, blk, ln);
  accumulate<CPL>(L, S, pts, grid, lds, ln);
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    if (ln[i].valid) out[S.out_off + ln[i].flat] = finish_score(L, S, ln[i]);
}

__device__ __forceinline__ bool better(double s, int64_t f, double bs, int64_t bf) {
  return (s > bs) || (s == bs && f < bf);
}

template <int CPL>
__global__ __launch_bounds__(kBlock) void score_best_kernel(
    LevelWork L, const ScanWork* __restrict__ scans, const double2* __restrict__ pts,
    const AngleEntry* __restrict__ angles, BestPartial* __restrict__ partials) {
  __shared__ double2 lds[kChunk];
  __shared__ double red_s[kBlock / 64];
  __shared__ int64_t red_f[kBlock / 64];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int scan = bid / L.blocks_per_scan;
  const int blk = bid - scan * L.blocks_per_scan;
  const ScanWork S = scans[scan];
  const float* grid = L.grid + (int64_t)S.grid_index * L.grid_stride;
  Lane ln[CPL];
  setup_lanes<CPL>(L, S, angles, blk, ln);
  accumulate<CPL>(L, S, pts, grid, lds, ln);
  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    if (!ln[i].valid) continue;
    const double s = finish_score(L, S, ln[i]);
    if (better(s, ln[i].flat, bs, bf)) {
      bs = s;
      bf = ln[i].flat;
    }
  }
  // wave reduce (64 lanes), then across the block's 4 waves
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double os = __shfl_down(bs, off, 64);
    const int64_t of = __shfl_down(bf, off, 64);
    if (better(os, of, bs, bf)) {
      bs = os;
      bf = of;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red_s[wave] = bs;
    red_f[wave] = bf;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w)
      if (better(red_s[w], red_f[w], bs, bf)) {
        bs = red_s[w];
        bf = red_f[w];
      }
    partials[(int64_t)scan * L.blocks_per_scan + blk] = BestPartial{bs, bf};
  }
}

__global__ __launch_bounds__(kBlock) void reduce_best_kernel(const BestPartial* __restrict__ in,
                                                             int32_t per, BestPartial* __restrict__ out) {
  __shared__ double red_s[kBlock / 64];
  __shared__ int64_t red_f[kBlock / 64];
  const int64_t w = blockIdx.x;
  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
  for (int i = threadIdx.x; i < per; i += kBlock) {
    const BestPartial p = in[w * per + i];
    if (better(p.score, p.flat, bs, bf)) {
      bs = p.score;
      bf = p.flat;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double os = __shfl_down(bs, off, 64);
    const int64_t of = __shfl_down(bf, off, 64);
    if (better(os, of, bs, bf)) {
      bs = os;
      bf = of;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red_s[wave] = bs;
    red_f[wave] = bf;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k)
      if (better(red_s[k], red_f[k], bs, bf)) {
        bs = red_s[k];
        bf = red_f[k];
      }
    out[w] = BestPartial{bs, bf};
  }
}

}  // namespace

hipError_t launch_score_all(const LevelWork& L, const ScanWork* d_scans, const double* d_pts_raw,
                            const AngleEntry* d_angles, double* d_out, int cpl,
                            hipStream_t stream) {
  const double2* d_pts = reinterpret_cast<const double2*>(d_pts_raw);
  const int64_t nblk = (int64_t)L.blocks_per_scan * L.n_scans;
  if (nblk <= 0 || nblk > INT32_MAX) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk), block(kBlock);
  switch (cpl) {
    case 1: hipLaunchKernelGGL(score_all_kernel<1>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out); break;
    case 2: hipLaunchKernelGGL(score_all_kernel<2>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out); break;
    case 4: hipLaunchKernelGGL(score_all_kernel<4>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_score_best(const LevelWork& L, const ScanWork* d_scans, const double* d_pts_raw,
                             const AngleEntry* d_angles, BestPartial* d_partials, int cpl,
                             hipStream_t stream) {
  const double2* d_pts = reinterpret_cast<const double2*>(d_pts_raw);
  const int64_t nblk = (int64_t)L.blocks_per_scan * L.n_scans;
  if (nblk <= 0 || nblk > INT32_MAX) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk), block(kBlock);
  switch (cpl) {
    case 1: hipLaunchKernelGGL(score_best_kernel<1>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_partials); break;
    case 2: hipLaunchKernelGGL(score_best_kernel<2>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_partials); break;
    case 4: hipLaunchKernelGGL(score_best_kernel<4>, grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_partials); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_reduce_best(const BestPartial* d_partials, int32_t blocks_per_scan,
                              int32_t n_windows, BestPartial* d_out, hipStream_t stream) {
  if (n_windows <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reduce_best_kernel, dim3(n_windows), dim3(kBlock), 0, stream, d_partials,
                     blocks_per_scan, d_out);
  return hipGetLastError();
}

}  // namespace csm
