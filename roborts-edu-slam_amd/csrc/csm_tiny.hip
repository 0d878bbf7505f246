// csm_tiny.hip — v8 "tiny window" scoring kernel: sub-cell window steps whose
// whole x (and y) span is under one cell, (n_space - 1) * f < 1 (the
// super-fine level of every shipped parameter set: 3 steps of 0.2 cells).
//
// Candidate (j, k) of angle a reads, for beam b, cell
// (trunc((lx + x_j) + 0.5), trunc((ly + y_k) + 0.5)) with x_j = x0 + j*f
// (correlate_scan_matcher.h:569-572, :637-662). With the span under a cell the
// columns of j = 0 .. n_space-1 take at most two values, ix_0 and ix_0 + 1
// (fp addition and trunc are monotone; the host checks (n_space - 1) * f < 1
// and the kernel checks each beam), rows likewise: a beam touches a 2 x 2
// block of cells. So the lanes are beams, not candidates: lane l rotates beam
// cb + l once, computes its n_space columns and rows with the reference's own
// expressions (no margin argument needed: the indices are exact), loads the
// 2 x 2 block with two 8-byte loads and adds, per candidate, the cell its
// offsets pick. A wave sums its (window, angle)'s beams 64 at a time; the
// candidates' sums meet across lanes at the end. Beams outside the zero-padded
// part of the grid (negative indices, far past the high edges) or wider than
// two cells take the cell-by-cell path with the reference's bounds check.
// Measured 0.128 ms per super-fine launch on config 2 (2048 windows x 21
// angles, 1081 beams) against 0.191 ms for the LDS-DMA row kernel; VALU-bound
// (the fp64 index expressions); two chunks per iteration measured the same.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_device.hpp"
#include "csm_tail.hpp"
#include "csm_internal.hpp"

namespace csm {
namespace {

typedef int32_t v2i __attribute__((ext_vector_type(2)));

template <int NS, bool BEST>
__global__ __launch_bounds__(64) void score_tiny_kernel(LevelWork L, const ScanWork* __restrict__ scans,
                                                        const double2* __restrict__ pts,
                                                        const AngleEntry* __restrict__ angles,
                                                        double* __restrict__ out,
                                                        BestPartial* __restrict__ partials) {
  constexpr int NC = NS * NS;
  static_assert(NC <= 64, "one candidate per lane in the epilogue");
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  dev::clear_word(L);
  const int win = bid / L.n_angles;
  const int a = bid - win * L.n_angles;
  const ScanWork S = scans[win];
  const AngleEntry ae = angles[S.angle_off + a];
  const int lane = threadIdx.x;
  const double f = L.step_cells;
  double xj[NS], yk[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    xj[j] = S.x0 + j * f;  // :569
    yk[j] = S.y0 + j * f;  // :572
  }
  const int sx = L.size_x, sy = L.size_y, pitch = L.pitch;
  // the fast path's 2 x 2 block stays inside the zero padding
  const int gx_hi = pitch - 2, gy_hi = sy + kGridiPadRows - 2;
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(L.gridi_stride * 4), 0x00020000);
  const double2* __restrict__ P = pts + S.pts_off;
  const int n_used = S.n_used, step = S.step;

  int64_t acc[NS][NS];
  int32_t part[NS][NS];  // <= 16 chunks of |value| < 2^26 before each fold
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[j][k] = part[j][k] = 0;
  double2 pn = P[(int64_t)min(lane, n_used - 1) * step];
  int chunk = 0;
  for (int cb = 0; cb < n_used; cb += 64, ++chunk) {
    const double2 p = pn;
    pn = P[(int64_t)min(cb + 64 + lane, n_used - 1) * step];
    const bool live = cb + lane < n_used;
    const double lx = ae.cosine * p.x - ae.sine * p.y;  // :179
    const double ly = ae.sine * p.x + ae.cosine * p.y;  // :180
    int gx[NS], gy[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      gx[j] = (int)((lx + xj[j]) + 0.5);  // :647
      gy[j] = (int)((ly + yk[j]) + 0.5);  // :648
    }
    const bool fast = gx[0] >= 0 && gy[0] >= 0 && gx[0] <= gx_hi && gy[0] <= gy_hi && gx[NS - 1] - gx[0] <= 1 &&
                      gy[NS - 1] - gy[0] <= 1;
    const int off = fast ? (gy[0] * pitch + gx[0]) * 4 : 0;
    const v2i r0 = __builtin_bit_cast(v2i, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 0));
    const v2i r1 = __builtin_bit_cast(v2i, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off + pitch * 4, 0, 0));
    if (live && fast) {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const v2i r = gy[k] != gy[0] ? r1 : r0;
#pragma unroll
        for (int j = 0; j < NS; ++j) part[j][k] += gx[j] != gx[0] ? r.y : r.x;
      }
    } else if (live) {  // cell by cell, the reference's bounds check (outside: 0)
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const bool in = (unsigned)gx[j] < (unsigned)sx && (unsigned)gy[k] < (unsigned)sy;
          part[j][k] += in ? gi[(int64_t)gy[k] * pitch + gx[j]] : 0;
        }
    }
    if ((chunk & 15) == 15) {
#pragma unroll
      for (int j = 0; j < NS; ++j)
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          acc[j][k] += part[j][k];
          part[j][k] = 0;
        }
    }
  }
  // candidate (j, k)'s sum over the lanes, into lane j * NS + k
  int64_t mine = 0;
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int64_t v = dev::wave_sum_i64(acc[j][k] + part[j][k]);
      if (lane == j * NS + k) mine = v;
    }
  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
  double lmax = -INFINITY;  // the fused finish (csm_tail.hpp): this lane's max, any NaN
  bool lnan = false;
  if (lane < NC) {
    const int j = lane / NS, k = lane - (lane / NS) * NS;
    const double accd = (double)(mine + (int64_t)n_used * L.outside_i) * L.int_scale;
    const double score = dev::penalized(L, S, accd, S.x0 + j * f /* :569 */, S.y0 + k * f /* :572 */, ae.angle);
    const int64_t flat = ((int64_t)a * NS + j) * NS + k;
    if (BEST) {
      bs = score;
      bf = flat;
    } else {
      tail::store_score(L, out + S.out_off + flat, score);
      lnan = score != score;
      lmax = score;
    }
  }
  if (!BEST && L.tail.on) {
    __shared__ __attribute__((aligned(16))) char tail_a[tail::kBytesA];
    __shared__ __attribute__((aligned(16))) char tail_b[tail::kBytesB];
    tail::finish(L, S, angles, out, a, lmax, lnan, tail_a, tail_b);
  }
  if (BEST) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double os = __shfl_down(bs, o, 64);
      const int64_t of = __shfl_down(bf, o, 64);
      if (dev::better(os, of, bs, bf)) {
        bs = os;
        bf = of;
      }
    }
    if (lane == 0) partials[(int64_t)win * L.blocks_per_scan + a] = BestPartial{bs, bf};
  }
}

template <int NS>
hipError_t launch_tiny(const LevelWork& L, const ScanWork* s, const double2* p, const AngleEntry* an, double* out,
                       BestPartial* part, unsigned nblk, hipStream_t stream) {
  if (part)
    hipLaunchKernelGGL((score_tiny_kernel<NS, true>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  else
    hipLaunchKernelGGL((score_tiny_kernel<NS, false>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  return hipGetLastError();
}

}  // namespace

bool tiny_supported(int ns, double f) { return ns >= 2 && ns <= 4 && f > 0.0 && (double)(ns - 1) * f < 1.0; }

hipError_t launch_score_tiny(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                             hipStream_t stream) {
  const int64_t nblk = (int64_t)L.n_scans * L.n_angles;
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || !tiny_supported(ns, L.step_cells) ||
      L.blocks_per_scan != L.n_angles || L.pitch < L.size_x + kGridiPadCols || L.gridi_stride * 4 >= INT32_MAX)
    return hipErrorInvalidValue;
  const double2* p = reinterpret_cast<const double2*>(d_pts);
  const unsigned n = (unsigned)nblk;
  switch (ns) {
    case 2: return launch_tiny<2>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 3: return launch_tiny<3>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 4: return launch_tiny<4>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace csm
