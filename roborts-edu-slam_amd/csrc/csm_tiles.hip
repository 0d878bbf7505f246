// csm_tiles.hip — beam-tile scoring kernel (v5, INT mode, integer window step).
//
// Hot path: GetResponse over the (theta, x, y) window (correlate_scan_matcher.h
// :552-584, 637-662) plus PenalizeResponse (:718-745), for windows whose step
// is a whole number of map cells (res == map resolution: the coarse levels of
// the sim YAML and of config 1).
//
// v4 (csm_kernels.hip) fetched, for every beam, the NS grid rows an angle group
// needs as 16-byte LDS-DMA pieces: ~0.8 KB per group per beam, bounded by the
// TA and LDS write rate. Consecutive beams of a scan land on neighbouring
// cells (0.25 deg apart: < 1 cell per beam below 10 m), so the patches of T
// consecutive beams overlap almost entirely. Here a group fetches ONE
// TH x 32-cell box that holds the patches of T = 8 beams (its rows and
// columns are the union of the beams' row/column ranges), and the group's
// lanes then read all T beams from it: DMA traffic per beam drops ~T-fold.
// A tile whose patches do not fit (a depth jump inside it) is fetched beam by
// beam with the same code.
//
// Status: exact (parity tests run it through CSM_KERNEL=v5) but not the
// default: on config 2 it took 8.3 ms per step for the coarse level against
// v4's 7.0 (profiles/r01): 87 VALU instructions per wave-beam (v4: 55),
// 192 VGPRs (2 waves per SIMD) leaving each tile's DMA wait exposed (37% of
// wave cycles in s_waitcnt), and bank conflicts on the box reads.
//
// Exactness. Lane (theta, j) computes its own column index ix_j with the
// reference's expression for every beam, as v4 does. The rows use iy_k =
// iy_0 + k, which holds when the window step is exactly 1 cell and
// v0 = (ly + y_0) + 0.5 is positive and at least 1e-9 from an integer (the
// rounding of (ly + y_k) + 0.5 against v0 + k is below 1e-10 cells for any
// map under 2^20 cells). Otherwise (and for a column outside the box) the
// lane takes the exact path for that beam: per-candidate indices and direct
// loads. Sums are exact integers, so beam order and tiling change nothing.
#include "csm_device.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

using namespace dev;
typedef __attribute__((address_space(3))) int32_t lds_i32;

template <int NS, int T, bool BEST>
__global__ __launch_bounds__(64) void score_tiles_kernel(LevelWork L, const ScanWork* __restrict__ scans,
                                                         const double2* __restrict__ pts,
                                                         const AngleEntry* __restrict__ angles,
                                                         double* __restrict__ out,
                                                         BestPartial* __restrict__ partials) {
  constexpr int G = 64 / NS;           // angle groups per wave
  constexpr int TW = 32;               // box columns (8 pieces of 4 cells)
  constexpr int TH = NS + 11;          // box rows: NS + drift of the row base across a tile
  constexpr int PPR = TW / 4;          // pieces per box row
  constexpr int NP = G * TH * PPR;     // pieces per box set
  constexpr int NI = (NP + 63) / 64;   // DMA instructions per fetch
  constexpr int BOX = TH * TW;         // ints per group box
  static_assert(NS + 5 <= TW, "a single beam's patch (+ margins, alignment) must fit a box");
  __shared__ __attribute__((aligned(16))) int32_t img[NI * 256];
  __shared__ __attribute__((aligned(16))) int32_t zblk[NS * TW];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int win = bid / L.blocks_per_scan;
  const int blk = bid - win * L.blocks_per_scan;
  const ScanWork S = scans[win];
  const int lane = threadIdx.x;
  const int g = lane / NS;
  const int ge = g < G ? g : G - 1;  // idle lanes shadow lane (G-1, NS-1)
  const int r = g < G ? lane - g * NS : NS - 1;
  const int a_raw = blk * G + ge;
  const bool valid = (g < G) && (a_raw < L.n_angles);
  const int a = a_raw < L.n_angles ? a_raw : 0;
  const AngleEntry ae = angles[S.angle_off + a];
  const double f = L.step_cells;    // == 1.0 (host)
  const double x_0 = S.x0 + 0 * f;  // :569 at j = 0
  const double x_r = S.x0 + r * f;  // :569 at j = r
  const double y_0 = S.y0 + 0 * f;  // :572 at k = 0
  const int sx = L.size_x, sy = L.size_y;
  const int pitch = L.pitch;
  const double2* __restrict__ P = pts + S.pts_off;
  const int step = S.step;
  const int n_used = S.n_used;
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(L.gridi_stride * 4), 0x00020000);
  const int zero_off = sy * pitch * 4;  // byte offset of the appended zero row
  const int xa_max = pitch - TW;        // host: pitch >= TW, pitch % 4 == 0

  for (int t = lane; t < NS * TW; t += 64) zblk[t] = 0;
  __syncthreads();

  double2 pw = P[(int64_t)min(lane, n_used - 1) * step];  // beams pbase .. pbase+63
  int pbase = 0;

  int64_t acci[NS];
  int32_t part[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    acci[k] = 0;
    part[k] = 0;
  }

  for (int tb = 0; tb < n_used; tb += T) {
    if (tb - pbase >= 64) {
      pbase = tb;
      pw = P[(int64_t)min(tb + lane, n_used - 1) * step];
    }
    const int nb = min(T, n_used - tb);
    // per beam: own column, group row base and column base, regularity
    int cxs[T], rys[T], x0s[T];
    bool rgs[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int b = tb + min(t, nb - 1);
      const int l = b - pbase;
      const double px = bcast_lane(pw.x, l), py = bcast_lane(pw.y, l);
      const double lx = ae.cosine * px - ae.sine * py;  // :179
      const double ly = ae.sine * px + ae.cosine * py;  // :180
      cxs[t] = (int)((lx + x_r) + 0.5);                 // :647 for j = r
      x0s[t] = (int)((lx + x_0) + 0.5);                 // :647 for j = 0
      const double v0 = (ly + y_0) + 0.5;               // :648 for k = 0
      rys[t] = (int)v0;
      const double fr = v0 - (double)rys[t];
      rgs[t] = (v0 > 0.0) && (fr >= 1e-9) && (fr <= 1.0 - 1e-9);
      __builtin_amdgcn_sched_barrier(0);  // one beam's temporaries at a time
    }
    // Does every group's tile fit one box? (group-uniform; ballot over the
    // wave.) If not, the tile is fetched and summed beam by beam.
    const unsigned all = (nb >= 32) ? ~0u : ((1u << nb) - 1u);
    bool fit;
    {
      int mnx = INT32_MAX, mxx = INT32_MIN, mny = INT32_MAX, mxy = INT32_MIN;
#pragma unroll
      for (int t = 0; t < T; ++t)
        if (t < nb) {
          mnx = min(mnx, x0s[t]);
          mxx = max(mxx, x0s[t]);
          mny = min(mny, rys[t]);
          mxy = max(mxy, rys[t]);
        }
      fit = (mxx - mnx) + NS + 2 + 3 <= TW && (mxy - mny) + NS <= TH;
    }
    const bool allfit = __ballot(!fit) == 0;
    const int nruns = allfit ? 1 : nb;
#pragma unroll 1
    for (int q = 0; q < nruns; ++q) {
      const unsigned mask = allfit ? all : (1u << q);
      int mnx = INT32_MAX, mxx = INT32_MIN, mny = INT32_MAX;
#pragma unroll
      for (int t = 0; t < T; ++t)
        if ((mask >> t) & 1u) {
          mnx = min(mnx, x0s[t]);
          mxx = max(mxx, x0s[t]);
          mny = min(mny, rys[t]);
        }
      const int bx0 = mnx - 1, bx1 = mxx + (NS - 1) + 1;  // +-1: a column may round off ix_0 + j
      const int xa = min(max(bx0, 0), xa_max) & ~3;
      const int by0 = mny;
      const int pack = (int)(((unsigned)(by0 + 32768) << 16) | (unsigned)xa);  // host: |by0| < 16000
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        // this lane's piece of fetch i: (group, box row, 4-cell piece in row)
        const int u = i * 64 + lane;
        const int gq = u / (TH * PPR);
        const int rem = u - gq * TH * PPR;
        const int rho = rem / PPR;
        const int q = rem - rho * PPR;
        const int gp = __builtin_amdgcn_ds_bpermute(min(gq * NS, 63) * 4, pack);
        const int row = (int)((unsigned)gp >> 16) - 32768 + rho;
        const int col = (gp & 0xFFFF) + 4 * q;
        const int off = (u < NP && (unsigned)row < (unsigned)sy) ? (row * pitch + col) * 4 : zero_off;
        buffer_load_lds16(rsrc, (lds_i32*)(img + i * 256), off);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): the boxes are in LDS
      __builtin_amdgcn_sched_barrier(0);
      const int lo = max(bx0, 0), hi = min(bx1, sx - 1);
      const bool fitx = lo > hi || (lo >= xa && hi < xa + TW);
      unsigned slow = 0;  // beams this lane must take the exact path for
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (!((mask >> t) & 1u)) continue;
        const int cx = cxs[t];
        const bool inx = (unsigned)cx < (unsigned)sx;
        const bool fast = rgs[t] && fitx && (rys[t] - by0 + NS <= TH) && (!inx || (unsigned)(cx - xa) < (unsigned)TW);
        const int32_t* base = (fast && inx) ? img + ge * BOX + (rys[t] - by0) * TW + (cx - xa) : zblk;
#pragma unroll
        for (int k = 0; k < NS; ++k) part[k] += base[k * TW];
        if (!fast) slow |= 1u << t;
        __builtin_amdgcn_sched_barrier(0);  // keeps one beam's reads in flight, not all T*NS
      }
      __builtin_amdgcn_sched_barrier(0);
#ifndef CSM_TILES_EXPERIMENT_NO_SLOW
      if (slow) {  // exact per-candidate path (rare): beams read zeros above, add them here
#pragma unroll 1
        for (int t = 0; t < T; ++t) {
          if (!((slow >> t) & 1u)) continue;
          const int b = tb + t;
          const double px = bcast_lane(pw.x, b - pbase), py = bcast_lane(pw.y, b - pbase);
          const double ly = ae.sine * px + ae.cosine * py;
          const int cx = cxs[t];
          const bool inx = (unsigned)cx < (unsigned)sx;
#pragma unroll
          for (int k = 0; k < NS; ++k) {
            const int gy = (int)((ly + (S.y0 + k * f)) + 0.5);
            const bool in = inx && (unsigned)gy < (unsigned)sy;
            part[k] += __builtin_amdgcn_raw_buffer_load_b32(rsrc, in ? (gy * pitch + cx) * 4 : zero_off, 0, 0);
          }
        }
      }
#endif
    }
    if (((tb + T) & 31) == 0 || tb + T >= n_used) {  // 32 * (2^26 - 1) < 2^31 (ensure_int_grid)
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        acci[k] += part[k];
        part[k] = 0;
      }
    }
  }

  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    if (valid) {
      const double acc = (double)(acci[k] + (int64_t)n_used * L.outside_i) * L.int_scale;
      const double yk = S.y0 + k * f;  // :572
      const double score = penalized(L, S, acc, x_r, yk, ae.angle);
      const int64_t flat = ((int64_t)a * NS + r) * NS + k;
      if (BEST) {
        if (better(score, flat, bs, bf)) {
          bs = score;
          bf = flat;
        }
      } else {
        out[S.out_off + flat] = score;
      }
    }
  }
  if (BEST) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double os = __shfl_down(bs, o, 64);
      const int64_t of = __shfl_down(bf, o, 64);
      if (better(os, of, bs, bf)) {
        bs = os;
        bf = of;
      }
    }
    if (lane == 0) partials[(int64_t)win * L.blocks_per_scan + blk] = BestPartial{bs, bf};
  }
}

}  // namespace

bool tiles_supported(int ns) { return ns == 13 || ns == 21; }

hipError_t launch_score_tiles(const LevelWork& L, const ScanWork* d_scans, const double* d_pts_raw,
                              const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                              int tile_beams, hipStream_t stream) {
  const double2* d_pts = reinterpret_cast<const double2*>(d_pts_raw);
  const int64_t nblk = (int64_t)L.blocks_per_scan * L.n_scans;
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || L.step_cells != 1.0 || L.pitch < 32 ||
      L.pitch % 4 != 0 || L.pitch >= 65536)
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk), block(64);
#define CSM_TILES_CASE(N, TB)                                                                              \
  if (ns == N && tile_beams == TB) {                                                                       \
    if (d_partials)                                                                                        \
      hipLaunchKernelGGL((score_tiles_kernel<N, TB, true>), grid, block, 0, stream, L, d_scans, d_pts,    \
                         d_angles, d_out, d_partials);                                                     \
    else                                                                                                   \
      hipLaunchKernelGGL((score_tiles_kernel<N, TB, false>), grid, block, 0, stream, L, d_scans, d_pts,   \
                         d_angles, d_out, d_partials);                                                     \
    return hipGetLastError();                                                                              \
  }
  CSM_TILES_CASE(13, 8)
  CSM_TILES_CASE(13, 4)
  CSM_TILES_CASE(21, 8)
  CSM_TILES_CASE(21, 4)
#undef CSM_TILES_CASE
  return hipErrorInvalidValue;
}

}  // namespace csm
