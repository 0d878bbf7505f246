// csm_pyramid.hip — kernels of the admissible multi-resolution search
// (csm_pyramid.hpp): max-pooled grid levels, node bounds, pruning/expansion.
//
// Exactness of the bound. A node at depth d covers candidates j in
// [j0, j0 + 2^d) (j0 = J 2^d), k likewise, at one angle. For a beam, the
// column a candidate reads is trunc(fl(fl(lx + x_j) + 0.5)) with
// x_j = fl(x0 + j) (correlate_scan_matcher.h:569,647; step exactly one cell).
// fp addition and trunc are monotone, so the columns of the node's
// candidates lie in [g0, trunc(t_j1)], g0 the anchor candidate's own column;
// t_j1 - t_j0 <= 2^d - 1 + (rounding < 2^-20), so trunc(t_j1) <= g0 + 2^d
// (for t < 0, trunc = ceil, and ceil(a + b) <= ceil(a) + ceil(b) gives the
// same bound). Level d stores at anchor g0 the maximum over [g0, g0 + 2^d],
// off-grid cells counting as the outside value (0 in the fixed-point copy),
// hence sum_beams level_d[anchor] >= the integer sum of every candidate of
// the node. The score is monotone in that sum ((double)(S + n outside_i) *
// 2^-E / divisor: exact scaling, monotone rounding), and the centre penalty
// (:718-745) multiplies by a factor in [0.45, 1] (0.45 = 0.5 * 0.9, its
// floors), so the bound is the raw score if >= 0 and 0.45 times it if < 0.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "csm_device.hpp"
#include "csm_pyramid.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

using dev::better;
using dev::penalized;

constexpr int kPB = 256;  // threads per block (4 waves)

__device__ __forceinline__ void node_decode(uint64_t nd, int& w, int& a, int& J, int& K) {
  w = (int)(nd >> 44);
  a = (int)((nd >> 32) & 0xFFF);
  J = (int)((nd >> 16) & 0xFFFF);
  K = (int)(nd & 0xFFFF);
}

__device__ __forceinline__ int64_t pyr_col(const PyrGrid& L, int xs) {
  return (int64_t)(xs & ((1 << L.lg) - 1)) * L.q + (xs >> L.lg);
}

// Level d (>= 1): anchor (x, y) = (xs - 2^d, ys - 2^d) holds the maximum of
// the source over anchors x + t, t in taps (d = 1: the grid at 0, 1, 2;
// d >= 2: level d - 1 at 0 and 2^(d-1)), rows likewise, quantised upwards to
// int16 (level 1 from the int32 grid: ceil(max / 2^qs); later levels take
// the max of already quantised values, the same thing). Every stored cell of
// the buffer is written (pad columns zero).
template <typename TS>
__global__ __launch_bounds__(256) void pyr_pool_kernel(PyrGrid src, PyrGrid dst, int t1, int t2, int ntaps,
                                                       int64_t total) {
  const TS* __restrict__ sg = (const TS*)src.g;
  int16_t* __restrict__ dg = (int16_t*)const_cast<void*>(dst.g);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t gidx = i / dst.stride;
    const int64_t r = i - gidx * dst.stride;
    const int ys = (int)(r / dst.pitch), c = (int)(r - (int64_t)ys * dst.pitch);
    const int ph = c / dst.q, qx = c - ph * dst.q;
    const int xs = (qx << dst.lg) + ph;  // logical column of storage column c
    int32_t m = 0;
    if (ph < (1 << dst.lg) && xs < dst.width && ys < dst.height) {
      const int ax = xs - dst.shift + src.shift, ay = ys - dst.shift + src.shift;
      const TS* g = sg + gidx * src.stride;
      const int tap[3] = {0, t1, t2};
      bool any = false;
      for (int ty = 0; ty < ntaps; ++ty) {
        const int yy = ay + tap[ty];
        for (int tx = 0; tx < ntaps; ++tx) {
          const int xx = ax + tap[tx];
          const bool in = (unsigned)xx < (unsigned)src.width && (unsigned)yy < (unsigned)src.height;
          const int32_t v = in ? (int32_t)g[(int64_t)yy * src.pitch + pyr_col(src, xx)] : 0;  // off-grid: outside
          m = any ? max(m, v) : v;
          any = true;
        }
      }
      const int dq = dst.qs - src.qs;  // quantise: ceil(m / 2^dq) (arithmetic shift floors)
      if (dq > 0) m = (m + (1 << dq) - 1) >> dq;
    }
    dg[i] = (int16_t)m;
  }
}

__global__ __launch_bounds__(256) void pyr_top_kernel(LevelWork L, int32_t nj, int64_t first, int64_t n,
                                                      uint64_t* __restrict__ out) {
  const int64_t per_angle = (int64_t)nj * nj;
  const int64_t per_window = per_angle * L.n_angles;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = first + i;
    const int64_t w = q / per_window;
    const int64_t rw = q - w * per_window;
    const int64_t a = rw / per_angle;
    const int64_t ra = rw - a * per_angle;
    const int64_t K = ra / nj, J = ra - K * nj;  // J fastest
    out[i] = pyr_node((uint32_t)w, (uint32_t)a, (uint32_t)J, (uint32_t)K);
  }
}

// A node's bound from its integer sum over the beams of a quantised level
// (units of 2^qs): the raw score if >= 0, 0.45 times it otherwise (the
// centre penalty's floor).
__device__ __forceinline__ double level_bound(const LevelWork& L, const ScanWork& S, int64_t sum, int qs,
                                              int32_t n_used) {
  const double acc = (double)((sum << qs) + (int64_t)n_used * L.outside_i) * L.int_scale;
  const double raw = acc / S.divisor;
  return (L.use_penalty && raw < 0.0) ? raw * 0.45 : raw;
}

template <int NT = kPB>
__device__ __forceinline__ void block_best(double v, int64_t f, uint64_t nd, PyrPartial* __restrict__ out) {
  __shared__ double rs[NT / 64];
  __shared__ int64_t rf[NT / 64];
  __shared__ uint64_t rn[NT / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_down(v, off, 64);
    const int64_t of = __shfl_down(f, off, 64);
    const uint64_t on = __shfl_down(nd, off, 64);
    if (better(ov, of, v, f)) {
      v = ov;
      f = of;
      nd = on;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    rs[wave] = v;
    rf[wave] = f;
    rn[wave] = nd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < NT / 64; ++k)
      if (better(rs[k], rf[k], v, f)) {
        v = rs[k];
        f = rf[k];
        nd = rn[k];
      }
    *out = PyrPartial{v, f, nd};
  }
}

// lpn lanes per node (blocks stride over the list; a node's lanes take every
// lpn-th beam and meet by shuffles): the sum over the scan's beams of the
// level-d value at the anchor candidate's cell (GetResponse :645-654 with the
// pooled level in place of the grid); d = 0 is the candidate's exact,
// penalised score. Integer sums: the split changes nothing. The list length
// is often only known on the device (n_dev) and far below the launch's
// upper bound (a few hundred nodes at the lower levels of a single query),
// so every block derives lpn from it: the most lanes per node, up to a wave,
// the grid can give every node, each lane's gather chain a fraction of the
// beams. Blocks past the list write an empty partial and leave.
template <typename T>
__global__ __launch_bounds__(kPB) void pyr_bound_kernel(LevelWork L, PyrGrid lev, int d,
                                                        const ScanWork* __restrict__ scans,
                                                        const AngleEntry* __restrict__ angles,
                                                        const double2* __restrict__ pts, int32_t n_used,
                                                        int32_t step, const uint64_t* __restrict__ nodes,
                                                        int64_t n_host, const unsigned long long* __restrict__ n_dev,
                                                        double* __restrict__ vals,
                                                        PyrPartial* __restrict__ partials,
                                                        unsigned long long* __restrict__ scored) {
  extern __shared__ double2 beams[];
  const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
  const int64_t threads = (int64_t)gridDim.x * kPB;
  int lpn = 1;  // a power of two, the same in every block
  while (lpn < 64 && n * (2 * lpn) <= threads && 2 * lpn <= n_used) lpn <<= 1;
  if (((int64_t)blockIdx.x * kPB) / lpn >= n) {  // no node for this block (uniform)
    if (threadIdx.x == 0) partials[blockIdx.x] = PyrPartial{-1.0e300, INT64_MAX, kPyrNoNode};
    return;
  }
  for (int b = threadIdx.x; b < n_used; b += kPB) beams[b] = pts[(int64_t)b * step];
  __syncthreads();
  if (scored && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(scored, (unsigned long long)n);
  double bv = -1.0e300;
  int64_t bf = INT64_MAX;
  uint64_t bn = kPyrNoNode;
  const int sh = lev.shift, W = lev.width, H = lev.height, pitch = lev.pitch, lg = lev.lg, qc = lev.q;
  const int pm = (1 << lg) - 1;
  const int sub = (int)(threadIdx.x & (lpn - 1));
  for (int64_t i = ((int64_t)blockIdx.x * kPB + threadIdx.x) / lpn; i < n; i += threads / lpn) {
    const uint64_t nd = nodes[i];
    int w, a, J, K;
    node_decode(nd, w, a, J, K);
    const int j0 = J << d, k0 = K << d;
    const bool valid = nd != kPyrNoNode && w < L.n_scans && a < L.n_angles && j0 < L.n_space && k0 < L.n_space;
    double v = -1.0e300;
    int64_t gflat = INT64_MAX;
    int64_t sum = 0;
    if (valid) {
      const ScanWork S = scans[w];
      const AngleEntry ae = angles[S.angle_off + a];
      const double x = S.x0 + j0 * L.step_cells;  // :569
      const double y = S.y0 + k0 * L.step_cells;  // :572
      const T* __restrict__ g = (const T*)lev.g + (int64_t)S.grid_index * lev.stride;
      auto cell = [&](int b) -> int32_t {
        const double2 p = beams[b];
        const double lx = ae.cosine * p.x - ae.sine * p.y;
        const double ly = ae.sine * p.x + ae.cosine * p.y;
        const int gx = (int)((lx + x) + 0.5) + sh;
        const int gy = (int)((ly + y) + 0.5) + sh;
        const bool in = (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
        const int64_t idx = (int64_t)gy * pitch + (int64_t)(gx & pm) * qc + (gx >> lg);
        const int32_t c = g[in ? idx : 0];
        return in ? c : 0;
      };
      int b = sub;
      for (; b + 7 * lpn < n_used; b += 8 * lpn) {  // 8 gathers in flight per lane
        int32_t c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = cell(b + u * lpn);
        // |c| < 2^26: eight fit an int32
        sum += (int64_t)(((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7])));
      }
      for (; b < n_used; b += lpn) sum += cell(b);
    }
    for (int o = lpn / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);  // the node's lanes (all valid or none)
    if (valid) {
      const ScanWork S = scans[w];
      const AngleEntry ae = angles[S.angle_off + a];
      const double x = S.x0 + j0 * L.step_cells;  // :569
      const double y = S.y0 + k0 * L.step_cells;  // :572
      sum <<= lev.qs;  // the quantised levels' unit
      const double acc = (double)(sum + (int64_t)n_used * L.outside_i) * L.int_scale;
      if (d == 0) {
        v = penalized(L, S, acc, x, y, ae.angle);
      } else {
        const double raw = acc / S.divisor;
        v = (L.use_penalty && raw < 0.0) ? raw * 0.45 : raw;
      }
      gflat = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + j0) * L.n_space + k0;
    }
    if (sub == 0) vals[i] = v;
    if (better(v, gflat, bv, bf)) {
      bv = v;
      bf = gflat;
      bn = nd;
    }
  }
  block_best(bv, bf, bn, partials + blockIdx.x);
}

// The whole top level at once, laid out as the exhaustive column kernel
// (csm_kernels.hip score_cols_kernel): lane = one (angle, J) column of a
// window, kt rows K per lane, so a beam's rotation and column are computed
// once per lane and shared by its rows, and adjacent J lanes gather adjacent
// phase-split cells. Writes every top node and its bound in list order
// ((window, angle, K, J), J fastest) and one best per block.
constexpr int kTopKT = 16;
constexpr int kTB = 64;  // one wave per block: a window's blocks, XCD-remapped, share one XCD's L2
template <typename T>
__global__ __launch_bounds__(kTB) void pyr_top_bound_kernel(LevelWork L, PyrGrid lev, int d, int32_t nj,
                                                            int32_t ktiles, int32_t kt, int32_t col_blocks,
                                                            const ScanWork* __restrict__ scans,
                                                            const AngleEntry* __restrict__ angles,
                                                            const double2* __restrict__ pts, int32_t n_used,
                                                            int32_t step, uint64_t* __restrict__ nodes,
                                                            double* __restrict__ vals,
                                                            PyrPartial* __restrict__ partials) {
  extern __shared__ double2 beams[];
  for (int b = threadIdx.x; b < n_used; b += kTB) beams[b] = pts[(int64_t)b * step];
  __syncthreads();
  const int per_window = col_blocks * ktiles;
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int w = bid / per_window;
  const int r = bid - w * per_window;
  const int cb = r / ktiles, ktile = r - cb * ktiles;
  const int col = cb * kTB + threadIdx.x;
  const bool valid = col < L.n_angles * nj;
  const int a = valid ? col / nj : 0;
  const int J = valid ? col - a * nj : 0;
  const int K0 = ktile * kt;
  const int krem = min(kt, nj - K0);
  const ScanWork S = scans[w];
  const AngleEntry ae = angles[S.angle_off + a];
  const double x = S.x0 + (J << d) * L.step_cells;  // :569
  double y[kTopKT];
#pragma unroll
  for (int kk = 0; kk < kTopKT; ++kk) y[kk] = S.y0 + ((K0 + kk) << d) * L.step_cells;  // :572
  const T* __restrict__ g = (const T*)lev.g + (int64_t)S.grid_index * lev.stride;
  const int sh = lev.shift, W = lev.width, H = lev.height, pitch = lev.pitch, lg = lev.lg, qc = lev.q;
  const int pm = (1 << lg) - 1;
  int64_t sum[kTopKT];
#pragma unroll
  for (int kk = 0; kk < kTopKT; ++kk) sum[kk] = 0;
  for (int b = 0; b < n_used; ++b) {
    const double2 p = beams[b];
    const double lx = ae.cosine * p.x - ae.sine * p.y;
    const double ly = ae.sine * p.x + ae.cosine * p.y;
    const int gx = (int)((lx + x) + 0.5) + sh;
    const bool inx = (unsigned)gx < (unsigned)W;
    const int64_t cx = (int64_t)(gx & pm) * qc + (gx >> lg);
    int32_t c[kTopKT];
#pragma unroll
    for (int kk = 0; kk < kTopKT; ++kk) {
      const int gy = (int)((ly + y[kk]) + 0.5) + sh;
      const bool in = inx && (unsigned)gy < (unsigned)H && kk < krem;
      const int32_t v = (int32_t)g[in ? (int64_t)gy * pitch + cx : 0];
      c[kk] = in ? v : 0;
    }
#pragma unroll
    for (int kk = 0; kk < kTopKT; ++kk) sum[kk] += c[kk];
  }
  double bv = -1.0e300;
  int64_t bf = INT64_MAX;
  uint64_t bn = kPyrNoNode;
  const int64_t wbase = ((int64_t)w * L.n_angles + a) * nj;
#pragma unroll
  for (int kk = 0; kk < kTopKT; ++kk) {
    if (valid && kk < krem) {
      const int K = K0 + kk;
      const double acc = (double)((sum[kk] << lev.qs) + (int64_t)n_used * L.outside_i) * L.int_scale;
      const double raw = acc / S.divisor;
      const double v = (L.use_penalty && raw < 0.0) ? raw * 0.45 : raw;
      const int64_t idx = (wbase + K) * nj + J;
      const uint64_t nd = pyr_node((uint32_t)w, (uint32_t)a, (uint32_t)J, (uint32_t)K);
      nodes[idx] = nd;
      vals[idx] = v;
      const int64_t gflat = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + (J << d)) * L.n_space + (K << d);
      if (better(v, gflat, bv, bf)) {
        bv = v;
        bf = gflat;
        bn = nd;
      }
    }
  }
  block_best<kTB>(bv, bf, bn, partials + bid);
}

// The top level as beam boxes (csm_box.hip's argument with node steps of 2^d
// cells). With step one cell the anchor column of node J is
// trunc(fl(fl(lx + fl(x0 + J 2^d)) + 0.5)); whenever the beam passes the box
// test (t_0 >= 0, fraction at least kTopBoxMargin from an integer, |t| < 2^24
// cells: the host's box_ok) it equals trunc(t_0) + J 2^d for every J, rows
// likewise. In the phase-split layout the anchors of J = 0, 1, ... are then
// adjacent cells of phase (trunc(t_0) + shift) mod 2^d, so a beam's nodes of
// one row K are nj consecutive int16 cells of the box copy (tb: level d, each
// phase's columns padded with zeros past the grid, 2^d nj zero rows below
// it) and one row piece per lane covers all nj x nj nodes in NL
// buffer_load_dwordx4 per beam, instead of nj^2 / 64 dword gathers. Rejected
// beams are summed node by node with pyr_top_bound_kernel's expressions
// afterwards; nodes, bounds and the best per wave are written exactly as that
// kernel writes them.
//
// Loads are dword-aligned: lane (K, c) loads the 16 bytes at element
// c0a + 8c (c0 = the row's node 0, c0a = c0 rounded down to even), NP =
// ceil((nj + 1) / 8) pieces per row. Element e then belongs to node
// e - (c0 - c0a): the beam's parity (uniform) picks the accumulator set, even
// (node 8c + i) or odd (node 8c + i - 1, folded across pieces through LDS at
// the end). Measured (config 3, d = 4, nj = 21): 1.58 ms per query against
// 2.9 ms for the gathers and 1.98 ms for an int32 copy (twice the bytes per
// beam); L2-bound (~15 TB/s of 64-byte requests, 96 % hits).
constexpr double kTopBoxMargin = 0x1p-20;

template <int NP, int NL>
__global__ __launch_bounds__(64) void pyr_topbox_kernel(LevelWork L, PyrGrid tb, int d, int32_t nj,
                                                          const ScanWork* __restrict__ scans,
                                                          const AngleEntry* __restrict__ angles,
                                                          const double2* __restrict__ pts, int32_t n_used,
                                                          int32_t step, int split, int32_t* __restrict__ sums,
                                                          int32_t* __restrict__ slab,
                                                          PyrPartial* __restrict__ partials) {
#ifndef CSM_TOPBOX_GB
#define CSM_TOPBOX_GB 4
#endif
  constexpr int GB = NL == 1 ? 8 : CSM_TOPBOX_GB;  // beams whose loads are issued together
  __shared__ int32_t odd_sum[32][8 * 5 + 8];
  // split > 1 (few windows): `split` waves per (window, angle), each over a
  // contiguous range of the beams, storing its sums in its own slab row;
  // pyr_topbox_final_kernel then adds the rows and bounds the nodes
  const int bid0 = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int bid = bid0 / split, part = bid0 - (bid0 / split) * split;
  const int w = bid / L.n_angles;
  const int a = bid - w * L.n_angles;
  const int b_lo = (int)((int64_t)n_used * part / split), b_hi = (int)((int64_t)n_used * (part + 1) / split);
  const ScanWork S = scans[w];
  const AngleEntry ae = angles[S.angle_off + a];
  const int lane = threadIdx.x;
  const int pitch2 = tb.pitch * 2;  // bytes per row
  const int sh = tb.shift, lg = tb.lg, pm = (1 << lg) - 1, W = tb.width, H = tb.height, qc = tb.q;
  const int sx = W - sh, sy = H - sh;
  const int zero_el = H * tb.pitch;  // element offset of the zero rows (even: pitch is)
  bool act[NL];
  int Ks[NL], cs[NL], voff[NL];
#pragma unroll
  for (int s = 0; s < NL; ++s) {
    const int i = s * 64 + lane;
    act[s] = i < nj * NP;
    Ks[s] = act[s] ? i / NP : 0;
    cs[s] = act[s] ? i - Ks[s] * NP : 0;
    voff[s] = ((Ks[s] << d) * pitch2) + 16 * cs[s];
  }
  const int16_t* g = (const int16_t*)tb.g + (int64_t)S.grid_index * tb.stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)g);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)g >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(tb.stride * 2), 0x00020000);
  const double x_0 = S.x0 + 0 * L.step_cells;  // :569, J = 0
  const double y_0 = S.y0 + 0 * L.step_cells;  // :572, K = 0
  // element offset of the beam's node (0, 0) (zero_el: reads zeros)
  auto test = [&](const double2 p, double& lx, double& ly, int& el) -> bool {
    lx = ae.cosine * p.x - ae.sine * p.y;  // :179
    ly = ae.sine * p.x + ae.cosine * p.y;  // :180
    const double tx = (lx + x_0) + 0.5;
    const double ty = (ly + y_0) + 0.5;
    const double fx = tx - floor(tx), fy = ty - floor(ty);
    const bool clean = tx >= 0.0 && ty >= 0.0 && fx >= kTopBoxMargin && fx <= 1.0 - kTopBoxMargin &&
                       fy >= kTopBoxMargin && fy <= 1.0 - kTopBoxMargin;
    const int ix0 = clean ? (int)tx : 0, iy0 = clean ? (int)ty : 0;
    const int xs = ix0 + sh, ys = iy0 + sh;
    el = (clean && ix0 < sx && iy0 < sy) ? ys * tb.pitch + (xs & pm) * qc + (xs >> lg) : zero_el;
    return clean;
  };
  typedef int32_t v4i __attribute__((ext_vector_type(4)));
  int32_t ae_[NL][8], ao_[NL][8];  // even / odd parity sums (|sum| <= 4096 * 2^14)
#pragma unroll
  for (int s = 0; s < NL; ++s)
#pragma unroll
    for (int t = 0; t < 8; ++t) ae_[s][t] = ao_[s][t] = 0;
  auto add8 = [&](int32_t (&acc)[8], const v4i v) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[2 * t] += (int32_t)((uint32_t)v[t] << 16) >> 16;  // low half: element 2t
      acc[2 * t + 1] += v[t] >> 16;                // high half: element 2t + 1
    }
  };
  uint64_t slow = 0;  // bit c: chunk c of this wave's range holds a rejected beam
  double2 pn = pts[(int64_t)min(b_lo + lane, n_used - 1) * step];
  for (int cb = b_lo; cb < b_hi; cb += 64) {
    const double2 p = pn;
    pn = pts[(int64_t)min(cb + 64 + lane, n_used - 1) * step];
    double lx, ly;
    int el;
    const bool clean = test(p, lx, ly, el);
    const bool live = cb + lane < b_hi;
    if (!live) el = zero_el;
    slow |= (uint64_t)(__builtin_amdgcn_ballot_w64(live && !clean) != 0) << min((cb - b_lo) >> 6, 63);
    const int nb = min(64, b_hi - cb);
    for (int r = 0; r < nb; r += GB) {  // beams past nb read the zero rows
      int so[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) so[u] = __builtin_amdgcn_readlane(el, r + u);
      v4i buf[GB][NL];
#pragma unroll
      for (int u = 0; u < GB; ++u)
#pragma unroll
        for (int s = 0; s < NL; ++s)
          buf[u][s] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[s], (so[u] & ~1) * 2, 0);
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        if (so[u] & 1) {  // uniform
#pragma unroll
          for (int s = 0; s < NL; ++s) add8(ao_[s], buf[u][s]);
        } else {
#pragma unroll
          for (int s = 0; s < NL; ++s) add8(ae_[s], buf[u][s]);
        }
      }
    }
  }
  // odd sums to their nodes: element 8c + t of row K is node 8c + t - 1
#pragma unroll
  for (int s = 0; s < NL; ++s)
    if (act[s])
#pragma unroll
      for (int t = 0; t < 8; ++t) odd_sum[Ks[s]][8 * cs[s] + t] = ao_[s][t];
  __syncthreads();
  int32_t acc[NL][8];
#pragma unroll
  for (int s = 0; s < NL; ++s)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int J = 8 * cs[s] + t;
      acc[s][t] = ae_[s][t] + ((act[s] && J + 1 < 8 * NP) ? odd_sum[Ks[s]][J + 1] : 0);
    }
  // rejected beams, node by node (pyr_top_bound_kernel's expressions)
  for (uint64_t m = slow; m != 0; m &= m - 1) {
    const int c0 = (int)__builtin_ctzll(m);
    const int c_end = c0 == 63 ? (b_hi - b_lo + 63) / 64 : c0 + 1;
    for (int c = c0; c < c_end; ++c) {
      const int cb = b_lo + c * 64;
      double lx, ly;
      int el;
      const bool clean = test(pts[(int64_t)min(cb + lane, n_used - 1) * step], lx, ly, el);
      for (uint64_t rej = __builtin_amdgcn_ballot_w64(cb + lane < b_hi && !clean); rej != 0; rej &= rej - 1) {
        const int l = (int)__builtin_ctzll(rej);  // uniform: one beam for the whole wave
        const double bx = dev::bcast_lane(lx, l);
        const double by = dev::bcast_lane(ly, l);
#pragma unroll
        for (int s = 0; s < NL; ++s) {
          const int gy = (int)((by + (S.y0 + (Ks[s] << d) * L.step_cells)) + 0.5) + sh;
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int J = 8 * cs[s] + t;
            const int gx = (int)((bx + (S.x0 + (J << d) * L.step_cells)) + 0.5) + sh;
            const bool in = act[s] && J < nj && (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
            const int32_t v = g[in ? (int64_t)gy * tb.pitch + (int64_t)(gx & pm) * qc + (gx >> lg) : 0];
            acc[s][t] += in ? v : 0;
          }
        }
      }
    }
  }
  double bv = -1.0e300;
  int64_t bf = INT64_MAX;
  uint64_t bn = kPyrNoNode;
  const int64_t wbase = ((int64_t)w * L.n_angles + a) * nj;
  if (split > 1) {  // partial sums of this beam range, plain stores (device-scope
                    // atomics from every split wave cost more than the beams)
    int32_t* row = slab + ((int64_t)bid * split + part) * nj * nj;
#pragma unroll
    for (int s = 0; s < NL; ++s)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int J = 8 * cs[s] + t, K = Ks[s];
        if (act[s] && J < nj) row[K * nj + J] = acc[s][t];
      }
    return;
  }
#pragma unroll
  for (int s = 0; s < NL; ++s) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int J = 8 * cs[s] + t, K = Ks[s];
      if (act[s] && J < nj) {
        const double v = level_bound(L, S, acc[s][t], tb.qs, n_used);
        sums[(wbase + K) * nj + J] = acc[s][t];  // the node is implicit in the index
        const uint64_t nd = pyr_node((uint32_t)w, (uint32_t)a, (uint32_t)J, (uint32_t)K);
        const int64_t gflat = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + (J << d)) * L.n_space + (K << d);
        if (better(v, gflat, bv, bf)) {
          bv = v;
          bf = gflat;
          bn = nd;
        }
      }
    }
  }
  block_best<64>(bv, bf, bn, partials + bid);
}

// After a split pyr_topbox_kernel: each (window, angle)'s node bounds from the
// summed integers and its best (one wave per (window, angle), as the
// unsplit kernel writes them).
__global__ __launch_bounds__(64) void pyr_topbox_final_kernel(LevelWork L, int d, int32_t nj, int qs, int32_t n_used,
                                                              const ScanWork* __restrict__ scans, int split,
                                                              const int32_t* __restrict__ slab,
                                                              int32_t* __restrict__ sums,
                                                              PyrPartial* __restrict__ partials) {
  const int bid = blockIdx.x;
  const int w = bid / L.n_angles;
  const int a = bid - w * L.n_angles;
  const ScanWork S = scans[w];
  const int64_t wbase = ((int64_t)w * L.n_angles + a) * nj;
  const int32_t* rows = slab + (int64_t)bid * split * nj * nj;
  double bv = -1.0e300;
  int64_t bf = INT64_MAX;
  uint64_t bn = kPyrNoNode;
  for (int i = threadIdx.x; i < nj * nj; i += 64) {
    const int K = i / nj, J = i - K * nj;
    int32_t sum = 0;  // |sum| <= 4096 beams * 2^15: the rows add up in int32
    for (int p = 0; p < split; ++p) sum += rows[(int64_t)p * nj * nj + i];
    sums[wbase * nj + i] = sum;
    const double v = level_bound(L, S, sum, qs, n_used);
    const int64_t gflat = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + (J << d)) * L.n_space + (K << d);
    if (better(v, gflat, bv, bf)) {
      bv = v;
      bf = gflat;
      bn = pyr_node((uint32_t)w, (uint32_t)a, (uint32_t)J, (uint32_t)K);
    }
  }
  block_best<64>(bv, bf, bn, partials + bid);
}

// tb (padded phase-split int16) from level d: every stored cell written,
// zero outside the level.
__global__ __launch_bounds__(256) void pyr_widen_kernel(PyrGrid src, PyrGrid dst, int64_t total) {
  const int16_t* __restrict__ sg = (const int16_t*)src.g;
  int16_t* __restrict__ dg = (int16_t*)const_cast<void*>(dst.g);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t gidx = i / dst.stride;
    const int64_t r = i - gidx * dst.stride;
    const int ys = (int)(r / dst.pitch), c = (int)(r - (int64_t)ys * dst.pitch);
    const int ph = c / dst.q, qx = c - ph * dst.q;
    const int xs = (qx << dst.lg) + ph;
    int16_t v = 0;
    if (ph < (1 << dst.lg) && xs < dst.width && ys < dst.height)
      v = sg[gidx * src.stride + (int64_t)ys * src.pitch + pyr_col(src, xs)];
    dg[i] = v;
  }
}

// merge (one block): fold the best partial into the incumbent. Otherwise
// block i picks the best of the i-th of gridDim.x equal segments of the
// partials (different windows / angle ranges: diverse probe roots) when it
// beats the incumbent (kPyrNoNode otherwise).
__global__ __launch_bounds__(kPB) void pyr_final_kernel(const PyrPartial* __restrict__ in, int64_t n, int merge,
                                                        BestPartial* __restrict__ inc,
                                                        uint64_t* __restrict__ probe) {
  const BestPartial cur = *inc;
  const int64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
  double v = -1.0e300;
  int64_t f = INT64_MAX;
  uint64_t nd = kPyrNoNode;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kPB) {
    const PyrPartial p = in[i];
    if (better(p.v, p.gflat, v, f)) {
      v = p.v;
      f = p.gflat;
      nd = p.node;
    }
  }
  __shared__ PyrPartial out;
  block_best(v, f, nd, &out);
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool win = out.gflat != INT64_MAX && better(out.v, out.gflat, cur.score, cur.flat);
    if (merge) {
      if (win) *inc = BestPartial{out.v, out.gflat};
    } else {
      probe[blockIdx.x] = win ? out.node : kPyrNoNode;
    }
  }
}

__global__ __launch_bounds__(256) void pyr_probe_kernel(int d, int n_probe, const uint64_t* __restrict__ probe,
                                                        uint64_t* __restrict__ out) {
  const int64_t per = (int64_t)1 << (2 * d);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < per * n_probe;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % per;
    const uint64_t nd = probe[t / per];
    int w, a, J, K;
    node_decode(nd, w, a, J, K);
    if (nd == kPyrNoNode) {
      out[t] = kPyrNoNode;
      continue;
    }
    const uint32_t dk = (uint32_t)(i >> d), dj = (uint32_t)(i & ((1 << d) - 1));  // J fastest
    const uint32_t j = ((uint32_t)J << d) + dj, k = ((uint32_t)K << d) + dk;
    out[t] = (j < 0x10000u && k < 0x10000u) ? pyr_node((uint32_t)w, (uint32_t)a, j, k) : kPyrNoNode;
  }
}

// Wave-aggregated append of each lane's kept children (mask bit 2 dk + dj).
__device__ __forceinline__ void append_children(int w, int a, int J, int K, uint32_t mask,
                                                uint64_t* __restrict__ out, unsigned long long* __restrict__ count,
                                                int64_t cap) {
  const int lane = threadIdx.x & 63;
  const int cnt = __builtin_popcount(mask);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  const int total = __shfl(incl, 63, 64);
  unsigned long long base = 0;
  if (lane == 63 && total > 0) base = atomicAdd(count, (unsigned long long)total);
  base = __shfl(base, 63, 64);
  int64_t o = (int64_t)base + (incl - cnt);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (mask & (1u << q)) {
      if (o < cap)
        out[o] = pyr_node((uint32_t)w, (uint32_t)a, (uint32_t)(2 * J + (q & 1)), (uint32_t)(2 * K + (q >> 1)));
      ++o;
    }
  }
}

// The incumbent as integer sums (one thread): level_bound is monotone in the
// sum, so with every window sharing one scan (divisor, beam count: the host
// checks) bound > score <=> sum >= thr[0] and bound >= score <=> sum >=
// thr[1] (INT32_MAX + 1: no such sum).
__device__ __forceinline__ void incumbent_thresholds(const LevelWork& L, const ScanWork& S, int qs, int32_t n_used,
                                                     const BestPartial& cur, int64_t* thr) {
  for (int strict = 1; strict >= 0; --strict) {
    int64_t lo = INT32_MIN, hi = (int64_t)INT32_MAX + 1;
    while (lo < hi) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      const double v = level_bound(L, S, mid, qs, n_used);
      if (strict ? v > cur.score : v >= cur.score) hi = mid;
      else lo = mid + 1;
    }
    thr[1 - strict] = lo;
  }
}

// The same thresholds once for a launch of many blocks (config 3's top level:
// tens of thousands of blocks would each repeat the search).
__global__ void pyr_threshold_kernel(LevelWork L, const ScanWork* __restrict__ scans, int qs, int32_t n_used,
                                     const BestPartial* __restrict__ inc, int64_t* __restrict__ thr) {
  incumbent_thresholds(L, scans[0], qs, n_used, *inc, thr);
}

// The children of top nodes [first, first + n) of pyr_topbox_kernel's
// implicit list ((window, angle, K, J), J fastest), from their integer sums
// against the incumbent's thresholds (incumbent_thresholds, each block's
// thread 0): the same test as better(bound, lowest, incumbent) without a
// division per node; only the few nodes at or above the incumbent decode
// their index.
__global__ __launch_bounds__(256) void pyr_expand_top_kernel(LevelWork L, int d, int32_t nj, int qs, int32_t n_used,
                                                             const ScanWork* __restrict__ scans,
                                                             const int64_t* __restrict__ thr_dev,
                                                             const int32_t* __restrict__ sums, int64_t first,
                                                             int64_t n, const BestPartial* __restrict__ inc,
                                                             uint64_t* __restrict__ out,
                                                             unsigned long long* __restrict__ count, int64_t cap) {
  __shared__ int64_t thr[2];
  const BestPartial cur = *inc;
  if (threadIdx.x == 0) {  // few blocks: each finds them (one launch less); many: pyr_threshold_kernel did
    if (thr_dev) {
      thr[0] = thr_dev[0];
      thr[1] = thr_dev[1];
    } else {
      incumbent_thresholds(L, scans[0], qs, n_used, cur, thr);
    }
  }
  __syncthreads();
  const int64_t t_gt = thr[0], t_ge = thr[1];
  const int h = d - 1;
  const int64_t per_angle = (int64_t)nj * nj;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + threadIdx.x;
    int w = 0, a = 0, J = 0, K = 0;
    uint32_t mask = 0;
    const int64_t q = first + i;
    const int64_t sum = i < n ? (int64_t)sums[q] : INT64_MIN;
    if (sum >= t_ge) {
      const int64_t wa = q / per_angle;
      const int64_t r = q - wa * per_angle;
      K = (int)(r / nj);
      J = (int)(r - (int64_t)K * nj);
      w = (int)(wa / L.n_angles);
      a = (int)(wa - (int64_t)w * L.n_angles);
      const int64_t lowest = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + (J << d)) * L.n_space + (K << d);
      if (sum >= t_gt || lowest < cur.flat) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int cj = 2 * J + (c & 1), ck = 2 * K + (c >> 1);
          if ((cj << h) < L.n_space && (ck << h) < L.n_space) mask |= 1u << c;
        }
      }
    }
    if (__builtin_amdgcn_ballot_w64(mask != 0) == 0) continue;  // uniform: the usual case
    append_children(w, a, J, K, mask, out, count, cap);
  }
}

// Children in the order (2J, 2K), (2J+1, 2K), (2J, 2K+1), (2J+1, 2K+1): J
// pairs adjacent, as the next level's gathers want them.
__global__ __launch_bounds__(256) void pyr_expand_kernel(LevelWork L, int d, const uint64_t* __restrict__ nodes,
                                                         const double* __restrict__ bounds, int64_t n_host,
                                                         const unsigned long long* __restrict__ n_dev,
                                                         const BestPartial* __restrict__ inc,
                                                         uint64_t* __restrict__ out,
                                                         unsigned long long* __restrict__ count, int64_t cap) {
  const BestPartial cur = *inc;
  const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
  const int h = d - 1;
  // whole waves step together (the append below is wave-wide)
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + threadIdx.x;
    int w = 0, a = 0, J = 0, K = 0;
    uint32_t mask = 0;  // children kept: bit (2 dk + dj)
    if (i < n) {
      const uint64_t nd = nodes[i];
      node_decode(nd, w, a, J, K);
      const double b = bounds[i];
      const int64_t lowest = (int64_t)w * L.n_cand + ((int64_t)a * L.n_space + (J << d)) * L.n_space + (K << d);
      if (nd != kPyrNoNode && better(b, lowest, cur.score, cur.flat)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cj = 2 * J + (q & 1), ck = 2 * K + (q >> 1);
          if ((cj << h) < L.n_space && (ck << h) < L.n_space) mask |= 1u << q;
        }
      }
    }
    append_children(w, a, J, K, mask, out, count, cap);  // one atomic per wave
  }
}

// A search's device state at its start: the incumbent at "none", the node
// counters zero (one launch in place of a copy and a memset).
__global__ __launch_bounds__(256) void pyr_init_kernel(BestPartial* __restrict__ inc,
                                                       unsigned long long* __restrict__ zero, int n) {
  if (threadIdx.x == 0) *inc = BestPartial{-1.7976931348623157e308, INT64_MAX};  // {-DBL_MAX, INT64_MAX}
  for (int i = threadIdx.x; i < n; i += blockDim.x) zero[i] = 0;
}

int blocks_for(int64_t n, int per) {
  int64_t b = (n + per - 1) / per;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

hipError_t launch_pyr_pool(const PyrGrid& src, const PyrGrid& dst, int d, int32_t n_grids, hipStream_t stream) {
  const int64_t total = dst.stride * n_grids;
  const int t1 = d == 1 ? 1 : (1 << (d - 1));
  const int t2 = d == 1 ? 2 : 0;
  const int ntaps = d == 1 ? 3 : 2;
  if (src.qs == 0)
    hipLaunchKernelGGL(pyr_pool_kernel<int32_t>, dim3(blocks_for(total, 256)), dim3(256), 0, stream, src, dst, t1, t2,
                       ntaps, total);
  else
    hipLaunchKernelGGL(pyr_pool_kernel<int16_t>, dim3(blocks_for(total, 256)), dim3(256), 0, stream, src, dst, t1, t2,
                       ntaps, total);
  return hipGetLastError();
}

hipError_t launch_pyr_top(const LevelWork& L, int32_t nj, int64_t first, int64_t n, uint64_t* out,
                          hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pyr_top_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, stream, L, nj, first, n, out);
  return hipGetLastError();
}

int pyr_blocks(int64_t upper) {
  int64_t b = (upper + kPB - 1) / kPB;
  if (b > 4096) b = 4096;  // 16 waves per CU; blocks stride over longer lists
  return (int)(b < 1 ? 1 : b);
}

// launch size: room for up to a wave per node of the upper bound (the kernel
// picks the lanes per node from the actual count)
int pyr_bound_blocks(int64_t upper, int32_t n_used) {
  (void)n_used;
  return pyr_blocks(upper >= INT64_MAX / 128 ? upper : upper * 64);
}

hipError_t launch_pyr_bound(const LevelWork& L, const PyrGrid& lev, int d, const ScanWork* scans,
                            const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                            const uint64_t* nodes, int64_t n, const unsigned long long* n_dev, int64_t upper,
                            double* vals, PyrPartial* partials, unsigned long long* scored, hipStream_t stream) {
  if (upper <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)pyr_bound_blocks(upper, n_used);
  const size_t lds = (size_t)n_used * sizeof(double2);
  const double2* p = reinterpret_cast<const double2*>(pts);
  if (lev.qs == 0)
    hipLaunchKernelGGL(pyr_bound_kernel<int32_t>, dim3(blocks), dim3(kPB), lds, stream, L, lev, d, scans, angles, p,
                       n_used, step, nodes, n, n_dev, vals, partials, scored);
  else
    hipLaunchKernelGGL(pyr_bound_kernel<int16_t>, dim3(blocks), dim3(kPB), lds, stream, L, lev, d, scans, angles, p,
                       n_used, step, nodes, n, n_dev, vals, partials, scored);
  return hipGetLastError();
}

hipError_t launch_pyr_final(const PyrPartial* partials, int64_t n, bool merge, int n_probe, BestPartial* inc,
                            uint64_t* probe, hipStream_t stream) {
  hipLaunchKernelGGL(pyr_final_kernel, dim3(merge ? 1 : n_probe), dim3(kPB), 0, stream, partials, n, merge ? 1 : 0,
                     inc, probe);
  return hipGetLastError();
}

int pyr_top_blocks(const LevelWork& L, int32_t nj, int32_t* ktiles, int32_t* kt, int32_t* col_blocks) {
  *ktiles = (nj + kTopKT - 1) / kTopKT;
  *kt = (nj + *ktiles - 1) / *ktiles;
  *col_blocks = (int32_t)(((int64_t)L.n_angles * nj + kTB - 1) / kTB);
  const int64_t b = (int64_t)L.n_scans * *col_blocks * *ktiles;
  return b > INT32_MAX ? -1 : (int)b;
}

hipError_t launch_pyr_top_bound(const LevelWork& L, const PyrGrid& lev, int d, int32_t nj, const ScanWork* scans,
                                const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                                uint64_t* nodes, double* vals, PyrPartial* partials, hipStream_t stream) {
  int32_t ktiles, kt, col_blocks;
  const int blocks = pyr_top_blocks(L, nj, &ktiles, &kt, &col_blocks);
  if (blocks <= 0) return hipErrorInvalidValue;
  if (lev.qs == 0)
    hipLaunchKernelGGL(pyr_top_bound_kernel<int32_t>, dim3(blocks), dim3(kTB), (size_t)n_used * sizeof(double2), stream,
                       L, lev, d, nj, ktiles, kt, col_blocks, scans, angles, reinterpret_cast<const double2*>(pts),
                       n_used, step, nodes, vals, partials);
  else
    hipLaunchKernelGGL(pyr_top_bound_kernel<int16_t>, dim3(blocks), dim3(kTB), (size_t)n_used * sizeof(double2), stream,
                       L, lev, d, nj, ktiles, kt, col_blocks, scans, angles, reinterpret_cast<const double2*>(pts),
                       n_used, step, nodes, vals, partials);
  return hipGetLastError();
}

int pyr_topbox_pieces(int32_t nj) { return (nj >= 1 && nj <= 32) ? (nj + 8) / 8 : 0; }

hipError_t launch_pyr_widen(const PyrGrid& src, const PyrGrid& dst, int32_t n_grids, hipStream_t stream) {
  if (src.qs == 0 || src.lg != dst.lg || dst.qs != src.qs) return hipErrorInvalidValue;
  const int64_t total = dst.stride * n_grids;
  hipLaunchKernelGGL(pyr_widen_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, stream, src, dst, total);
  return hipGetLastError();
}

// fewest beams a split top-level wave takes (each split wave adds its nj^2
// node sums with global atomics)
constexpr int kTopboxMinBeams = 32;

hipError_t launch_pyr_topbox(const LevelWork& L, const PyrGrid& tb, int d, int32_t nj, const ScanWork* scans,
                             const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                             int32_t* sums, int32_t* slab, PyrPartial* partials, hipStream_t stream,
                             int* split_out) {
  const int np = pyr_topbox_pieces(nj);
  const int64_t blocks = (int64_t)L.n_scans * L.n_angles;
  if (np == 0 || blocks <= 0 || blocks > INT32_MAX || n_used < 1 || n_used > 4096 || tb.qs == 0 ||
      tb.stride * 2 >= INT32_MAX || tb.pitch % 2 != 0)
    return hipErrorInvalidValue;
  const int nl = (nj * np + 63) / 64;
  const double2* p = reinterpret_cast<const double2*>(pts);
  // few (window, angle) pairs: split each one's beams over up to 16 waves (at
  // least 128 beams each) so the launch fills the chip
  int split = 1;
  while (split < kPyrTopMaxSplit && blocks * split < 4096 && n_used / (2 * split) >= kTopboxMinBeams) split *= 2;
  if (split > 1 && !slab) split = 1;
  if (split_out) *split_out = split;
  hipError_t e;
  const unsigned grid = (unsigned)(blocks * split);
  bool launched = false;
#define CSM_TOPBOX(NP, NL)                                                                                         \
  if (!launched && np == NP && nl == NL) {                                                                       \
    hipLaunchKernelGGL((pyr_topbox_kernel<NP, NL>), dim3(grid), dim3(64), 0, stream, L, tb, d, nj, scans, angles, \
                       p, n_used, step, split, sums, slab, partials);                                             \
    launched = true;                                                                                              \
  }
  CSM_TOPBOX(1, 1)
  CSM_TOPBOX(2, 1)
  CSM_TOPBOX(3, 1)
  CSM_TOPBOX(3, 2)
  CSM_TOPBOX(4, 2)
  CSM_TOPBOX(5, 3)
#undef CSM_TOPBOX
  if (!launched) return hipErrorInvalidValue;
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (split > 1)
    hipLaunchKernelGGL(pyr_topbox_final_kernel, dim3((unsigned)blocks), dim3(64), 0, stream, L, d, nj, tb.qs, n_used,
                       scans, split, slab, sums, partials);
  return hipGetLastError();
}

hipError_t launch_pyr_expand_top(const LevelWork& L, int d, int32_t nj, int qs, int32_t n_used, const ScanWork* scans,
                                 const int32_t* sums, int64_t first, int64_t n, const BestPartial* inc,
                                 int64_t* thr, uint64_t* out, unsigned long long* count, int64_t cap,
                                 hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  // a block per 256 nodes up to 65536 blocks: the loop is one dependent load
  // per iteration, so few iterations per thread
  const int blocks = blocks_for(n, 256);
  const bool shared_thr = blocks > 1024;
  if (shared_thr) hipLaunchKernelGGL(pyr_threshold_kernel, dim3(1), dim3(1), 0, stream, L, scans, qs, n_used, inc, thr);
  hipLaunchKernelGGL(pyr_expand_top_kernel, dim3(blocks), dim3(256), 0, stream, L, d, nj, qs, n_used, scans,
                     shared_thr ? (const int64_t*)thr : nullptr, sums, first, n, inc, out, count, cap);
  return hipGetLastError();
}

hipError_t launch_pyr_init(BestPartial* inc, unsigned long long* zero, int n, hipStream_t stream) {
  hipLaunchKernelGGL(pyr_init_kernel, dim3(1), dim3(256), 0, stream, inc, zero, n);
  return hipGetLastError();
}

hipError_t launch_pyr_probe(int d, int n_probe, const uint64_t* probe, uint64_t* out, hipStream_t stream) {
  const int64_t n = ((int64_t)1 << (2 * d)) * n_probe;
  hipLaunchKernelGGL(pyr_probe_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, stream, d, n_probe, probe, out);
  return hipGetLastError();
}

hipError_t launch_pyr_expand(const LevelWork& L, int d, const uint64_t* nodes, const double* bounds, int64_t n,
                             const unsigned long long* n_dev, int64_t upper, const BestPartial* inc, uint64_t* out,
                             unsigned long long* count, int64_t cap, hipStream_t stream) {
  if (upper <= 0) return hipSuccess;
  hipLaunchKernelGGL(pyr_expand_kernel, dim3(pyr_blocks(upper)), dim3(256), 0, stream, L, d, nodes, bounds, n, n_dev,
                     inc, out, count, cap);
  return hipGetLastError();
}

}  // namespace csm
