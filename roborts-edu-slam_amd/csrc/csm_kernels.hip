// csm_kernels.hip — CDNA4 (gfx950) kernels of the correlative scan matcher.
//
// Hot path replaced: the theta x X x Y x beam loops of
// MultiResolutionCorrelateScanMatcher::ScanMatch / GetResponse
// (correlate_scan_matcher.h:552-584, 637-662) plus PenalizeResponse (:718-745).
//
// The general-purpose kernels, the fallbacks of the specialised families
// (csm_box.hip one-cell steps, csm_phase.hip sub-cell steps, csm_tiny.hip
// sub-cell spans, csm_split.hip few-window launches):
//   v2 score_cols_kernel   any window and any grid: lane = (theta, x) column,
//                          fp64 sums in the reference's beam order for any fp32
//                          grid, or exact fixed-point sums (INT mode)
//   v4 score_rowsd_kernel  INT mode, windows whose x-span fits a row segment:
//                          row segments staged in LDS by LDS-DMA
//   reduce_best_kernel     per-window argmax of the block partials
// (r03 retired v1, lane per candidate, and v3, register-staged row segments:
// every window they took, v2 or v4 takes, and no selection reached them.)
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
// LevelWork::clear_word: block 0, lane 0 of a scoring kernel clears it.
__device__ __forceinline__ void clear_word(const LevelWork& L) {
  if (L.clear_word && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(L.clear_word), (uint64_t)(uint32_t)L.clear_tag << 32,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // {count 0, tag} (dev::clear_word)
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// Divisor (:659) and centre penalty (:718-745) of one candidate.
__device__ __forceinline__ double penalized(const LevelWork& L, const ScanWork& S, double acc,
                                           double x, double y, double angle) {
  double score = acc / S.divisor;
  if (L.use_penalty) {
    // util::DoubleEqual(score, 0.0) with kDoubleTolerance = 1e-6.
    const bool is_zero = (score < 0.0) ? (score >= -1e-06) : (score <= 1e-06);
    if (!is_zero) {
      const double dx = x - S.cx, dy = y - S.cy;
      double d2 = dx * dx + dy * dy;
      d2 *= (L.mres * L.mres);
      double dp = 1.0 - (L.dist_gain * d2 / (L.size / 2));
      dp = dp < 0.5 ? 0.5 : dp;  // std::max(dp, 0.5)
      double da = angle - S.ct;
      da = da * da;
      double ap = 1.0 - (0.25 * da / 0.349);
      ap = ap < 0.9 ? 0.9 : ap;
      score = score * (dp * ap);
    }
  }
  return score;
}

__device__ __forceinline__ bool better(double s, int64_t f, double bs, int64_t bf) {
  return (s > bs) || (s == bs && f < bf);
}

// ---- v2: column kernel ------------------------------------------------------
// One wave per block; lane = one (theta, x) column of the window, KT rows of
// y per lane (KT == n_space for the front-end windows, so no row is wasted).
// Per beam a lane rotates the point once (LUT entry :179-180) and truncates
// the x index once (:647); only the y index (:648) is per candidate. The beam
// is wave-uniform (scalar load). The loop body has no branches: all KT loads
// of a beam are in flight together.
//
// INT mode: cells are read from an exact fixed-point copy holding
// (value - outside) * 2^E through a buffer descriptor; an out-of-grid offset
// fails the hardware range check and reads 0, i.e. exactly `outside`, which is
// added back as n_used * outside * 2^E at the end. Sums run in 32-bit chunks
// folded into 64-bit; csm_set_grid enables the mode only when that integer
// sum equals the reference's sequential fp64 sum bit for bit.
template <int KT, bool INT, bool BEST>
__global__ __launch_bounds__(64) void score_cols_kernel(
    LevelWork L, const ScanWork* __restrict__ scans, const double2* __restrict__ pts,
    const AngleEntry* __restrict__ angles, double* __restrict__ out,
    BestPartial* __restrict__ partials) {
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  clear_word(L);
  const int win = bid / L.blocks_per_scan;
  const int r = bid - win * L.blocks_per_scan;
  const int cb = r / L.ktiles;
  const int kt = r - cb * L.ktiles;
  const ScanWork S = scans[win];
  const int lane = threadIdx.x;
  const int col = cb * 64 + lane;
  const bool valid = col < L.n_cols;
  const int colc = valid ? col : 0;
  const int a = colc / L.n_space;
  const int j = colc - a * L.n_space;
  const AngleEntry ae = angles[S.angle_off + a];
  const double x = S.x0 + j * L.step_cells;  // :569
  const int k0 = kt * KT;
  double y[KT];
#pragma unroll
  for (int kk = 0; kk < KT; ++kk) y[kk] = S.y0 + (k0 + kk) * L.step_cells;  // :572
  const int sx = L.size_x, sy = L.size_y;
  const int64_t gofs = (int64_t)S.grid_index * L.grid_stride;
  const double2* __restrict__ P = pts + S.pts_off;
  const int step = S.step;
  const int n_used = S.n_used;
  double accd[KT];
  int64_t acci[KT];
#pragma unroll
  for (int kk = 0; kk < KT; ++kk) {
    accd[kk] = 0.0;
    acci[kk] = 0;
  }
  if (INT) {
    const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
    const int32_t* gbase = (const int32_t*)(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)gbase, (short)0, (int)(L.gridi_stride * 4), 0x00020000);
    const int sx4 = L.pitch * 4;  // row stride of gridi (bytes)
    // Cells of beam b for every row of this lane (KT buffer loads in flight).
    // The host guarantees |gy| * 4 * pitch < 2^30 for every candidate of the
    // window (run_windows), so gy * sx4 never wraps: a row outside [0, sy)
    // gives an offset < 0 or >= 4*pitch*sy, and an x outside [0, sx) adds -2^30;
    // both fail the descriptor's range check and read 0 (= `outside`).
    auto load_beam = [&](int b, int32_t (&v)[KT]) {
      const double2 p = P[(int64_t)b * step];
      const double lx = ae.cosine * p.x - ae.sine * p.y;
      const double ly = ae.sine * p.x + ae.cosine * p.y;
      const int gx = (int)((lx + x) + 0.5);
      const int gx4 = ((unsigned)gx < (unsigned)sx) ? gx * 4 : -(1 << 30);
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        const int gy = (int)((ly + y[kk]) + 0.5);
        v[kk] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, __mul24(gy, sx4) + gx4, 0, 0);
      }
    };
    constexpr int kFold = 32;  // 32 * 2^26 <= 2^31: int32 chunk sums cannot overflow
    // two register sets, beams alternate between them: beam b+1's loads are
    // in flight while beam b is summed, with no register copies in between
    int32_t va[KT], vb[KT];
    load_beam(0, va);
    for (int base = 0; base < n_used; base += kFold) {
      const int nb = min(kFold, n_used - base);
      int32_t part[KT];
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) part[kk] = 0;
      for (int b = 0; b < nb; b += 2) {
        load_beam(min(base + b + 1, n_used - 1), vb);
        // keep the sums below the next beam's loads: the waits then leave
        // those KT loads in flight (vmcnt(KT)) instead of draining them
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) part[kk] += va[kk];
        load_beam(min(base + b + 2, n_used - 1), va);
        __builtin_amdgcn_sched_barrier(0);
        if (b + 1 < nb) {
#pragma unroll
          for (int kk = 0; kk < KT; ++kk) part[kk] += vb[kk];
        }
      }
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) acci[kk] += part[kk];
      // kFold is even, so every chunk but the last ends with va holding beam
      // base + kFold, the next chunk's first; only the last chunk can be odd.
    }
  } else {
    const float* __restrict__ gf = L.grid + gofs;
    const float outside = L.outside;
    auto load_beam = [&](int b, float (&v)[KT]) {
      const double2 p = P[(int64_t)b * step];
      const double lx = ae.cosine * p.x - ae.sine * p.y;
      const double ly = ae.sine * p.x + ae.cosine * p.y;
      const int gx = (int)((lx + x) + 0.5);
      const bool inx = (unsigned)gx < (unsigned)sx;
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        const int gy = (int)((ly + y[kk]) + 0.5);
        const bool inb = inx & ((unsigned)gy < (unsigned)sy);
        const float g = gf[inb ? gy * sx + gx : 0];
        v[kk] = inb ? g : outside;  // :651
      }
    };
    float v[KT];
    load_beam(0, v);
    for (int b = 0; b < n_used; ++b) {
      float vn[KT];
      load_beam(min(b + 1, n_used - 1), vn);
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        accd[kk] += (double)v[kk];  // :652, beam order
        v[kk] = vn[kk];
      }
    }
  }
  const int krem = min(KT, L.n_space - k0);
  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
#pragma unroll
  for (int kk = 0; kk < KT; ++kk) {
    if (kk < krem && valid) {
      const double acc =
          INT ? (double)(acci[kk] + (int64_t)n_used * L.outside_i) * L.int_scale : accd[kk];
      const double score = penalized(L, S, acc, x, y[kk], ae.angle);
      const int64_t flat = ((int64_t)a * L.n_space + j) * L.n_space + (k0 + kk);
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
    for (int off = 32; off > 0; off >>= 1) {
      const double os = __shfl_down(bs, off, 64);
      const int64_t of = __shfl_down(bf, off, 64);
      if (better(os, of, bs, bf)) {
        bs = os;
        bf = of;
      }
    }
    if (lane == 0) partials[(int64_t)win * L.blocks_per_scan + r] = BestPartial{bs, bf};
  }
}

// 16-byte buffer load written straight into LDS at lds + 16 * lane. The
// builtin has no host-side form; the guard only keeps hipcc's host pass (which
// must still emit the kernel's launch stub) from seeing it.
__device__ __forceinline__ void buffer_load_lds16(__amdgpu_buffer_rsrc_t rsrc,
                                                  __attribute__((address_space(3))) int32_t* lds,
                                                  int voffset) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, lds, 16, voffset, 0, 0, 0);
#endif
}

// ---- v4: row-segment kernel, LDS-DMA staging (INT mode) --------------------
// For one beam and one angle the endpoint cells of a window's candidates form
// a separable set: ix depends only on the x step j, iy only on the y step k
// (:647-648). With lane (theta, r) of an angle group of NS lanes:
//   * the group's NS grid rows iy_r are each needed over the same short x-span
//     [xs, xs + SEG) (SEG = 4*SQ cells > (n_space-1)*f + 1, chosen by the host),
//     so a wave fetches its R = G*NS row segments as R*SQ 16-byte pieces; the
//     pieces are dealt to lanes row-major (lane l of load instruction i takes
//     piece 64*i + l), so one instruction covers ~64/SQ whole row segments and
//     touches few cache lines (a lane-per-row deal made every lane hit its own
//     line: 64 lines per instruction, measured slower than v2). Each piece's
//     row address comes from its owner lane by ds_bpermute, and the pieces are
//     parked in an LDS tile, one row per segment;
//   * lane (theta, j = r) computes its exact ix_r (reference arithmetic) and
//     reads column ix_r - xs of each of its group's NS tile rows: NS LDS reads
//     at immediate offsets.
// Per beam a wave issues ceil(R*SQ/64) gathers for R*NS candidates (v2: NS
// gathers for 64 candidates; TA-busy ~85% there, profiles/r01). A cell outside
// the grid reads 0 (= `outside`, pre-subtracted): rows through the buffer range
// check, x through a zero pad column of the tile. A lane whose x-span ever
// exceeds SEG (impossible for the host's SEG; kept as a guard) is recomputed
// exactly after the loop.
//
// The 16-byte pieces go straight into LDS by global_load_lds_dwordx4 (dest =
// wave-uniform base + 16 * lane): no VGPR staging and no ds_write_b128 (13
// LDS cycles each, the largest LDS cost of r01's register-staged form). Pieces are dealt row-major, so the LDS image is [row][SEG] with rows
// contiguous; beams alternate between two images (DMA of beam b+1 in flight
// while beam b is summed, counted vmcnt). DMA has no range check: rows outside
// the grid point at the zero row the host appends to gridi, columns outside
// the grid read a zero block.
// BS waves per block split a window's beams into BS contiguous ranges (low
// wave counts per launch otherwise: the super-fine level is one wave per
// window); their integer sums meet in LDS, exact in any order.
template <int NS, int SQ, bool BEST, int BS>
__global__ __launch_bounds__(64 * BS) void score_rowsd_kernel(
    LevelWork L, const ScanWork* __restrict__ scans, const double2* __restrict__ pts,
    const AngleEntry* __restrict__ angles, double* __restrict__ out,
    BestPartial* __restrict__ partials) {
  constexpr int G = 64 / NS;           // angle groups per wave
  constexpr int R = G * NS;            // row segments per beam
  constexpr int SEG = 4 * SQ;          // cells per row segment
  constexpr int NP = R * SQ;           // 16-byte pieces per beam
  constexpr int NI = (NP + 63) / 64;   // DMA instructions per beam
  constexpr int IMG = NI * 256;        // ints per image
  typedef __attribute__((address_space(3))) int32_t lds_i32;
  // two images as distinct objects, so the compiler's LDS-DMA wait tracking
  // can tell a read of one from the DMA still writing the other
  __shared__ __attribute__((aligned(16))) int32_t img0_s[BS * IMG];
  __shared__ __attribute__((aligned(16))) int32_t img1_s[BS * IMG];
  __shared__ __attribute__((aligned(16))) int32_t img2_s[BS * IMG];
  __shared__ __attribute__((aligned(16))) int32_t zblk[NS * SEG];
  __shared__ int64_t xsum[(BS - 1) * 64 * NS + 1];  // waves 1.. -> wave 0
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  clear_word(L);
  const int win = bid / L.blocks_per_scan;
  const int blk = bid - win * L.blocks_per_scan;
  const ScanWork S = scans[win];
  const int lane = BS > 1 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  const int wv = BS > 1 ? (int)(threadIdx.x >> 6) : 0;  // BS == 1: images at fixed LDS addresses
  int32_t* const img0 = img0_s + wv * IMG;
  int32_t* const img1 = img1_s + wv * IMG;
  int32_t* const img2 = img2_s + wv * IMG;
  const int g = lane / NS;
  // idle lanes (g >= G) shadow lane (G-1, NS-1): identical LDS addresses
  // broadcast instead of adding bank conflicts
  const int ge = g < G ? g : G - 1;
  const int r = g < G ? lane - g * NS : NS - 1;
  const int a_raw = blk * G + ge;
  const bool valid = (g < G) && (a_raw < L.n_angles);
  const int a = a_raw < L.n_angles ? a_raw : 0;
  const AngleEntry ae = angles[S.angle_off + a];
  const double f = L.step_cells;
  const double x_0 = S.x0 + 0 * f;  // :569 at j = 0
  const double x_r = S.x0 + r * f;  // :569 at j = r
  const double y_r = S.y0 + r * f;  // :572 at k = r
  const int sx = L.size_x, sy = L.size_y;
  const int pitch = L.pitch;
  const int xs_max = sx - SEG;  // host: sx >= SEG
  const double2* __restrict__ P = pts + S.pts_off;
  const int step = S.step;
  const int n_used = S.n_used;
  const int b_lo = (int)((int64_t)n_used * wv / BS);  // this wave's beams
  const int b_hi = (int)((int64_t)n_used * (wv + 1) / BS);
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(L.gridi_stride * 4), 0x00020000);
  const int pitch4 = pitch * 4;
  const int zero_off = sy * pitch4;  // byte offset of the appended zero row

  int src4[NI], qofs[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int p = i * 64 + lane;
    const bool act = p < NP;
    const int rho = act ? p / SQ : 0;
    src4[i] = rho * 4;
    qofs[i] = act ? 16 * (p - rho * SQ) : -1;  // bytes into the segment; -1: idle piece
  }
  for (int t = lane; t < NS * SEG; t += 64) zblk[t] = 0;
  __syncthreads();

  // Beam points, 64 at a time in registers (lane l holds beam pbase + l) and
  // broadcast by readlane: no scalar load (and its lgkmcnt(0) drain of the
  // LDS queue) per beam.
  double2 pw = P[(int64_t)max(0, min(b_lo + lane, b_hi - 1)) * step];
  int pbase = b_lo;
  auto bcast = [](double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  };
  auto point = [&](int b) {
    const int l = b - pbase;
    double2 p;
    p.x = bcast(pw.x, l);
    p.y = bcast(pw.y, l);
    return p;
  };

  auto image = [&](int buf) -> int32_t* { return buf == 0 ? img0 : (buf == 1 ? img1 : img2); };
  // Beam b into image buf: issue this lane's DMA pieces; return the LDS byte
  // address of this lane's column in its group's k = 0 row.
  auto prep = [&](int b, int buf, lds_i32*& rd, bool& bad) {
    const double2 p = point(b);
    const double lx = ae.cosine * p.x - ae.sine * p.y;  // :179
    const double ly = ae.sine * p.x + ae.cosine * p.y;  // :180
    const int ix0 = (int)((lx + x_0) + 0.5);
    const int ixr = (int)((lx + x_r) + 0.5);
    const int iyr = (int)((ly + y_r) + 0.5);
    const int xs = min(max(ix0, 0), xs_max);
    const int rowoff = ((unsigned)iyr < (unsigned)sy) ? __mul24(iyr, pitch4) + xs * 4 : zero_off;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int o = __builtin_amdgcn_ds_bpermute(src4[i], rowoff);
      buffer_load_lds16(rsrc, (lds_i32*)(image(buf) + i * 256), qofs[i] < 0 ? zero_off : o + qofs[i]);
    }
    const int pos = ixr - xs;
    const bool inx = (unsigned)ixr < (unsigned)sx;
    bad |= inx & ((unsigned)pos >= (unsigned)SEG);
    lds_i32* row0 = (lds_i32*)(image(buf) + ge * NS * SEG);
    rd = inx ? row0 + pos : (lds_i32*)&zblk[0];
  };
  // The reads are inline asm: hipcc's wait insertion treats every LDS read as
  // aliasing any LDS-DMA in flight and drains vmcnt(0), serialising the
  // pipeline; the explicit vmcnt(NI) before these reads is the real fence.
  auto consume = [&](const lds_i32* rd, int32_t (&part)[NS]) {
    typedef int32_t v2i __attribute__((ext_vector_type(2)));
    v2i w[(NS + 1) / 2];  // rows 2h, 2h+1; untouched until the lgkmcnt(0) below
    const uint32_t a = (uint32_t)(uintptr_t)rd;
#pragma unroll
    for (int h = 0; h < (NS + 1) / 2; ++h) {
      const int k = 2 * h;
      if (k + 1 < NS && (k + 1) * SEG <= 255) {  // two rows per instruction (dword offsets)
        asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3"
                     : "=v"(w[h]) : "v"(a), "i"(k * SEG), "i"((k + 1) * SEG));
      } else if (k + 1 < NS) {
        asm volatile("ds_read_b32 %0, %2 offset:%3\n\tds_read_b32 %1, %2 offset:%4"
                     : "=&v"(w[h].x), "=&v"(w[h].y) : "v"(a), "i"(k * SEG * 4), "i"((k + 1) * SEG * 4));
      } else {
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(w[h].x) : "v"(a), "i"(k * SEG * 4));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int h = 0; h < (NS + 1) / 2; ++h) {
      asm volatile("" : "+v"(w[h]));
      part[2 * h] += w[h].x;
      if (2 * h + 1 < NS) part[2 * h + 1] += w[h].y;
    }
  };

  int64_t acci[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acci[k] = 0;
  bool bad = false;
  // Three images: beam b is summed while the DMAs of b+1 and b+2 are in
  // flight (vmcnt(2*NI)). Chunks of 30 beams keep beam -> image static
  // (30 * (2^26 - 1) < 2^31, ensure_int_grid).
  constexpr int kFold = 30;
  constexpr short kWait2 = (short)(0xF70 | (2 * NI));  // needs 2*NI < 16
  static_assert(2 * NI < 16, "vmcnt field");
  lds_i32 *r0 = nullptr, *r1 = nullptr, *r2 = nullptr;
  if (b_hi > b_lo) {
    prep(b_lo, 0, r0, bad);
    prep(min(b_lo + 1, b_hi - 1), 1, r1, bad);
  }
  for (int base = b_lo; base < b_hi; base += kFold) {
    const int nb = min(kFold, b_hi - base);
    if (base != pbase) {  // this chunk preps beams base+2 .. base+kFold+1
      pbase = base;
      pw = P[(int64_t)min(base + lane, b_hi - 1) * step];
    }
    int32_t part[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) part[k] = 0;
    for (int b = 0; b < nb; b += 3) {
      prep(min(base + b + 2, b_hi - 1), 2, r2, bad);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(kWait2);
      __builtin_amdgcn_sched_barrier(0);
      consume(r0, part);
      __builtin_amdgcn_sched_barrier(0);
      prep(min(base + b + 3, b_hi - 1), 0, r0, bad);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(kWait2);
      __builtin_amdgcn_sched_barrier(0);
      if (b + 1 < nb) consume(r1, part);
      __builtin_amdgcn_sched_barrier(0);
      prep(min(base + b + 4, b_hi - 1), 1, r1, bad);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(kWait2);
      __builtin_amdgcn_sched_barrier(0);
      if (b + 2 < nb) consume(r2, part);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) acci[k] += part[k];
  }
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): no DMA outlives the workgroup
  if (bad) {  // guard (never taken for the host's SEG): exact per-cell recompute
#pragma unroll
    for (int k = 0; k < NS; ++k) acci[k] = 0;
    for (int b = b_lo; b < b_hi; ++b) {
      const double2 p = P[(int64_t)b * step];
      const double lx = ae.cosine * p.x - ae.sine * p.y;
      const double ly = ae.sine * p.x + ae.cosine * p.y;
      const int gx = (int)((lx + x_r) + 0.5);
      const bool inx = (unsigned)gx < (unsigned)sx;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int gy = (int)((ly + (S.y0 + k * f)) + 0.5);
        const bool in = inx && (unsigned)gy < (unsigned)sy;
        acci[k] += gi[in ? (int64_t)gy * pitch + gx : (int64_t)sy * pitch];
      }
    }
  }
  if constexpr (BS > 1) {  // the other waves' sums into wave 0
    if (wv > 0) {
#pragma unroll
      for (int k = 0; k < NS; ++k) xsum[((wv - 1) * NS + k) * 64 + lane] = acci[k];
    }
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int w2 = 1; w2 < BS; ++w2)
#pragma unroll
      for (int k = 0; k < NS; ++k) acci[k] += xsum[((w2 - 1) * NS + k) * 64 + lane];
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

template <int KT>
static hipError_t launch_cols_kt(const LevelWork& L, const ScanWork* d_scans, const double2* d_pts,
                                 const AngleEntry* d_angles, double* d_out, BestPartial* d_partials,
                                 hipStream_t stream) {
  const int64_t nblk = (int64_t)L.blocks_per_scan * L.n_scans;
  if (nblk <= 0 || nblk > INT32_MAX) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk), block(64);
  if (d_partials) {
    if (L.int_mode)
      hipLaunchKernelGGL((score_cols_kernel<KT, true, true>), grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out, d_partials);
    else
      hipLaunchKernelGGL((score_cols_kernel<KT, false, true>), grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out, d_partials);
  } else {
    if (L.int_mode)
      hipLaunchKernelGGL((score_cols_kernel<KT, true, false>), grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out, d_partials);
    else
      hipLaunchKernelGGL((score_cols_kernel<KT, false, false>), grid, block, 0, stream, L, d_scans, d_pts, d_angles, d_out, d_partials);
  }
  return hipGetLastError();
}

hipError_t launch_score_cols(const LevelWork& L, const ScanWork* d_scans, const double* d_pts_raw,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials,
                             int kt, hipStream_t stream) {
  const double2* d_pts = reinterpret_cast<const double2*>(d_pts_raw);
#define CSM_KT_CASE(K) \
  case K: return launch_cols_kt<K>(L, d_scans, d_pts, d_angles, d_out, d_partials, stream);
  switch (kt) {
    CSM_KT_CASE(1) CSM_KT_CASE(2) CSM_KT_CASE(3) CSM_KT_CASE(4) CSM_KT_CASE(5) CSM_KT_CASE(6)
    CSM_KT_CASE(7) CSM_KT_CASE(8) CSM_KT_CASE(9) CSM_KT_CASE(10) CSM_KT_CASE(11)
    CSM_KT_CASE(12) CSM_KT_CASE(13) CSM_KT_CASE(14) CSM_KT_CASE(15) CSM_KT_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef CSM_KT_CASE
}

// Row-segment instantiations (n_space, SQ): the sim-YAML levels (13,4) (11,2)
// (3,1), param_config.h's coarse (9,5) and config 1's window (21,6) at 5 cm.
#define CSM_ROWS_LIST(X) X(13, 4) X(11, 2) X(3, 1) X(9, 5) X(21, 6)

int rows_pick_sq(int ns, int need_seg) {
#define CSM_ROWS_PICK(N, Q) \
  if (ns == N && 4 * Q >= need_seg) return Q;
  CSM_ROWS_LIST(CSM_ROWS_PICK)
#undef CSM_ROWS_PICK
  return 0;
}

// Waves per block of the LDS-DMA row kernel: launches of fewer than 4096
// blocks (the super-fine level: one block per window) split each window's
// beams over up to 8 waves, towards 16 waves per SIMD; at most 64 KB of LDS
// per block (three images and the cross-wave sums per wave). Measured on the
// fine level (6144 blocks), a 4-way split was 7% slower than none.
int rows_beam_split(int64_t blocks) {
  int bs = 1;
  if (blocks >= 4096) return 1;
  while (bs < 8 && blocks * bs < 16384) bs *= 2;
  return bs;
}
template <int NS, int SQ>
constexpr int rows_bs_cap() {
  constexpr int NP = (64 / NS) * NS * SQ;
  constexpr int IMG = (NP + 63) / 64 * 256;
  int bs = 8;
  while (bs > 1 && bs * (3 * IMG * 4 + NS * 64 * 8) > 64 * 1024) bs /= 2;
  return bs;
}
template <int NS, int SQ, int B>
hipError_t launch_rowsd(const LevelWork& L, const ScanWork* d_scans, const double2* d_pts,
                        const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, dim3 grid,
                        hipStream_t stream) {
  if constexpr (B > rows_bs_cap<NS, SQ>()) {
    return launch_rowsd<NS, SQ, rows_bs_cap<NS, SQ>()>(L, d_scans, d_pts, d_angles, d_out, d_partials, grid,
                                                        stream);
  } else {
    if (d_partials)
      hipLaunchKernelGGL((score_rowsd_kernel<NS, SQ, true, B>), grid, dim3(64 * B), 0, stream, L, d_scans, d_pts,
                         d_angles, d_out, d_partials);
    else
      hipLaunchKernelGGL((score_rowsd_kernel<NS, SQ, false, B>), grid, dim3(64 * B), 0, stream, L, d_scans, d_pts,
                         d_angles, d_out, d_partials);
    return hipGetLastError();
  }
}

hipError_t launch_score_rows(const LevelWork& L, const ScanWork* d_scans, const double* d_pts_raw,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials,
                             int ns, int sq, hipStream_t stream) {
  const double2* d_pts = reinterpret_cast<const double2*>(d_pts_raw);
  const int64_t nblk = (int64_t)L.blocks_per_scan * L.n_scans;
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || L.size_x < 4 * sq) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  const int bs = rows_beam_split(nblk);
#define CSM_ROWSD_LAUNCH(N, Q, B) \
  return launch_rowsd<N, Q, B>(L, d_scans, d_pts, d_angles, d_out, d_partials, grid, stream)
#define CSM_ROWS_CASE(N, Q)                     \
  if (ns == N && sq == Q) {                     \
    if (bs == 1) CSM_ROWSD_LAUNCH(N, Q, 1);     \
    if (bs == 2) CSM_ROWSD_LAUNCH(N, Q, 2);     \
    if (bs == 4) CSM_ROWSD_LAUNCH(N, Q, 4);     \
    CSM_ROWSD_LAUNCH(N, Q, 8);                  \
  }
  CSM_ROWS_LIST(CSM_ROWS_CASE)
#undef CSM_ROWS_CASE
#undef CSM_ROWSD_LAUNCH
  return hipErrorInvalidValue;
}

// max |x| + |y| over a batch's points (csm_load_scans_async): the bound
// int_mode_ok needs, found on the device while the batch uploads instead of
// by the host reading every point. Non-negative doubles order like their
// bits, and a NaN's bits exceed +inf's, so an integer max keeps NaN.
__global__ __launch_bounds__(256) void points_maxabs_kernel(const double2* __restrict__ p, int64_t n,
                                                            unsigned long long* __restrict__ out) {
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double2 q = p[i];
    const double a = fabs(q.x) + fabs(q.y);
    const unsigned long long b = __builtin_bit_cast(unsigned long long, a);
    m = b > m ? b : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

hipError_t launch_points_maxabs(const double* pts, int64_t n, unsigned long long* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(points_maxabs_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     reinterpret_cast<const double2*>(pts), n, out);
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

// ---- grid analysis / fixed-point copy (csm_set_grid) -----------------------
namespace csm {
namespace {

// Per cell: finite? smallest power of two the value is a multiple of, and |v|.
// Pass 1: each block reduces its cells in registers, then across its waves in
// LDS, and writes one partial (no atomics: thousands of same-address atomics
// serialised the old version at ~0.3 ms for a 3000 x 3000 map).
__global__ __launch_bounds__(256) void analyze_grid_kernel(const float* __restrict__ g, int64_t n,
                                                           GridStats* __restrict__ partials) {
  int min_g = INT32_MAX;
  uint32_t max_bits = 0;
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t u = __float_as_uint(g[i]) & 0x7FFFFFFFu;
    const uint32_t e = u >> 23, m = u & 0x7FFFFFu;
    if (e == 0xFF) {
      bad = 1;
      continue;
    }
    if (u == 0) continue;
    const uint32_t mm = (e == 0) ? m : (m | 0x800000u);
    const int gexp = ((e == 0) ? -149 : (int)e - 150) + __builtin_ctz(mm);
    min_g = min(min_g, gexp);
    max_bits = max(max_bits, u);
  }
  for (int off = 32; off > 0; off >>= 1) {
    min_g = min(min_g, __shfl_down(min_g, off, 64));
    max_bits = max(max_bits, (uint32_t)__shfl_down((int)max_bits, off, 64));
    bad |= __shfl_down(bad, off, 64);
  }
  __shared__ GridStats w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = GridStats{min_g, max_bits, bad, 0};
  __syncthreads();
  if (threadIdx.x == 0) {
    GridStats r = w[0];
    for (int k = 1; k < 4; ++k) {
      r.min_gexp = min(r.min_gexp, w[k].min_gexp);
      r.max_abs_bits = max(r.max_abs_bits, w[k].max_abs_bits);
      r.nonfinite |= w[k].nonfinite;
    }
    partials[blockIdx.x] = r;
  }
}

// Pass 2: one block folds the partials into st[0].
__global__ __launch_bounds__(256) void analyze_reduce_kernel(const GridStats* __restrict__ partials, int np,
                                                             GridStats* __restrict__ st) {
  int min_g = INT32_MAX;
  uint32_t max_bits = 0;
  int bad = 0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    const GridStats p = partials[i];
    min_g = min(min_g, p.min_gexp);
    max_bits = max(max_bits, p.max_abs_bits);
    bad |= p.nonfinite;
  }
  for (int off = 32; off > 0; off >>= 1) {
    min_g = min(min_g, __shfl_down(min_g, off, 64));
    max_bits = max(max_bits, (uint32_t)__shfl_down((int)max_bits, off, 64));
    bad |= __shfl_down(bad, off, 64);
  }
  __shared__ GridStats w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = GridStats{min_g, max_bits, bad, 0};
  __syncthreads();
  if (threadIdx.x == 0) {
    GridStats r = w[0];
    for (int k = 1; k < 4; ++k) {
      r.min_gexp = min(r.min_gexp, w[k].min_gexp);
      r.max_abs_bits = max(r.max_abs_bits, w[k].max_abs_bits);
      r.nonfinite |= w[k].nonfinite;
    }
    st[0] = r;
  }
}

// gi = (g - outside) * 2^E, exact when the host accepted E.
// gi[y * pitch + x] = (g[y * sx + x] - outside) * 2^E; pad cells (x >= sx)
// and the appended zero row y = sy (what DMA reads for rows off the grid) = 0.
__global__ __launch_bounds__(256) void fixed_point_kernel(const float* __restrict__ g, int32_t sx,
                                                          int32_t sy, int32_t pitch, float outside,
                                                          double scale, int32_t* __restrict__ gi,
                                                          int32_t pad_rows) {
  const int64_t n = (int64_t)pitch * (sy + pad_rows);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t y = i / pitch;
    const int x = (int)(i - y * pitch);
    gi[i] = (x < sx && y < sy) ? (int32_t)(((double)g[y * sx + x] - (double)outside) * scale) : 0;
  }
}

}  // namespace

hipError_t launch_analyze_grid(const float* g, int64_t n, GridStats* d_stats, hipStream_t stream) {
  // d_stats holds 1 + kAnalyzeBlocks entries: the result, then the partials
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, kAnalyzeBlocks));
  hipLaunchKernelGGL(analyze_grid_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, n, d_stats + 1);
  hipLaunchKernelGGL(analyze_reduce_kernel, dim3(1), dim3(256), 0, stream, d_stats + 1, (int)blocks, d_stats);
  return hipGetLastError();
}

hipError_t launch_fixed_point(const float* g, int32_t sx, int32_t sy, int32_t pitch, float outside,
                              int int_exp, int32_t* gi, hipStream_t stream, bool pad) {
  const int32_t pad_rows = pad ? kGridiPadRows : 0;
  const int64_t n = (int64_t)pitch * (sy + pad_rows);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(fixed_point_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0,
                     stream, g, sx, sy, pitch, outside, ldexp(1.0, int_exp), gi, pad_rows);
  return hipGetLastError();
}

namespace {
// Incremental refresh of a resident grid (csm_update_grid_cells): each entry
// rewrites one fp32 cell and, when the exact fixed-point copy exists, its
// int32 image with the fixed_point_kernel's expression. Duplicate indices
// carry the same value, so their order does not matter.
__global__ __launch_bounds__(256) void update_cells_kernel(const CellUpdate* __restrict__ u, int64_t n,
                                                           float* __restrict__ g, int32_t sx,
                                                           int32_t* __restrict__ gi, int32_t pitch,
                                                           float outside, double scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const CellUpdate c = u[i];
    g[c.index] = c.value;
    if (gi) {
      const int32_t y = c.index / sx;
      const int32_t x = c.index - y * sx;
      gi[(int64_t)y * pitch + x] = (int32_t)(((double)c.value - (double)outside) * scale);
    }
  }
}
}  // namespace

hipError_t launch_update_cells(const CellUpdate* d_updates, int64_t n, float* g, int32_t sx, int32_t* gi,
                               int32_t pitch, float outside, int int_exp, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(update_cells_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_updates, n, g, sx, gi,
                     pitch, outside, ldexp(1.0, int_exp));
  return hipGetLastError();
}

}  // namespace csm
