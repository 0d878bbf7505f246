// csm_box.hip — v6 "box" scoring kernel: window levels whose step is exactly
// one map cell (the coarse level of every shipped parameter set at its own map
// resolution, e.g. simulatin_param.yaml's 0.05 m window on a 0.05 m map).
//
// With step 1, candidate (j, k) of angle a reads, for beam b, cell
// (ix_j, iy_k) = (trunc((lx + x_j) + 0.5), trunc((ly + y_k) + 0.5))
// (correlate_scan_matcher.h:637-662 with x_j = x0 + j, y_k = y0 + k, :569/:572).
// Whenever t = (lx + x0) + 0.5 is non-negative with a fraction at least
// kBoxMargin away from an integer, ix_j = trunc(t) + j for every j (see
// kBoxMargin for the rounding argument): the beam's cells form one
// n_space x n_space box of the grid. The fixed-point grid (gridi) is padded
// with zero columns and rows, so the box is n_space row pieces of 16 bytes
// that one buffer_load_dwordx4 per lane fetches: lane (k, q) loads row
// iy0 + k, cells ix0 + 4q .. ix0 + 4q + 3, and adds them to its four
// candidates (j = 4q .. 4q+3, k). The box corner is one scalar per beam
// (soffset), so a beam costs one vector-memory instruction, one readlane and
// four integer adds per wave: no LDS, no per-lane address arithmetic.
// Beams that fail the test (off the grid on the low side, or a fraction
// within the margin of a rounding boundary) read the zero
// block and are summed afterwards cell by cell with the reference's own
// expressions, so the scores are the reference's bit for bit in every case.
//
// Tiled mode (L.tile_n > 0, best only): a one-cell-step window wider than 16
// (the loop-closure windows, 321^2 and 401^2) is covered by 16 x 16 tiles at
// offsets (ox, oy) = (min(16 ti, n - 16), min(16 tj, n - 16)), one wave per
// (window, tile, angle): the last tile of an axis is shifted back to the edge
// (overlapping candidates score identically). Candidate (j, k) of a tile is the
// window's (ox + j, oy + k), formed as x0 + (ox + j) * f like the reference's
// x_j, and its flat index is the window's, so the per-window reduction keeps
// the lowest index among equal scores across tiles.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "csm_device.hpp"
#include "csm_tail.hpp"
#include "csm_internal.hpp"

namespace csm {
namespace {

typedef int32_t v4i __attribute__((ext_vector_type(4)));

// Rounding argument. Host: every |x_j|, |lx + x_j|, |t_j| < 2^24 cells
// (use_int's R * 4 * pitch < 2^30, pitch >= 16). With T = lx + x0 + 0.5 (real)
// and x_j = fl(x0 + j) = x0 + j + d_j, |d_j| <= 2^-29, the reference's
// t_j = fl(fl(lx + x_j) + 0.5) = T + j + E_j with |E_j| <= 3 * 2^-29 < 2^-27.
// The kernels test t = fl(lx + h), h = fl(fl(x0 + 0.5) + pad) (one add per
// beam and axis instead of two; pad: the columns the layout holds before the
// grid's first, 0 but for the pair strips' kStripPadLo), t = T + pad + E with
// |E| <= 2^-27. If t >= 0 and frac(t) is in [2^-20, 1 - 2^-20], T + pad is
// positive and T more than 2^-20 - 2^-27 > |E_j| from an integer, so the
// padded cell of candidate j is floor(T) + j + pad = trunc(t) + j. Without
// padding that is the reference's trunc(t_j) + pad; with it, a t_j in (-1, 0)
// (trunc 0) lands on column -1, which repeats column 0, and t_j < -1 on the
// outside index. The same for rows.
constexpr double kBoxMargin = 0x1p-20;

// Beams per run-list segment: the list of one segment lives in LDS.
#ifndef CSM_RUN_SEG
#define CSM_RUN_SEG 1152
#endif
constexpr int kRunSeg = CSM_RUN_SEG;
#ifndef CSM_BOX_PF
#define CSM_BOX_PF 6
#endif
constexpr int kPF = CSM_BOX_PF;  // chunks of beam points in flight while a run list is built
// the pair kernel's list build: ILP form (below) and its points in flight
#ifndef CSM_PAIR_ILP
#define CSM_PAIR_ILP 1
#endif
#ifndef CSM_PAIR_PF
#define CSM_PAIR_PF 4
#endif
// Runs in flight per wave (16 measured no better; one load per beam instead of
// per run: 2.28 vs 1.02 ms, profiles/r01)
constexpr int kD = 8;
static_assert(kRunSeg % 64 == 0, "segments of whole 64-beam chunks");


// One wave's view of its (window, angle): the beam points, the box test and
// the per-segment run list.
struct BoxWave {
  const ScanWork& S;
  const AngleEntry& ae;
  const double2* __restrict__ P;
  int step, n_used, lane, sx, sy, pitch4, zero_off;  // pitch4: bytes per grid row
  double x_0, y_0;  // x_ox, y_oy: the tile's first candidate
  int cell_shift = 2;  // log2 bytes per cell: 2 for gridi (int32), 0 for the palette grid (bytes)
  int strip_bytes = 0, copy_bytes = 0;  // strip copies (offsets<true>): bytes per strip and per copy
  int nspan = 0;  // candidates per axis of the wave (box_test's far test; 0: off)
  // cells before the grid's first that the layout holds (kStripPadLo in the
  // pair strips): box corners and t are counted from column / row -pad
  int pad = 0;
  double hx = x_0 + 0.5 + pad, hy = y_0 + 0.5 + pad;  // box_test's t, one add per axis (rounding argument)
  // a beam point's byte offset step: full-rate 24-bit multiplies (the host
  // keeps every scan under 2^24 points and step * 16 under 2^24: box_points_ok)
  uint32_t step16 = (uint32_t)step * 16u;

  // The box test of one beam point; on success (ix0, iy0) is the box corner.
  // far: every cell the beam reads for this wave's candidates is off the
  // grid's low side (t_j <= -1 for every j < nspan on one axis, so trunc(t_j)
  // <= -1 by the rounding argument above): the beam adds the outside value,
  // zero in gridi, to every candidate, and needs no cell-by-cell pass.
  __device__ __forceinline__ bool box_test(const double2 p, double& lx, double& ly, int& ix0, int& iy0,
                                           bool& far) const {
    lx = ae.cosine * p.x - ae.sine * p.y;  // :179
    ly = ae.sine * p.x + ae.cosine * p.y;  // :180
    const double tx = lx + hx;  // the reference's (lx + x_0) + 0.5 within 2^-27 cells
    const double ty = ly + hy;
    // v_fract_f64: tx - floor(tx), exact below 2^52; it differs (1 - 2^-53 for
    // 1.0) only for tiny negative t, which the t >= 0 test rejects either way
    const double fx = __builtin_amdgcn_fract(tx);
    const double fy = __builtin_amdgcn_fract(ty);
    const bool clean = tx >= 0.0 && ty >= 0.0 && fx >= kBoxMargin && fx <= 1.0 - kBoxMargin &&
                       fy >= kBoxMargin && fy <= 1.0 - kBoxMargin;
    const double lim = (double)(pad - nspan) - kBoxMargin;
    far = nspan > 0 && (tx <= lim || ty <= lim);
    ix0 = clean ? (int)tx : 0;
    iy0 = clean ? (int)ty : 0;
    return clean;
  }
  // Lane l: the box byte offset of beam cb + l (the zero block for beams past
  // n_used, boxes wholly past the grid's high edges and rejected beams).
  // slow: bit c marks 64-beam chunk c as holding a rejected beam (bit 63:
  // some chunk >= 63), for the cell-by-cell pass at the end.
  // STRIP: the offset in the strip copies (csm_palette.hip) of the box's first
  // row piece: copy c = -(ix0 / 4) mod 4 puts cells (ix0 & ~3) .. +15 in one
  // 16-byte strip row, and the corner's byte phase ix0 & 3 rides in the low
  // bits (the piece itself is 16-byte aligned).
  template <bool STRIP = false>
  __device__ __forceinline__ int offsets(const double2 p, int cb, uint64_t& slow) const {
    double lx, ly;
    int ix0, iy0;
    bool far;
    const bool clean = box_test(p, lx, ly, ix0, iy0, far);
    const bool live = cb + lane < n_used;
    const uint64_t rej = __builtin_amdgcn_ballot_w64(live && !clean && !far);
    if (rej) slow |= 1ull << min(cb >> 6, 63);
    int o;
    if (STRIP) {  // (kStripShift: 4 or 1 cells between copies)
      constexpr int S = kStripShift, LS = S == 4 ? 2 : 0;
      const int c = (-(ix0 >> LS)) & (kStripCopies - 1);
      const int xs = (ix0 & ~(S - 1)) + S * c;
      // 24-bit products (box_pair_strips_ok: copies of whole 16-byte rows,
      // copy_bytes / 16 and strip_bytes below 2^24)
      o = (int)(__umul24((uint32_t)c, (uint32_t)copy_bytes >> 4) << 4) +
          (int)__umul24((uint32_t)(xs >> 4), (uint32_t)strip_bytes) + iy0 * 16 + (ix0 & (S - 1));
    } else {
      o = iy0 * pitch4 + (ix0 << cell_shift);
    }
    return (live && clean && ix0 < sx + pad && iy0 < sy + pad) ? o : zero_off;
  }
  __device__ __forceinline__ double2 point(int cb) const {
    const uint32_t i = (uint32_t)min(cb + lane, n_used - 1);
    return *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(P) + __umul24(i, step16));
  }

  // Run list of beams [s0, s1): consecutive beams with the same box corner
  // (common: at a few metres, neighbouring beams of a 0.25 deg scanner land in
  // the same cell) form one run, (corner offset, count) at run_off / run_cnt;
  // runs of boxes wholly off the grid and of rejected beams are dropped (they
  // read zeros). Slots from `scratch` on take the non-run lanes' writes
  // (branch-free). Returns the run count.
  template <int PF = kPF, typename CT = int32_t, bool STRIP = false, bool ILP = false>
  __device__ __forceinline__ int build_runs(int s0, int s1, int32_t* run_off, CT* run_cnt, int scratch,
                                            uint64_t& slow) const {
    int nruns = 0;
    // points of PF chunks in flight: the list build is latency-bound
    // otherwise (one dependent load per 64 beams)
    double2 pq[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {  // issued in the order the loop consumes them
      pq[u] = point(s0 + 64 * u);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int cb0 = s0; cb0 < s1; cb0 += 64 * PF) {
      // ILP: the PF chunks' box tests first (independent dependency chains
      // the compiler interleaves), then the next PF chunks' points are issued
      // and the run edges found while they are in flight
      int offv[PF];
      if constexpr (ILP) {
#pragma unroll
        for (int u = 0; u < PF; ++u) offv[u] = offsets<STRIP>(pq[u], cb0 + 64 * u, slow);
#pragma unroll
        for (int u = 0; u < PF; ++u) pq[u] = point(cb0 + 64 * (u + PF));
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        // no early exit: a chunk at or past s1 adds no run (live is false for
        // every lane), and an exit here made the compiler drain vmcnt(0) per
        // chunk instead of keeping PF chunks of points in flight
        const int cb = cb0 + 64 * u;
        int off;
        if constexpr (ILP) {
          off = offv[u];
        } else {
          const double2 pcur = pq[u];
          pq[u] = point(cb + 64 * PF);
          __builtin_amdgcn_sched_barrier(0);
          off = offsets<STRIP>(pcur, cb, slow);
        }
        const bool live = cb + lane < s1;
        // previous beam's corner (lane 0: none)
        const int prev = __builtin_amdgcn_mov_dpp(off, 0x138, 0xF, 0xF, false);  // wave_shr:1
        const bool edge = live && (lane == 0 || off != prev);  // a new corner starts here
        const uint64_t E = __builtin_amdgcn_ballot_w64(edge);
        const int nlive = min(64, s1 - cb);
        const uint64_t above = lane == 63 ? 0ull : (E >> (lane + 1)) << (lane + 1);
        const int next = above ? (int)__builtin_ctzll(above) : nlive;
        const bool head = edge && off != zero_off;
        const uint64_t Hm = __builtin_amdgcn_ballot_w64(head);
        const int rank = __builtin_popcountll(Hm & ((1ull << lane) - 1));
        const int slot = head ? nruns + rank : scratch + lane;
        run_off[slot] = off;
        run_cnt[slot] = (CT)(next - lane);  // 1..64
        nruns += __builtin_popcountll(Hm);
      }
    }
    return nruns;
  }
};

// Rejected beams, cell by cell with the reference's expressions: only the
// marked chunks are revisited, and only their rejected beams summed into the
// lane's candidates (j = 4q .. 4q+3, row k). Beams go four at a time, their 16
// gathers issued together (one at a time, a wave near the grid's low edge
// paid a dependent round trip per beam: 20 % of the pair kernel's time).
template <int NS>
__device__ __forceinline__ void slow_beams(const BoxWave& B, const LevelWork& L, const int32_t* gi, uint64_t slow,
                                           int k, int q, int ox, int oy, int64_t (&acc)[4]) {
  const double f = L.step_cells;
  const int64_t zero_cell = (int64_t)B.sy * L.pitch;  // first of the zero rows
  const double yk = B.S.y0 + (oy + k) * f;           // :572
  double xj[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) xj[t] = B.S.x0 + (ox + 4 * q + t) * f;  // :569
  for (uint64_t m = slow; m != 0; m &= m - 1) {
    const int c0 = (int)__builtin_ctzll(m);
    const int c_end = c0 == 63 ? (B.n_used + 63) / 64 : c0 + 1;
    for (int c = c0; c < c_end; ++c) {
      const int cb = c * 64;
      double lx, ly;
      int ix0, iy0;
      bool far;
      const bool clean = B.box_test(B.point(cb), lx, ly, ix0, iy0, far);
      uint64_t rej = __builtin_amdgcn_ballot_w64(cb + B.lane < B.n_used && !clean && !far);
      while (rej != 0) {  // uniform
        int32_t v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool have = rej != 0;
          const int l = have ? (int)__builtin_ctzll(rej) : 0;  // uniform: one beam for the whole wave
          rej &= rej - 1;
          const double bx = dev::bcast_lane(lx, l);
          const double by = dev::bcast_lane(ly, l);
          const int gy = (int)((by + yk) + 0.5);
          const bool iny = have && (unsigned)gy < (unsigned)B.sy;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int gx = (int)((bx + xj[t]) + 0.5);
            const bool in = iny && (unsigned)gx < (unsigned)B.sx && 4 * q + t < NS;
            v[u][t] = gi[in ? (int64_t)gy * L.pitch + gx : zero_cell];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[t] += v[u][t];
      }
    }
  }
}

// Scores of the lane's candidates (j = 4q .. 4q+3, row k) from their integer
// sums: written out, or reduced to the wave's best.
template <int NS, bool BEST>
__device__ __forceinline__ void box_epilogue(const LevelWork& L, const ScanWork& S, const AngleEntry& ae, int win,
                                             int a, bool act, int k, int q, int ox, int oy, int nsf,
                                             const int64_t (&acc)[4], double* __restrict__ out,
                                             BestPartial* __restrict__ partials, const AngleEntry* angles,
                                             char* ldsA, char* ldsB) {
  const double f = L.step_cells;
  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
  double lmax = -INFINITY;  // the fused finish (csm_tail.hpp): this lane's max, any NaN
  bool lnan = false;
  const double yk = S.y0 + (oy + k) * f;  // :572
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int j = 4 * q + t;
    if (act && j < NS) {
      const double accd = (double)(acc[t] + (int64_t)S.n_used * L.outside_i) * L.int_scale;
      const double xj = S.x0 + (ox + j) * f;  // :569
      const double score = dev::penalized(L, S, accd, xj, yk, ae.angle);
      const int64_t flat = ((int64_t)a * nsf + ox + j) * nsf + oy + k;
      if (BEST) {
        if (dev::better(score, flat, bs, bf)) {
          bs = score;
          bf = flat;
        }
      } else {
        tail::store_score(L, out + S.out_off + flat, score);
        lnan |= score != score;
        lmax = (score > lmax) ? score : lmax;
      }
    }
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
    if (threadIdx.x == 0) partials[(int64_t)win * L.blocks_per_scan + a] = BestPartial{bs, bf};
  } else if (L.tail.on) {
    tail::finish(L, S, angles, out, a, lmax, lnan, ldsA, ldsB);
  }
}

template <int NS, int D, bool BEST>
__global__ __launch_bounds__(64) void score_box_kernel(LevelWork L, const ScanWork* __restrict__ scans,
                                                       const double2* __restrict__ pts,
                                                       const AngleEntry* __restrict__ angles,
                                                       double* __restrict__ out,
                                                       BestPartial* __restrict__ partials) {
  constexpr int NQ = (NS + 3) / 4;  // 16-byte pieces per box row
  static_assert(NS * NQ <= 64, "one box row piece per lane");
  static_assert(64 % D == 0 && 32 % D == 0, "loads in flight divide the fold block");
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  dev::clear_word(L);
  const int wt = bid / L.n_angles;  // window (untiled) or (window, tile)
  const int a = bid - wt * L.n_angles;
  int win = wt, ox = 0, oy = 0, nsf = NS;
  if (L.tile_n > 0) {
    const int tpw = L.tile_n * L.tile_n;
    win = wt / tpw;
    const int t = wt - win * tpw;
    const int ti = t / L.tile_n;
    nsf = L.tile_ns;
    ox = min(ti * NS, nsf - NS);
    oy = min((t - ti * L.tile_n) * NS, nsf - NS);
  }
  const ScanWork S = scans[win];
  const AngleEntry ae = angles[S.angle_off + a];
  const int lane = threadIdx.x;
  const bool act = lane < NS * NQ;
  // idle lanes repeat row 0's addresses (no extra cache lines)
  const int k = act ? lane / NQ : 0;
  const int q = act ? lane - k * NQ : lane % NQ;
  const int pitch4 = L.pitch * 4;
  const BoxWave B{S, ae, pts + S.pts_off, S.step, S.n_used, lane, L.size_x, L.size_y, pitch4,
                  L.size_y * pitch4 /* first of the zero rows */, S.x0 + ox * L.step_cells /* :569, j = ox */,
                  S.y0 + oy * L.step_cells /* :572, k = oy */, 2, 0, 0, NS};
  const int n_used = S.n_used;
  const int zero_off = B.zero_off;
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(L.gridi_stride * 4), 0x00020000);
  const int voff = k * pitch4 + 16 * q;

  auto load = [&](int soff) { return __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0); };
  int64_t acc[4] = {0, 0, 0, 0};
  uint64_t slow = 0;
  v4i buf[D];
  // Run list: a run is one load whose values are added count times. Lists
  // are built per segment of kRunSeg beams (list, padding, then one scratch
  // slot per lane for the branch-free list writes).
  constexpr int kScratch = kRunSeg + 64 + 2 * D;
  __shared__ __attribute__((aligned(16))) int32_t run_off[kScratch + 64];
  __shared__ __attribute__((aligned(16))) int32_t run_cnt[kScratch + 64];
  static_assert(sizeof(run_off) >= tail::kBytesA && sizeof(run_cnt) >= tail::kBytesB, "the fused finish's LDS");
  for (int s0 = 0; s0 < n_used; s0 += kRunSeg) {
    const int s1 = min(n_used, s0 + kRunSeg);
    const int nruns = B.build_runs(s0, s1, run_off, run_cnt, kScratch, slow);
    // whole groups of D, then empty runs (zero block, count 0) far enough
    // past the list for the issue-ahead window below
    const int npad = (nruns + D - 1) / D * D;
    for (int i = nruns + lane; i < npad + 64 + D; i += 64) {
      run_off[i] = zero_off;
      run_cnt[i] = 0;
    }
    __syncthreads();
    if (npad == 0) continue;
    // lane i of cA: count of run rb + i; of wI: corner of run rb + D + i
    // (loads are issued exactly D runs ahead of their use)
    int rb = 0;
    int cA = run_cnt[lane];
    int wI = run_off[D + lane];
#pragma unroll
    for (int j = 0; j < D; ++j) buf[j] = load(run_off[j]);
    for (int r0 = 0; r0 < npad; r0 += D) {
      int so[D], cn[D];
#pragma unroll
      for (int j = 0; j < D; ++j) {
        cn[j] = __builtin_amdgcn_readlane(cA, r0 + j - rb);
        so[j] = __builtin_amdgcn_readlane(wI, r0 + j - rb);
      }
#pragma unroll
      for (int j = 0; j < D; ++j) {
        v4i v = buf[j];
        asm volatile("" : "+v"(v));  // consume run r0+j here, in order
        acc[0] += (int64_t)cn[j] * v.x;
        acc[1] += (int64_t)cn[j] * v.y;
        acc[2] += (int64_t)cn[j] * v.z;
        acc[3] += (int64_t)cn[j] * v.w;
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
        buf[j] = load(so[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (((r0 + D) & 63) == 0) {  // slide the register windows by 64 runs
        rb += 64;
        cA = run_cnt[rb + lane];
        wI = run_off[rb + D + lane];
      }
    }
    __syncthreads();  // the next segment rewrites the list
  }
  slow_beams<NS>(B, L, gi, slow, k, q, ox, oy, acc);
  box_epilogue<NS, BEST>(L, S, ae, wt, a, act, k, q, ox, oy, nsf, acc, out, partials, angles,
                         reinterpret_cast<char*>(run_off), reinterpret_cast<char*>(run_cnt));
}

// CSM_BOX_TRACE builds: s_memtime stamps of the pair kernel's phases for a
// sample of waves (every 61st block), read by tools/box_trace.py through
// csm_debug_box_trace: [0] entry, [1] first list build starts, [2] build,
// [3] sort, [4] accumulate (cycles summed over segments), [5] the sums'
// transpose done, [6] the cell-by-cell pass done, [7] exit, [8] runs, [9]
// pairs (padded), [10] beams, [11] XCC/SE/CU id (HW_ID).
#ifdef CSM_BOX_TRACE
constexpr int kBoxTraceWaves = 4096;
__device__ unsigned long long g_box_trace[kBoxTraceWaves][12];
__device__ int g_box_trace_n;
#define BOX_STAMP() ((unsigned long long)__builtin_amdgcn_s_memtime())
#endif

// v11 "pair" box kernel (n_space <= 13, palettes of at most kPairMaxPal
// values, r04). It reads the box through the grid's palette: a scan-match grid
// holds few distinct values (unknown, occupied and the blur kernel's levels),
// so every cell is a byte, the index of its value in the palette (L.pal_vals,
// 0 = the outside value), and a run's count times the value is an exact fp64
// FMA (every product and partial sum an integer below 2^53). Two changes to
// the r04 one-run-per-row palette form (v10, retired in r05), one per bound it
// hit (TA 0.66, VALU 0.70 of the kernel's cycles, profiles/r04):
//  - the box rows come from the strip copies of the index grid: a run's 13
//    rows are 208 contiguous bytes of one strip (2.5 cache lines per run, not
//    14 row-major), so the texture-address unit tags a fifth of the lines;
//  - runs of equal count go in pairs (the segment's run list is counting-
//    sorted by count): with indices below 16, one v_lshl_or per 4 cells makes
//    the pair's code a | b << s, and a 256-entry table of V[a] + V[b] turns
//    one lookup and one FMA into two runs' worth. The sums stay exact: every
//    product and partial sum is an integer below 2^53 (|V| < 2^26, counts <=
//    64, 1081 beams), so they equal the int64 sums of the other kernels.
// An odd bin's last run pairs with the zero run (offset zero_off, index 0).
constexpr int kPairPD = 2;  // pairs of one slot per step
#ifndef CSM_PAIR_SEG
#define CSM_PAIR_SEG 576
#endif
constexpr int kPairSeg = CSM_PAIR_SEG;
static_assert(kPairSeg % 64 == 0 && (kPairSeg + 128) * 4 >= 16 * 16 * 8,
              "whole 64-beam chunks; the sums' transpose (16 x 16 int64) reuses the run list");

// waves per SIMD the pair kernel's register allocation aims for
// (__launch_bounds__'s second argument on AMD: minimum waves per execution unit);
// 0: the compiler's choice (114 VGPRs). r05 A/B at B = 1081: 4 waves (98
// VGPRs) made the kernel 0.632 -> 0.734 ms, seg 448 with 5 waves 0.687 ms
// (profiles/r05/experiments/ab_pair_waves.txt)
#ifndef CSM_PAIR_WAVES
#define CSM_PAIR_WAVES 0
#endif
#if CSM_PAIR_WAVES > 0
#define CSM_PAIR_BOUNDS __launch_bounds__(64, CSM_PAIR_WAVES)
#else
#define CSM_PAIR_BOUNDS __launch_bounds__(64)
#endif
// 8 x byte B of w (a pair code's byte offset in the 8-byte pair table): one
// SDWA shift for every byte (the compiler folds byte 0 into the code's OR with
// a mask and a separate shift, and the OR itself then into two instructions)
template <int B>
__device__ __forceinline__ uint32_t byte_x8(uint32_t w) {
  static_assert(B >= 0 && B < 4, "a byte of a dword");
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
        : "=v"(r) : "v"(w));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
        : "=v"(r) : "v"(w));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
        : "=v"(r) : "v"(w));
  else
    asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
        : "=v"(r) : "v"(w));
  return r;
}

// The run-free form (NORUN) for short scans: at the reference's default beam
// rule (every 10th beam, B = 109) neighbouring beams rarely share a box corner
// (104 runs for 108 beams, profiles/r06/experiments/box_trace_b109.txt), so
// the run list and its counting sort (17 % of a wave there) buy nothing.
// NORUN pairs consecutive beams, each with count 1: pair p is beams 2p and
// 2p + 1 of the segment, in beam order. The sums are the same exact integers.
constexpr int kPairNoRunBeams = 128;

template <int NS, bool BEST, bool NORUN = false>
__global__ CSM_PAIR_BOUNDS void score_box_pair_kernel(LevelWork L, const ScanWork* __restrict__ scans,
                                                            const double2* __restrict__ pts,
                                                            const AngleEntry* __restrict__ angles,
                                                            double* __restrict__ out,
                                                            BestPartial* __restrict__ partials) {
  static_assert(NS >= 1 && NS <= kPalMaxSpace, "corner phase (<= 3) + NS cells within one 16-byte row piece");
  static_assert(kPairPD == 2, "a slot's step: one ds_read_b128 of pair offsets, one u16 of counts");
#ifdef CSM_BOX_TRACE
  unsigned long long tr[12] = {BOX_STAMP(), 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tq = 0;
#endif
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  dev::clear_word(L);
  const int win = bid / L.n_angles;
  const int a = bid - win * L.n_angles;
  const ScanWork S = scans[win];
  const AngleEntry ae = angles[S.angle_off + a];
  const int lane = threadIdx.x;
  const int k = lane & 15, slot = lane >> 4;
  const int zero_off = (kStripPadLo + L.size_y) * 16;  // copy 0, strip 0, first zero row
  BoxWave B{S, ae, pts + S.pts_off, S.step, S.n_used, lane, L.size_x, L.size_y, 0, zero_off, S.x0 /* :569 */,
            S.y0 /* :572 */, 0, L.strip_bytes, L.strip_copy_bytes, NS, kStripPadLo};
  const int n_used = S.n_used;
  // pair table: tab[a | b << sh] = V[a] + V[b]
  const int sh = L.pal_n <= 8 ? 3 : 4;
  __shared__ double tab[256];
  for (int i = lane; i < 256; i += 64) {
    const int ia = i & ((1 << sh) - 1), ib = i >> sh;
    tab[i] = (ia < L.pal_n && ib < L.pal_n) ? (double)L.pal_vals[ia] + (double)L.pal_vals[ib] : 0.0;
  }
  const uint8_t* pg = L.pal_strips + (int64_t)S.grid_index * L.strip_grid_bytes;
  const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)pg);
  const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)pg >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)phi << 32) | plo), (short)0, (int)L.strip_grid_bytes, 0x00020000);
  // rows past the box read the last row again (no new lines); their lanes'
  // sums are never read (the exchange below takes rows k < NS only)
  const int krow = min(k, NS - 1) * 16;
  // a box row piece's offset: 16-byte aligned when every row sits at byte 0
  // of its strip row (kStripShift 1), its low bits the byte phase otherwise
  constexpr int kPieceMask = kStripShift == 1 ? ~0 : ~15;

  double acc[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) acc[j] = 0.0;
  uint64_t slow = 0;
  constexpr int kStepPairs = 4 * kPairPD;  // pairs per step: slot s takes pairs [g + 2s, g + 2s + 2)
  constexpr int kScratch = kPairSeg + 64;
  constexpr int kPairSlots = kPairSeg + 64 + 4 * kStepPairs;  // pair members incl. odd-bin partners + padding
  __shared__ __attribute__((aligned(16))) int32_t run_off[kScratch + 64];
  __shared__ uint8_t run_cnt[kScratch + 64];
  __shared__ __attribute__((aligned(16))) int32_t pair_off[kPairSlots];  // pair p: members 2p, 2p + 1
  __shared__ __attribute__((aligned(16))) uint8_t pair_cnt[kPairSlots / 2];
  __shared__ int32_t bin[64];  // counting sort by run count (1..64)
  static_assert(sizeof(run_off) >= tail::kBytesA && sizeof(pair_off) >= tail::kBytesB, "the fused finish's LDS");
  for (int s0 = 0; s0 < n_used; s0 += kPairSeg) {
#ifdef CSM_BOX_TRACE
    tq = BOX_STAMP();
    if (s0 == 0) tr[1] = tq;
#endif
    int npad;
    if constexpr (NORUN) {
      // beam i of the segment's box offset at pair_off[i]; past the segment,
      // through the look-ahead step's pairs, the zero run
      const int s1 = min(n_used, s0 + kPairSeg);
      npad = ((s1 - s0 + 1) / 2 + kStepPairs - 1) / kStepPairs * kStepPairs;
      const int s_end = s0 + 2 * (npad + kStepPairs);
      for (int cb = s0; cb < s_end; cb += 128) {
        const double2 p0 = B.point(cb), p1 = B.point(cb + 64);
        const int o0 = B.offsets<true>(p0, cb, slow);
        const int o1 = B.offsets<true>(p1, cb + 64, slow);
        pair_off[cb - s0 + lane] = cb + lane < s1 ? o0 : zero_off;
        if (cb + 64 < s_end) pair_off[cb + 64 - s0 + lane] = cb + 64 + lane < s1 ? o1 : zero_off;
      }
      __syncthreads();
#ifdef CSM_BOX_TRACE
      tr[2] += BOX_STAMP() - tq;
      tq = BOX_STAMP();
      tr[8] += s1 - s0;
      tr[9] += npad;
#endif
    } else {
    const int nruns = B.build_runs<CSM_PAIR_PF, uint8_t, true, CSM_PAIR_ILP != 0>(
        s0, min(n_used, s0 + kPairSeg), run_off, run_cnt, kScratch, slow);
    bin[lane] = 0;
    __syncthreads();
#ifdef CSM_BOX_TRACE
    tr[2] += BOX_STAMP() - tq;
    tq = BOX_STAMP();
    tr[8] += nruns;
#endif
    for (int i = lane; i < nruns; i += 64) atomicAdd(&bin[run_cnt[i] - 1], 1);
    __syncthreads();
    // bin b: ceil(h / 2) pairs from slot 2 * (pairs of the bins below)
    const int h = bin[lane];
    const int pb = (h + 1) >> 1;
    int incl = pb;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const int npairs = __shfl(incl, 63, 64);
    const int base = 2 * (incl - pb);
    bin[lane] = base;
    if (h & 1) pair_off[base + h] = zero_off;  // the odd bin's last run pairs with the zero run
    // whole steps, then one step of empty pairs (zero runs, count 0) that the
    // look-ahead reads of the last step take
    npad = (npairs + kStepPairs - 1) / kStepPairs * kStepPairs;
    for (int p = npairs + lane; p < npad + kStepPairs; p += 64) {
      pair_off[2 * p] = zero_off;
      pair_off[2 * p + 1] = zero_off;
      pair_cnt[p] = 0;
    }
    __syncthreads();
    for (int i = lane; i < nruns; i += 64) {
      const int c = run_cnt[i];
      const int s = atomicAdd(&bin[c - 1], 1);
      pair_off[s] = run_off[i];
      if ((s & 1) == 0) pair_cnt[s >> 1] = (uint8_t)c;
    }
    __syncthreads();
#ifdef CSM_BOX_TRACE
    tr[3] += BOX_STAMP() - tq;
    tq = BOX_STAMP();
    tr[9] += npad;
#endif
    }
#if defined(CSM_PAL_DIAG) && CSM_PAL_DIAG >= 1  // timing diagnostic (wrong scores): the run lists only
    if (false) {
#else
    if (npad > 0) {
#endif
      int4 offs = *reinterpret_cast<const int4*>(&pair_off[4 * slot]);  // (A0, B0, A1, B1)
      uint32_t cnts = NORUN ? 0x0101u : (uint32_t)*reinterpret_cast<const uint16_t*>(&pair_cnt[2 * slot]);
      v4i dA[kPairPD], dB[kPairPD];
      dA[0] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (offs.x & kPieceMask), 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // issued in the order the loop consumes them
      dB[0] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (offs.y & kPieceMask), 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      dA[1] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (offs.z & kPieceMask), 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      dB[1] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (offs.w & kPieceMask), 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      for (int g = 0; g < npad; g += kStepPairs) {
        // the next step's pairs of this slot (the padding covers the last step's)
        const int4 noffs = *reinterpret_cast<const int4*>(&pair_off[2 * (g + kStepPairs) + 4 * slot]);
        const uint32_t ncnts =
            NORUN ? 0x0101u : (uint32_t)*reinterpret_cast<const uint16_t*>(&pair_cnt[g + kStepPairs + 2 * slot]);
        const int curA[2] = {offs.x, offs.z}, curB[2] = {offs.y, offs.w};
        const int nxtA[2] = {noffs.x, noffs.z}, nxtB[2] = {noffs.y, noffs.w};
#pragma unroll
        for (int p = 0; p < kPairPD; ++p) {
          // the pair's two rows, each shifted by its corner's byte phase, then
          // merged into codes a | b << sh (indices < 16: no carry between bytes)
          const v4i xa = dA[p], xb = dB[p];
          uint32_t w[4];
          if constexpr (kStripShift == 1) {  // every row at byte 0 of its strip row
            w[0] = (uint32_t)xa.x | ((uint32_t)xb.x << sh);
            w[1] = (uint32_t)xa.y | ((uint32_t)xb.y << sh);
            w[2] = (uint32_t)xa.z | ((uint32_t)xb.z << sh);
            w[3] = (uint32_t)xa.w | ((uint32_t)xb.w << sh);
          } else {
            const uint32_t sa = (uint32_t)curA[p] & 3u, sb = (uint32_t)curB[p] & 3u;
            w[0] = __builtin_amdgcn_alignbyte((uint32_t)xa.y, (uint32_t)xa.x, sa) |
                   (__builtin_amdgcn_alignbyte((uint32_t)xb.y, (uint32_t)xb.x, sb) << sh);
            w[1] = __builtin_amdgcn_alignbyte((uint32_t)xa.z, (uint32_t)xa.y, sa) |
                   (__builtin_amdgcn_alignbyte((uint32_t)xb.z, (uint32_t)xb.y, sb) << sh);
            w[2] = __builtin_amdgcn_alignbyte((uint32_t)xa.w, (uint32_t)xa.z, sa) |
                   (__builtin_amdgcn_alignbyte((uint32_t)xb.w, (uint32_t)xb.z, sb) << sh);
            w[3] = __builtin_amdgcn_alignbyte(0u, (uint32_t)xa.w, sa) |
                   (__builtin_amdgcn_alignbyte(0u, (uint32_t)xb.w, sb) << sh);
          }
          const double c = (double)((cnts >> (8 * p)) & 0xFFu);
          dA[p] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (nxtA[p] & kPieceMask), 0, 0);
          dB[p] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, krow + (nxtB[p] & kPieceMask), 0, 0);
          const char* tb = reinterpret_cast<const char*>(tab);
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            const uint32_t wj = w[j >> 2];
            const uint32_t o = (j & 3) == 0 ? byte_x8<0>(wj) : (j & 3) == 1 ? byte_x8<1>(wj)
                             : (j & 3) == 2 ? byte_x8<2>(wj) : byte_x8<3>(wj);
            acc[j] = __builtin_fma(c, *reinterpret_cast<const double*>(tb + o), acc[j]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        offs = noffs;
        cnts = ncnts;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the look-ahead loads past the list land
    }
    __syncthreads();  // the next segment rewrites the lists
#ifdef CSM_BOX_TRACE
    tr[4] += BOX_STAMP() - tq;
#endif
  }
  // the four run slots of row k meet, then the sums go to the (row, piece)
  // layout of the v6 epilogue through LDS (the run list's space)
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    acc[j] += __shfl_xor(acc[j], 16, 64);
    acc[j] += __shfl_xor(acc[j], 32, 64);
  }
  int64_t* xch = reinterpret_cast<int64_t*>(run_off);
  if (slot == 0 && k < NS) {
#pragma unroll
    for (int j = 0; j < NS; ++j) xch[k * 16 + j] = (int64_t)acc[j];
  }
  __syncthreads();
  const int kk = lane >> 2, q = lane & 3;
  int64_t mine[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) mine[t] = (kk < NS && 4 * q + t < NS) ? xch[kk * 16 + 4 * q + t] : 0;
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
#ifdef CSM_BOX_TRACE
  tr[5] = BOX_STAMP();
#endif
  slow_beams<NS>(B, L, gi, slow, kk, q, 0, 0, mine);
#ifdef CSM_BOX_TRACE
  tr[6] = BOX_STAMP();
#endif
  box_epilogue<NS, BEST>(L, S, ae, win, a, kk < NS, kk, q, 0, 0, NS, mine, out, partials, angles,
                         reinterpret_cast<char*>(run_off), reinterpret_cast<char*>(pair_off));
#ifdef CSM_BOX_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tr[7] = BOX_STAMP();
#ifdef CSM_BOX_TRACE_XCD  // per-XCD balance (tools/box_trace.py --xcd): the dispatch slot and the exit wall clock
  tr[10] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
  tr[11] = (unsigned long long)blockIdx.x;
#else
  tr[10] = (unsigned long long)n_used;
  tr[11] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
#endif
  if (bid % 61 == 0 && lane == 0) {
    const int i = atomicAdd(&g_box_trace_n, 1);
    if (i < kBoxTraceWaves)
      for (int j = 0; j < 12; ++j) g_box_trace[i][j] = tr[j];
  }
#endif
}

template <int NS>
hipError_t launch_pair(const LevelWork& L, const ScanWork* s, const double2* p, const AngleEntry* an, double* out,
                       BestPartial* part, unsigned nblk, hipStream_t stream) {
  const bool norun = L.max_n_used > 0 && L.max_n_used <= kPairNoRunBeams;
  if (part && norun)
    hipLaunchKernelGGL((score_box_pair_kernel<NS, true, true>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  else if (part)
    hipLaunchKernelGGL((score_box_pair_kernel<NS, true>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  else if (norun)
    hipLaunchKernelGGL((score_box_pair_kernel<NS, false, true>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out,
                       part);
  else
    hipLaunchKernelGGL((score_box_pair_kernel<NS, false>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  return hipGetLastError();
}

template <int NS>
hipError_t launch_ns(const LevelWork& L, const ScanWork* s, const double2* p, const AngleEntry* an, double* out,
                     BestPartial* part, unsigned nblk, hipStream_t stream) {
  if (part)
    hipLaunchKernelGGL((score_box_kernel<NS, kD, true>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  else
    hipLaunchKernelGGL((score_box_kernel<NS, kD, false>), dim3(nblk), dim3(64), 0, stream, L, s, p, an, out, part);
  return hipGetLastError();
}

}  // namespace

bool box_supported(int ns) { return ns >= 9 && ns <= 16; }
bool box_pair_supported(int ns) { return ns >= 9 && ns <= kPalMaxSpace; }

hipError_t launch_score_box_pair(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                                 const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                                 hipStream_t stream) {
  const int64_t nblk = (int64_t)L.n_scans * L.n_angles;
  const StripGeom G = strip_geom(L.size_x, L.size_y);
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || L.step_cells != 1.0 || L.blocks_per_scan != L.n_angles ||
      L.tile_n > 0 || L.pal_n < 1 || L.pal_n > kPairMaxPal || !L.pal_strips || !L.pal_vals ||
      L.strip_bytes != G.strip_bytes || L.strip_copy_bytes != G.copy_bytes || L.strip_grid_bytes != G.grid_bytes ||
      G.grid_bytes > INT32_MAX || (int64_t)L.size_y * 16 > INT32_MAX)
    return hipErrorInvalidValue;
  const double2* p = reinterpret_cast<const double2*>(d_pts);
  const unsigned n = (unsigned)nblk;
  switch (ns) {
    case 9: return launch_pair<9>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 10: return launch_pair<10>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 11: return launch_pair<11>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 12: return launch_pair<12>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 13: return launch_pair<13>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_score_box(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                            const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                            hipStream_t stream) {
  // tiled: n_scans windows of tile_ns, tile_n^2 tiles of ns each (best only)
  const int64_t tiles = L.tile_n > 0 ? (int64_t)L.tile_n * L.tile_n : 1;
  const int64_t nblk = (int64_t)L.n_scans * tiles * L.n_angles;
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || L.step_cells != 1.0 || L.blocks_per_scan != L.n_angles ||
      L.pitch < L.size_x + kGridiPadCols || L.pitch % 4 != 0)
    return hipErrorInvalidValue;
  if (L.tile_n > 0 && (!d_partials || ns != 16 || L.tile_ns < ns || (int64_t)(L.tile_n - 1) * ns >= L.tile_ns ||
                       (int64_t)L.tile_n * ns < L.tile_ns))
    return hipErrorInvalidValue;
  const double2* p = reinterpret_cast<const double2*>(d_pts);
  const unsigned n = (unsigned)nblk;
  switch (ns) {
    case 9: return launch_ns<9>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 10: return launch_ns<10>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 11: return launch_ns<11>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 12: return launch_ns<12>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 13: return launch_ns<13>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 14: return launch_ns<14>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 15: return launch_ns<15>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    case 16: return launch_ns<16>(L, d_scans, p, d_angles, d_out, d_partials, n, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace csm

#ifdef CSM_BOX_TRACE
// Trace readout for tools/box_trace.py: copies and resets the stamps.
extern "C" int csm_debug_box_trace(unsigned long long* out, int max_waves) {
  int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(csm::g_box_trace_n), sizeof(int)) != hipSuccess) return -1;
  n = n < csm::kBoxTraceWaves ? n : csm::kBoxTraceWaves;
  n = n < max_waves ? n : max_waves;
  if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::g_box_trace), (size_t)n * 12 * sizeof(unsigned long long)) !=
                   hipSuccess)
    return -1;
  const int zero = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(csm::g_box_trace_n), &zero, sizeof(int));
  return n;
}
#endif
