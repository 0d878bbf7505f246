// csm_phase.hip — v7 "phase" scoring kernel: window levels whose step f is
// below one map cell (the fine level of every shipped parameter set on a
// 5 cm map: 11 steps of f = 0.4 cells).
//
// Candidate (j, k) of angle a reads, for beam b, cell
// (trunc((lx + x_j) + 0.5), trunc((ly + y_k) + 0.5)) with x_j = x0 + j*f
// (correlate_scan_matcher.h:569-572, :637-662). Write t = (lx + x0) + 0.5 =
// X + phase (X = floor(t)). The column of candidate j is then
// X + floor(phase + j*f): as the phase runs over [0, 1) the offsets change
// only at the breakpoints ceil(j*f) - j*f, so inside a bucket q between two
// breakpoints the columns are X + ox[q][j], fixed. A beam is thus a C x C box
// of cells (C = max ox + 1) at corner (X, Y) plus a bucket pair (qx, qy), and
// it adds box cell (ox[qy][k], ox[qx][j]) to candidate (j, k).
//
// So the kernel sums boxes per bucket pair — C*C cells per beam instead of
// NS*NS candidate reads — and expands the pair sums to candidates once, at
// the end. One wave per (window, angle):
//   1. classify every beam (rotation, phases, buckets, margin test), count it
//      into its pair, scatter its box corner into the pair's list in LDS
//      (lists padded to whole groups of SL beams);
//   2. walk the lists: lane (slot, box row, piece) gathers a 16-byte row
//      piece of its slot's beam box, one group of SL beams per wave
//      instruction, kD groups in flight; where a list entry ends the lanes'
//      int32 partials go into the pair's int64 box sums psum[pair][cell]
//      (LDS, kept over the whole scan: segments add into the same sums);
//   3. once per scan, candidate (j, k) = sum over pairs of
//      psum[pair][ox[qy][k]][ox[qx][j]].
// Sums are exact integers over the fixed-point grid (gridi), so their order
// is free (csm_set_grid). Rounding, as for the box kernel (csm_box.hip): the
// computed t_j is within 2^-27 of T + j*f (T = lx + x0 + 0.5, real), so a
// phase at least 2^-20 from every bucket edge gives trunc(t_j) =
// X + floor(phase + j*f) exactly. Beams that fail (a phase inside a margin,
// t < 0) are summed cell by cell with the reference's expressions.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_device.hpp"
#include "csm_tail.hpp"
#include "csm_internal.hpp"

namespace csm {
namespace {

#ifndef CSM_PHASE_SEG
#define CSM_PHASE_SEG 576  // r03: 576: 0.352 ms per fine launch, 768: 0.364, 384: 0.381, 1152: 0.415
#endif
constexpr int kSeg = CSM_PHASE_SEG;  // beams classified per segment (lists in LDS)
// groups per list entry: a lane's int32 partial sums one slot over at most
// kEntG groups, |value| < 2^26 each, before it goes into the pair's int64 sums
constexpr int kEntG = 31;
static_assert(kEntG * ((1LL << 26) - 1) < 2147483647LL, "a lane's int32 partial");
constexpr int kChunks = kSeg / 64;   // 64-beam chunks per segment, classified in registers
#ifndef CSM_PHASE_DEPTH
// r03 (int64 pair sums, list entries read a block ahead): 4: 0.352 ms per fine
// launch, 8: 0.357-0.359, 16: 0.396 (r02: 8: 0.418-0.423, 16: 0.426, 4: 0.424)
#define CSM_PHASE_DEPTH 4
#endif
constexpr int kD = CSM_PHASE_DEPTH;  // groups of loads in flight
static_assert(kD <= 32, "int32 partial sums fold every kD groups");
// gentry[lane & (kD - 1)] and the group-window slides index by masking
static_assert((kD & (kD - 1)) == 0, "CSM_PHASE_DEPTH must be a power of two");
static_assert(kSeg % 64 == 0, "CSM_PHASE_SEG must be whole 64-beam chunks");

typedef int32_t v4i __attribute__((ext_vector_type(4)));

// waves per SIMD the register allocation aims for (__launch_bounds__'s
// second argument on AMD: minimum waves per execution unit)
#ifndef CSM_PHASE_WAVES
#define CSM_PHASE_WAVES 4
#endif

// ST: the box rows come from the strip copies of gridi (L.istrips, r04): a
// beam's 5 rows are 160 contiguous bytes of one strip instead of 5 rows of the
// row-major grid, so a load instruction's lanes touch about half the 64-byte
// segments (the texture-address unit's cost per instruction follows them).
// KCH: 64-beam chunks classified per segment, all in flight at once. kChunks
// (a 576-beam segment) for full scans; 2 for short ones (levels of <= 128
// beams, kPhaseShortBeams: the reference's default every-10th-beam rule), which
// would otherwise load and classify seven dead chunks per wave.
constexpr int kPhaseShortBeams = 128;

template <int NS, int C, int NQ, bool BEST, bool ST, int KCH = kChunks>
__global__ __launch_bounds__(64, CSM_PHASE_WAVES) void score_phase_kernel(LevelWork L, PhaseTable T,
                                                         const ScanWork* __restrict__ scans,
                                                         const double2* __restrict__ pts,
                                                         const AngleEntry* __restrict__ angles,
                                                         double* __restrict__ out,
                                                         BestPartial* __restrict__ partials) {
  constexpr int NP = NQ * NQ;   // bucket pairs
  constexpr int NPC = (C + 3) / 4;  // 16-byte pieces per box row
  constexpr int LPS = C * NPC;  // lanes per slot: one row piece each
  constexpr int SL = 64 / LPS;  // beams (slots) per wave instruction
  constexpr int PC = C * C;     // int64 box sums per pair
  static_assert(LPS <= 64 && NP <= 64 && NS <= kPhaseMaxSpace && NQ <= kPhaseMaxBuckets, "layout");
  static_assert(2 * NP + 1 < 256, "group tags are bytes");
  // padded lists, whole kD blocks of groups and two blocks of issue-ahead slack
  constexpr int kList = 64 * KCH + NP * (SL - 1) + 3 * SL * kD + 64;  // a segment is 64 * KCH beams
  constexpr int kMaxGroups = kList / SL + 1;
  __shared__ int32_t list[kList];
  __shared__ int32_t cursor[NP];
  __shared__ int32_t ngroups_s;
  // group tag: 2 * pair + (entry within the pair & 1), so the tag changes
  // exactly where an entry ends; the groups past the lists carry 2 * NP
  // (pair NP: a dummy row of psum nobody reads)
  __shared__ uint8_t gtag[kMaxGroups];
  __shared__ __attribute__((aligned(16))) int64_t psum[(NP + 1) * PC];  // per pair, box cell (row, column): the whole scan's sums
  static_assert(sizeof(psum) >= tail::kBytesA + tail::kBytesB, "the fused finish's LDS (csm_tail.hpp)");
  __shared__ int8_t oxs[NQ][kPhaseMaxSpace];

  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  dev::clear_word(L);
  const int win = bid / L.n_angles;
  const int a = bid - win * L.n_angles;
  const ScanWork S = scans[win];
  const AngleEntry ae = angles[S.angle_off + a];
  const int lane = threadIdx.x;
  // lane (slot, box row cv, piece ch); lanes past SL slots repeat slot 0's
  // row 0 piece 0 (same cache lines) and never fold into accum
  const bool cact = lane < SL * LPS;
  const int slot = cact ? lane / LPS : 0;
  const int within = cact ? lane - slot * LPS : 0;
  const int cv = within / NPC;  // box row (y offset)
  const int ch = within - cv * NPC;
  const double f = L.step_cells;
  const double x_0 = S.x0 + 0 * f;  // :569 at j = 0
  const double y_0 = S.y0 + 0 * f;  // :572 at k = 0
  const int sx = L.size_x, sy = L.size_y;
  const int pitch4 = L.pitch * 4;
  constexpr int kRowB = kIStripCells * 4;   // strip row bytes
  static_assert(!ST || 4 * NPC <= kIStripCells + 4, "a box row's pieces stay within its strip row and the next");
  // the strip form counts columns and rows from -kIStripPadLo (t and the box
  // corner shifted by it: the padding holds what the reference's truncation
  // reads there)
  constexpr int kPad = ST ? kIStripPadLo : 0;
  const int zero_off = ST ? (kPad + sy) * kRowB : sy * pitch4;  // first of the zero rows (strip form: copy 0, strip 0)
  const double2* __restrict__ P = pts + S.pts_off;
  const int step = S.step;
  const int n_used = S.n_used;
  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const int32_t* gsrc = ST ? L.istrips + (int64_t)S.grid_index * (L.istrip_grid_bytes / 4) : gi;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gsrc);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gsrc >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, ST ? (int)L.istrip_grid_bytes : (int)(L.gridi_stride * 4),
      0x00020000);
  const int voff = ST ? cv * kRowB + ch * 16 : cv * pitch4 + ch * 16;

  for (int i = lane; i < NQ * kPhaseMaxSpace; i += 64) oxs[i / kPhaseMaxSpace][i % kPhaseMaxSpace] =
      T.ox[i / kPhaseMaxSpace][i % kPhaseMaxSpace];
  for (int i = lane; i < (NP + 1) * PC; i += 64) psum[i] = 0;

  auto bucket = [&](double ph, bool& ok) -> int {
    int q = 0;
    bool hit = false;
#pragma unroll
    for (int b = 0; b < NQ; ++b) {
      const bool in = b < T.nq && ph >= T.lo[b] && ph <= T.hi[b];
      q = in ? b : q;
      hit |= in;
    }
    ok = ok && hit;
    return q;
  };
  // Beam cb + lane (live below lim): its box offset and pair (pair < 0: it adds
  // nothing here — not live, box wholly past the grid's high edges, or rejected).
  auto classify = [&](const double2 p, int cb, int lim, double& lx, double& ly, bool& rejected) -> int2 {
    lx = ae.cosine * p.x - ae.sine * p.y;  // :179
    ly = ae.sine * p.x + ae.cosine * p.y;  // :180
    const double tx = (lx + x_0) + (0.5 + kPad);  // (a shift by kPad within 2^-28 cells)
    const double ty = (ly + y_0) + (0.5 + kPad);
    bool ok = tx >= 0.0 && ty >= 0.0;
    // v_fract_f64: tx - floor(tx), exact below 2^52; it differs (1 - 2^-53 for
    // 1.0) only for tiny negative t, which the t >= 0 test rejects either way
    const double fx = __builtin_amdgcn_fract(tx);
    const double fy = __builtin_amdgcn_fract(ty);
    int qx, qy;
    if (T.uniform) {  // equal-width buckets (PhaseTable::uniform)
      const double nqd = (double)T.nq;
      const double sx_ = fx * nqd, sy_ = fy * nqd;
      const double rx = __builtin_amdgcn_fract(sx_), ry = __builtin_amdgcn_fract(sy_);
      qx = (int)(sx_ - rx);
      qy = (int)(sy_ - ry);
      ok = ok && rx >= T.ulo && rx <= T.uhi && ry >= T.ulo && ry <= T.uhi && qx < T.nq && qy < T.nq;
    } else {
      qx = bucket(fx, ok);
      qy = bucket(fy, ok);
    }
    const bool live = cb + lane < lim;
    // far: every candidate's cell is off the grid's low side on one axis
    // (t_j = t + j*f <= -1 for all j, with the rounding margin): the beam adds
    // the outside value (zero in gridi) everywhere and skips the exact pass
    const double lim_far = kPad - 1.0 - (NS - 1) * f - 0x1p-20;
    const bool far = tx <= lim_far || ty <= lim_far;
    rejected = live && !ok && !far;
    const int ix0 = ok ? (int)tx : 0;
    const int iy0 = ok ? (int)ty : 0;
    const bool use = live && ok && ix0 < sx + kPad && iy0 < sy + kPad;
    int o;
    if (ST) {  // copy c = (ix0 / 4) mod 2 puts cells (ix0 & ~3) .. +7 in one strip row
      const int c = (ix0 >> 2) & 1;
      const int xs = (ix0 & ~3) + 4 * c;
      o = c * L.istrip_copy_bytes + (xs >> 3) * L.istrip_bytes + iy0 * kRowB + (ix0 & 3) * 4;
    } else {
      o = iy0 * pitch4 + ix0 * 4;
    }
    return make_int2(use ? o : 0, use ? qx * NQ + qy : -1);
  };
  auto point = [&](int b) { return P[(int64_t)min(b, n_used - 1) * step]; };

  // per lane: its candidates' box offsets in every bucket, 4 bits each
  constexpr int NC = NS * NS;
  constexpr int R = (NC + 63) / 64;
  __syncthreads();  // oxs, psum
  uint32_t oxj[R], oyk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = lane + 64 * r;
    const int j = t < NC ? t / NS : 0;
    const int k = t < NC ? t - j * NS : 0;
    oxj[r] = 0;
    oyk[r] = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      oxj[r] |= (uint32_t)oxs[q][j] << (4 * q);
      oyk[r] |= (uint32_t)oxs[q][k] << (4 * q);
    }
  }
  int64_t sum[R];
#pragma unroll
  for (int r = 0; r < R; ++r) sum[r] = 0;
  const int lane_cell = cv * C + 4 * ch;  // this lane's first box cell in a pair's sums

  uint64_t slow = 0;  // bit c: 64-beam chunk c holds a rejected beam (bit 63: some chunk >= 63)
  static_assert(KCH >= 1 && KCH <= kChunks, "segments of at most kSeg beams");
  for (int s0 = 0; s0 < n_used; s0 += 64 * KCH) {
    const int s1 = min(n_used, s0 + 64 * KCH);
    // 1a. every point of the segment in flight at once, then classify into
    // registers (offset, pair) and count per pair
    double2 pq[KCH];
#pragma unroll
    for (int u = 0; u < KCH; ++u) pq[u] = point(s0 + 64 * u + lane);
    if (lane < NP) cursor[lane] = 0;
    __syncthreads();
    int offr[KCH], pairr[KCH];
#pragma unroll
    for (int u = 0; u < KCH; ++u) {
      const int cb = s0 + 64 * u;
      double lx, ly;
      bool rej;
      const int2 c = classify(pq[u], cb, s1, lx, ly, rej);
      slow |= (uint64_t)(__builtin_amdgcn_ballot_w64(rej) != 0) << min(cb >> 6, 63);
      offr[u] = c.x;
      pairr[u] = c.y;
      if (c.y >= 0) atomicAdd(&cursor[c.y], 1);
    }
    __syncthreads();
    // 1b. lists: pair p gets whole groups of SL beams, its groups split into
    // entries of at most kEntG groups (a lane's partial fits int32)
    {
      const int cnt = lane < NP ? cursor[lane] : 0;
      const int g = (cnt + SL - 1) / SL;
      int gi_ = g;  // inclusive scan over lanes
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int tg = __shfl_up(gi_, o, 64);
        if (lane >= o) gi_ += tg;
      }
      const int g0p = gi_ - g;
      if (lane < NP) {
        cursor[lane] = g0p * SL;
        for (int k = 0; k < g; ++k) gtag[g0p + k] = (uint8_t)(2 * lane + ((k / kEntG) & 1));
      }
      if (lane == NP - 1) ngroups_s = gi_;
    }
    __syncthreads();
    const int ngroups = __builtin_amdgcn_readfirstlane(ngroups_s);
    // Whole blocks of kD groups and no branch in the unrolled loop below, so
    // the compiler keeps exactly kD loads in flight across iterations.
    // Padding entries, the groups past the lists and the issue-ahead slack
    // read the zero block; the groups past the lists go to the dummy pair.
    const int ng_pad = (ngroups + kD - 1) / kD * kD;
    for (int i = lane; i < (ng_pad + 2 * kD) * SL; i += 64) list[i] = zero_off;
    for (int i = ngroups + lane; i < ng_pad + kD; i += 64) gtag[i] = (uint8_t)(2 * NP);
    __syncthreads();
    // 1c. scatter box corners into their pair's list
#pragma unroll
    for (int u = 0; u < KCH; ++u)
      if (pairr[u] >= 0) list[atomicAdd(&cursor[pairr[u]], 1)] = offr[u];
    __syncthreads();
    // 2. gather: group g = list entries g*SL .. g*SL + SL - 1 (slot s takes
    // g*SL + s); one 16-byte row piece per lane (buffer_load_dwordx4: the TA
    // coalesces a slot's row into its cache lines, a dword gather costs an
    // access per lane). Where an entry ends (a uniform branch), the lanes add
    // their int32 partials into the pair's int64 box sums (ds_add_u64; the
    // cells past the box, columns >= C, are not kept).
    if (ngroups > 0) {
      v4i buf[kD];
#pragma unroll
      for (int j = 0; j < kD; ++j) {  // issued in order: the loop consumes buf[0] first
        buf[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, list[j * SL + slot] + voff, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      int32_t part[4] = {0, 0, 0, 0};
      int t_prev = __builtin_amdgcn_readfirstlane((int)gtag[0]);
      // (r04: adding slot pairs in registers first, half the lanes and half
      // the same-address atomics, took the isolated 4096-window launch from
      // 0.508 to 0.573 ms: the shuffles cost more than the conflicts)
      auto flush = [&](int tag) {  // uniform tag: pair tag >> 1
        int64_t* dst = psum + (tag >> 1) * PC + lane_cell;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (cact && 4 * ch + t < C)
            __hip_atomic_fetch_add(dst + t, (int64_t)part[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          part[t] = 0;
        }
      };
      int gev = gtag[lane & (kD - 1)];
      // the list entries (this lane's slot) whose loads a block issues are read
      // a block ahead, so no load waits on its address's LDS read
      int lcur[kD];
#pragma unroll
      for (int j = 0; j < kD; ++j) lcur[j] = list[(kD + j) * SL + slot];
      for (int g0 = 0; g0 < ng_pad; g0 += kD) {
        const int gev_next = gtag[g0 + kD + (lane & (kD - 1))];  // next block's tags
        int lnext[kD];
#pragma unroll
        for (int j = 0; j < kD; ++j) lnext[j] = list[(g0 + 2 * kD + j) * SL + slot];
#pragma unroll
        for (int j = 0; j < kD; ++j) {
          const int tj = __builtin_amdgcn_readlane(gev, j);
          if (tj != t_prev) flush(t_prev);  // uniform: only where an entry ends
          t_prev = tj;
          v4i v = buf[j];
          asm volatile("" : "+v"(v));  // consume group g0 + j here, in order
          part[0] += v.x;
          part[1] += v.y;
          part[2] += v.z;
          part[3] += v.w;
          buf[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lcur[j] + voff, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < kD; ++j) lcur[j] = lnext[j];
        gev = gev_next;
      }
      flush(t_prev);
    }
    __syncthreads();  // the next segment rewrites the lists
  }
  // 3. the pairs' box sums into the candidates: candidate (j, k) takes box
  // cell (ox[qy][k], ox[qx][j]) of pair (qx, qy), once for the whole scan
  for (int pr = 0; pr < NP; ++pr) {
    const int qx = pr / NQ, qy = pr - (pr / NQ) * NQ;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int u = (oxj[r] >> (4 * qx)) & 15;
      const int v = (oyk[r] >> (4 * qy)) & 15;
      sum[r] += psum[pr * PC + v * C + u];
    }
  }

  // rejected beams, cell by cell with the reference's expressions, four beams
  // at a time (their gathers issued together)
  for (uint64_t m = slow; m != 0; m &= m - 1) {
    const int c0 = (int)__builtin_ctzll(m);
    const int c_end = c0 == 63 ? (n_used + 63) / 64 : c0 + 1;
    for (int c = c0; c < c_end; ++c) {
      const int cb = c * 64;
      double lx, ly;
      bool rej;
      (void)classify(point(cb + lane), cb, n_used, lx, ly, rej);
      uint64_t rm = __builtin_amdgcn_ballot_w64(rej);
      while (rm != 0) {  // uniform
        int32_t v[4][R];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool have = rm != 0;
          const int l = have ? (int)__builtin_ctzll(rm) : 0;  // uniform: one beam for the whole wave
          rm &= rm - 1;
          const double bx = dev::bcast_lane(lx, l);
          const double by = dev::bcast_lane(ly, l);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int t = lane + 64 * r;
            const int j = t < NC ? t / NS : 0, k = t < NC ? t - (t / NS) * NS : 0;
            const int gx = (int)((bx + (S.x0 + j * f)) + 0.5);
            const int gy = (int)((by + (S.y0 + k * f)) + 0.5);
            const bool in = have && t < NC && (unsigned)gx < (unsigned)sx && (unsigned)gy < (unsigned)sy;
            v[u][r] = gi[in ? (int64_t)gy * L.pitch + gx : (int64_t)sy * L.pitch];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int r = 0; r < R; ++r) sum[r] += v[u][r];
      }
    }
  }

  double bs = -1.0e300;
  int64_t bf = INT64_MAX;
  double lmax = -INFINITY;  // the fused finish (csm_tail.hpp): this lane's max, any NaN
  bool lnan = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = lane + 64 * r;
    if (t < NC) {
      const int j = t / NS, k = t - (t / NS) * NS;
      const double accd = (double)(sum[r] + (int64_t)n_used * L.outside_i) * L.int_scale;
      const double xj = S.x0 + j * f;  // :569
      const double yk = S.y0 + k * f;  // :572
      const double score = dev::penalized(L, S, accd, xj, yk, ae.angle);
      const int64_t flat = ((int64_t)a * NS + j) * NS + k;
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
  if (!BEST && L.tail.on) {
    __syncthreads();  // psum's last reads are done: the finisher's LDS
    tail::finish(L, S, angles, out, a, lmax, lnan, reinterpret_cast<char*>(psum),
                 reinterpret_cast<char*>(psum) + tail::kBytesA);
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

template <int NS, int C, int NQ, bool ST, int KCH>
hipError_t launch_phase_k(const LevelWork& L, const PhaseTable& T, const ScanWork* s, const double2* p,
                          const AngleEntry* an, double* out, BestPartial* part, unsigned nblk, hipStream_t stream) {
  if (part)
    hipLaunchKernelGGL((score_phase_kernel<NS, C, NQ, true, ST, KCH>), dim3(nblk), dim3(64), 0, stream, L, T, s, p,
                       an, out, part);
  else
    hipLaunchKernelGGL((score_phase_kernel<NS, C, NQ, false, ST, KCH>), dim3(nblk), dim3(64), 0, stream, L, T, s, p,
                       an, out, part);
  return hipGetLastError();
}

template <int NS, int C, int NQ, bool ST>
hipError_t launch_phase(const LevelWork& L, const PhaseTable& T, const ScanWork* s, const double2* p,
                        const AngleEntry* an, double* out, BestPartial* part, unsigned nblk, hipStream_t stream) {
  if (L.max_n_used > 0 && L.max_n_used <= kPhaseShortBeams)
    return launch_phase_k<NS, C, NQ, ST, kPhaseShortBeams / 64>(L, T, s, p, an, out, part, nblk, stream);
  return launch_phase_k<NS, C, NQ, ST, kChunks>(L, T, s, p, an, out, part, nblk, stream);
}

}  // namespace

// Instantiated shape: the fine level of the shipped parameter sets on a 5 cm
// map (11 steps of 0.4 cells: 5 buckets, 5 x 5 boxes). Other sub-cell windows
// use the row-segment kernel.
bool phase_supported(int ns, int cells, int nq) { return ns == 11 && cells == 5 && nq == 5; }

hipError_t launch_score_phase(const LevelWork& L, const PhaseTable& T, const ScanWork* d_scans, const double* d_pts,
                              const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                              hipStream_t stream) {
  const int64_t nblk = (int64_t)L.n_scans * L.n_angles;
  if (nblk <= 0 || nblk > INT32_MAX || !L.int_mode || !(L.step_cells < 1.0) || L.blocks_per_scan != L.n_angles ||
      L.pitch < L.size_x + kGridiPadCols || L.pitch % 4 != 0 || !phase_supported(ns, T.cells, T.nq) ||
      T.cells > kGridiPadCols + 1)
    return hipErrorInvalidValue;
  for (int q = 0; q < T.nq; ++q)
    for (int j = 0; j < ns; ++j)
      if (T.ox[q][j] < 0 || T.ox[q][j] >= T.cells) return hipErrorInvalidValue;
  const double2* p = reinterpret_cast<const double2*>(d_pts);
  if (L.istrips) {
    const StripGeom G = istrip_geom(L.size_x, L.size_y);
    if (L.istrip_bytes != G.strip_bytes || L.istrip_copy_bytes != G.copy_bytes || L.istrip_grid_bytes != G.grid_bytes ||
        G.grid_bytes > INT32_MAX)
      return hipErrorInvalidValue;
    return launch_phase<11, 5, 5, true>(L, T, d_scans, p, d_angles, d_out, d_partials, (unsigned)nblk, stream);
  }
  return launch_phase<11, 5, 5, false>(L, T, d_scans, p, d_angles, d_out, d_partials, (unsigned)nblk, stream);
}

}  // namespace csm
