// csm_tail.hpp — the fast finish fused into the scoring launch (r05).
//
// The separate fast finish (finish_fast_kernel, csm_finish.hip) was one more
// dependent launch after every scoring launch of the 3-level driver: six per
// config-2 step, ~40 us each, most of it the launch's ramp and the latency of
// its one round of blocks. Here the scoring launch finishes each window
// itself. Every (window, angle) wave stores its scores write-through (sc1),
// then its angle's max, waits for the stores (vmcnt(0)) and counts in on its
// window's counter with one agent-scope atomic; the wave whose add returns
// n_angles - 1 finishes the window, reading the scores with sc1 loads: the
// hand-off form of MI355X_MICROARCH.md (inter-workgroup visibility, Valid
// forms row 1: every byte stored sc1 and drained before the counter, every
// load of them sc1, the last arriver told by its add's return value). Its
// decisions are the fast finish's (correlate_scan_matcher.h:607-611,670-710,
// 887-1003): no sort where no tie can change an output, otherwise the window
// goes to the exact pass (finish_kernel) exactly as before. One wave works a
// window: the candidates stream through registers in passes, the compacted
// sets sit in the scoring kernel's own LDS (its lists are dead by then).
#pragma once

#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

namespace csm {

constexpr int kSysWriteThrough = 17;  // buffer cache policy sc0 | sc1: system-coherent, written through L2

// One wave stores a window's FinishOut, assembled in LDS (src), to dst: the
// pieces `lists` selects and the seal (kind = writer | lists << 2, and the
// checksum of those pieces and the tag, csm_internal.hpp). Into host memory
// (A.host_flag) as write-through sc0 sc1 stores, nothing left dirty in the
// XCD's L2; plain stores otherwise (device memory, copied back after the launch).
__device__ __forceinline__ void emit_sealed(const FinishArgs& A, const FinishOut* src, FinishOut* dst, int lists,
                                            uint32_t writer, int lane) {
  static_assert(sizeof(FinishOut) == 560 && offsetof(FinishOut, pos_idx) == 64 &&
                    offsetof(FinishOut, ang_idx) == 144 && offsetof(FinishOut, pos_score) == 224 &&
                    offsetof(FinishOut, ang_score) == 384 &&
                    offsetof(FinishOut, seal_tag_kind) == 16 * kFinishSealPiece,
                "FinishOut pieces: header 0-3, pos_idx 4-8, ang_idx 9-13, pos_score 14-23, ang_score 24-33, seal 34");
  const int n_pieces = finish_n_pieces(lists);
  const uint64_t tk = (uint64_t)(uint32_t)A.flag_value | ((uint64_t)(writer | (uint32_t)lists << 2) << 32);
  const int pc = lane < n_pieces ? finish_piece(lane, lists) : kFinishSealPiece;
  int4 piece = lane < n_pieces ? reinterpret_cast<const int4*>(src)[pc] : make_int4(0, 0, 0, 0);
  uint64_t h = lane < n_pieces ? finish_piece_hash(pc, (uint32_t)piece.x, (uint32_t)piece.y, (uint32_t)piece.z,
                                                   (uint32_t)piece.w)
                               : 0ull;
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  h += finish_seal_share(tk);
  if (lane == n_pieces) piece = make_int4((int32_t)(uint32_t)tk, (int32_t)(uint32_t)(tk >> 32), (int32_t)(uint32_t)h,
                                          (int32_t)(uint32_t)(h >> 32));
  if (lane > n_pieces) return;
  if (A.host_flag) {
    const uint64_t base = (uint64_t)(uintptr_t)dst;
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)bhi << 32) | blo), (short)0, (int)sizeof(FinishOut), 0x00020000);
    typedef int32_t v4i_t __attribute__((ext_vector_type(4)));
    const v4i_t v = {piece.x, piece.y, piece.z, piece.w};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, pc * 16, 0, kSysWriteThrough);
  } else {
    reinterpret_cast<int4*>(dst)[pc] = piece;
  }
}

// The pending seal of a window the exact pass owes (kSealPending), written
// through to host memory; the host defers such a window to after the join.
__device__ __forceinline__ void store_pending_seal(const FinishArgs& A, FinishOut* dst) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, (int)sizeof(FinishOut), 0x00020000);
  const uint64_t tk = (uint64_t)(uint32_t)A.flag_value | ((uint64_t)kSealPending << 32);
  typedef int32_t v2i_t __attribute__((ext_vector_type(2)));
  const v2i_t v = {(int32_t)(uint32_t)tk, (int32_t)(uint32_t)(tk >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)offsetof(FinishOut, seal_tag_kind), 0, kSysWriteThrough);
}

namespace tail {

constexpr int kCap = 128;     // compacted candidates (the positional set, the near-best set); more: exact pass
constexpr int kAngles = 32;   // angle rows staged in LDS for FindBest's sums (more: read from memory)
constexpr int kLevels = 8;    // thresholds best - {0.01, 0.02, ..., 0.64}, then everything > bound
// The finisher's LDS, two 16-byte aligned regions of the scoring kernel:
// A: compacted keys (+4 padding) | their indices | ranked indices;
// B: ranked keys | FinishOut | angle cos | angle sin.
constexpr int kBytesA = (kCap + 4) * 8 + kCap * 4 + kCap * 4;
constexpr int kBytesB = kCap * 8 + (int)sizeof(FinishOut) + 2 * kAngles * 8;
static_assert(kBytesA % 16 == 0 && (kCap * 8) % 16 == 0 && sizeof(FinishOut) % 16 == 0, "16-byte pieces");

__device__ __forceinline__ double load_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A score's store: write-through (sc1) when the launch finishes its windows.
__device__ __forceinline__ void store_score(const LevelWork& L, double* p, double v) {
  if (L.tail.on)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(v, o, 64);
    v = (t > v) ? t : v;
  }
  return v;
}

// Append window w to the exact pass's list. Block 0 of the launch clears the
// header to {0, tag} as its first store, agent-scope (dev::clear_word); an
// append waits until that clear is visible (in practice it always is: block 0
// is dispatched first and a window finishes only after all of its waves), then
// takes a slot with one atomic add. (A compare-and-swap restart of the header
// per tag serialised ~250 appends of a super-fine launch: 1.4 ms at B = 109.)
// The wait is bounded (~2^20 sleeps, tens of ms): a clear that never arrives
// is a broken invariant and traps the launch (an error the host sees) instead
// of hanging it.
__device__ __forceinline__ void list_append(int32_t* list, int32_t tag, int32_t w) {
  for (int spins = 0; __hip_atomic_load(list + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag; ++spins) {
    if (spins == (1 << 20)) __builtin_trap();
    __builtin_amdgcn_s_sleep(2);
  }
  const int at = __hip_atomic_fetch_add(list, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  list[2 + at] = w;
}

// Every wave of a tail launch calls this after its scores are stored with
// store_score: lmax / lnan are this lane's max over its stored scores and
// whether any was NaN. ldsA / ldsB: kBytesA / kBytesB of the kernel's LDS,
// 16-byte aligned, free once its scores are computed.
__device__ __forceinline__ void finish(const LevelWork& L, const ScanWork& S, const AngleEntry* __restrict__ angles,
                                    const double* __restrict__ scores, int a, double lmax, bool lnan, char* ldsA,
                                    char* ldsB) {
  const int lane = threadIdx.x & 63;
  const TailArgs& T = L.tail;
  const FinishArgs& A = T.A;
  const int w = S.reserved;
  const int na = L.n_angles;
  // this angle's max (NaN: a NaN score)
  const double m = wave_max(lmax);
  const bool anan = __ballot(lnan) != 0;
  if (lane == 0)
    __hip_atomic_store(T.ang_max + (int64_t)w * na + a, anan ? __builtin_nan("") : m, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every score and the max stored (sc1, drained)
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(T.win_ctr + w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old != na - 1) return;  // not the window's last wave
  if (lane == 0) __hip_atomic_store(T.win_ctr + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  const int n = (int)A.n_cand;
  const int ns = A.n_space, nss = ns * ns;
  const double* sc = scores + S.out_off;
  double* ck = reinterpret_cast<double*>(ldsA);
  int* ci = reinterpret_cast<int*>(ldsA + (kCap + 4) * 8);
  int* si = ci + kCap;
  double* sk = reinterpret_cast<double*>(ldsB);
  FinishOut* so = reinterpret_cast<FinishOut*>(ldsB + kCap * 8);
  double* acs = reinterpret_cast<double*>(ldsB + kCap * 8 + sizeof(FinishOut));
  double* asn = acs + kAngles;
  const bool want_pos = !(A.skip_lists & 1), want_ang = !(A.skip_lists & 2);
  const int lists = (want_pos ? 1 : 0) | (want_ang ? 2 : 0);

  // 1. best = the front of the sorted candidates (:607): the angles' maxima
  double best = -INFINITY;
  bool bad = false;
  for (int t = lane; t < na; t += 64) {
    const double v = load_sc1(T.ang_max + (int64_t)w * na + t);
    bad |= (v != v);
    best = (v > best) ? v : best;
  }
  best = wave_max(best);
  bool flag = __ballot(bad) != 0 || n <= 0;
  const double lo = best - 0.1;
  const double bound = (0.5 < lo) ? 0.5 : lo;  // std::min(best - 0.1, 0.5) (:912,:986)
  // level k < 7: s > bound and s - best >= -0.01 * 2^k; level 7: s > bound
  auto level_of = [&](double s) {
    const double d = s - best;
    double dl = 0.01;
    int lv = 0;
#pragma unroll
    for (int k = 0; k < kLevels - 1; ++k, dl *= 2.0) lv += (d < -dl) ? 1 : 0;
    return (s > bound) ? lv : kLevels;
  };
  constexpr int U = 8;  // score loads in flight per lane
  // 2. one pass over the scores: level counts (16 bits a level per lane, two
  // 64-bit words) and, speculatively, the candidates of levels 0..kSpec
  // compacted (lanes in index order) -- the positional set is almost always
  // among them; the smallest level whose cumulative count reaches 20 (or all
  // > bound) is then known
  constexpr int kSpec = 3;
  int Lsel = 0, nC = 0, nS = 0;
  if (!flag) {
    uint64_t c0 = 0, c1 = 0;
    for (int base = 0; base < n; base += 64 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + 64 * u + lane;
        v[u] = i < n ? load_sc1(sc + i) : -INFINITY;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + 64 * u + lane;
        const int lv = level_of(v[u]);  // -INFINITY padding: no level
        const uint64_t one = 1ull << (16 * (lv & 3));
        c0 += lv < 4 ? one : 0ull;
        c1 += (lv >= 4 && lv < kLevels) ? one : 0ull;
        const bool in = lv <= kSpec;
        const uint64_t mm = __ballot(in);
        if (in) {
          const int p = nS + __popcll(mm & ((1ull << lane) - 1));
          if (p < kCap) {
            ck[p] = v[u];
            ci[p] = i;
          }
        }
        nS += __popcll(mm);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c0 += __shfl_xor(c0, o, 64);
      c1 += __shfl_xor(c1, o, 64);
    }
    int cnt[kLevels];
#pragma unroll
    for (int k = 0; k < kLevels; ++k) cnt[k] = (int)(((k < 4 ? c0 : c1) >> (16 * (k & 3))) & 0xFFFF);
    Lsel = want_pos ? kLevels - 1 : 0;
    int cum = 0;
    for (int k = 0; want_pos && k < kLevels; ++k) {
      cum += cnt[k];
      if (cum >= kCovPoints) {
        Lsel = k;
        break;
      }
    }
    for (int k = 0; k <= Lsel; ++k) nC += cnt[k];
    flag = nC > kCap;
  }
  // 3. the set, compacted, ranked by value: rank = elements greater; an
  // equal value where the order decides flags the window
  if (!flag) {
    if (Lsel <= kSpec && nS <= kCap) {  // from the speculative list: its levels <= Lsel, kept in order
      __syncthreads();
      int at = 0;
      for (int t0 = 0; t0 < nS; t0 += 64) {
        const int t = t0 + lane;
        const double x = t < nS ? ck[t] : -INFINITY;
        const int ix = t < nS ? ci[t] : 0;
        const bool in = t < nS && level_of(x) <= Lsel;
        const uint64_t mm = __ballot(in);
        __syncthreads();  // every lane has read its entry before the list is rewritten
        if (in) {
          const int p = at + __popcll(mm & ((1ull << lane) - 1));
          ck[p] = x;
          ci[p] = ix;
        }
        at += __popcll(mm);
        __syncthreads();
      }
    } else {  // a second pass
      int at = 0;
      for (int base = 0; base < n; base += 64 * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = base + 64 * u + lane;
          v[u] = i < n ? load_sc1(sc + i) : -INFINITY;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = base + 64 * u + lane;
          const bool in = level_of(v[u]) <= Lsel;  // padding never qualifies
          const uint64_t mm = __ballot(in);
          if (in) {
            const int p = at + __popcll(mm & ((1ull << lane) - 1));
            ck[p] = v[u];
            ci[p] = i;
          }
          at += __popcll(mm);
        }
      }
    }
    if (lane < 4) ck[nC + lane] = -INFINITY;  // the rank loop reads 4 at a time
    __syncthreads();
    bool tie = false;
    for (int t = lane; t < nC; t += 64) {
      const double x = ck[t];
      int r = 0, eq = 0;
      for (int j = 0; j < nC; j += 4) {
        const double2 u01 = *reinterpret_cast<const double2*>(&ck[j]);
        const double2 u23 = *reinterpret_cast<const double2*>(&ck[j + 2]);
        r += ((u01.x > x) ? 1 : 0) + ((u01.y > x) ? 1 : 0) + ((u23.x > x) ? 1 : 0) + ((u23.y > x) ? 1 : 0);
        eq += ((u01.x == x) ? 1 : 0) + ((u01.y == x) ? 1 : 0) + ((u23.x == x) ? 1 : 0) + ((u23.y == x) ? 1 : 0);
      }
      const double d = x - best;
      const bool inF = d < 0.0 ? d >= -1e-2 : d <= 1e-2;  // DoubleEqual(s, best, 1e-2)
      tie |= eq > 1 && (inF || (want_pos && r <= kCovPoints));
      sk[r] = x;  // distinct ranks whenever nothing is flagged
      si[r] = ci[t];
    }
    flag = __ballot(tie) != 0;
  }
  const double f = A.step_cells;
  auto cx = [&](int idx) { return S.x0 + ((idx / ns) % ns) * f; };
  auto cy = [&](int idx) { return S.y0 + (idx % ns) * f; };
  if (!flag) {
    for (int t = lane; t < na && t < kAngles; t += 64) {
      const AngleEntry ae = angles[S.angle_off + t];
      acs[t] = ae.cosine;
      asn[t] = ae.sine;
    }
    __syncthreads();
    // FindBestCandidate (:676-707), the same sequential sums as finish_kernel
    double bxl = 0.0, byl = 0.0;
    if (lane == 0) {
      double ax = 0.0, ay = 0.0, thx = 0.0, thy = 0.0, ssum = 0.0;
      int count = 0;
      for (int r = 0; r < nC; ++r) {
        const double s = sk[r];
        const double d = s - best;
        if (!(d < 0.0 ? d >= -1e-2 : d <= 1e-2)) break;
        const int idx = si[r];
        const int aa = idx / nss;
        const double ca = aa < kAngles ? acs[aa] : angles[S.angle_off + aa].cosine;
        const double sa = aa < kAngles ? asn[aa] : angles[S.angle_off + aa].sine;
        ax += cx(idx) * s;
        ay += cy(idx) * s;
        thx += ca * s;
        thy += sa * s;
        ssum += s;
        count++;
      }
      const int fi0 = si[0];
      so->front_idx = fi0;
      so->count = count;
      so->best_score = best;
      so->thx = thx;
      so->thy = thy;
      so->ssum = ssum;
      if (count > 1) {
        bxl = ax / ssum;
        byl = ay / ssum;
      } else {
        bxl = cx(fi0);
        byl = cy(fi0);
      }
      so->best_x = bxl;
      so->best_y = byl;
      so->n_pos = want_pos ? min(nC, kCovPoints) : 0;
    }
    const double bx = __shfl(bxl, 0, 64), by = __shfl(byl, 0, 64);
    // positional list (:915-928): the sorted prefix with score > bound, <= 20
    if (want_pos && lane < min(nC, kCovPoints)) {
      so->pos_idx[lane] = si[lane];
      so->pos_score[lane] = sk[lane];
    }
    // 4. angular list (:990-1003): near the best, score >= bound
    if (!want_ang) {
      if (lane == 0) so->n_ang = 0;
    } else {
      const double tol = A.lin_tol;
      // the candidates the test can pass: columns j with |x0 + j f - bx| <= tol
      // and rows likewise, one cell of margin each way (the test itself, the
      // reference's expressions, decides), over every angle
      auto span = [&](double c0, double bc, int& lo, int& hi) {
        const double l = std::floor((bc - fabs(tol) - c0) / f) - 1.0, h = std::ceil((bc + fabs(tol) - c0) / f) + 1.0;
        lo = l < 0.0 ? 0 : (l > ns - 1 ? ns : (int)l);
        hi = h < 0.0 ? -1 : (h > ns - 1 ? ns - 1 : (int)h);
      };
      int j0, j1, k0, k1;
      span(S.x0, bx, j0, j1);
      span(S.y0, by, k0, k1);
      const int nj = j1 >= j0 ? j1 - j0 + 1 : 0, nk = k1 >= k0 ? k1 - k0 + 1 : 0;
      const int per = nj * nk, total = per * na;
      int nN = 0;
      for (int t0 = 0; t0 < total; t0 += 64) {
        const int t = t0 + lane;
        int i = 0;
        double v = -INFINITY;
        if (t < total) {
          const int aa = t / per, r = t - aa * per, jj = r / nk;
          i = (aa * ns + j0 + jj) * ns + k0 + (r - jj * nk);
          v = load_sc1(sc + i);
        }
        bool in = false;
        if (v >= bound) {  // padding (-inf) never qualifies
          const double dx = cx(i) - bx, dy = cy(i) - by;
          const bool ex = dx < 0.0 ? dx >= -fabs(tol) : dx <= fabs(tol);
          const bool ey = dy < 0.0 ? dy >= -fabs(tol) : dy <= fabs(tol);
          in = ex && ey;
        }
        const uint64_t mm = __ballot(in);
        if (in) {
          const int p = nN + __popcll(mm & ((1ull << lane) - 1));
          if (p < kCap) {
            ck[p] = v;
            ci[p] = i;
          }
        }
        nN += __popcll(mm);
      }
      if (nN > kCap) {
        flag = true;
      } else {
        if (lane < 4) ck[nN + lane] = -INFINITY;
        __syncthreads();
        bool tie = false;
        for (int t = lane; t < nN; t += 64) {
          const double x = ck[t];
          int r = 0, eq = 0;
          for (int j = 0; j < nN; j += 4) {
            const double2 u01 = *reinterpret_cast<const double2*>(&ck[j]);
            const double2 u23 = *reinterpret_cast<const double2*>(&ck[j + 2]);
            r += ((u01.x > x) ? 1 : 0) + ((u01.y > x) ? 1 : 0) + ((u23.x > x) ? 1 : 0) + ((u23.y > x) ? 1 : 0);
            eq += ((u01.x == x) ? 1 : 0) + ((u01.y == x) ? 1 : 0) + ((u23.x == x) ? 1 : 0) + ((u23.y == x) ? 1 : 0);
          }
          tie |= eq > 1 && r <= kCovPoints;
          if (r < kCovPoints) {
            so->ang_idx[r] = ci[t];
            so->ang_score[r] = x;
          }
        }
        flag = __ballot(tie) != 0;
        if (lane == 0) so->n_ang = min(nN, kCovPoints);
      }
    }
  }
  if (!flag) {
    __syncthreads();  // the LDS FinishOut is complete
    emit_sealed(A, so, T.out + w, lists, kSealFast, lane);
    if (lane == 0) A.need_exact[w] = 0;
  } else if (lane == 0) {  // the exact pass takes this window
    A.need_exact[w] = 1;
    list_append(A.exact_list, A.flag_value, w);
    if (A.host_fast_flag) store_pending_seal(A, T.out + w);
  }
  // count in; the level-part's last window signals the host (DESIGN §7 "Host signals")
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    const int t = __hip_atomic_fetch_add(T.level_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == T.n_windows - 1) {
      __hip_atomic_store(T.level_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t head =
          __hip_atomic_load(reinterpret_cast<uint64_t*>(A.exact_list), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int cnt = (uint32_t)(head >> 32) == (uint32_t)A.flag_value ? (int)(uint32_t)head : 0;
      if (cnt == 0 && A.host_flag)  // nothing for the exact pass: it returns at once
        __hip_atomic_store(A.host_flag, A.flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (A.host_fast_flag)  // every window sealed or pending: the settled ones complete now
        __hip_atomic_store(A.host_fast_flag, A.flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace tail
}  // namespace csm
