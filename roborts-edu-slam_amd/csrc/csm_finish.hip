// csm_finish.hip — device-side finish of a window: the reference's
// std::sort(candidates, greater) (correlate_scan_matcher.h:607) reproduced
// EXACTLY (same permutation, ties included), then the three ordered scans
// that consume the sorted candidates: FindBestCandidate's prefix
// (:670-710) and the candidate lists of ComputePositionalCovariance
// (:911-928) and ComputeAngularCovariance (:985-1003).
//
// Why an emulation and not a GPU sort: the winner among exactly tied scores,
// the averaged best pose and both covariances depend on the order std::sort
// leaves tied candidates in, and real grids tie constantly (sub-cell window
// steps land many candidates on the same cells). libstdc++'s std::sort is
// deterministic given the comparison outcomes:
//   introsort loop (threshold 16, depth limit 2*floor(log2 n)); pivot = median
//   of (first+1, mid, last-1) swapped to first; unguarded Hoare partition;
//   heap sort at depth 0; final insertion sort.
// Segments left by the loop are ordered relative to each other (left >= pivot
// >= right), so the final insertion sort equals an independent stable sort of
// each leaf segment, and segments can be processed in any order. The unguarded
// partition is computed in parallel: with l_k the k-th position (ascending)
// whose key is not > pivot and r_k the k-th position (descending) whose key is
// not < pivot, the sequential loop swaps exactly the pairs (l_k, r_k) with
// l_k < r_k and returns cut = min(l_{p+1}, r_p) for p such pairs.
// The formulation is validated against libstdc++ in tests/wave_sort_model.py.
//
// Layout: one 4-wave workgroup per window, segments in per-level LDS lists. A
// segment of more than 64 elements is partitioned by one wave in LDS; a segment of at most 64 is
// loaded into registers (lane = element) and finished there: its whole
// introsort recursion (ballot / bpermute partitions) and the stable sort of
// its leaves, then written back once.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>

#include "csm_device.hpp"
#include "csm_tail.hpp"
#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {

namespace {

// Waves per window of the exact path. Segments are handed out level by level
// with barriers in between (an earlier version pulled them from a spin-locked
// LDS stack and, rarely, spun past its iteration bound).
constexpr int kWaves = kFinishWaves;
// Partial sort (positions past what the ordered scans read stay unsorted) for
// windows of at least this many candidates; kNearRounds: tighten the second
// stage's limit to the 20th near-best score (20 block-wide rounds) instead of
// every element >= bound.
#ifndef CSM_PARTIAL_MIN
#define CSM_PARTIAL_MIN 256
#endif
#ifndef CSM_NEAR_ROUNDS
#define CSM_NEAR_ROUNDS 0
#endif
constexpr int kPartialMinCand = CSM_PARTIAL_MIN;
constexpr bool kNearRounds = CSM_NEAR_ROUNDS != 0;

struct Seg {
  int32_t first, last, depth;
};

// CSM_FINISH_TRACE builds: wall-clock stamps of the exact pass's phases for
// the first kTraceWindows windows that take it (tools/finish_trace.py).
#ifdef CSM_FINISH_TRACE
constexpr int kTraceWindows = 256;
__device__ unsigned long long g_trace[kTraceWindows][10];
__device__ int g_trace_n;
// per stage-1 level: [2 l] = wall clock at the level's start, [2 l + 1] =
// segments in it << 32 | the first segment's length (csm_debug_finish_levels)
constexpr int kTraceLevels = 16;
__device__ unsigned long long g_ltrace[kTraceWindows][2 * kTraceLevels];
#define CSM_STAMP(i)                                          \
  do {                                                        \
    if (threadIdx.x == 0 && tr >= 0) g_trace[tr][i] = wall_clock64(); \
  } while (0)
#else
#define CSM_STAMP(i) \
  do {               \
  } while (0)
#endif

struct WaveScratch {      // per-wave LDS scratch of the register sort
  uint8_t T[72], U[72];   // lane of the k-th right / left stop
  Seg st[40];             // sub-segment stack
};

static_assert(sizeof(WaveScratch) <= kFinishWaveScratch, "finish_layout wave scratch");

struct Shared {           // misc block of the LDS carve (finish_layout: kFinishMisc bytes)
  int plim, top, pending, pad;
  double bx, by;
  int ndef, cnt_a, cnt_b, nan;
  double red[kWaves];
  int wl[kWaves], wr[kWaves];  // partition_block: per-wave counts
  int fail;                    // partition_block: first rank that is not a pair
};
static_assert(sizeof(Shared) <= kFinishMisc, "finish_layout misc block");

// Block-wide reductions (all threads of the 4-wave block must call them).
__device__ double block_max(double v, Shared* sh, int wave) {
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  __syncthreads();  // sh->red is free
  if ((threadIdx.x & 63) == 0) sh->red[wave] = v;
  __syncthreads();
  double r = sh->red[0];
  for (int i = 1; i < kWaves; ++i) r = sh->red[i] > r ? sh->red[i] : r;
  return r;
}
__device__ int block_sum_i(int v, Shared* sh, int wave) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh->red[wave] = (double)v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < kWaves; ++i) r += sh->red[i];
  return (int)r;
}

__device__ __forceinline__ bool gt(double a, double b) { return a > b; }  // comp = greater

__device__ __forceinline__ void swap_kv(double* k, uint16_t* v, int a, int b) {
  const double tk = k[a];
  k[a] = k[b];
  k[b] = tk;
  const uint16_t tv = v[a];
  v[a] = v[b];
  v[b] = tv;
}

// std::__move_median_to_first(result, a, b, c) — lane 0 only.
__device__ void move_median_to_first(double* k, uint16_t* v, int result, int a, int b, int c) {
  if (gt(k[a], k[b])) {
    if (gt(k[b], k[c])) swap_kv(k, v, result, b);
    else if (gt(k[a], k[c])) swap_kv(k, v, result, c);
    else swap_kv(k, v, result, a);
  } else if (gt(k[a], k[c])) swap_kv(k, v, result, a);
  else if (gt(k[b], k[c])) swap_kv(k, v, result, c);
  else swap_kv(k, v, result, b);
}

// std::__adjust_heap / __push_heap / heap sort of [first, last) — one lane.
__device__ void adjust_heap(double* k, uint16_t* v, int base, int hole, int len, double vk, uint16_t vv) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (gt(k[base + second], k[base + second - 1])) second--;
    k[base + hole] = k[base + second];
    v[base + hole] = v[base + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    k[base + hole] = k[base + second - 1];
    v[base + hole] = v[base + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && gt(k[base + parent], vk)) {
    k[base + hole] = k[base + parent];
    v[base + hole] = v[base + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  k[base + hole] = vk;
  v[base + hole] = vv;
}

__device__ void heap_sort(double* k, uint16_t* v, int first, int last) {
  const int len = last - first;
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      adjust_heap(k, v, first, parent, len, k[first + parent], v[first + parent]);
      if (parent == 0) break;
    }
  }
  while (last - first > 1) {
    --last;
    const double vk = k[last];
    const uint16_t vv = v[last];
    k[last] = k[first];
    v[last] = v[first];
    adjust_heap(k, v, first, 0, last - first, vk, vv);
  }
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t below_mask(int lane) {
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}
__device__ __forceinline__ uint64_t above_mask(int lane) {
  return lane == 63 ? 0ull : (~0ull << (lane + 1));
}
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double read_lane(double x, int l) {
  const uint64_t u = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int read_lane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- large segments: one wave, LDS -------------------------------------------
// Parallel std::__unguarded_partition(first+1, last, pivot=first). lpos/rpos
// are the window-sized scratch arrays; this segment uses [first, last). One
// pass ranks both stop kinds from the left: lpos[k] = the k-th left stop
// (l_k), rposl[g] = the g-th right stop from the LEFT, so the k-th from the
// right is r_k = rposl[totR + 1 - k] (no counting pass for totR first).
// Every pass takes kU chunks of 64 per iteration, their LDS reads issued
// together (one wave works a segment alone: nothing else hides the latency);
// ranks are still assigned chunk by chunk in order.
constexpr int kU = 4;
__device__ int partition_lds(double* k, uint16_t* v, uint16_t* lpos_all, uint16_t* rpos_all,
                             int first, int last) {
  const int lane = lane_id();
  const int m = last - first;
  const int cap = m / 2 + 2;  // pairs <= m/2; ranks up to pairs + 1 are read
  uint16_t* lpos = lpos_all + first - 1;   // ranks are 1-based
  uint16_t* rposl = rpos_all + first - 1;  // right stops, ranked from the left
  const double P = k[first];
  int cntL = 0, cntR = 0;
  for (int base = first + 1; base < last; base += 64 * kU) {
    double key[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = base + 64 * u + lane;
      key[u] = p < last ? k[p] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = base + 64 * u + lane;
      const bool ok = p < last;
      const bool isL = ok && !gt(key[u], P);
      const bool isR = ok && !gt(P, key[u]);
      const uint64_t mL = __ballot(isL), mR = __ballot(isR);
      const int rl = cntL + popc(mL & below_mask(lane)) + 1;
      const int rr = cntR + popc(mR & below_mask(lane)) + 1;
      if (isL) lpos[rl] = (uint16_t)p;
      if (isR) rposl[rr] = (uint16_t)p;
      cntL += popc(mL);
      cntR += popc(mR);
    }
  }
  const int totL = cntL, totR = cntR;
  const int kmax = min(min(totL, totR), cap);
  // the pairs (l_k < r_k) are a prefix of the ranks: l_k rises, r_k falls
  int npairs = 0;
  bool open = true;
  for (int kb = 1; open && kb <= kmax; kb += 64 * kU) {
    int lp[kU], rp[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int kk = kb + 64 * u + lane;
      lp[u] = kk <= kmax ? (int)lpos[kk] : 0;
      rp[u] = kk <= kmax ? (int)rposl[totR + 1 - kk] : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int kk = kb + 64 * u + lane;
      const uint64_t mk = __ballot(kk <= kmax && lp[u] < rp[u]);
      if (open) npairs += popc(mk);
      open = open && mk == ~0ull;
    }
  }
  int cut = INT32_MAX;
  if (npairs + 1 <= totL) cut = lpos[npairs + 1];
  if (npairs >= 1) cut = min(cut, (int)rposl[totR + 1 - npairs]);
  // the swapped positions are all distinct: the kU chunks' swaps are independent
  for (int kb = 1; kb <= npairs; kb += 64 * kU) {
    int lp[kU], rp[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int kk = kb + 64 * u + lane;
      lp[u] = kk <= npairs ? (int)lpos[kk] : -1;
      rp[u] = kk <= npairs ? (int)rposl[totR + 1 - kk] : -1;
    }
    double kl[kU], kr[kU];
    uint16_t vl[kU], vr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (lp[u] >= 0) {
        kl[u] = k[lp[u]];
        kr[u] = k[rp[u]];
        vl[u] = v[lp[u]];
        vr[u] = v[rp[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (lp[u] >= 0) {
        k[lp[u]] = kr[u];
        k[rp[u]] = kl[u];
        v[lp[u]] = vr[u];
        v[rp[u]] = vl[u];
      }
    }
  }
  return uni(cut);
}

// The same partition by the whole 4-wave block, for a level holding one
// large segment (the partial sort's chain down to the prefix): each wave
// ranks both stop kinds of a contiguous quarter from the quarter's left, into
// the quarter's own part of the scratch (one pass); after one barrier the
// global rank k maps to (the wave holding it, its local rank) through the
// waves' counts. The pairs, the cut and the swaps are the single-wave pass's.
constexpr int kCoopMin = 256;
__device__ int partition_block(double* k, uint16_t* v, uint16_t* lpos_all, uint16_t* rpos_all, int first,
                               int last, Shared* sh, int wave) {
  const int lane = lane_id();
  const int m = last - first;
  const int cap = m / 2 + 2;
  if (threadIdx.x == 0) {
    move_median_to_first(k, v, first, first + 1, first + m / 2, last - 1);
    sh->fail = INT32_MAX;
  }
  __syncthreads();
  const double P = k[first];
  const int cq = ((m - 1 + 63) / 64 + kWaves - 1) / kWaves;  // 64-chunks per quarter
  auto q_lo = [&](int w) { return min(first + 1 + w * cq * 64, last); };
  const int q0 = q_lo(wave), q1 = q_lo(wave + 1);
  int cL = 0, cR = 0;  // local ranks: wave w's j-th left stop at lpos_all[q0 - 1 + j]
  for (int base = q0; base < q1; base += 64 * kU) {
    double key[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = base + 64 * u + lane;
      key[u] = p < q1 ? k[p] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = base + 64 * u + lane;
      const bool ok = p < q1;
      const bool isL = ok && !gt(key[u], P);
      const bool isR = ok && !gt(P, key[u]);
      const uint64_t mL = __ballot(isL), mR = __ballot(isR);
      const int rl = cL + popc(mL & below_mask(lane)) + 1;
      const int rr = cR + popc(mR & below_mask(lane)) + 1;
      if (isL) lpos_all[q0 - 1 + rl] = (uint16_t)p;
      if (isR) rpos_all[q0 - 1 + rr] = (uint16_t)p;
      cL += popc(mL);
      cR += popc(mR);
    }
  }
  if (lane == 0) {
    sh->wl[wave] = cL;
    sh->wr[wave] = cR;
  }
  __syncthreads();
  int offL[kWaves + 1], offR[kWaves + 1];  // counts of the earlier quarters
  offL[0] = offR[0] = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    offL[w + 1] = offL[w] + sh->wl[w];
    offR[w + 1] = offR[w] + sh->wr[w];
  }
  const int totL = offL[kWaves], totR = offR[kWaves];
  auto lpos = [&](int kk) -> int {  // l_k, kk in [1, totL]
    int w = 0;
#pragma unroll
    for (int t = 1; t < kWaves; ++t) w += kk > offL[t] ? 1 : 0;
    return lpos_all[q_lo(w) - 1 + (kk - offL[w])];
  };
  auto rpos = [&](int kk) -> int {  // r_k: the (totR + 1 - k)-th right stop from the left
    const int g = totR + 1 - kk;
    int w = 0;
#pragma unroll
    for (int t = 1; t < kWaves; ++t) w += g > offR[t] ? 1 : 0;
    return rpos_all[q_lo(w) - 1 + (g - offR[w])];
  };
  const int kmax = min(min(totL, totR), cap);
  for (int kk = 1 + (int)threadIdx.x; kk <= kmax; kk += 64 * kWaves)
    if (!(lpos(kk) < rpos(kk))) {  // ranks past the pairs fail from here on
      atomicMin(&sh->fail, kk);
      break;
    }
  __syncthreads();
  const int f = sh->fail;
  const int npairs = f == INT32_MAX ? kmax : f - 1;
  int cut = INT32_MAX;
  if (npairs + 1 <= totL) cut = lpos(npairs + 1);
  if (npairs >= 1) cut = min(cut, rpos(npairs));
  __syncthreads();  // every thread read the cut before the swaps move elements
  for (int kk = 1 + (int)threadIdx.x; kk <= npairs; kk += 64 * kWaves) swap_kv(k, v, lpos(kk), rpos(kk));
  __syncthreads();
  return cut;
}

// ---- small segments: one wave, registers ----------------------------------------
// Finishes [base, base+m), m <= 64, entirely: introsort recursion from depth
// `depth`, heap sort where a sub-segment runs out of depth, stable sort of the
// leaves, one write back.
__device__ void sort_small(double* keys, uint16_t* vals, int base, int m, int depth, WaveScratch* ws) {
  const int lane = lane_id();
  double k = lane < m ? keys[base + lane] : 0.0;
  int v = lane < m ? (int)vals[base + lane] : 0;
  uint64_t starts = 1ull;   // starts of final segments (relative)
  uint64_t heaped = 0ull;   // lanes of heap-sorted sub-segments (already ordered)
  int sp = 0;
  if (lane == 0) ws->st[0] = Seg{0, m, depth};
  sp = 1;
  while (sp > 0) {
    --sp;
    const Seg s = ws->st[sp];
    const int f = uni(s.first), l = uni(s.last), d = uni(s.depth);
    const int len = l - f;
    if (len <= 16) {
      starts |= 1ull << f;
      continue;
    }
    if (d == 0) {  // std::__partial_sort(first, last, last): heap sort on one lane
      if (lane < m) {
        keys[base + lane] = k;
        vals[base + lane] = (uint16_t)v;
      }
      if (lane == 0) heap_sort(keys, vals, base + f, base + l);
      if (lane < m) {
        k = keys[base + lane];
        v = vals[base + lane];
      }
      starts |= 1ull << f;
      const uint64_t seg = ((l == 64) ? ~0ull : ((1ull << l) - 1)) & ~((1ull << f) - 1);
      heaped |= seg;
      continue;
    }
    // __move_median_to_first(f, f+1, mid, l-1)
    const int a = f + 1, b = f + len / 2, c = l - 1;
    const double ka = read_lane(k, a), kb = read_lane(k, b), kc = read_lane(k, c);
    int sel;
    if (gt(ka, kb)) sel = gt(kb, kc) ? b : (gt(ka, kc) ? c : a);
    else sel = gt(ka, kc) ? a : (gt(kb, kc) ? c : b);
    const double kf = read_lane(k, f), ks = read_lane(k, sel);
    const int vf = read_lane_i(v, f), vs = read_lane_i(v, sel);
    if (lane == f) {
      k = ks;
      v = vs;
    } else if (lane == sel) {
      k = kf;
      v = vf;
    }
    const double P = ks;
    const bool inr = lane > f && lane < l;
    const bool isL = inr && !gt(k, P);
    const bool isR = inr && !gt(P, k);
    const uint64_t mL = __ballot(isL), mR = __ballot(isR);
    const int totL = popc(mL), totR = popc(mR);
    const int rL = popc(mL & below_mask(lane)) + 1;  // rank ascending
    const int rR = popc(mR & above_mask(lane)) + 1;  // rank from the right
    if (isR) ws->T[rR] = (uint8_t)lane;
    if (isL) ws->U[rL] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int pL = (isL && rL <= totR) ? (int)ws->T[rL] : -1;
    const int pR = (isR && rR <= totL) ? (int)ws->U[rR] : 64;
    const bool swL = isL && pL > lane;   // l_k < r_k
    const bool swR = isR && pR < lane;
    const int npairs = popc(__ballot(swL));
    int cut = INT32_MAX;
    if (npairs + 1 <= totL) cut = ws->U[npairs + 1];
    if (npairs >= 1) cut = min(cut, (int)ws->T[npairs]);
    cut = uni(cut);
    const int src = swL ? pL : (swR ? pR : lane);
    k = __shfl(k, src, 64);
    v = __shfl(v, src, 64);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane == 0) {
      ws->st[sp] = Seg{cut, l, d - 1};
      ws->st[sp + 1] = Seg{f, cut, d - 1};
    }
    sp += 2;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  // stable sort of each leaf (the final insertion sort restricted to it)
  const uint64_t bnd = starts | ((m == 64) ? 0ull : (1ull << m));
  const uint64_t le_mask = bnd & above_mask(lane);
  const int le = le_mask ? __builtin_ctzll(le_mask) : 64;
  const uint64_t ls_mask = bnd & (below_mask(lane) | (1ull << lane));
  const int ls = 63 - __builtin_clzll(ls_mask ? ls_mask : 1ull);
  const bool active = lane < m && !((heaped >> lane) & 1ull);
  int rank = 0;
  for (int t = 0; t < 16; ++t) {  // every lane shuffles: sources must be active lanes
    const int j = ls + t;
    const bool okj = active && j < le;
    const double kj = __shfl(k, okj ? j : lane, 64);
    if (okj) rank += (gt(kj, k) || (kj == k && j < lane)) ? 1 : 0;
  }
  const int dest = active ? ls + rank : lane;
  if (lane < m) {
    keys[base + dest] = k;
    vals[base + dest] = (uint16_t)v;
  }
}

}  // namespace

// The exact pass over one window (4 waves). Waves 1-3 return before the
// list scans; the caller's barrier joins them. Inlined into finish_kernel
// (as a call it took 211 VGPRs and scratch; inlined 129 and none, r04).
__device__ __forceinline__ void finish_window(const FinishArgs& A, const ScanWork* __restrict__ scans,
                              const AngleEntry* __restrict__ angles, const double* __restrict__ scores,
                              FinishOut* __restrict__ out, const int w, char* smem) {
  const int n = (int)A.n_cand;
#ifdef CSM_FINISH_TRACE
  __shared__ int tr_s;
  if (threadIdx.x == 0) {
    tr_s = atomicAdd(&g_trace_n, 1);
    if (tr_s >= kTraceWindows) tr_s = -1;
  }
  __syncthreads();
  const int tr = tr_s;
  if (threadIdx.x == 0 && tr >= 0) g_trace[tr][9] = (unsigned long long)n;
#endif
  CSM_STAMP(0);
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const FinishLayout Lo = finish_layout(n);
  Shared* sh = reinterpret_cast<Shared*>(smem);
  WaveScratch* ws = reinterpret_cast<WaveScratch*>(smem + Lo.wave_scratch) + wave;
  double* keys = reinterpret_cast<double*>(smem + Lo.keys);
  uint16_t* vals = reinterpret_cast<uint16_t*>(smem + Lo.vals);
  uint16_t* lpos = reinterpret_cast<uint16_t*>(smem + Lo.lpos);
  uint16_t* rpos = reinterpret_cast<uint16_t*>(smem + Lo.rpos);
  Seg* stack = reinterpret_cast<Seg*>(smem + Lo.stack);

  const double* sc = scores + (int64_t)w * (A.score_stride ? A.score_stride : A.n_cand);
  // Load, and the limits of the partial sort: max, NaN, and the FindBest
  // prefix size (every element with DoubleEqual(s, max, 1e-2): the prefix is
  // exactly that set, in sorted order).
  double lmax = -INFINITY;
  bool lnan = false;
  for (int i = threadIdx.x; i < n; i += 64 * kWaves) {
    const double x = sc[i];
    keys[i] = x;
    vals[i] = (uint16_t)i;
    lnan |= x != x;
    lmax = x > lmax ? x : lmax;
  }
  lmax = block_max(lmax, sh, wave);
  CSM_STAMP(1);
  if (threadIdx.x == 0) {
    sh->nan = 0;
    sh->cnt_a = 0;
    sh->cnt_b = 0;
    sh->ndef = 0;
  }
  __syncthreads();
  if (__ballot(lnan) != 0 && lane == 0) atomicOr(&sh->nan, 1);
  {
    int c = 0;
    for (int i = threadIdx.x; i < n; i += 64 * kWaves) {
      const double d = keys[i] - lmax;
      c += (d < 0.0 ? d >= -1e-2 : d <= 1e-2) ? 1 : 0;
    }
    c = wave_sum_i(c);
    if (lane == 0) atomicAdd(&sh->cnt_a, c);
  }
  // Level-synchronous introsort: every segment of a level is independent, so
  // the waves take them round-robin, children go to the next level's list
  // (LDS atomic add, no lock), a barrier separates levels. Depth decreases at
  // every partition, so there are at most 2*floor(log2 n) + 2 levels.
  // Partial: a segment starting at or past sh->plim is set aside (positions
  // past the limit are never read, and no element crosses a segment boundary
  // afterwards), kept for the second stage in the deferred list.
  const int half = (n / 16 + 64) / 2;  // finish_layout: the stack region holds two lists
  Seg* cur = stack;
  Seg* nxt = stack + half;
  Seg* deferred = reinterpret_cast<Seg*>(smem + Lo.defer);
  __syncthreads();
  if (threadIdx.x == 0) {
    int lg = 0;
    while ((2 << lg) <= n) ++lg;  // floor(log2 n)
    cur[0] = Seg{0, n, 2 * lg};
    sh->top = 1;      // segments in cur
    sh->pending = 0;  // segments appended to nxt
    sh->pad = 0;
    // stage 1: FindBest's prefix and the positional list's 20
    // (small windows sort whole: the limits' extra passes cost more there)
    const bool full = sh->nan || A.order_out != nullptr || n < kPartialMinCand;
    const int need = (A.skip_lists & 1) ? 1 : kCovPoints;  // the positional list reads 20
    sh->plim = full ? n : min(n, max(sh->cnt_a, need));
  }
  __syncthreads();
  CSM_STAMP(2);
  // A child segment goes to the next level's list, or straight to the
  // deferred list when it starts at or past the limit: a level then holds only
  // the segments that are partitioned, so the partial sort's chain (one live
  // segment per level) takes the whole block's partition_block, not one wave.
  auto push = [&](const Seg& c) {  // one lane
    if (c.first >= sh->plim) {
      const int at = atomicAdd(&sh->ndef, 1);
      if (at < kFinishDefer) deferred[at] = c;
      else sh->pad = 1;  // cannot happen: at most one straddling segment per level
    } else {
      const int at = atomicAdd(&sh->pending, 1);
      if (at < half) nxt[at] = c;
      else sh->pad = 1;  // list overflow: cannot happen for the layout's capacity
    }
  };
  auto run_levels = [&]() {
    const int plim = sh->plim;
    for (int level = 0;; ++level) {
      const int ncur = sh->top;
#ifdef CSM_FINISH_TRACE
      if (threadIdx.x == 0 && tr >= 0 && level < kTraceLevels && plim == sh->plim) {
        g_ltrace[tr][2 * level] = wall_clock64();
        g_ltrace[tr][2 * level + 1] =
            ((unsigned long long)ncur << 32) | (unsigned)(ncur > 0 ? cur[0].last - cur[0].first : 0);
      }
#endif
      if (ncur == 0) break;
      if (level > 64) {  // cannot happen (depth bound); reported as count = -1
        if (threadIdx.x == 0) sh->pad = 1;
        break;
      }
      const Seg s0 = cur[0];
      if (ncur == 1 && s0.first < plim && s0.last - s0.first > kCoopMin && s0.depth > 0) {
        // one large segment: the whole block partitions it
        const int cut = partition_block(keys, vals, lpos, rpos, s0.first, s0.last, sh, wave);
        if (threadIdx.x == 0) {
          push(Seg{cut, s0.last, s0.depth - 1});
          push(Seg{s0.first, cut, s0.depth - 1});
        }
      } else
      for (int i = wave; i < ncur; i += kWaves) {
        const Seg s = cur[i];
        const int first = uni(s.first), last = uni(s.last), depth = uni(s.depth);
        const int len = last - first;
        if (first >= plim) {  // set aside for the second stage
          if (lane == 0) {
            const int at = atomicAdd(&sh->ndef, 1);
            if (at < kFinishDefer) deferred[at] = s;
            else sh->pad = 1;  // cannot happen: at most one straddling segment per level
          }
        } else if (len <= 64) {
          if (len > 1) sort_small(keys, vals, first, len, depth, ws);
        } else if (depth == 0) {
          if (lane == 0) heap_sort(keys, vals, first, last);
        } else {
          if (lane == 0) move_median_to_first(keys, vals, first, first + 1, first + len / 2, last - 1);
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          const int cut = partition_lds(keys, vals, lpos, rpos, first, last);
          if (lane == 0) {
            push(Seg{cut, last, depth - 1});
            push(Seg{first, cut, depth - 1});
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        sh->top = sh->pad ? 0 : sh->pending;
        sh->pending = 0;
      }
      Seg* t = cur;
      cur = nxt;
      nxt = t;
      __syncthreads();
    }
  };
  run_levels();
  __syncthreads();
  CSM_STAMP(3);
#ifdef CSM_FINISH_TRACE
  if (threadIdx.x == 0 && tr >= 0) g_trace[tr][8] = (unsigned long long)sh->plim;
#endif

  // ---- ordered scans over the sorted candidates -----------------------------
  const ScanWork S = scans[w];
  const int ns = A.n_space;
  const int nss = ns * ns;
  const double f = A.step_cells;
  auto cx = [&](int idx) { return S.x0 + ((idx / ns) % ns) * f; };
  auto cy = [&](int idx) { return S.y0 + (idx % ns) * f; };
  const double best = keys[0];
  FinishOut* o = reinterpret_cast<FinishOut*>(smem + Lo.fout);  // stored sealed at the end (emit_sealed)
  // The window's angle rows (cos, sin) in LDS for FindBest's sequential sums:
  // one dependent global load per prefix element made the loop latency-bound
  // (the super-fine level's prefix holds most of its 189 candidates). The
  // partition scratch (lpos .. stack) is free until stage 2 rewrites it.
  const int n_ang = n / nss;
  double2* acs = reinterpret_cast<double2*>(smem + Lo.lpos);
  const bool staged = (size_t)n_ang * sizeof(double2) <= Lo.fout - Lo.lpos;  // (not into the FinishOut)
  if (staged)
    for (int t = threadIdx.x; t < n_ang; t += 64 * kWaves) {
      const AngleEntry ae = angles[S.angle_off + t];
      acs[t] = make_double2(ae.cosine, ae.sine);
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    // FindBestCandidate (:670-710): sequential sums over the tied prefix.
    double ax = 0.0, ay = 0.0, thx = 0.0, thy = 0.0, ssum = 0.0;
    int count = 0;
    for (int i = 0; i < n; ++i) {
      const double s = keys[i];
      const double d = s - best;
      const bool eq = d < 0.0 ? d >= -1e-2 : d <= 1e-2;  // DoubleEqual(s, best, 1e-2)
      if (!eq) break;
      const int idx = vals[i];
      const int a = idx / nss;
      const AngleEntry ae = staged ? AngleEntry{0.0, acs[a].x, acs[a].y} : angles[S.angle_off + a];
      ax += cx(idx) * s;
      ay += cy(idx) * s;
      thx += ae.cosine * s;
      thy += ae.sine * s;
      ssum += s;
      count++;
    }
    const int fi = vals[0];
    o->front_idx = fi;
    o->count = count;
    o->best_score = best;
    o->thx = thx;
    o->thy = thy;
    o->ssum = ssum;
    if (count > 1) {  // :700-707 (atan2 of thy/ssum, thx/ssum is left to the host)
      sh->bx = ax / ssum;
      sh->by = ay / ssum;
    } else {
      sh->bx = cx(fi);
      sh->by = cy(fi);
    }
    o->best_x = sh->bx;
    o->best_y = sh->by;
  }
  __syncthreads();
  CSM_STAMP(4);
  const double bx = sh->bx, by = sh->by;
  const double lo = best - 0.1;
  const double bound = (0.5 < lo) ? 0.5 : lo;  // std::min(best - 0.1, 0.5) (:912,:986)
  const double tol = A.lin_tol;
  auto near_best = [&](int idx) {
    const double dx = cx(idx) - bx, dy = cy(idx) - by;
    const bool ex = dx < 0.0 ? dx >= -fabs(tol) : dx <= fabs(tol);
    const bool ey = dy < 0.0 ? dy >= -fabs(tol) : dy <= fabs(tol);
    return ex && ey;
  };
  const bool want_pos = !(A.skip_lists & 1), want_ang = !(A.skip_lists & 2);
  // Stage 2: the angular list reads the sorted order of every element with
  // score >= bound while it still needs near-best ones: all of them when at
  // most 20 are near the best, else up to the 20th near one in sorted order,
  // i.e. every element scoring at least the 20th largest near-best score.
  if (want_ang) {  // uniform over the block
    int cm = 0, cr = 0;
    for (int i = threadIdx.x; i < n; i += 64 * kWaves) {
      const double x = keys[i];
      const bool above = x >= bound;
      cr += above ? 1 : 0;
      cm += (above && near_best(vals[i])) ? 1 : 0;
    }
    cm = wave_sum_i(cm);
    cr = wave_sum_i(cr);
    if (lane == 0) atomicAdd(&sh->cnt_b, cr);
    if (threadIdx.x == 0) sh->top = 0;
    __syncthreads();
    if (lane == 0) atomicAdd(&sh->top, cm);  // reuse: |M|
    __syncthreads();
    int p2 = sh->cnt_b;  // every element >= bound
    if (kNearRounds && sh->top > kCovPoints && sh->plim < n) {
      // 20th largest near-best score: rounds of "largest below the previous"
      double v = INFINITY;
      int got = 0;
      while (got < kCovPoints) {
        double m = -INFINITY;
        for (int i = threadIdx.x; i < n; i += 64 * kWaves) {
          const double x = keys[i];
          if (x >= bound && x < v && x > m && near_best(vals[i])) m = x;
        }
        m = block_max(m, sh, wave);
        int c = 0;
        for (int i = threadIdx.x; i < n; i += 64 * kWaves) c += (keys[i] == m && near_best(vals[i])) ? 1 : 0;
        c = block_sum_i(c, sh, wave);
        got += c;
        v = m;
      }
      int c = 0;
      for (int i = threadIdx.x; i < n; i += 64 * kWaves) c += keys[i] >= v ? 1 : 0;
      p2 = block_sum_i(c, sh, wave);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = sh->plim;
      sh->plim = max(old, min(n, p2));
      int nd = 0;
      const int ndef = min(sh->ndef, kFinishDefer);
      for (int i = 0; i < ndef; ++i)
        if (deferred[i].first < sh->plim) cur[nd++] = deferred[i];
      sh->ndef = 0;
      sh->top = sh->pad ? 0 : nd;
      sh->pending = 0;
    }
    __syncthreads();
    run_levels();
    __syncthreads();
  }
  CSM_STAMP(5);
  if (A.order_out)
    for (int i = threadIdx.x; i < n; i += 64 * kWaves) A.order_out[(int64_t)w * n + i] = vals[i];
  if (threadIdx.x == 0 && sh->pad) o->count = -1;
  if (wave != 0) return;

  // positional list (:915-928): the sorted prefix with score > bound, <= 20
  {
    int npos = 0;
    for (int base = 0; want_pos && base < n && npos < kCovPoints; base += 64) {
      const int p = base + lane;
      const bool ok = p < n && keys[p] > bound;
      const uint64_t m = __ballot(ok);
      const int run = (m == ~0ull) ? 64 : __ffsll((long long)~m) - 1;  // prefix length in chunk
      if (lane < run && npos + lane < kCovPoints) {
        o->pos_idx[npos + lane] = vals[p];
        o->pos_score[npos + lane] = keys[p];
      }
      npos += run;
      if (run < 64) break;
    }
    if (lane == 0) o->n_pos = min(npos, kCovPoints);
  }
  // angular list (:990-1003): score >= bound and (x, y) within lin_tol of the best
  {
    int nang = 0;
    for (int base = 0; want_ang && base < n && nang < kCovPoints; base += 64) {
      const int p = base + lane;
      bool ok = false;
      bool above = false;
      if (p < n) {
        const double s = keys[p];
        above = s >= bound;
        if (above) ok = near_best(vals[p]);
      }
      const uint64_t m = __ballot(ok);
      const int r = nang + popc(m & below_mask(lane));
      if (ok && r < kCovPoints) {
        o->ang_idx[r] = vals[p];
        o->ang_score[r] = keys[p];
      }
      nang += popc(m);
      if (__ballot(above) != ~0ull) break;  // sorted: nothing later is >= bound
    }
    if (lane == 0) o->n_ang = min(nang, kCovPoints);
  }
  // the LDS FinishOut (thread 0's header, the lanes' list entries) to memory, sealed
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  emit_sealed(A, o, out + w, (want_pos ? 1 : 0) | (want_ang ? 2 : 0), kSealExact, lane);
  CSM_STAMP(6);
}

// scores: window-major, n_cand per window (penalty applied). 4 waves/window.
// With the fast finish's list of flagged windows, a small grid walks the list
// (a block per window of all n_windows cost ~50 us of dispatch at 2048
// windows even though almost every block exits at once).
__device__ __forceinline__ void finish_entry(const FinishArgs& A, const ScanWork* __restrict__ scans,
                                             const AngleEntry* __restrict__ angles, const double* __restrict__ scores,
                                             FinishOut* __restrict__ out, char* smem) {
  if (A.exact_list) {
    // {count, tag} in one load: a pass whose launch's list has been reset by
    // the slot's next scoring launch (another tag) had nothing to do
    const uint64_t head = __hip_atomic_load(reinterpret_cast<uint64_t*>(A.exact_list), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    const int cnt = (uint32_t)(head >> 32) == (uint32_t)A.flag_value ? (int)(uint32_t)head : 0;
    for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
      finish_window(A, scans, angles, scores, out, A.exact_list[2 + i], smem);
      __syncthreads();  // the next window reuses the LDS carve
    }
    if (A.host_flag && cnt > 0) {  // (nothing flagged: the fast pass signalled the host)
      // every block's sealed FinishOut stores complete, then the last block
      // signals the host (the ordering argument: DESIGN §7 "Host signals")
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add(A.done_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == (int)gridDim.x - 1) {
          __hip_atomic_store(A.done_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(A.host_flag, A.flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    return;
  }
  const int w = blockIdx.x;
  if (A.need_exact && A.need_exact[w] == 0) return;  // the fast finish settled this window
  finish_window(A, scans, angles, scores, out, w, smem);
}

__global__ __launch_bounds__(64 * kWaves) void finish_kernel(FinishArgs A, const ScanWork* __restrict__ scans,
                                                             const AngleEntry* __restrict__ angles,
                                                             const double* __restrict__ scores,
                                                             FinishOut* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  finish_entry(A, scans, angles, scores, out, smem);
}

// ---- fast finish: no sort when no tie can matter ----------------------------
// Everything the sorted candidates feed is decided by the elements with
// score >= bound = min(best - 0.1, 0.5) (:912,:986; FindBestCandidate's
// prefix, s >= best - 0.01, lies above it): the FindBest prefix (all of it, in
// sorted order: its sums are order-dependent), the first 20 with score > bound
// (:915-928) and the first 20 near the best with score >= bound (:990-1003).
// std::sort leaves distinct scores in strictly decreasing order, so if none of
// the scores these read repeats (nor the value just past a list's 20th), they
// are fixed by value alone:
//   1. max, NaN check; counts above eight thresholds best - delta;
//   2. the smallest threshold holding 20 elements > bound (or all of them):
//      compacted (<= kFastCap), ranked by value in LDS (rank = elements
//      greater), which gives the prefix and the positional list;
//   3. FindBest's sums -> (bx, by); the near-best elements >= bound compacted
//      (<= kFastNearCap) and ranked the same way for the angular list.
// A repeat where order decides, a NaN or an oversized set flags the window
// for finish_kernel's exact std::sort emulation, which runs next and skips
// every other window. One block of T threads per window; each thread holds
// its V = ceil(n / T) scores in registers (loaded once, all in flight: the
// passes re-reading the scores from L2 were latency-bound, one round trip per
// 256 candidates per pass), and the window's angle rows sit in LDS for the
// sequential FindBest sums. T = 1024 for launches of few windows (the
// reference's single-scan levels), 256 otherwise.
#ifndef CSM_EXACT_GRID
#define CSM_EXACT_GRID 512  // blocks of a listed exact pass (they walk the list of flagged windows)
#endif
constexpr int kFastCap = 512;      // compacted candidates of step 2
constexpr int kFastNearCap = 512;  // compacted near-best candidates of step 3
constexpr int kFastLevels = 8;     // thresholds best - {0.01, 0.02, ..., 0.64}, then everything > bound
constexpr int kFastAngles = 256;   // angle rows staged in LDS (more: read from memory)
__device__ __forceinline__ double wave_max_d(double v) {
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(v, o, 64);
    v = (t > v) ? t : v;
  }
  return v;
}

// Host signal (A.host_flag): every block's FinishOut stores complete (write-
// through sc0 sc1 stores to the coherent host buffer, each wave waits for
// them), the blocks count in; the last one, if no window was flagged for the
// exact pass, stores the flag value itself -- the exact launch behind it then
// returns at once and is off the host's critical path. The count-in is
// relaxed: the host reads every window through its seal, so a flag seen
// before a window's stores costs a spin, never a wrong result (DESIGN §7
// "Host signals"; a per-block system-scope release, one L2 write-back per
// block, cost 25-50 us per launch).
__device__ __forceinline__ void fast_signal(const FinishArgs& A) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(A.done_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      __hip_atomic_store(A.done_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // flag() counts with device-scope atomics before each block's add
      if (__hip_atomic_load(A.exact_list, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        __hip_atomic_store(A.host_flag, A.flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (A.host_fast_flag)  // every header is in: settled windows complete now
        __hip_atomic_store(A.host_fast_flag, A.flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int T, int V>
__device__ __forceinline__ void finish_fast_body(const FinishArgs& A, const ScanWork* __restrict__ scans,
                                                 const AngleEntry* __restrict__ angles,
                                                 const double* __restrict__ scores, FinishOut* __restrict__ out);

#ifdef CSM_TRACE_FASTBLK
// per block: start, end (wall clock), hw id, then the phase stamps 16-25 of its
// window (plain stores: no same-address atomics; tools/fast_blocks.py)
constexpr int kFastBlkTrace = 4096;
__device__ unsigned long long g_fast_blk[kFastBlkTrace][16];
__device__ int g_fast_cand;  // record launches of this many candidates only (0: every launch)
#undef CSM_TS_MIN
#undef CSM_TS_MAX
#define CSM_TS_MIN(slot) CSM_TS_MAX(slot)
#define CSM_TS_MAX(slot)                                                            \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < kFastBlkTrace &&                           \
        (g_fast_cand == 0 || A.n_cand == g_fast_cand))                              \
      g_fast_blk[blockIdx.x][(slot) - 13] = (unsigned long long)wall_clock64();     \
  } while (0)
#endif

template <int T, int V>
__global__ __launch_bounds__(T) void finish_fast_kernel(FinishArgs A, const ScanWork* __restrict__ scans,
                                                        const AngleEntry* __restrict__ angles,
                                                        const double* __restrict__ scores,
                                                        FinishOut* __restrict__ out) {
  CSM_TS_MIN(16);
#ifdef CSM_TRACE_FASTBLK
  const unsigned long long t_start = wall_clock64();
#endif
  finish_fast_body<T, V>(A, scans, angles, scores, out);
  CSM_TS_MAX(24);  // body done
  if (A.host_flag) fast_signal(A);
  CSM_TS_MAX(25);  // signalled
#ifdef CSM_TRACE_FASTBLK
  if (threadIdx.x == 0 && blockIdx.x < kFastBlkTrace && (g_fast_cand == 0 || A.n_cand == g_fast_cand)) {
    g_fast_blk[blockIdx.x][0] = t_start;
    g_fast_blk[blockIdx.x][1] = wall_clock64();
    g_fast_blk[blockIdx.x][2] = __smid();
  }
#endif
}

template <int T, int V>
__device__ __forceinline__ void finish_fast_body(const FinishArgs& A, const ScanWork* __restrict__ scans,
                                                 const AngleEntry* __restrict__ angles,
                                                 const double* __restrict__ scores, FinishOut* __restrict__ out) {
  constexpr int NW = T / 64;
  // LDS lists sized to what the instantiation can hold (n <= V * T): a block
  // of the 189- and 1331-candidate levels then fits 8 to a CU, so a part's
  // 2048 windows take one round of blocks, not two (23.2 KB of LDS a block
  // allowed 7). The caps only decide when the exact pass takes a window.
  constexpr int CAP = V * T < kFastCap ? V * T : kFastCap;
  constexpr int NCAP = V * T < kFastNearCap ? V * T : kFastNearCap;
  constexpr int ACAP = T == 128 ? 64 : (V * T < kFastAngles ? V * T : kFastAngles);
  __shared__ __attribute__((aligned(16))) double ck[CAP + 4];  // step 2 candidates (value, index), then ...
  __shared__ int ci[CAP];
  __shared__ double sk[CAP];   // ... sorted by value (rank order)
  __shared__ int si[CAP];
  __shared__ __attribute__((aligned(16))) double nk[NCAP + 4];
  __shared__ int ni[NCAP];
  __shared__ double acs[ACAP], asn[ACAP];
  __shared__ double red[NW];
  __shared__ int cnt_s[kFastLevels];
  __shared__ int nC_s, nN_s, flag_s;
  __shared__ double sbx, sby;
  // FinishOut is assembled in LDS and stored once at the end (34 16-byte
  // stores): written field by field it was dozens of scattered stores, to
  // pinned host memory on the few-window path, each barrier after them
  // waiting for their completions.
  __shared__ __attribute__((aligned(16))) FinishOut so;
  const int w = blockIdx.x;
  const int n = (int)A.n_cand;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* sc = scores + (int64_t)w * (A.score_stride ? A.score_stride : A.n_cand);
  int32_t* need = A.need_exact + w;
  auto flag = [&]() {  // thread 0: the exact pass takes this window
    *need = 1;
    if (A.exact_list) A.exact_list[2 + atomicAdd(A.exact_list, 1)] = w;
    if (A.host_fast_flag) store_pending_seal(A, out + w);  // the exact pass owes it
  };
  // the scores, every load in flight (index clamped, value masked after)
  double v[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = tid + k * T;
    const double x = sc[min(i, n - 1)];
    v[k] = i < n ? x : -INFINITY;
  }
  const ScanWork S = scans[w];
  const int ns = A.n_space;
  const int nss = ns * ns;
  CSM_TS_MAX(17);  // score loads issued
  {
    const int na = min(n / nss, ACAP);
    for (int t = tid; t < na; t += T) {
      const AngleEntry ae = angles[S.angle_off + t];
      acs[t] = ae.cosine;
      asn[t] = ae.sine;
    }
  }
  if (tid < kFastLevels) cnt_s[tid] = 0;
  if (tid == 0) {
    nC_s = 0;
    nN_s = 0;
    flag_s = 0;
  }

  // 1. best = the front of the sorted candidates (:607); NaN anywhere: exact path
  double m = -INFINITY;
  bool nan = false;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    nan |= (v[k] != v[k]);
    m = (v[k] > m) ? v[k] : m;
  }
  m = wave_max_d(m);
  if (lane == 0) red[wave] = m;
  if (__ballot(nan) != 0 && lane == 0) flag_s = 1;
  __syncthreads();
  double best = red[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) best = fmax(best, red[q]);
  CSM_TS_MAX(18);  // max reduced
  if (flag_s || n <= 0) {
    if (tid == 0) flag();
    return;
  }
  const double lo = best - 0.1;
  const double bound = (0.5 < lo) ? 0.5 : lo;  // std::min(best - 0.1, 0.5) (:912,:986)
  // level k < 7: s > bound and s - best >= -0.01 * 2^k; level 7: s > bound
  // smallest level holding s (kFastLevels: none), branch-free: d >= -dl holds
  // from the first level on (dl doubles), so the level counts the failures
  auto level_of = [&](double s) {
    const double d = s - best;
    double dl = 0.01;
    int lv = 0;
#pragma unroll
    for (int k = 0; k < kFastLevels - 1; ++k, dl *= 2.0) lv += (d < -dl) ? 1 : 0;
    return (s > bound) ? lv : kFastLevels;
  };
  int lv[V];
  {
    // per-lane counts packed 16 bits a level (levels 0-3 in c0, 4-7 in c1; a
    // wave counts at most 64 * V < 2^16 per level), added across the wave in
    // two 64-bit words: vector work only. (Per-level ballots and scalar
    // popcounts kept the CU's one scalar unit busy for every wave: ~4.6 us
    // of a coarse window's block, tools/fast_blocks.py.)
    static_assert(64 * V < 65536, "16-bit level counts");
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      lv[k] = level_of(v[k]);  // -INFINITY padding: no level
      const uint64_t one = 1ull << (16 * (lv[k] & 3));
      c0 += lv[k] < 4 ? one : 0ull;
      c1 += (lv[k] >= 4 && lv[k] < kFastLevels) ? one : 0ull;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c0 += __shfl_xor(c0, o, 64);
      c1 += __shfl_xor(c1, o, 64);
    }
    if (lane < kFastLevels) {
      const int t = (int)(((lane < 4 ? c0 : c1) >> (16 * (lane & 3))) & 0xFFFF);
      if (t) atomicAdd(&cnt_s[lane], t);
    }
  }
  __syncthreads();
  CSM_TS_MAX(19);  // level counts
  // 2. the smallest level whose cumulative count reaches 20 (or all > bound);
  // without the positional list, level 0 (exactly FindBest's prefix set)
  const bool want_pos = !(A.skip_lists & 1), want_ang = !(A.skip_lists & 2);
  int L = want_pos ? kFastLevels - 1 : 0, cum = 0;
  for (int k = 0; want_pos && k < kFastLevels; ++k) {
    cum += cnt_s[k];
    if (cum >= kCovPoints) {
      L = k;
      break;
    }
  }
  int nC = 0;
  for (int k = 0; k <= L; ++k) nC += cnt_s[k];
  if (nC > CAP) {
    if (tid == 0) flag();
    return;
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = tid + k * T;
    const bool in = lv[k] <= L;  // padding never qualifies
    const uint64_t mm = __ballot(in);
    if (mm) {  // wave-uniform
      int base = 0;
      if (lane == 0) base = atomicAdd(&nC_s, popc(mm));
      base = uni(base);
      if (in) {
        const int p = base + popc(mm & below_mask(lane));
        ck[p] = v[k];
        ci[p] = i;
      }
    }
  }
  if (tid < 4 && nC + tid < CAP + 4) ck[nC + tid] = -INFINITY;  // the rank loop's padding (nC known)
  __syncthreads();
  // rank = elements greater; any equal value where the order decides: exact
  // path (the prefix, the positional 20 and the value just past them)
  // (ck padded with -inf to a multiple of 4: read 4 at a time, 2 LDS loads)
  for (int t = tid; t < nC; t += T) {
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
    if (eq > 1 && (inF || (want_pos && r <= kCovPoints))) flag_s = 1;
    sk[r] = x;  // distinct ranks whenever nothing is flagged
    si[r] = ci[t];
  }
  __syncthreads();
  CSM_TS_MAX(20);  // compacted and ranked
  if (flag_s) {
    if (tid == 0) flag();
    return;
  }
  const double f = A.step_cells;
  auto cx = [&](int idx) { return S.x0 + ((idx / ns) % ns) * f; };
  auto cy = [&](int idx) { return S.y0 + (idx % ns) * f; };
  FinishOut* const o = &so;
  // Only the pieces the host reads are stored: the header, plus the lists the
  // level keeps (skip_lists) -- 64 B per window instead of 544 B on a level
  // whose lists are dead, the bytes that cross to host memory with a host signal.
  const int lists = (want_pos ? 1 : 0) | (want_ang ? 2 : 0);
  auto emit = [&]() {  // all threads: the LDS FinishOut and its seal to out[w]
    __syncthreads();
    if (wave == 0) emit_sealed(A, &so, out + w, lists, kSealFast, lane);
  };
  if (tid == 0) {  // :676-707, the same sequential sums as finish_kernel
    double ax = 0.0, ay = 0.0, thx = 0.0, thy = 0.0, ssum = 0.0;
    int count = 0;
    for (int r = 0; r < nC; ++r) {
      const double s = sk[r];
      const double d = s - best;
      if (!(d < 0.0 ? d >= -1e-2 : d <= 1e-2)) break;
      const int idx = si[r];
      const int a = idx / nss;
      const double ca = a < ACAP ? acs[a] : angles[S.angle_off + a].cosine;
      const double sa = a < ACAP ? asn[a] : angles[S.angle_off + a].sine;
      ax += cx(idx) * s;
      ay += cy(idx) * s;
      thx += ca * s;
      thy += sa * s;
      ssum += s;
      count++;
    }
    const int fi0 = si[0];
    o->front_idx = fi0;
    o->count = count;
    o->best_score = best;
    o->thx = thx;
    o->thy = thy;
    o->ssum = ssum;
    if (count > 1) {
      sbx = ax / ssum;
      sby = ay / ssum;
    } else {
      sbx = cx(fi0);
      sby = cy(fi0);
    }
    o->best_x = sbx;
    o->best_y = sby;
    o->n_pos = want_pos ? min(nC, kCovPoints) : 0;
  }
  // positional list (:915-928): the sorted prefix with score > bound, <= 20
  if (want_pos && tid < min(nC, kCovPoints)) {
    o->pos_idx[tid] = si[tid];
    o->pos_score[tid] = sk[tid];
  }
  __syncthreads();
  CSM_TS_MAX(21);  // prefix sums and positional list
  // 3. angular list (:990-1003): near the best, score >= bound
  if (!want_ang) {
    if (tid == 0) o->n_ang = 0;
    emit();
    if (tid == 0) *need = 0;
    return;
  }
  const double bx = sbx, by = sby, tol = A.lin_tol;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = tid + k * T;
    const double s = v[k];
    bool in = false;
    if (s >= bound) {  // padding (-inf) never qualifies
      const double dx = cx(i) - bx, dy = cy(i) - by;
      const bool ex = dx < 0.0 ? dx >= -fabs(tol) : dx <= fabs(tol);
      const bool ey = dy < 0.0 ? dy >= -fabs(tol) : dy <= fabs(tol);
      in = ex && ey;
    }
    const uint64_t mm = __ballot(in);
    if (mm) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&nN_s, popc(mm));
      base = uni(base);
      if (in) {
        const int p = base + popc(mm & below_mask(lane));
        if (p < NCAP) {
          nk[p] = s;
          ni[p] = i;
        }
      }
    }
  }
  __syncthreads();
  CSM_TS_MAX(22);  // near-best compacted
  const int nN = nN_s;
  if (nN > NCAP) {
    if (tid == 0) flag();
    return;
  }
  if (tid < 4) nk[nN + tid] = -INFINITY;  // the rank loop's padding
  __syncthreads();
  for (int t = tid; t < nN; t += T) {
    const double x = nk[t];
    int r = 0, eq = 0;
    for (int j = 0; j < nN; j += 4) {  // (nk padded with -inf like ck)
      const double2 u01 = *reinterpret_cast<const double2*>(&nk[j]);
      const double2 u23 = *reinterpret_cast<const double2*>(&nk[j + 2]);
      r += ((u01.x > x) ? 1 : 0) + ((u01.y > x) ? 1 : 0) + ((u23.x > x) ? 1 : 0) + ((u23.y > x) ? 1 : 0);
      eq += ((u01.x == x) ? 1 : 0) + ((u01.y == x) ? 1 : 0) + ((u23.x == x) ? 1 : 0) + ((u23.y == x) ? 1 : 0);
    }
    if (eq > 1 && r <= kCovPoints) flag_s = 1;
    if (r < kCovPoints) {
      o->ang_idx[r] = ni[t];
      o->ang_score[r] = x;
    }
  }
  __syncthreads();
  CSM_TS_MAX(23);  // near-best ranked
  if (tid == 0) o->n_ang = min(nN, kCovPoints);
  if (flag_s) {  // (flag_s is read after the barrier above: uniform)
    if (tid == 0) flag();
    return;
  }
  emit();
  if (tid == 0) *need = 0;
}

// Scores per thread of the fast finish's instantiations: the smallest V with
// V * T >= n (n <= kFinishMaxCand = 10240).
template <int T, int V>
hipError_t launch_fast_tv(const FinishArgs& A, const ScanWork* s, const AngleEntry* a, const double* sc,
                          FinishOut* o, int32_t nw, hipStream_t stream) {
  hipLaunchKernelGGL((finish_fast_kernel<T, V>), dim3(nw), dim3(T), 0, stream, A, s, a, sc, o);
  return hipGetLastError();
}

hipError_t launch_fast(const FinishArgs& A, const ScanWork* s, const AngleEntry* a, const double* sc, FinishOut* o,
                       int32_t nw, hipStream_t stream) {
  const int64_t n = A.n_cand;
  if (nw <= (A.wide_windows ? A.wide_windows : kFinishWideWindows)) {  // few windows: 16 waves per window
    if (n <= 1024) return launch_fast_tv<1024, 1>(A, s, a, sc, o, nw, stream);
    if (n <= 2048) return launch_fast_tv<1024, 2>(A, s, a, sc, o, nw, stream);
    if (n <= 4096) return launch_fast_tv<1024, 4>(A, s, a, sc, o, nw, stream);
    if (n <= 6144) return launch_fast_tv<1024, 6>(A, s, a, sc, o, nw, stream);
    return launch_fast_tv<1024, 10>(A, s, a, sc, o, nw, stream);
  }
  if (n <= 256) return launch_fast_tv<256, 1>(A, s, a, sc, o, nw, stream);
  if (n <= 512) return launch_fast_tv<256, 2>(A, s, a, sc, o, nw, stream);
  if (n <= 1024) return launch_fast_tv<256, 4>(A, s, a, sc, o, nw, stream);
  // two waves a window (20 KB of LDS, ~80 VGPRs): 8 blocks a CU, where
  // <256, 6> held 7 (66 VGPRs, 23.2 KB)
  if (n <= 1408) return launch_fast_tv<128, 11>(A, s, a, sc, o, nw, stream);
  if (n <= 1536) return launch_fast_tv<256, 6>(A, s, a, sc, o, nw, stream);
  if (n <= 2560) return launch_fast_tv<256, 10>(A, s, a, sc, o, nw, stream);
  if (n <= 5120) return launch_fast_tv<256, 20>(A, s, a, sc, o, nw, stream);
  return launch_fast_tv<256, 40>(A, s, a, sc, o, nw, stream);
}

hipError_t launch_finish(const FinishArgs& A, const ScanWork* d_scans, const AngleEntry* d_angles,
                         const double* d_scores, FinishOut* d_out, int32_t n_windows, hipStream_t stream,
                         hipStream_t exact_stream, hipEvent_t ev_fast, bool fast_done) {
  const size_t lds = finish_lds_bytes(A.n_cand);
  if (A.n_cand <= 0 || A.n_cand > kFinishMaxCand || lds > 160 * 1024 || n_windows <= 0) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
#ifdef CSM_FINISH_TRACE
    const int max_dyn = 156 * 1024;  // + static trace slot
#else
    const int max_dyn = 160 * 1024;
#endif
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&finish_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, max_dyn);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const bool listed = A.need_exact && A.exact_list && !A.order_out;
  if (listed && !A.host_flag) {  // with a host signal the scoring launch zeroed the count
    hipError_t e = hipMemsetAsync(A.exact_list, 0, 2 * sizeof(int32_t), stream);  // {count 0, tag 0}
    if (e != hipSuccess) return e;
  }
  if (A.need_exact && !A.order_out && !fast_done) {  // fast pass first; the exact pass only where it flagged
    hipError_t e = launch_fast(A, d_scans, d_angles, d_scores, d_out, n_windows, stream);
    if (e != hipSuccess) return e;
  }
  hipStream_t xs = stream;
  if (exact_stream && exact_stream != stream && A.need_exact && !A.order_out && ev_fast) {
    hipError_t e;
    if ((e = hipEventRecord(ev_fast, stream)) != hipSuccess || (e = hipStreamWaitEvent(exact_stream, ev_fast, 0)) != hipSuccess)
      return e;
    xs = exact_stream;
  }
  FinishArgs B = A;
  if (!A.host_flag) B.flag_value = 0;       // the tag the memset above left
  if (A.order_out) B.need_exact = nullptr;  // the permutation hook always sorts
  if (!listed) B.exact_list = nullptr;
  const dim3 grid(listed ? std::min(n_windows, CSM_EXACT_GRID) : n_windows);
  hipLaunchKernelGGL(finish_kernel, grid, dim3(64 * kWaves), lds, xs, B, d_scans, d_angles, d_scores, d_out);
  return hipGetLastError();
}

}  // namespace csm

#ifdef CSM_TRACE_SMALL
// Trace readout of the fast finish's stamps (slots 16-25; tools/small_trace.py).
extern "C" int csm_debug_fast_trace(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::dev::g_small_trace), 64 * 8) != hipSuccess) return -1;
  unsigned long long init[64] = {0};
  init[0] = init[16] = ~0ull;
  return hipMemcpyToSymbol(HIP_SYMBOL(csm::dev::g_small_trace), init, 64 * 8) == hipSuccess ? 0 : -1;
}
#endif

#ifdef CSM_TRACE_FASTBLK
// Per-block (start, end, hw id, phase stamps) of the last fast-finish launch
// (of n_cand candidates if selected; tools/fast_blocks.py).
extern "C" int csm_debug_fast_select(int n_cand) {
  return hipMemcpyToSymbol(HIP_SYMBOL(csm::g_fast_cand), &n_cand, sizeof(int)) == hipSuccess ? 0 : -1;
}
extern "C" int csm_debug_fast_blocks(unsigned long long* out, int max_blocks) {
  const int n = max_blocks < csm::kFastBlkTrace ? max_blocks : csm::kFastBlkTrace;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::g_fast_blk), (size_t)n * 16 * 8) == hipSuccess ? n : -1;
}
#endif

#ifdef CSM_FINISH_TRACE
// Trace readout for tools/finish_trace.py: copies and resets the stamps.
extern "C" int csm_debug_finish_levels(unsigned long long* out, int max_windows) {
  int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(csm::g_trace_n), sizeof(int)) != hipSuccess) return -1;
  n = n < csm::kTraceWindows ? n : csm::kTraceWindows;
  n = n < max_windows ? n : max_windows;
  if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::g_ltrace),
                                   (size_t)n * 2 * csm::kTraceLevels * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return n;
}

extern "C" int csm_debug_finish_trace(unsigned long long* out, int max_windows) {
  int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(csm::g_trace_n), sizeof(int)) != hipSuccess) return -1;
  n = n < max_windows ? n : max_windows;
  n = n < csm::kTraceWindows ? n : csm::kTraceWindows;
  if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::g_trace), (size_t)n * 10 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  const int zero = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(csm::g_trace_n), &zero, sizeof(int));
  return n;
}
#endif
