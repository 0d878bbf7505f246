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
// Layout: one 256-thread workgroup (4 waves) per window. The waves pull
// segments from a shared LDS stack (spin lock). A segment of more than 64
// elements is partitioned by one wave in LDS; a segment of at most 64 is
// loaded into registers (lane = element) and finished there: its whole
// introsort recursion (ballot / bpermute partitions) and the stable sort of
// its leaves, then written back once.
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {

namespace {

constexpr int kWaves = 4;

struct Seg {
  int32_t first, last, depth;
};

struct WaveScratch {      // per-wave LDS scratch of the register sort
  uint8_t T[72], U[72];   // lane of the k-th right / left stop
  Seg st[40];             // sub-segment stack
};

static_assert(sizeof(WaveScratch) <= kFinishWaveScratch, "finish_layout wave scratch");

struct Shared {           // misc block of the LDS carve (finish_layout: 64 B + waves)
  int lock, top, pending, pad;
  double bx, by;
};

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

// ---- shared work stack ------------------------------------------------------
__device__ __forceinline__ void lock(Shared* sh) {
  for (int spins = 0; atomicCAS(&sh->lock, 0, 1) != 0; ++spins) {
    if (spins > (1 << 24)) {  // bounded: a stuck lock aborts the window
      sh->pad = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void unlock(Shared* sh) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  atomicExch(&sh->lock, 0);
}

// ---- large segments: one wave, LDS -------------------------------------------
// Parallel std::__unguarded_partition(first+1, last, pivot=first). lpos/rpos
// are the window-sized scratch arrays; this segment uses [first, first+cap).
__device__ int partition_lds(double* k, uint16_t* v, uint16_t* lpos_all, uint16_t* rpos_all,
                             int first, int last) {
  const int lane = lane_id();
  const int m = last - first;
  const int cap = m / 2 + 2;  // pairs <= m/2; ranks up to pairs + 1 are read
  uint16_t* lpos = lpos_all + first - 1;  // ranks are 1-based
  uint16_t* rpos = rpos_all + first - 1;
  const double P = k[first];
  int totR = 0;
  for (int base = first + 1; base < last; base += 64) {
    const int p = base + lane;
    const bool ok = p < last;
    const bool isR = ok && !gt(P, ok ? k[p] : 0.0);
    totR += popc(__ballot(isR));
  }
  int cntL = 0, cntR = 0;
  for (int base = first + 1; base < last; base += 64) {
    const int p = base + lane;
    const bool ok = p < last;
    const double key = ok ? k[p] : 0.0;
    const bool isL = ok && !gt(key, P);
    const bool isR = ok && !gt(P, key);
    const uint64_t mL = __ballot(isL), mR = __ballot(isR);
    const int rl = cntL + popc(mL & below_mask(lane)) + 1;
    const int rr = totR - (cntR + popc(mR & below_mask(lane))) ;  // rank from the right
    if (isL && rl <= cap) lpos[rl] = (uint16_t)p;
    if (isR && rr <= cap) rpos[rr] = (uint16_t)p;
    cntL += popc(mL);
    cntR += popc(mR);
  }
  const int totL = cntL;
  const int kmax = min(min(totL, totR), cap);
  int npairs = 0;
  for (int kb = 1; kb <= kmax; kb += 64) {
    const int kk = kb + lane;
    const bool okp = kk <= kmax && lpos[kk] < rpos[kk];
    const uint64_t mk = __ballot(okp);
    npairs += popc(mk);
    if (mk != ~0ull) break;
  }
  int cut = INT32_MAX;
  if (npairs + 1 <= totL) cut = lpos[npairs + 1];
  if (npairs >= 1) cut = min(cut, (int)rpos[npairs]);
  for (int kb = 1; kb <= npairs; kb += 64) {
    const int kk = kb + lane;
    if (kk <= npairs) swap_kv(k, v, lpos[kk], rpos[kk]);
  }
  return uni(cut);
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

// scores: window-major, n_cand per window (penalty applied). 4 waves/window.
__global__ __launch_bounds__(64 * kWaves) void finish_kernel(FinishArgs A, const ScanWork* __restrict__ scans,
                                                             const AngleEntry* __restrict__ angles,
                                                             const double* __restrict__ scores,
                                                             FinishOut* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = blockIdx.x;
  const int n = (int)A.n_cand;
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

  const double* sc = scores + (int64_t)w * A.n_cand;
  for (int i = threadIdx.x; i < n; i += 64 * kWaves) {
    keys[i] = sc[i];
    vals[i] = (uint16_t)i;
  }
  if (threadIdx.x == 0) {
    int lg = 0;
    while ((2 << lg) <= n) ++lg;  // floor(log2 n)
    stack[0] = Seg{0, n, 2 * lg};
    sh->lock = 0;
    sh->top = 1;
    sh->pending = 1;
    sh->pad = 0;
  }
  __syncthreads();

  // introsort loop, segments pulled by whichever wave is free (bounded: a
  // window never needs more than ~n iterations per wave)
  for (int iter = 0;; ++iter) {
    if (iter > 4 * n + (1 << 16) || sh->pad) {
      sh->pad = 1;  // reported as count = -1: the host fails the call loudly
      break;
    }
    int got = 0, pend = 0;
    Seg s{0, 0, 0};
    if (lane == 0) {
      lock(sh);
      if (sh->top > 0) {
        s = stack[--sh->top];
        got = 1;
      }
      pend = sh->pending;
      unlock(sh);
    }
    got = uni(got);
    if (!got) {
      if (uni(pend) == 0) break;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    const int first = uni(s.first), last = uni(s.last), depth = uni(s.depth);
    const int len = last - first;
    int delta = -1;  // change of `pending` when this segment is done
    Seg c0{0, 0, 0}, c1{0, 0, 0};
    if (len <= 64) {
      if (len > 1) sort_small(keys, vals, first, len, depth, ws);
    } else if (depth == 0) {
      if (lane == 0) heap_sort(keys, vals, first, last);
    } else {
      if (lane == 0) move_median_to_first(keys, vals, first, first + 1, first + len / 2, last - 1);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const int cut = partition_lds(keys, vals, lpos, rpos, first, last);
      c0 = Seg{cut, last, depth - 1};
      c1 = Seg{first, cut, depth - 1};
      delta = 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) {
      lock(sh);
      if (delta > 0) {
        stack[sh->top++] = c0;
        stack[sh->top++] = c1;
      }
      sh->pending += delta;
      unlock(sh);
    }
  }
  __syncthreads();
  if (A.order_out)
    for (int i = threadIdx.x; i < n; i += 64 * kWaves) A.order_out[(int64_t)w * n + i] = vals[i];
  if (wave != 0) return;

  // ---- ordered scans over the sorted candidates (wave 0) ---------------------
  const ScanWork S = scans[w];
  const int ns = A.n_space;
  const int nss = ns * ns;
  const double f = A.step_cells;
  auto cx = [&](int idx) { return S.x0 + ((idx / ns) % ns) * f; };
  auto cy = [&](int idx) { return S.y0 + (idx % ns) * f; };
  const double best = keys[0];
  FinishOut* o = out + w;
  if (lane == 0) {
    // FindBestCandidate (:670-710): sequential sums over the tied prefix.
    double ax = 0.0, ay = 0.0, thx = 0.0, thy = 0.0, ssum = 0.0;
    int count = 0;
    for (int i = 0; i < n; ++i) {
      const double s = keys[i];
      const double d = s - best;
      const bool eq = d < 0.0 ? d >= -1e-2 : d <= 1e-2;  // DoubleEqual(s, best, 1e-2)
      if (!eq) break;
      const int idx = vals[i];
      const AngleEntry ae = angles[S.angle_off + idx / nss];
      ax += cx(idx) * s;
      ay += cy(idx) * s;
      thx += ae.cosine * s;
      thy += ae.sine * s;
      ssum += s;
      count++;
    }
    const int fi = vals[0];
    o->front_idx = fi;
    o->count = sh->pad ? -1 : count;
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
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const double bx = sh->bx, by = sh->by;
  const double lo = best - 0.1;
  const double bound = (0.5 < lo) ? 0.5 : lo;  // std::min(best - 0.1, 0.5) (:912,:986)
  // positional list (:915-928): the sorted prefix with score > bound, <= 20
  {
    int npos = 0;
    for (int base = 0; base < n && npos < kCovPoints; base += 64) {
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
    const double tol = A.lin_tol;
    int nang = 0;
    for (int base = 0; base < n && nang < kCovPoints; base += 64) {
      const int p = base + lane;
      bool ok = false;
      bool above = false;
      if (p < n) {
        const double s = keys[p];
        above = s >= bound;
        if (above) {
          const int idx = vals[p];
          const double dx = cx(idx) - bx, dy = cy(idx) - by;
          const bool ex = dx < 0.0 ? dx >= -fabs(tol) : dx <= fabs(tol);
          const bool ey = dy < 0.0 ? dy >= -fabs(tol) : dy <= fabs(tol);
          ok = ex && ey;
        }
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
}

hipError_t launch_finish(const FinishArgs& A, const ScanWork* d_scans, const AngleEntry* d_angles,
                         const double* d_scores, FinishOut* d_out, int32_t n_windows, hipStream_t stream) {
  const size_t lds = finish_lds_bytes(A.n_cand);
  if (A.n_cand <= 0 || A.n_cand > kFinishMaxCand || lds > 160 * 1024 || n_windows <= 0) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&finish_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(finish_kernel, dim3(n_windows), dim3(64 * kWaves), lds, stream, A, d_scans,
                     d_angles, d_scores, d_out);
  return hipGetLastError();
}

}  // namespace csm
