// csm_finish.hip — device-side finish of a window: the reference's
// std::sort(candidates, greater) (correlate_scan_matcher.h:607) reproduced
// EXACTLY (same permutation, ties included), then the three ordered scans
// that consume the sorted candidates: FindBestCandidate's prefix
// (:670-710) and the candidate lists of ComputePositionalCovariance
// (:911-928) and ComputeAngularCovariance (:985-1003).
//
// Why an emulation and not a GPU sort: the winner among exactly tied scores,
// the averaged best pose and both covariances depend on the order std::sort
// leaves tied candidates in, and synthetic/real grids tie constantly (sub-cell
// window steps land many candidates on the same cells). libstdc++'s std::sort
// is deterministic given the comparison outcomes:
//   introsort loop (threshold 16, depth limit 2*floor(log2 n)); pivot = median
//   of (first+1, mid, last-1) swapped to first; unguarded Hoare partition;
//   heap sort at depth 0; final insertion sort.
// Segments left by the loop are ordered relative to each other (left >= pivot
// >= right), so the final insertion sort equals an independent stable
// insertion sort of each leaf segment. The unguarded partition is computed in
// parallel by one wave: with l_k the k-th position (ascending) whose key is
// not > pivot and r_k the k-th position (descending) whose key is not <
// pivot, the sequential loop swaps exactly the pairs (l_k, r_k) with
// l_k < r_k and returns cut = min(l_{p+1}, r_p) for p such pairs.
// The model is validated against libstdc++ in tests/introsort_ref.py.
//
// One 64-lane workgroup (one wave) per window; keys, indices and scratch in LDS.
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {

namespace {

struct Seg {
  int32_t first, last, depth;
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

// std::__adjust_heap / __push_heap / heap sort of [first, last) — lane 0 only.
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

__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t lanes_below() {
  const int lane = threadIdx.x;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Parallel std::__unguarded_partition(first+1, last, pivot=first) of one wave.
// lpos/rpos hold positions of left/right stops by rank (1-based), up to cap.
__device__ int partition(double* k, uint16_t* v, uint16_t* lpos, uint16_t* rpos, int cap,
                         int first, int last) {
  const int lane = threadIdx.x;
  const double P = k[first];
  // pass 1: total right stops
  int totR = 0;
  for (int base = first + 1; base < last; base += 64) {
    const int p = base + lane;
    const bool ok = p < last;
    const double key = ok ? k[p] : 0.0;
    const bool isR = ok && !gt(P, key);
    totR += popc(__ballot(isR));
  }
  // pass 2: ranks, scatter the first `cap` stops of each side
  int cntL = 0, cntR = 0, totL = 0;
  for (int base = first + 1; base < last; base += 64) {
    const int p = base + lane;
    const bool ok = p < last;
    const double key = ok ? k[p] : 0.0;
    const bool isL = ok && !gt(key, P);
    const bool isR = ok && !gt(P, key);
    const uint64_t mL = __ballot(isL), mR = __ballot(isR);
    const int rl = cntL + popc(mL & lanes_below()) + 1;
    const int rr_incl = cntR + popc(mR & lanes_below()) + 1;  // right stops at positions <= p
    const int rr = totR - rr_incl + 1;                        // rank from the right
    if (isL && rl <= cap) lpos[rl] = (uint16_t)p;
    if (isR && rr <= cap) rpos[rr] = (uint16_t)p;
    cntL += popc(mL);
    cntR += popc(mR);
  }
  totL = cntL;
  __syncthreads();
  // number of swapped pairs: ranks k with l_k < r_k (a prefix of k)
  const int kmax = min(min(totL, totR), cap);
  int npairs = 0;
  for (int kb = 1; kb <= kmax; kb += 64) {
    const int kk = kb + lane;
    const bool okp = kk <= kmax && lpos[kk] < rpos[kk];
    const uint64_t m = __ballot(okp);
    npairs += popc(m);
    if (m != ~0ull) break;
  }
  // cut = min(l_{npairs+1}, r_{npairs})
  int cut = INT32_MAX;
  if (npairs + 1 <= totL) cut = lpos[npairs + 1];
  if (npairs >= 1) cut = min(cut, (int)rpos[npairs]);
  __syncthreads();
  for (int kb = 1; kb <= npairs; kb += 64) {
    const int kk = kb + lane;
    if (kk <= npairs) swap_kv(k, v, lpos[kk], rpos[kk]);
  }
  __syncthreads();
  return cut;
}

}  // namespace

// scores: window-major, n_cand per window (penalty applied). One wave/window.
__global__ __launch_bounds__(64) void finish_kernel(FinishArgs A, const ScanWork* __restrict__ scans,
                                                   const AngleEntry* __restrict__ angles,
                                                   const double* __restrict__ scores,
                                                   FinishOut* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = blockIdx.x;
  const int n = (int)A.n_cand;
  const int lane = threadIdx.x;
  const FinishLayout Lo = finish_layout(n);
  const int cap = Lo.cap;
  int& sp = *reinterpret_cast<int*>(smem);                    // misc: stack pointer
  double* bxy = reinterpret_cast<double*>(smem + 16);         // misc: best (x, y)
  double* keys = reinterpret_cast<double*>(smem + Lo.keys);
  uint16_t* vals = reinterpret_cast<uint16_t*>(smem + Lo.vals);
  uint16_t* lpos = reinterpret_cast<uint16_t*>(smem + Lo.lpos);
  uint16_t* rpos = reinterpret_cast<uint16_t*>(smem + Lo.rpos);
  uint32_t* bounds = reinterpret_cast<uint32_t*>(smem + Lo.bounds);
  const int nwords = Lo.nwords;
  Seg* stack = reinterpret_cast<Seg*>(smem + Lo.stack);

  const double* sc = scores + (int64_t)w * A.n_cand;
  for (int i = lane; i < n; i += 64) {
    keys[i] = sc[i];
    vals[i] = (uint16_t)i;
  }
  for (int i = lane; i < nwords; i += 64) bounds[i] = 0u;
  if (lane == 0) {
    int lg = 0;
    while ((2 << lg) <= n) ++lg;  // floor(log2 n)
    stack[0] = Seg{0, n, 2 * lg};
    sp = 1;
  }
  __syncthreads();

  // introsort loop over an explicit stack of segments (order is irrelevant:
  // segments are independent; each child inherits depth-1 as in the loop).
  while (true) {
    __syncthreads();
    const int top = sp;
    if (top == 0) break;
    const Seg s = stack[top - 1];
    __syncthreads();
    if (lane == 0) sp = top - 1;
    if (lane == 0) atomicOr(&bounds[s.first >> 5], 1u << (s.first & 31));
    const int len = s.last - s.first;
    if (len <= 16) continue;  // leaf
    if (s.depth == 0) {
      if (lane == 0) heap_sort(keys, vals, s.first, s.last);
      continue;
    }
    if (lane == 0) {
      const int mid = s.first + len / 2;
      move_median_to_first(keys, vals, s.first, s.first + 1, mid, s.last - 1);
    }
    __syncthreads();
    const int cut = partition(keys, vals, lpos, rpos, cap, s.first, s.last);
    if (lane == 0) {
      int t = sp;
      stack[t++] = Seg{cut, s.last, s.depth - 1};
      stack[t++] = Seg{s.first, cut, s.depth - 1};
      sp = t;
    }
  }
  __syncthreads();

  // final insertion sort == stable insertion sort of every segment
  for (int base = 0; base < n; base += 64) {
    const int p = base + lane;
    const bool start = p < n && ((bounds[p >> 5] >> (p & 31)) & 1u);
    if (start) {
      int end = p + 1;
      while (end < n && !((bounds[end >> 5] >> (end & 31)) & 1u)) ++end;
      for (int i = p + 1; i < end; ++i) {
        const double vk = keys[i];
        const uint16_t vv = vals[i];
        int j = i;
        while (j > p && gt(vk, keys[j - 1])) {
          keys[j] = keys[j - 1];
          vals[j] = vals[j - 1];
          --j;
        }
        keys[j] = vk;
        vals[j] = vv;
      }
    }
  }
  __syncthreads();

  // ---- ordered scans over the sorted candidates -------------------------
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
    o->count = count;
    o->best_score = best;
    o->thx = thx;
    o->thy = thy;
    o->ssum = ssum;
    if (count > 1) {  // :700-707 (atan2 of thy/ssum, thx/ssum is left to the host)
      bxy[0] = ax / ssum;
      bxy[1] = ay / ssum;
    } else {
      bxy[0] = cx(fi);
      bxy[1] = cy(fi);
    }
    o->best_x = bxy[0];
    o->best_y = bxy[1];
  }
  __syncthreads();
  const double bx = bxy[0], by = bxy[1];
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
      const int r = nang + popc(m & lanes_below());
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
  hipLaunchKernelGGL(finish_kernel, dim3(n_windows), dim3(64), lds, stream, A, d_scans, d_angles,
                     d_scores, d_out);
  return hipGetLastError();
}

}  // namespace csm
