// csm_gridmap.hip — HIP kernels of the device-resident occupancy-grid maps
// (SURVEY.md 8f rows f1 and f4). Host bookkeeping and the C ABI are in
// csm_gridmap.cpp; the reference code each kernel replaces is cited per kernel
// (paths relative to the reference root).
//
// Cells are separate arrays in HBM (prob, pass, hit, update_index, touched),
// row-major with the map's row length. Every cell update is done by exactly one
// thread per scan, in the reference's per-cell event order, so float results
// are the reference's bit for bit; raises to a maximum (the blur splat) use
// integer atomicMax on the float bits, valid because probabilities are never
// negative.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_gridmap_internal.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ bool in_map(const GmCells& C, int x, int y, int tol) {
  // PointInMap(x, y, half_kernel_size_ + 1) (grid_map_base.h:344-352) on ints
  return x > tol && x < C.size_x - tol && y > tol && y < C.size_y - tol;
}

// ---- cell functions (grid_map_cell.h) -----------------------------------------------
__device__ __forceinline__ void cell_set_occupied(const GmCells& C, const GmOps& P, int64_t i) {
  if (P.kind == kGmCount) {  // CountCellFunctions::UpdateSetOccupied :94-101
    const float h = C.hit[i] + (1.0f + P.occu_factor);
    const float p = C.pass[i] + (1.0f + P.free_factor);
    float v = h / p;
    if (v > 1.0f) v = 1.0f;
    C.hit[i] = h;
    C.pass[i] = p;
    C.prob[i] = v;
  } else {  // ProbabilityCellFunctions::UpdateSetOccupied :339-343
    float v = C.prob[i] + P.occu_factor;
    if (v > 1.0f) v = 1.0f;
    C.prob[i] = v;
  }
}
__device__ __forceinline__ void cell_set_free(const GmCells& C, const GmOps& P, int64_t i) {
  if (P.kind == kGmCount) {  // :103-106
    const float p = C.pass[i] + (1.0f + P.free_factor);
    C.pass[i] = p;
    C.prob[i] = C.hit[i] / p;
  } else {  // :345-349
    float v = C.prob[i] - P.free_factor;
    if (v < 0.0f) v = 0.0f;
    C.prob[i] = v;
  }
}
__device__ __forceinline__ void cell_unset_free(const GmCells& C, const GmOps& P, int64_t i) {
  if (P.kind == kGmCount) {  // :108-111
    const float p = C.pass[i] - (1.0f + P.free_factor);
    C.pass[i] = p;
    C.prob[i] = C.hit[i] / p;
  } else {  // :351-355
    float v = C.prob[i] + P.free_factor;
    if (v > 1.0f) v = 1.0f;
    C.prob[i] = v;
  }
}
// ProbabilityCellFunctions::SetGridProbability (:361-365) as a max: the
// splat only ever raises values, so applying raises in any order gives the
// sequential result.
__device__ __forceinline__ void raise_prob(float* prob, int64_t i, float p) {
  if (prob[i] < p) atomicMax(reinterpret_cast<unsigned int*>(prob + i), __float_as_uint(p));
}
// The fixed-point mirror (GmCells::fpm) of a cell: the fixed_point_kernel's
// expression (csm_kernels.hip). The map is monotone in the value, so raising
// the mirror to the max of the raises keeps it equal to the raised cell.
__device__ __forceinline__ int32_t fixed_of(const GmCells& C, float p) {
  return (int32_t)(((double)p - (double)C.fpm_outside) * C.fpm_scale);
}
__device__ __forceinline__ void raise_mirror(const GmCells& C, int64_t x, int64_t y, float p) {
  if (!C.fpm) return;
  int32_t* a = C.fpm + y * C.fpm_pitch + x;
  const int32_t q = fixed_of(C, p);
  if (*a < q) atomicMax(a, q);
}

// LineVisitor::ErgodLineBresenhami (occu_grid_map.h:125-188) in closed form:
// after the reference's swaps, iteration t visits x0 + t and has taken
// floor((2 t dy + dx) / (2 dx)) y steps (its error term stays in [-dx, dx)).
struct Line {
  int x0, y0, dx, dy, ystep;
  bool steep;
  __device__ Line(int ax, int ay, int bx, int by) {
    steep = abs(by - ay) > abs(bx - ax);
    if (steep) {
      int t = ax;
      ax = ay;
      ay = t;
      t = bx;
      bx = by;
      by = t;
    }
    if (ax > bx) {
      int t = ax;
      ax = bx;
      bx = t;
      t = ay;
      ay = by;
      by = t;
    }
    x0 = ax;
    y0 = ay;
    dx = bx - ax;
    dy = abs(by - ay);
    ystep = ay < by ? 1 : -1;
  }
  __device__ __forceinline__ void at(int t, int& x, int& y) const {
    const int c = dx ? (int)((2ll * t * dy + dx) / (2ll * dx)) : 0;
    const int X = x0 + t, Y = y0 + ystep * c;
    x = steep ? Y : X;
    y = steep ? X : Y;
  }
};

// Blur splat, just_update_occu mode (SetCellOccuBlur :531-576 with
// just_update_occu_): one thread per (endpoint, kernel cell).
__global__ __launch_bounds__(kThreads) void blur_splat_kernel(const GmEnd* __restrict__ ends, int n, GmCells C,
                                                               int hk, const float* __restrict__ ktab, int tol) {
  const int ks = 2 * hk + 1, k2 = ks * ks;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (g >= (int64_t)n * k2) return;
  const int b = (int)(g / k2), k = (int)(g - (int64_t)b * k2);
  const GmEnd e = ends[b];
  if (!in_map(C, e.x, e.y, tol)) return;  // CellUpdate :476-478
  const int64_t ci = (int64_t)e.y * C.row + e.x;
  if (!(C.uidx[ci] < e.occu_idx)) return;  // :534
  if (k == 0) {  // SetGridProbability(center, 1.0f) :544
    raise_prob(C.prob, ci, 1.0f);
    raise_mirror(C, e.x, e.y, 1.0f);
  }
  const int i = k % ks - hk, j = k / ks - hk;  // kernel_index = (i+hk) + ks*(j+hk) :563
  const int64_t c = (int64_t)(e.y + j) * C.row + (e.x + i);
  const float p = ktab[k];  // (float)(kernel_value * cell_occu_prob_offset_) :567
  if (p <= 1.0f) {
    raise_prob(C.prob, c, p);
    raise_mirror(C, e.x + i, e.y + j, p);
  }
  C.touched[c] = 1;  // map_update_point_.push_back :571
}

// Occupied endpoints without lines (SetCellOccu :512-529): the first endpoint
// of the scan in a cell takes the update (update_index_ guard as an atomic max).
__global__ __launch_bounds__(kThreads) void occupied_once_kernel(const GmEnd* __restrict__ ends, int n, GmCells C,
                                                                  GmOps P, int tol) {
  const int b = blockIdx.x * kThreads + threadIdx.x;
  if (b >= n) return;
  const GmEnd e = ends[b];
  if (!in_map(C, e.x, e.y, tol)) return;
  const int64_t ci = (int64_t)e.y * C.row + e.x;
  C.touched[ci] = 1;
  const int old = atomicMax(C.uidx + ci, e.occu_idx);
  if (old < e.occu_idx) {
    if (old == e.free_idx) cell_unset_free(C, P, ci);
    cell_set_occupied(C, P, ci);
  }
}

// Lines + endpoints, pass 1 (UpdateMapByRange :312-321 without
// just_update_occu_): one wave per ray, lanes over the line. Each line cell
// learns the first ray that crosses it (key: scan sequence, then the lowest
// ray), each endpoint cell that some ray ends in it this scan.
__global__ __launch_bounds__(kThreads) void line_events_kernel(const GmEnd* __restrict__ ends, int n, int sx,
                                                                int sy, GmCells C, uint64_t* __restrict__ fkey,
                                                                uint32_t* __restrict__ oseq, uint32_t seq, int tol) {
  const int b = blockIdx.x * (kThreads / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= n) return;
  const GmEnd e = ends[b];
  const Line L(sx, sy, e.x, e.y);
  const uint64_t key = ((uint64_t)seq << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)b);
  for (int t = lane; t <= L.dx; t += 64) {
    int x, y;
    L.at(t, x, y);
    if (!in_map(C, x, y, tol)) continue;  // CellUpdate :476-478 per line cell
    const int64_t c = (int64_t)y * C.row + x;
    atomicMax(reinterpret_cast<unsigned long long*>(fkey + c), (unsigned long long)key);
    C.touched[c] = 1;
  }
  if (lane == 0 && in_map(C, e.x, e.y, tol)) oseq[(int64_t)e.y * C.row + e.x] = seq;
}

// Pass 2: the first ray through a cell applies the cell's whole event
// sequence of this scan. A ray's own endpoint lies on its line, so every
// endpoint cell was crossed first: free (SetCellFree :499-510), then, if some
// ray ends there, unset-free + occupied (SetCellOccu :512-529).
__global__ __launch_bounds__(kThreads) void line_apply_kernel(const GmEnd* __restrict__ ends, int n, int sx, int sy,
                                                               GmCells C, GmOps P, const uint64_t* __restrict__ fkey,
                                                               const uint32_t* __restrict__ oseq, uint32_t seq,
                                                               int tol) {
  const int b = blockIdx.x * (kThreads / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= n) return;
  const GmEnd e = ends[b];
  const Line L(sx, sy, e.x, e.y);
  const uint64_t key = ((uint64_t)seq << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)b);
  for (int t = lane; t <= L.dx; t += 64) {
    int x, y;
    L.at(t, x, y);
    if (!in_map(C, x, y, tol)) continue;
    const int64_t c = (int64_t)y * C.row + x;
    if (fkey[c] != key) continue;
    int u = C.uidx[c];
    if (u < e.free_idx) {
      cell_set_free(C, P, c);
      u = e.free_idx;
    }
    if (oseq[c] == seq && u < e.occu_idx) {
      if (u == e.free_idx) cell_unset_free(C, P, c);
      cell_set_occupied(C, P, c);
      u = e.occu_idx;
    }
    C.uidx[c] = u;
  }
}

// MapFeedbackResponsePenalty (occu_grid_map.h:331-392): one wave per checked
// ray; a ray counts once if any line cell is occupied farther than the bound
// tolerance from its endpoint (CheckOccuLineVisitorCallback :447-471; the
// per-ray result saturates at 1). min_d2: smallest squared cell distance whose
// sqrt exceeds the tolerance (host).
__global__ __launch_bounds__(kThreads) void feedback_kernel(const GmEnd* __restrict__ ends, int n, int sx, int sy,
                                                             GmCells C, GmOps P, int use_blur, float occu_offset_f,
                                                             double occu_offset, int64_t min_d2,
                                                             int* __restrict__ count) {
  const int b = blockIdx.x * (kThreads / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= n) return;
  (void)occu_offset_f;
  const GmEnd e = ends[b];
  const Line L(sx, sy, e.x, e.y);
  bool hit = false;
  for (int t = lane; t <= L.dx; t += 64) {
    int x, y;
    L.at(t, x, y);
    if (x < 0 || y < 0 || x >= C.size_x || y >= C.size_y) continue;  // defined: not occupied
    const int64_t c = (int64_t)y * C.row + x;
    bool occ;
    if (use_blur) {
      occ = (double)C.prob[c] > occu_offset;
    } else if (P.kind == kGmCount) {  // CountCellFunctions::GetGridStates :125-136
      occ = C.pass[c] >= P.min_pass && !(C.prob[c] < P.occu_threshold);
    } else {  // ProbabilityCellFunctions::GetGridStates :367-375
      occ = C.prob[c] > 0.5f;
    }
    if (occ) {
      const int64_t dx = (int64_t)e.x - x, dy = (int64_t)e.y - y;
      if (dx * dx + dy * dy >= min_d2) hit = true;
    }
  }
  if (__builtin_amdgcn_ballot_w64(hit) != 0 && lane == 0) atomicAdd(count, 1);
}

// `new CellType[n]{default_cell_prob_}` (grid_map_base.h:160,214): element 0
// from default_cell_prob_, the others default-constructed (kDefaultCellProb).
__global__ __launch_bounds__(kThreads) void fresh_kernel(GmCells C, int64_t n, float first) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    C.prob[i] = i == 0 ? first : 0.5f;
    if (C.pass) {
      C.pass[i] = 0.0f;
      C.hit[i] = 0.0f;
    }
    C.uidx[i] = -1;
    C.touched[i] = 0;
  }
}

// Reset (grid_map_base.h:95-103) or, with only_touched, ResetValueSpeedup
// over map_update_point_ (:112-117); clear_touched: the list is cleared
// afterwards (InitMapWithRangeVec :237; Reset() alone keeps it).
__global__ __launch_bounds__(kThreads) void reset_kernel(GmCells C, int64_t n, float v, int only_touched,
                                                          int clear_touched) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    if (only_touched && !C.touched[i]) continue;
    C.prob[i] = v;
    if (C.fpm) {
      const int64_t y = i / C.row;
      C.fpm[y * C.fpm_pitch + (i - y * C.row)] = fixed_of(C, v);
    }
    if (C.pass) {
      C.pass[i] = 0.0f;
      C.hit[i] = 0.0f;
    }
    C.uidx[i] = -1;
    if (clear_touched) C.touched[i] = 0;
  }
}

// ExtendSize (grid_map_base.h:182-244): old rows to their place in the grown
// grid; map_update_point_ keeps its linear indices, so the touched flags are
// copied linearly.
__global__ __launch_bounds__(kThreads) void extend_copy_kernel(GmCells O, GmCells N, int gx, int gy) {
  const int64_t n_old = (int64_t)O.row * O.size_y;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n_old; i += (int64_t)gridDim.x * kThreads) {
    const int r = (int)(i / O.row), x = (int)(i - (int64_t)r * O.row);
    const int64_t d = (int64_t)(gy + r) * N.row + (gx + x);
    N.prob[d] = O.prob[i];
    if (N.pass) {
      N.pass[d] = O.pass[i];
      N.hit[d] = O.hit[i];
    }
    N.uidx[d] = O.uidx[i];
    N.touched[i] = O.touched[i];
  }
}

unsigned grid_for(int64_t n) {
  int64_t b = (n + kThreads - 1) / kThreads;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

hipError_t gm_launch_fresh(const GmCells& C, int64_t n, float first, hipStream_t s) {
  hipLaunchKernelGGL(fresh_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, C, n, first);
  return hipGetLastError();
}
hipError_t gm_launch_reset(const GmCells& C, int64_t n, float v, bool only_touched, bool clear_touched,
                           hipStream_t s) {
  hipLaunchKernelGGL(reset_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, C, n, v, only_touched ? 1 : 0,
                     clear_touched ? 1 : 0);
  return hipGetLastError();
}
hipError_t gm_launch_extend_copy(const GmCells& O, const GmCells& N, int gx, int gy, hipStream_t s) {
  hipLaunchKernelGGL(extend_copy_kernel, dim3(grid_for((int64_t)O.row * O.size_y)), dim3(kThreads), 0, s, O, N, gx,
                     gy);
  return hipGetLastError();
}
hipError_t gm_launch_blur(const GmEnd* ends, int n, const GmCells& C, int hk, const float* ktab, int tol,
                          hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t total = (int64_t)n * (2 * hk + 1) * (2 * hk + 1);
  hipLaunchKernelGGL(blur_splat_kernel, dim3((unsigned)((total + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                     ends, n, C, hk, ktab, tol);
  return hipGetLastError();
}
hipError_t gm_launch_occupied(const GmEnd* ends, int n, const GmCells& C, const GmOps& P, int tol, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(occupied_once_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                     ends, n, C, P, tol);
  return hipGetLastError();
}
hipError_t gm_launch_lines(const GmEnd* ends, int n, int sx, int sy, const GmCells& C, const GmOps& P,
                           uint64_t* fkey, uint32_t* oseq, uint32_t seq, int tol, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n + 3) / 4);
  hipLaunchKernelGGL(line_events_kernel, dim3(nb), dim3(kThreads), 0, s, ends, n, sx, sy, C, fkey, oseq, seq, tol);
  hipLaunchKernelGGL(line_apply_kernel, dim3(nb), dim3(kThreads), 0, s, ends, n, sx, sy, C, P, fkey, oseq, seq, tol);
  return hipGetLastError();
}
hipError_t gm_launch_feedback(const GmEnd* ends, int n, int sx, int sy, const GmCells& C, const GmOps& P,
                              int use_blur, double occu_offset, int64_t min_d2, int* count, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(feedback_kernel, dim3((unsigned)((n + 3) / 4)), dim3(kThreads), 0, s, ends, n, sx, sy, C, P,
                     use_blur, (float)occu_offset, occu_offset, min_d2, count);
  return hipGetLastError();
}

}  // namespace csm
