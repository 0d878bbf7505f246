// csm_palette.hip — the palette copy of the fixed-point grid, read by the v10
// palette box kernel (csm_box.hip).
//
// A scan-match grid holds a handful of distinct cell values: the unknown
// value (0 in gridi, which stores value - outside), the occupied value and
// the levels of the blur splat (occu_grid_map.h:83-105,531-576: a cell keeps
// the max of kernel * offset). The palette is those values, 0 first then
// ascending, and the copy holds every cell's index into it, one byte per cell
// in gridi's own layout (same pitch, same zero columns and rows). A grid with
// more than kPalMax distinct values has no palette (the box kernels read
// gridi itself).
//
//   pal_collect_kernel  each block dedupes its slice of cells in an LDS hash
//                       and lists its values (or marks an overflow)
//   pal_merge_kernel    one block merges the lists, sorts them, writes the
//                       palette and its size
//   pal_index_kernel    every cell's index by binary search in the palette
//   pal_strips_kernel   (palettes of at most kPairMaxPal values) the strip
//                       copies the v11 pair box kernel reads
//   istrips_kernel      the strip copies of gridi itself that the phase
//                       kernel reads (8-cell strips, two copies)
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_internal.hpp"

namespace csm {
namespace {

constexpr int kPalHash = 1024;            // LDS hash slots (>= 2 * (kPalMax + 256))
constexpr int32_t kPalEmpty = INT32_MIN;  // never a gridi value (|value| < 2^26)
constexpr int kPalCollectBlocks = 1024;
constexpr int kPalList = kPalMax + 1;     // per block: count, then values

__device__ __forceinline__ uint32_t pal_hash(int32_t v) { return ((uint32_t)v * 2654435761u) >> 22; }

// Insert v (non-zero) into the LDS set; `count` counts the distinct values.
__device__ __forceinline__ void pal_insert(int32_t* key, int32_t* count, int32_t v) {
  if (v == 0 || *(volatile int32_t*)count > kPalMax) return;
  uint32_t h = pal_hash(v);
  for (int probe = 0; probe < kPalHash; ++probe) {
    const int32_t k = key[h];
    if (k == v) return;
    if (k == kPalEmpty) {
      const int32_t old = atomicCAS(&key[h], kPalEmpty, v);
      if (old == kPalEmpty) {
        atomicAdd(count, 1);
        return;
      }
      if (old == v) return;
    }
    h = (h + 1) & (kPalHash - 1);
  }
}

__global__ __launch_bounds__(256) void pal_collect_kernel(const int4* __restrict__ g, int64_t n4, int64_t per4,
                                                          int32_t* __restrict__ lists) {
  __shared__ int32_t key[kPalHash];
  __shared__ int32_t count, pos;
  for (int i = threadIdx.x; i < kPalHash; i += 256) key[i] = kPalEmpty;
  if (threadIdx.x == 0) {
    count = 0;
    pos = 0;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per4, b1 = min(n4, b0 + per4);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) {
    const int4 v = g[i];
    pal_insert(key, &count, v.x);
    pal_insert(key, &count, v.y);
    pal_insert(key, &count, v.z);
    pal_insert(key, &count, v.w);
  }
  __syncthreads();
  int32_t* out = lists + (int64_t)blockIdx.x * kPalList;
  if (count > kPalMax) {
    if (threadIdx.x == 0) out[0] = kPalMax + 1;
    return;
  }
  for (int i = threadIdx.x; i < kPalHash; i += 256)
    if (key[i] != kPalEmpty) out[1 + atomicAdd(&pos, 1)] = key[i];
  if (threadIdx.x == 0) out[0] = count;
}

__global__ __launch_bounds__(256) void pal_merge_kernel(const int32_t* __restrict__ lists, int nb,
                                                        int32_t* __restrict__ vals, int32_t* __restrict__ state) {
  __shared__ int32_t key[kPalHash];
  __shared__ int32_t sorted[256];
  __shared__ int32_t count, pos, over;
  for (int i = threadIdx.x; i < kPalHash; i += 256) key[i] = kPalEmpty;
  if (threadIdx.x == 0) {
    count = 0;
    pos = 0;
    over = 0;
  }
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int32_t* in = lists + (int64_t)b * kPalList;
    const int32_t c = in[0];
    if (c > kPalMax) {
      if (threadIdx.x == 0) over = 1;
      break;  // uniform: every thread read the same count
    }
    for (int i = threadIdx.x; i < c; i += 256) pal_insert(key, &count, in[1 + i]);
  }
  __syncthreads();
  // index 0 is the zero value: at most kPalMax - 1 others
  if (over || count > kPalMax - 1) {
    if (threadIdx.x == 0) state[0] = kPalMax + 1;
    return;
  }
  sorted[threadIdx.x] = INT32_MAX;
  __syncthreads();
  for (int i = threadIdx.x; i < kPalHash; i += 256)
    if (key[i] != kPalEmpty) sorted[atomicAdd(&pos, 1)] = key[i];
  __syncthreads();
  // bitonic sort of the 256 slots (padding INT32_MAX sorts last)
  const int t = threadIdx.x;
  for (int size = 2; size <= 256; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int o = t ^ stride;
      if (o > t) {
        const bool up = (t & size) == 0;
        const int32_t x = sorted[t], y = sorted[o];
        if ((x > y) == up) {
          sorted[t] = y;
          sorted[o] = x;
        }
      }
      __syncthreads();
    }
  }
  if (t == 0) vals[0] = 0;
  if (t < count) vals[1 + t] = sorted[t];
  if (t == 0) state[0] = count + 1;
}

__global__ __launch_bounds__(256) void pal_index_kernel(const int4* __restrict__ g, int64_t n4,
                                                        const int32_t* __restrict__ vals,
                                                        const int32_t* __restrict__ state,
                                                        uint32_t* __restrict__ idx4) {
  __shared__ int32_t sv[kPalMax];
  const int m = state[0];
  if (m < 1 || m > kPalMax) return;  // no palette: nothing to index
  for (int i = threadIdx.x; i < m; i += 256) sv[i] = vals[i];
  __syncthreads();
  auto find = [&](int32_t v) -> uint32_t {
    if (v == 0) return 0u;
    int lo = 1, hi = m - 1;  // sv[1..m-1] ascending; v is one of them
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sv[mid] < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    return (uint32_t)lo;
  };
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 v = g[i];
    idx4[i] = find(v.x) | (find(v.y) << 8) | (find(v.z) << 16) | (find(v.w) << 24);
  }
}

// Strip copies of the palette index grid (v11 pair box kernel): copy c holds
// cell x of row y at byte (x + kStripPadLo + kStripShift c) of its strip row,
// strips kStripW bytes wide with their rows contiguous (row y of strip t at
// (t * rows + kStripPadLo + y) * 16). One thread writes one 16-byte strip row;
// cells off the grid are index 0 but for column -1 and row -1, which repeat
// column 0 and row 0 (kStripPadLo).
__global__ __launch_bounds__(256) void pal_strips_kernel(const uint8_t* __restrict__ idx, int pitch, int sx,
                                                         int sy, int rows, int n_strips, int64_t idx_stride,
                                                         int64_t grid_bytes, int n_grids, uint4* __restrict__ out) {
  const int64_t per_copy = (int64_t)n_strips * rows;
  const int64_t total = (int64_t)n_grids * kStripCopies * per_copy;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t g = i / (kStripCopies * per_copy);
    const int64_t r = i - g * kStripCopies * per_copy;
    const int c = (int)(r / per_copy);
    const int64_t sr = r - (int64_t)c * per_copy;
    const int t = (int)(sr / rows);
    const int y = (int)(sr - (int64_t)t * rows) - kStripPadLo;
    const uint8_t* src = idx + g * idx_stride + (int64_t)max(y, 0) * pitch;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (y >= -1 && y < sy) {
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const int x = kStripW * t + b - kStripShift * c - kStripPadLo;
        const uint32_t v = (x >= -1 && x < sx) ? src[max(x, 0)] : 0u;
        w[b >> 2] |= v << (8 * (b & 3));
      }
    }
    out[(g * grid_bytes + (int64_t)c * per_copy * kStripW) / 16 + sr] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Strip copies of gridi (the phase kernel's strip form): copy c holds cell x
// of row y at cell x + kIStripPadLo + 4c of its 8-cell strip row, row y at
// strip row y + kIStripPadLo; column -1 repeats column 0 and row -1 row 0,
// other cells off the grid are 0 (the outside value). One thread per 16-byte
// half row.
__global__ __launch_bounds__(256) void istrips_kernel(const int32_t* __restrict__ gi, int pitch, int sx, int sy,
                                                      int rows, int n_strips, int64_t gi_stride, int64_t grid_ints,
                                                      int n_grids, int4* __restrict__ out) {
  const int64_t per_copy = (int64_t)n_strips * rows * 2;  // half rows
  const int64_t total = (int64_t)n_grids * kIStripCopies * per_copy;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t g = i / (kIStripCopies * per_copy);
    const int64_t r = i - g * kIStripCopies * per_copy;
    const int c = (int)(r / per_copy);
    const int64_t hr = r - (int64_t)c * per_copy;  // half row within the copy
    const int64_t sr = hr >> 1;
    const int t = (int)(sr / rows);
    const int y = (int)(sr - (int64_t)t * rows) - kIStripPadLo;
    const int x0 = kIStripCells * t + 4 * (int)(hr & 1) - 4 * c - kIStripPadLo;
    const int32_t* src = gi + g * gi_stride + (int64_t)max(y, 0) * pitch;
    int v[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int x = x0 + b;
      v[b] = (y >= -1 && y < sy && x >= -1 && x < sx) ? src[max(x, 0)] : 0;
    }
    out[(g * grid_ints + (int64_t)c * per_copy * 4) / 4 + hr] = make_int4(v[0], v[1], v[2], v[3]);
  }
}

}  // namespace

StripGeom istrip_geom(int size_x, int size_y) {
  StripGeom G{};
  G.rows = kIStripPadLo + size_y + kIStripPadRows;
  // a box row starts at cell (ix & ~3) + 4c <= kIStripPadLo + size_x - 1 + 4 in
  // copy c (ix the padded column), phase <= 3
  G.n_strips = (kIStripPadLo + size_x + 3) / kIStripCells + 1;
  G.strip_bytes = (int64_t)G.rows * kIStripCells * 4;
  G.copy_bytes = G.strip_bytes * G.n_strips;
  G.grid_bytes = G.copy_bytes * kIStripCopies;
  return G;
}

hipError_t launch_build_istrips(const int32_t* gridi, int pitch, int size_x, int size_y, int64_t gridi_stride,
                                int n_grids, int32_t* out, hipStream_t stream) {
  const StripGeom G = istrip_geom(size_x, size_y);
  if (!gridi || !out || n_grids < 1 || pitch < size_x) return hipErrorInvalidValue;
  const int64_t total = (int64_t)n_grids * kIStripCopies * G.n_strips * G.rows * 2;
  const int64_t blocks = (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
  hipLaunchKernelGGL(istrips_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, gridi, pitch, size_x, size_y,
                     G.rows, G.n_strips, gridi_stride, G.grid_bytes / 4, n_grids, reinterpret_cast<int4*>(out));
  return hipGetLastError();
}

StripGeom strip_geom(int size_x, int size_y) {
  StripGeom G{};
  G.rows = kStripPadLo + size_y + kStripPadRows;
  // a box row piece starts at (ix & ~(S - 1)) + S c <= kStripPadLo + size_x - 1 + 16 - S
  // in copy c (S = kStripShift, ix the padded column)
  G.n_strips = (kStripPadLo + size_x + 15 - kStripShift) / kStripW + 1;
  G.strip_bytes = (int64_t)G.rows * kStripW;
  G.copy_bytes = G.strip_bytes * G.n_strips;
  G.grid_bytes = G.copy_bytes * kStripCopies;
  return G;
}

hipError_t launch_build_strips(const uint8_t* idx, int pitch, int size_x, int size_y, int64_t idx_stride,
                               int n_grids, uint8_t* out, hipStream_t stream) {
  const StripGeom G = strip_geom(size_x, size_y);
  if (!idx || !out || n_grids < 1 || pitch < size_x) return hipErrorInvalidValue;
  const int64_t total = (int64_t)n_grids * kStripCopies * G.n_strips * G.rows;
  const int64_t blocks = (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
  hipLaunchKernelGGL(pal_strips_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, idx, pitch, size_x, size_y,
                     G.rows, G.n_strips, idx_stride, G.grid_bytes, n_grids, reinterpret_cast<uint4*>(out));
  return hipGetLastError();
}

int64_t pal_scratch_ints(int64_t n) {
  const int64_t n4 = n / 4;
  const int64_t nb = n4 <= 0 ? 1 : (n4 + 4095) / 4096 < kPalCollectBlocks ? (n4 + 4095) / 4096 : kPalCollectBlocks;
  return nb * kPalList;
}

hipError_t launch_build_palette(const int32_t* gridi, int64_t n, int32_t* scratch, int32_t* vals, int32_t* state,
                                uint8_t* idx, hipStream_t stream) {
  if (n <= 0 || n % 4 != 0 || !gridi || !scratch || !vals || !state || !idx) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  const int nb = (int)(pal_scratch_ints(n) / kPalList);
  const int64_t per4 = (n4 + nb - 1) / nb;
  const int4* g = reinterpret_cast<const int4*>(gridi);
  hipLaunchKernelGGL(pal_collect_kernel, dim3(nb), dim3(256), 0, stream, g, n4, per4, scratch);
  hipLaunchKernelGGL(pal_merge_kernel, dim3(1), dim3(256), 0, stream, scratch, nb, vals, state);
  const int64_t blocks = (n4 + 255) / 256 < 8192 ? (n4 + 255) / 256 : 8192;
  hipLaunchKernelGGL(pal_index_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, n4, vals, state,
                     reinterpret_cast<uint32_t*>(idx));
  return hipGetLastError();
}

}  // namespace csm
