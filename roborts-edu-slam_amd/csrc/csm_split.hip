// csm_split.hip — scoring kernel for launches of few windows (the reference's
// own calling pattern: one scan, three levels, ScanMatchers::ScanMatch
// scan_matchers.h:238-256 through slam_processor.cpp:143 / :301), at any
// window step: the shipped 1 cm fine map gives integer steps of 5 and 2 cells
// and a one-cell super-fine level (config/simulatin_param.yaml:28,51-70),
// the real robot's 2.5 cm map steps of 2, 0.8 and 0.4 cells.
//
// One window has only 189-5070 candidates, so the throughput kernels (one wave
// per (window, angle)) leave most of the chip idle on it. Here the work is cut
// three ways: a lane is one candidate (its flat enumeration index q =
// (a * n + j) * n + k, correlate_scan_matcher.h:552-583), a 256-lane block a
// chunk of 256 consecutive candidates, and a window's beams are split over
// `splits` blocks per chunk (<= 32 beams each). Every lane recomputes its
// beam endpoints with the reference's expressions (LUT rotation :179-180,
// cell :647-648, x_j / y_k :569-572), so no margin argument is needed at any
// step size, and gathers (value - outside) * 2^E from the fixed-point grid
// (out-of-grid cells fail the buffer range check and read 0 = `outside`).
// The int32 partial sums go to a slab; the last block of a chunk to arrive
// (agent-scope release/acquire around one counter, cdna_hip_programming.md
// "in-launch split-K reduction") adds the splits in int64 and writes the
// penalised scores (:659, :718-745). Integer sums are exact, so the split
// changes nothing: scores equal the reference's bit for bit.
//
// A single window whose angle table fits travels in the kernel arguments
// (no copies before the launch); block 0 writes it to the device buffers the
// finish reads, and zeroes the finish's flagged-window count.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_device.hpp"
#include "csm_internal.hpp"

#pragma clang fp contract(off)

namespace csm {
namespace {

constexpr int kT = kSplitThreads;
constexpr int kUnroll = 8;

__global__ __launch_bounds__(kT) void score_split_kernel(LevelWork L, SplitWork W, const ScanWork* __restrict__ scans,
                                                         const double2* __restrict__ pts,
                                                         const AngleEntry* __restrict__ angles,
                                                         double* __restrict__ out) {
  __shared__ int32_t sh_last[1];
  const int tid = threadIdx.x;
  if (blockIdx.x == 0) {
    if (W.clear_word && tid == 0) *W.clear_word = 0;
    if (W.inline_window) {
      if (tid == 0) *W.scans_out = W.sw;
      for (int t = tid; t < L.n_angles; t += kT) W.angles_out[t] = W.ang[t];
    }
  }
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);  // a chunk's splits share an XCD
  const int split = bid % W.splits;
  const int rest = bid / W.splits;
  const int chunk = rest % W.chunks;
  const int win = rest / W.chunks;
  const ScanWork S = W.inline_window ? W.sw : scans[win];
  const AngleEntry* __restrict__ ang = W.inline_window ? W.ang : angles + S.angle_off;

  const int ns = L.n_space;
  const int nss = ns * ns;
  const int q = chunk * kT + tid;
  const bool valid = q < L.n_cand;
  const int qc = valid ? q : 0;
  const int a = qc / nss;
  const int r = qc - a * nss;
  const int j = r / ns;
  const int k = r - j * ns;
  const AngleEntry ae = ang[a];
  const double f = L.step_cells;
  const double x = S.x0 + j * f;  // :569
  const double y = S.y0 + k * f;  // :572

  const int32_t* gi = L.gridi + (int64_t)S.grid_index * L.gridi_stride;
  const uint32_t glo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)gi);
  const uint32_t ghi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)gi >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)ghi << 32) | glo), (short)0, (int)(L.gridi_stride * 4), 0x00020000);
  const int sx = L.size_x, sy = L.size_y;
  const int sx4 = L.pitch * 4;
  const double2* __restrict__ P = pts + S.pts_off;
  const int step = S.step;
  const int lo = (int)((int64_t)split * S.n_used / W.splits);
  const int hi = (int)((int64_t)(split + 1) * S.n_used / W.splits);

  // <= 32 beams of |value| < 2^26: the int32 sum cannot overflow (host check)
  int32_t acc = 0;
  for (int b0 = lo; b0 < hi; b0 += kUnroll) {
    int32_t v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int b = min(b0 + u, hi - 1);
      const double2 p = P[(int64_t)b * step];
      const double lx = ae.cosine * p.x - ae.sine * p.y;  // :179
      const double ly = ae.sine * p.x + ae.cosine * p.y;  // :180
      const int gx = (int)((lx + x) + 0.5);               // :647
      const int gy = (int)((ly + y) + 0.5);               // :648
      // off the grid (x, y or a beam past hi): an offset that fails the range check
      const bool in = ((unsigned)gx < (unsigned)sx) & ((unsigned)gy < (unsigned)sy) & (b0 + u < hi);
      const int off = in ? gy * sx4 + gx * 4 : -(1 << 30);
      v[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) acc += v[u];
  }

  // slab hand-off: plain stores, release, one ticket per chunk
  const int64_t cidx = (int64_t)win * W.chunks + chunk;
  int32_t* slab = W.slab + cidx * W.splits * kT;
  slab[split * kT + tid] = acc;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int ticket = __hip_atomic_fetch_add(W.arrive + cidx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_last[0] = ticket == W.splits - 1;
  }
  __syncthreads();
  if (!sh_last[0]) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W.arrive[cidx] = 0;  // ready for the next launch (kernel boundary orders it)
  }
  __syncthreads();
  int64_t sum = 0;
  for (int s = 0; s < W.splits; ++s) sum += slab[s * kT + tid];
  if (valid) {
    const double accd = (double)(sum + (int64_t)S.n_used * L.outside_i) * L.int_scale;
    out[S.out_off + q] = dev::penalized(L, S, accd, x, y, ae.angle);
  }
}

}  // namespace

hipError_t launch_score_split(const LevelWork& L, const SplitWork& W, const ScanWork* d_scans, const double* d_pts,
                              const AngleEntry* d_angles, double* d_out, hipStream_t stream) {
  const int64_t chunks = (L.n_cand + kT - 1) / kT;
  const int64_t nblk = (int64_t)L.n_scans * chunks * W.splits;
  if (!L.int_mode || nblk <= 0 || nblk > INT32_MAX || W.chunks != chunks || W.splits < 1 || !W.slab ||
      !W.arrive || L.pitch % 4 != 0 || L.n_cand > INT32_MAX)
    return hipErrorInvalidValue;
  if (W.inline_window && (L.n_scans != 1 || L.n_angles > kSplitArgAngles || !W.scans_out || !W.angles_out))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(score_split_kernel, dim3((unsigned)nblk), dim3(kT), 0, stream, L, W, d_scans,
                     reinterpret_cast<const double2*>(d_pts), d_angles, d_out);
  return hipGetLastError();
}

}  // namespace csm
