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
// (one agent-scope counter, write-through slab stores and loads) adds the
// splits in int64 and writes the
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
  CSM_TS_MIN(0);
  if (blockIdx.x == 0) {
    if (W.clear_word && tid == 0)
      __hip_atomic_store(reinterpret_cast<uint64_t*>(W.clear_word), (uint64_t)(uint32_t)W.clear_tag << 32,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // {count 0, tag} (dev::clear_word)
    if (W.inline_window) {
      if (tid == 0) *W.scans_out = W.sw;
      for (int t = tid; t < L.n_angles; t += kT) W.angles_out[t] = W.ang[t];
    }
  }
  // xcd_remap gives each XCD a contiguous range of about nwg / 8 blocks, so a
  // chunk's consecutive splits usually share an XCD, but a chunk may straddle
  // two ranges. The slab hand-off does not rely on sharing one: the partials
  // are stored write-through (sc1) and the last block reads them with sc1
  // loads that miss the local L2, so a block on another XCD sees them.
  const int bid = dev::xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid % W.splits;
  const int rest = bid / W.splits;
  const int chunk = rest % W.chunks;
  const int win = rest / W.chunks;
  const ScanWork S = W.inline_window ? W.sw : scans[win];
  const AngleEntry* __restrict__ ang = W.inline_window ? W.ang : angles + S.angle_off;

  // Lanes run x-fastest inside a row of the window (item i = (a * n + k) * n
  // + j), not in flat order: at a 5-cell step the flat order (y fastest)
  // sends every lane of a gather to its own row, the x order lets ~13 lanes
  // share 2-3 cache lines. The candidate's flat index is (a * n + j) * n + k.
  const int ns = L.n_space;
  const int nss = ns * ns;
  const int i = chunk * kT + tid;
  const bool valid = i < L.n_cand;
  const int ic = valid ? i : 0;
  const int a = ic / nss;
  const int r = ic - a * nss;
  const int k = r / ns;
  const int j = r - k * ns;
  const int q = (a * ns + j) * ns + k;
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

  CSM_TS_MAX(1);  // gathers issued and summed
  // Slab hand-off without fences (MI355X_MICROARCH.md, hand-offs with sc1
  // loads in place of the acquire, first row): every slab store and load is
  // an agent-scope (sc1, write-through / L1-bypassing) access, every storing
  // wave waits for its stores, one lane per block adds to the chunk's counter
  // behind a barrier, and the block whose add returned splits - 1 reads the
  // slab after that add has returned (the barrier passes it on). A release /
  // acquire fence pair here cost ~3.4 us on the level's critical path.
  const int64_t cidx = (int64_t)win * W.chunks + chunk;
  int32_t* slab = W.slab + cidx * W.splits * kT;
  const uint32_t slo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)slab);
  const uint32_t shi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)slab >> 32));
  const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)shi << 32) | slo), (short)0, W.splits * kT * 4, 0x00020000);
  constexpr int kSc1 = 16;  // cache policy sc1: write-through stores, L1-bypassing loads
  __builtin_amdgcn_raw_buffer_store_b32(acc, srsrc, (split * kT + tid) * 4, 0, kSc1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int ticket = __hip_atomic_fetch_add(W.arrive + cidx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_last[0] = ticket == W.splits - 1;
  }
  __syncthreads();
  CSM_TS_MAX(2);  // tickets drawn
  if (!sh_last[0]) return;
  if (tid == 0)  // ready for the next launch (the kernel boundary orders it)
    __hip_atomic_store(W.arrive + cidx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // every split's partial in flight at once (sc1 loads), then the int64 sum
  int64_t sum = 0;
  for (int s0 = 0; s0 < W.splits; s0 += kUnroll) {
    int32_t v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      v[u] = __builtin_amdgcn_raw_buffer_load_b32(srsrc, s0 + u < W.splits ? ((s0 + u) * kT + tid) * 4 : -(1 << 30), 0,
                                                  kSc1);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) sum += v[u];
  }
  if (valid) {
    const double accd = (double)(sum + (int64_t)S.n_used * L.outside_i) * L.int_scale;
    out[S.out_off + q] = dev::penalized(L, S, accd, x, y, ae.angle);
  }
  CSM_TS_MAX(3);  // chunk reduced, scores written
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

#ifdef CSM_TRACE_SMALL
// Trace readout for tools/small_trace.py: copies the stamps, then resets them
// (slot 0 and 16 to the maximum for the min stamps, the rest to 0).
extern "C" int csm_debug_small_trace(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(csm::dev::g_small_trace), 64 * 8) != hipSuccess) return -1;
  unsigned long long init[64] = {0};
  init[0] = init[16] = ~0ull;
  return hipMemcpyToSymbol(HIP_SYMBOL(csm::dev::g_small_trace), init, 64 * 8) == hipSuccess ? 0 : -1;
}
#endif
