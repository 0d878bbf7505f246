// csm_device.hpp — device helpers shared by the scoring kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "csm_internal.hpp"

namespace csm {
namespace dev {

// XCD-aware, bijective block remap (cdna_hip_programming.md T1): blocks that
// share a logical neighbourhood (one window) land on one XCD's L2.
// LevelWork::clear_word: block 0, lane 0 of a scoring kernel clears it. An
// agent-scope store: the fused finish's appends (csm_tail.hpp list_append) on
// other XCDs wait for it and add to the same word inside this launch, so it
// must not sit dirty in block 0's XCD L2 (a later write-back would also undo
// their adds).
__device__ __forceinline__ void clear_word(const LevelWork& L) {
  if (L.clear_word && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(L.clear_word), (uint64_t)(uint32_t)L.clear_tag << 32,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // {count 0, tag}
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// Divisor (:659) and centre penalty (:718-745) of one candidate.
__device__ __forceinline__ double penalized(const LevelWork& L, const ScanWork& S, double acc, double x,
                                           double y, double angle) {
  double score = acc / S.divisor;
  if (L.use_penalty) {
    // util::DoubleEqual(score, 0.0) with kDoubleTolerance = 1e-6.
    const bool is_zero = (score < 0.0) ? (score >= -1e-06) : (score <= 1e-06);
    if (!is_zero) {
      const double dx = x - S.cx, dy = y - S.cy;
      double d2 = dx * dx + dy * dy;
      d2 *= (L.mres * L.mres);
      double dp = 1.0 - (L.dist_gain * d2 / (L.size / 2));
      dp = dp < 0.5 ? 0.5 : dp;  // std::max(dp, 0.5)
      double da = angle - S.ct;
      da = da * da;
      double ap = 1.0 - (0.25 * da / 0.349);
      ap = ap < 0.9 ? 0.9 : ap;
      score = score * (dp * ap);
    }
  }
  return score;
}

__device__ __forceinline__ bool better(double s, int64_t f, double bs, int64_t bf) {
  return (s > bs) || (s == bs && f < bf);
}

// 16-byte buffer load written straight into LDS at lds + 16 * lane. The
// builtin has no host-side form; the guard only keeps hipcc's host pass (which
// must still emit the kernel's launch stub) from seeing it.
__device__ __forceinline__ void buffer_load_lds16(__amdgpu_buffer_rsrc_t rsrc,
                                                  __attribute__((address_space(3))) int32_t* lds,
                                                  int voffset) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, lds, 16, voffset, 0, 0, 0);
#endif
}

__device__ __forceinline__ double bcast_lane(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Cross-lane sums without the LDS unit (ds_bpermute): DPP within a row of 16
// lanes, v_permlane16_swap / v_permlane32_swap (CDNA4) across rows. For sums
// whose order does not matter only: exact integers (the kernels' fixed-point
// sums, also when held in doubles below 2^53).
// Lane l's value plus lane (l ^ 16)'s / (l ^ 32)'s: a swap of x with itself
// leaves (x, partner) in one of the two results and (partner, x) in the other
// for every lane, so their sum is x + partner in every lane.
template <bool ROWS32>
__device__ __forceinline__ uint64_t swap_sum_u64(uint64_t u) {
  const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
  if constexpr (ROWS32) {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return (((uint64_t)h[0] << 32) | l[0]) + (((uint64_t)h[1] << 32) | l[1]);
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return (((uint64_t)h[0] << 32) | l[0]) + (((uint64_t)h[1] << 32) | l[1]);
  }
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t u) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
// The sum of v over the wave, in every lane (two's-complement int64: exact).
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
  uint64_t u = (uint64_t)v;
  u += dpp_u64<0xB1>(u);   // quad_perm [1,0,3,2]: pairs
  u += dpp_u64<0x4E>(u);   // quad_perm [2,3,0,1]: quads
  u += dpp_u64<0x141>(u);  // row_half_mirror: 8 lanes
  u += dpp_u64<0x140>(u);  // row_mirror: the row of 16
  u = swap_sum_u64<false>(u);  // two rows
  u = swap_sum_u64<true>(u);   // the wave
  return (int64_t)u;
}

// CSM_TRACE_SMALL builds: wall-clock stamps (100 MHz) of the few-window
// kernels' phases, min over blocks for slot 0 and max for the others
// (tools/small_trace.py reads them through csm_debug_small_trace).
#ifdef CSM_TRACE_SMALL
static __device__ unsigned long long g_small_trace[64];  // one per translation unit
#define CSM_TS_MIN(slot)                                                   \
  do {                                                                     \
    if (threadIdx.x == 0) atomicMin(&::csm::dev::g_small_trace[slot], wall_clock64()); \
  } while (0)
#define CSM_TS_MAX(slot)                                                   \
  do {                                                                     \
    if (threadIdx.x == 0) atomicMax(&::csm::dev::g_small_trace[slot], wall_clock64()); \
  } while (0)
#else
#define CSM_TS_MIN(slot) \
  do {                   \
  } while (0)
#define CSM_TS_MAX(slot) \
  do {                   \
  } while (0)
#endif

}  // namespace dev
}  // namespace csm
