// csm_trig.hip — a level's angle rows' cos/sin on the device.
//
// The host plans each window's angles θ_i = start + i·ares
// (AngleSearchLookUpTable::UpdateLookUpTable correlate_scan_matcher.h:161-172)
// and, on this path, leaves cos θ_i / sin θ_i to this kernel: glibc 2.35's
// sincos restated operation for operation (libm_sincos.hpp) over the table
// taken from the host's libm, so every row equals what ::sincos returns on the
// host, bit for bit. Rows outside the restated domain (|θ| >= 105414350, or
// not finite) were computed by the host and are left as copied.
//
// One lane per row: ~90 binary64 operations and four 8-byte table loads each;
// a coarse level of 2048 windows × 30 angles is 61 k rows, ~1 k waves.
#include <hip/hip_runtime.h>

#include "csm_internal.hpp"
#include "libm_sincos.hpp"

namespace csm {

__global__ __launch_bounds__(256) void angle_trig_kernel(AngleEntry* __restrict__ rows, int64_t n,
                                                         const double* __restrict__ tab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = rows[i].angle;
  if (!libm::sincos_device_ok(a)) return;
  double s, c;
  libm::sincos(a, tab, &s, &c);
  rows[i].cosine = c;
  rows[i].sine = s;
}

// The rows whole, from each window's ScanWork: θ_a = (ct - offset) + a·ares
// in plan_window_into's operations (csm_launch.cpp; correlate_scan_matcher.h
// :161-168), then its sincos. Every row of the launch must be inside the
// restated domain (the plan checks each window's end angles). Replaces the
// rows' host-to-device copy (24 bytes a row).
__global__ __launch_bounds__(256) void angle_rows_kernel(const ScanWork* __restrict__ sw, int64_t n, int n_angles,
                                                         double offset, double ares, AngleEntry* __restrict__ rows,
                                                         const double* __restrict__ tab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t w = i / n_angles;
  const int a = (int)(i - w * n_angles);
  const ScanWork& S = sw[w];
  const double start = S.ct - offset;
  const double th = start + a * ares;
  double s, c;
  libm::sincos(th, tab, &s, &c);
  AngleEntry& r = rows[S.angle_off + a];
  r.angle = th;
  r.cosine = c;
  r.sine = s;
}

hipError_t launch_angle_rows(const ScanWork* d_sw, int nw, int n_angles, double offset, double ares, AngleEntry* d_rows,
                             const double* d_tab, hipStream_t stream) {
  const int64_t n = (int64_t)nw * n_angles;
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  if (blocks > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(angle_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_sw, n, n_angles, offset, ares,
                     d_rows, d_tab);
  return hipGetLastError();
}

hipError_t launch_angle_trig(AngleEntry* d_rows, int64_t n, const double* d_tab, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  if (blocks > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(angle_trig_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_rows, n, d_tab);
  return hipGetLastError();
}

}  // namespace csm
