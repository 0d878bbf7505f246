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

hipError_t launch_angle_trig(AngleEntry* d_rows, int64_t n, const double* d_tab, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  if (blocks > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(angle_trig_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_rows, n, d_tab);
  return hipGetLastError();
}

}  // namespace csm
