// ta_probe.hip — vector-memory address-path cost per load instruction by
// access pattern (design input for the box kernels: how the texture-address
// work of one buffer_load scales with the cache lines its lanes touch).
// Every wave issues kIters loads of the pattern over an L2-resident buffer;
// the kernel time over many waves gives ns per wave-instruction chip-wide.
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/ta_probe.hip -o tools/ubench/ta_probe && tools/ubench/ta_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kIters = 256;
constexpr int kBytes = 2 << 20;  // 2 MiB: L2-resident

// lane offset of pattern p (bytes); `it` varies the rows so loads differ
__device__ __forceinline__ int lane_off(int p, int lane, int it) {
  const int row = 2048;  // bytes per "grid row"
  const int r0 = (it * 37) & 511;
  switch (p) {
    case 0: return r0 * row + 16 * lane;                                  // contiguous 1 KB
    case 1: return (r0 + lane) * row;                                     // 64 rows, 16-B aligned
    case 2: return (r0 + lane) * row + 4;                                 // 64 rows, 4-B offset, inside a 64-B line
    case 3: return (r0 + lane) * row + 52;                                // 64 rows, straddles a 64-B line
    case 4: return (r0 + (lane >> 2)) * row + 16 * (lane & 3);            // 16 rows x 64 B aligned
    case 5: return (r0 + (lane >> 2)) * row + 16 * (lane & 3) + 4;        // 16 rows x 64 B, 4-B offset
    case 6: return (r0 + (lane & 15)) * row + 16 * (lane >> 4) + 100;     // 16 rows x 64 B (other lane order)
    case 7: return (r0 + (lane >> 3)) * row + 16 * (lane & 7);            // 8 rows x 128 B aligned
    case 8: return (r0 + (lane & 15)) * row;                             // 16 rows, 4 lanes per address
    case 9: return (r0 + (lane >> 1)) * row + 64 * (lane & 1) + 4;        // 32 rows, 2 lanes x (64+..)
    default: return 0;
  }
}

template <int W>
__global__ __launch_bounds__(64) void probe(const int* __restrict__ buf, int p, int* __restrict__ out) {
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, kBytes, 0x00020000);
  const int lane = threadIdx.x;
  const int wofs = (blockIdx.x & 7) * 64;  // a few distinct column bases
  int acc = 0;
#pragma unroll 8
  for (int it = 0; it < kIters; ++it) {
    const int o = lane_off(p, lane, it + blockIdx.x) + wofs;
    if (W == 16) {
      v4i v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, 0);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    } else {
      acc ^= __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0);
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  int* buf;
  int* out;
  CHECK(hipMalloc(&buf, kBytes + 4096));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 1, kBytes + 4096));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int blocks = 61440;
  const char* names[] = {"contig1KB", "64rows_al16", "64rows_off4", "64rows_straddle64", "16rows_x64B_al",
                         "16rows_x64B_off4", "16rows_x64B_perm+100", "8rows_x128B_al", "16rows_4lanes_same",
                         "32rows_x2"};
  for (int w : {16, 4}) {
    for (int p = 0; p < 10; ++p) {
      for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipEventRecord(a));
        if (w == 16)
          hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(64), 0, 0, buf, p, out);
        else
          hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(64), 0, 0, buf, p, out);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep == 1)
          std::printf("b%-2d %-22s %8.3f ms  %7.3f ns/wave-inst chip  %6.1f cyc/inst/CU@2.4GHz\n", w, names[p], ms,
                      ms * 1e6 / ((double)blocks * kIters), ms * 1e-3 * 2.4e9 * 256 / ((double)blocks * kIters));
      }
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
