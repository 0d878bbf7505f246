// Micro-benchmark: the cost of the box kernel's row-piece loads (csm_box.hip)
// by load width and active lanes. Every wave walks a random-walk of box
// corners over a 2000 x 2000 int32 grid (L2/MALL-resident, like config 2's
// gridi) and issues one load per corner per lane, 8 in flight, summing the
// values. Reports ns per wave-instruction across the chip and the derived
// cycles per instruction per CU.
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/box_loads.hip -o build/box_loads && build/box_loads
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kSX = 2016, kSY = 2000;  // pitch, rows
constexpr int kIters = 2048;

template <int W, int ACTIVE>
__global__ __launch_bounds__(64) void box_loads(const int* __restrict__ g, int* __restrict__ out, int seed) {
  const int lane = threadIdx.x;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, kSX * kSY * 4, 0x00020000);
  // lane (row, piece): rows of the box, W-dword pieces
  constexpr int PER_ROW = (16 + W - 1) / W;
  const int row = lane / PER_ROW, piece = lane % PER_ROW;
  const int voff = row * kSX * 4 + piece * W * 4;
  unsigned s = seed * 2654435761u + blockIdx.x * 40503u;
  int cx = 100 + (int)(s % 1700), cy = 100 + (int)((s >> 11) % 1700);
  int acc = 0;
  for (int it = 0; it < kIters; it += 8) {
    int so[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s = s * 1664525u + 1013904223u;
      cx += (int)((s >> 20) % 5) - 2;  // neighbouring beams: corners a few cells apart
      cy += (int)((s >> 24) % 5) - 2;
      cx = cx < 0 ? 0 : (cx > kSX - 32 ? kSX - 32 : cx);
      cy = cy < 0 ? 0 : (cy > kSY - 32 ? kSY - 32 : cy);
      so[j] = __builtin_amdgcn_readfirstlane(cy * kSX * 4 + cx * 4);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ACTIVE >= 64 || lane < ACTIVE) {
        if constexpr (W == 4) {
          auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, so[j], 0);
          acc += v[0] + v[1] + v[2] + v[3];
        } else if constexpr (W == 3) {
          auto v = __builtin_amdgcn_raw_buffer_load_b96(rsrc, voff, so[j], 0);
          acc += v[0] + v[1] + v[2];
        } else if constexpr (W == 2) {
          auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, so[j], 0);
          acc += v[0] + v[1];
        } else {
          acc += __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, so[j], 0);
        }
      }
    }
  }
  out[blockIdx.x * 64 + lane] = acc;
}

template <int W, int ACTIVE>
void run(const int* g, int* out, const char* name) {
  const int blocks = 256 * 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((box_loads<W, ACTIVE>), dim3(blocks), dim3(64), 0, 0, g, out, 1);  // warm
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((box_loads<W, ACTIVE>), dim3(blocks), dim3(64), 0, 0, g, out, r + 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double insts = (double)blocks * kIters;
  const double cyc_per_inst_cu = ms * 1e-3 * 2.4e9 * 256 / insts;
  std::printf("%-28s %8.3f ms  %6.2f cyc/inst/CU  %7.1f B/lane  %6.1f useful B/cyc/CU\n", name, ms, cyc_per_inst_cu,
              4.0 * W, (double)ACTIVE * 4 * W / cyc_per_inst_cu);
}

int main() {
  int* g;
  int* out;
  hipMalloc(&g, (size_t)kSX * kSY * 4);
  hipMalloc(&out, 256 * 16 * 64 * 4);
  hipMemset(g, 1, (size_t)kSX * kSY * 4);
  run<4, 64>(g, out, "dwordx4 x64 lanes");
  run<4, 52>(g, out, "dwordx4 x52 lanes");
  run<4, 39>(g, out, "dwordx4 x39 lanes");
  run<3, 64>(g, out, "dwordx3 x64 lanes");
  run<2, 64>(g, out, "dwordx2 x64 lanes");
  run<1, 64>(g, out, "dword   x64 lanes");
  run<1, 16>(g, out, "dword   x16 lanes");
  return 0;
}
