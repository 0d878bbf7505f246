// Micro-benchmark: TA cost of the box kernel's 13-row x 64-byte row-piece
// load (52 lanes of buffer_load_dwordx4, csm_box.hip) by how the row windows
// sit in 128-byte lines: (a) corners at any dword (1.47 lines per row),
// (b) two copies of the grid, the second shifted by 64 bytes, each corner
// read from the copy where its row window fits one line (1 line per row,
// twice the footprint), (c) every corner line-aligned (the lower bound).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/box_lines.hip -o build/box_lines && build/box_lines
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kSX = 2016, kSY = 2000;  // pitch (dwords, 128-byte aligned rows: 63 lines), rows
constexpr int kIters = 2048;

template <int MODE>
__global__ __launch_bounds__(64) void box_lines(const int* __restrict__ g, int* __restrict__ out, int seed) {
  const int lane = threadIdx.x;
  const int bytes = kSX * kSY * 4 * (MODE == 1 ? 2 : 1);
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, bytes, 0x00020000);
  const int row = lane < 52 ? lane / 4 : 0, piece = lane < 52 ? lane % 4 : 0;
  const int voff = row * kSX * 4 + piece * 16;
  unsigned s = seed * 2654435761u + blockIdx.x * 40503u;
  int cx = 100 + (int)(s % 1700), cy = 100 + (int)((s >> 11) % 1700);
  int acc = 0;
  for (int it = 0; it < kIters; it += 8) {
    int so[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s = s * 1664525u + 1013904223u;
      cx += (int)((s >> 20) % 5) - 2;
      cy += (int)((s >> 24) % 5) - 2;
      cx = cx < 0 ? 0 : (cx > kSX - 64 ? kSX - 64 : cx);
      cy = cy < 0 ? 0 : (cy > kSY - 32 ? kSY - 32 : cy);
      int x = cx;
      int base = 0;
      if (MODE == 1 && (x & 31) > 16) {  // the shifted copy: window at x + 16 there
        base = kSX * kSY * 4;
        x += 16;
      }
      if (MODE == 2) x &= ~31;
      so[j] = __builtin_amdgcn_readfirstlane(base + cy * kSX * 4 + x * 4);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, so[j], 0);
      acc += v[0] + v[1] + v[2] + v[3];
    }
  }
  out[blockIdx.x * 64 + lane] = acc;
}

template <int MODE>
void run(const int* g, int* out, const char* name) {
  const int blocks = 256 * 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((box_lines<MODE>), dim3(blocks), dim3(64), 0, 0, g, out, 1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((box_lines<MODE>), dim3(blocks), dim3(64), 0, 0, g, out, r + 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double insts = (double)blocks * kIters;
  std::printf("%-44s %8.3f ms  %6.2f cyc/inst/CU\n", name, ms, ms * 1e-3 * 2.4e9 * 256 / insts);
}

int main() {
  int* g;
  int* out;
  hipMalloc(&g, (size_t)kSX * kSY * 4 * 2);
  hipMalloc(&out, 256 * 16 * 64 * 4);
  hipMemset(g, 1, (size_t)kSX * kSY * 4 * 2);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(g, out, "(a) corners at any dword");
    run<1>(g, out, "(b) two copies, window in one line");
    run<2>(g, out, "(c) line-aligned corners (bound)");
  }
  return 0;
}
