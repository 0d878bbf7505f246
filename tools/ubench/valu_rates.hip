// Micro-benchmark: issue cost of the VALU instructions the scoring kernels
// use, one wave per SIMD (4 waves per CU), 1 CU-resident block per CU.
// Prints cycles per wave-instruction (s_memtime deltas).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define N_ITER 4096
#define REP8(x) x x x x x x x x

template <int OP>
__global__ __launch_bounds__(256) void k(int* out, int s, long long* cyc) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  long long b0 = a0, b1 = a1, b2 = a2, b3 = a3;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_ITER; ++i) {
    if constexpr (OP == 0) {  // v_add_u32 x4 per rep
      REP8(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "s"(s));)
    } else if constexpr (OP == 1) {  // v_mad_i64_i32
      REP8(asm volatile("v_mad_i64_i32 %0, s[0:1], %4, %5, %0\n v_mad_i64_i32 %1, s[0:1], %4, %5, %1\n v_mad_i64_i32 %2, s[0:1], %4, %5, %2\n v_mad_i64_i32 %3, s[0:1], %4, %5, %3" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(a0), "s"(s) : "s0", "s1");)
    } else if constexpr (OP == 2) {  // v_dot2_u32_u16
      REP8(asm volatile("v_dot2_u32_u16 %0, %4, %5, %0\n v_dot2_u32_u16 %1, %4, %5, %1\n v_dot2_u32_u16 %2, %4, %5, %2\n v_dot2_u32_u16 %3, %4, %5, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(s), "s"(s));)
    } else if constexpr (OP == 3) {  // v_dot2c_i32_i16
      REP8(asm volatile("v_dot2c_i32_i16 %0, %5, %4\n v_dot2c_i32_i16 %1, %5, %4\n v_dot2c_i32_i16 %2, %5, %4\n v_dot2c_i32_i16 %3, %5, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(s), "s"(s));)
    } else if constexpr (OP == 4) {  // v_readlane_b32 (to distinct SGPRs)
      REP8(asm volatile("v_readlane_b32 s2, %0, 1\n v_readlane_b32 s3, %0, 2\n v_readlane_b32 s4, %0, 3\n v_readlane_b32 s5, %0, 4" :: "v"(a0) : "s2", "s3", "s4", "s5");)
    } else if constexpr (OP == 5) {  // v_fma_f64
      REP8(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(d0));)
    } else if constexpr (OP == 6) {  // v_mad_u32_u24
      REP8(asm volatile("v_mad_u32_u24 %0, %4, %5, %0\n v_mad_u32_u24 %1, %4, %5, %1\n v_mad_u32_u24 %2, %4, %5, %2\n v_mad_u32_u24 %3, %4, %5, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(s), "s"(s));)
    } else if constexpr (OP == 7) {  // v_add_co_u32 + v_addc_co_u32 (int64 add) x2
      REP8(asm volatile("v_add_co_u32 %0, vcc, %0, %4\n v_addc_co_u32 %1, vcc, %1, 0, vcc\n v_add_co_u32 %2, vcc, %2, %4\n v_addc_co_u32 %3, vcc, %3, 0, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(s) : "vcc");)
    } else if constexpr (OP == 8) {  // v_mul_lo_u32
      REP8(asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "s"(s));)
    } else if constexpr (OP == 9) {  // v_pk_fma_f32
      REP8(asm volatile("v_pk_fma_f32 %0, %0, %4, %0\n v_pk_fma_f32 %1, %1, %4, %1\n v_pk_fma_f32 %2, %2, %4, %2\n v_pk_fma_f32 %3, %3, %4, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(d0));)
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + (int)(b0 + b1 + b2 + b3) + (int)(d0 + d1 + d2 + d3);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int* out, long long* cyc, int nblk) {
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, 3, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, 3, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double instr = (double)N_ITER * 32 * (nblk / 256);  // per SIMD (4 waves per block, 256 CUs)
  // memtime ticks at 100 MHz on CDNA; wall clock gives the shader clock view
  printf("%-18s %8.3f ms  %7.2f ns/wave-instr  memtime %lld\n", name, ms, ms * 1e6 / instr, c);
}

int main(int argc, char** argv) {
  int* out;
  long long* cyc;
  const int nblk = argc > 1 ? atoi(argv[1]) : 256;  // 256: one 4-wave block per CU
  hipMalloc(&out, nblk * 256 * sizeof(int));
  hipMalloc(&cyc, nblk * sizeof(long long));
  run<0>("v_add_u32", out, cyc, nblk);
  run<1>("v_mad_i64_i32", out, cyc, nblk);
  run<2>("v_dot2_u32_u16", out, cyc, nblk);
  run<3>("v_dot2c_i32_i16", out, cyc, nblk);
  run<4>("v_readlane_b32", out, cyc, nblk);
  run<5>("v_fma_f64", out, cyc, nblk);
  run<6>("v_mad_u32_u24", out, cyc, nblk);
  run<7>("add_co/addc", out, cyc, nblk);
  run<8>("v_mul_lo_u32", out, cyc, nblk);
  run<9>("v_pk_fma_f32", out, cyc, nblk);
  return 0;
}
