// Host<->device round-trip latency on one stream: what a single-scan
// 3-level match pays per level (launch, completion seen by the host).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <immintrin.h>

__global__ void empty_kernel(int* p) { if (threadIdx.x == 0 && p) p[0] += 1; }
__global__ void flag_kernel(int* host_flag, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0)
    __hip_atomic_store(host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev, evb;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  hipEventCreateWithFlags(&evb, hipEventDisableTiming | hipEventBlockingSync);
  int* d; hipMalloc(&d, 4096);
  int* h; hipHostMalloc((void**)&h, 4096, hipHostMallocDefault);
  int* hc; hipHostMalloc((void**)&hc, 4096, hipHostMallocCoherent);
  char* hbuf; hipHostMalloc((void**)&hbuf, 1 << 16, hipHostMallocDefault);
  const int N = 2000;
  std::vector<double> a, b, c, dd, e, f, g, k2;
  for (int i = 0; i < 50; ++i) { hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d); hipStreamSynchronize(s); }
  for (int i = 0; i < N; ++i) {  // launch + hipEventSynchronize
    double t = now_us(); hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d); hipEventRecord(ev, s); hipEventSynchronize(ev); a.push_back(now_us() - t);
  }
  for (int i = 0; i < N; ++i) {  // launch + blocking-sync event
    double t = now_us(); hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d); hipEventRecord(evb, s); hipEventSynchronize(evb); b.push_back(now_us() - t);
  }
  for (int i = 0; i < N; ++i) {  // launch + hipEventQuery spin
    double t = now_us(); hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d); hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause();
    c.push_back(now_us() - t);
  }
  for (int i = 0; i < N; ++i) {  // launch + host flag (default pinned)
    double t = now_us(); hipLaunchKernelGGL(flag_kernel, 1, 64, 0, s, h, i + 1);
    while (__atomic_load_n(h, __ATOMIC_ACQUIRE) != i + 1) _mm_pause();
    dd.push_back(now_us() - t);
  }
  hipStreamSynchronize(s);
  for (int i = 0; i < N; ++i) {  // launch + host flag (coherent pinned)
    double t = now_us(); hipLaunchKernelGGL(flag_kernel, 1, 64, 0, s, hc, i + 1);
    while (__atomic_load_n(hc, __ATOMIC_ACQUIRE) != i + 1) _mm_pause();
    e.push_back(now_us() - t);
  }
  hipStreamSynchronize(s);
  for (int i = 0; i < N; ++i) {  // D2H 512 B copy + event sync
    double t = now_us(); hipMemcpyAsync(hbuf, d, 512, hipMemcpyDeviceToHost, s); hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause();
    f.push_back(now_us() - t);
  }
  for (int i = 0; i < N; ++i) {  // H2D 17 KB copy + kernel + spin
    double t = now_us(); hipMemcpyAsync(d, hbuf, 1024, hipMemcpyHostToDevice, s); hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d); hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause();
    g.push_back(now_us() - t);
  }
  for (int i = 0; i < N; ++i) {  // 3 kernels back to back + spin
    double t = now_us();
    for (int j = 0; j < 3; ++j) hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d);
    hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause();
    k2.push_back(now_us() - t);
  }
  double tl = now_us();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_kernel, 1, 64, 0, s, d);
  double launch_cost = (now_us() - tl) / N;
  hipStreamSynchronize(s);
  std::printf("{\"launch_event_sync_us\": %.2f, \"launch_blocking_event_us\": %.2f, \"launch_query_spin_us\": %.2f, "
              "\"launch_host_flag_default_us\": %.2f, \"launch_host_flag_coherent_us\": %.2f, "
              "\"d2h_512B_spin_us\": %.2f, \"h2d_1KB_kernel_spin_us\": %.2f, \"three_kernels_spin_us\": %.2f, "
              "\"launch_call_cpu_us\": %.2f}\n",
              med(a), med(b), med(c), med(dd), med(e), med(f), med(g), med(k2), launch_cost);
  return 0;
}
