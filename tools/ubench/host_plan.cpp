// Host cost of the 3-level driver's per-window work on the GPU box's CPUs
// (no kernels): glibc sincos per call, the pool's plan of a 2048-window level
// into pageable and pinned rows, and the ScanWork fill, serial and pooled.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I include
//   -I roborts-edu-slam_amd/csrc -I /opt/rocm/include tools/ubench/host_plan.cpp
//   -L roborts-edu-slam_amd/lib -lroborts_csm -L /opt/rocm/lib -lamdhip64 -lpthread
#include <algorithm>
#include <cstdio>
#include <vector>

#include "csm_host.hpp"

using namespace csmh;

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int nw = 2048, reps = 200;
  csm_host_plan plan{};
  context_host_plan(0, 0, 1, &plan);
  std::printf("plan: threads %d numa %d cpus %d quota %d\n", plan.threads, plan.numa_node, plan.n_cpus, plan.quota_cpus);
  {  // sincos
    double acc = 0;
    const int N = 4000000;
    const double t0 = now_ms();
    for (int i = 0; i < N; ++i) {
      double s, c;
      ::sincos(-3.0 + i * (6.0 / N), &s, &c);
      acc += s + c;
    }
    std::printf("sincos %.2f ns/call (%g)\n", (now_ms() - t0) * 1e6 / N, acc);
  }
  ThreadPool pool(plan.threads, plan);
  void* pinned = nullptr;
  if (hipHostMalloc(&pinned, (size_t)nw * 30 * sizeof(AngleEntry) + (size_t)nw * sizeof(ScanWork), 0) != hipSuccess) return 1;
  std::vector<AngleEntry> pageable((size_t)nw * 30);
  for (int na : {30, 21, 11}) {
    for (int where = 0; where < 2; ++where) {
      AngleEntry* rows = where ? (AngleEntry*)pinned : pageable.data();
      for (int threads : {1, 4, 8, plan.threads}) {
        std::vector<double> t;
        for (int r = 0; r < reps; ++r) {
          const double t0 = now_ms();
          pool.run(nw, threads, [&](int i) {
            const double start = 0.001 * i + r * 1e-7 - 0.35;
            AngleEntry* o = rows + (size_t)i * na;
            for (int a = 0; a < na; ++a) {
              o[a].angle = start + a * 0.0175;
              ::sincos(o[a].angle, &o[a].sine, &o[a].cosine);
            }
          });
          t.push_back(now_ms() - t0);
        }
        std::printf("plan %d windows x %2d angles, %s rows, %2d threads: median %.1f us\n", nw, na,
                    where ? "pinned  " : "pageable", threads, med(t) * 1e3);
      }
    }
  }
  {  // ScanWork fill into pinned staging, serial
    ScanWork* sw = (ScanWork*)((char*)pinned + (size_t)nw * 30 * sizeof(AngleEntry));
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) {
      const double t0 = now_ms();
      for (int i = 0; i < nw; ++i) {
        ScanWork& s = sw[i];
        s.pts_off = i * 1081;
        s.angle_off = (int64_t)i * 30;
        s.out_off = (int64_t)i * 5072;
        s.n_used = 109;
        s.step = 10;
        s.divisor = 100.0 + r;
        s.x0 = s.y0 = s.cx = s.cy = s.ct = 0.5 * i;
        s.reserved = i;
        s.grid_index = 0;
      }
      t.push_back(now_ms() - t0);
    }
    std::printf("ScanWork fill %d (%zu B each) serial into pinned: median %.1f us\n", nw, sizeof(ScanWork), med(t) * 1e3);
  }
  return 0;
}
