// sincos_check: the restated glibc sincos (csrc/libm_sincos.hpp) against this
// machine's ::sincos, bit for bit, over N seeded arguments per thread.
//   g++ -O2 -ffp-contract=off -pthread -I roborts-edu-slam_amd/csrc \
//       tools/ubench/sincos_check.cpp -o tools/ubench/sincos_check -ldl
//   tools/ubench/sincos_check [N_per_thread] [threads]
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "libm_sincos_table.hpp"

int main(int argc, char** argv) {
  const long long n = argc > 1 ? std::atoll(argv[1]) : 10000000LL;
  const int th = argc > 2 ? std::atoi(argv[2]) : 8;
  static double tab[csm::libm::kSincosTableDoubles];
  if (!csm::libm::locate_sincos_table(tab)) {
    std::printf("table: not found\n");
    return 2;
  }
  std::vector<long long> bad((size_t)th, 0);
  std::vector<std::thread> ts;
  for (int t = 0; t < th; ++t)
    ts.emplace_back([&, t] { bad[(size_t)t] = csm::libm::check_sincos(tab, n, 0x5eed0000ull + (uint64_t)t); });
  for (auto& t : ts) t.join();
  long long sum = 0;
  for (long long b : bad) sum += b;
  std::printf("arguments %lld (+ %d edge cases per thread), mismatches %lld\n", n * th, 4 * 129 * 2, sum);
  return sum == 0 ? 0 : 1;
}
