// libm_sincos_table.hpp — find glibc's __sincostab in the libm this process
// has mapped, and check that the restated sincos (libm_sincos.hpp) equals the
// host's ::sincos with it. Host only.
//
// The table is not exported; it sits in libm's read-only segment. It is
// located by its first five doubles (entry 0 = {0, 0, 1, 0}, entry 1's sin
// hi word), which must occur exactly once in the object that holds
// ::sincos, and every entry is then checked against sin/cos(k/128). A libm
// that does not pass (another version, another layout) leaves the device
// path off and the host keeps calling ::sincos.
#pragma once

#include <dlfcn.h>
#include <link.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>

#include "libm_sincos.hpp"

namespace csm {
namespace libm {

namespace detail {
struct Find {
  const void* fn;        // an address inside the object (::sincos)
  const double* found;   // the table, when it is found once
  int hits;
};

inline bool in_object(const dl_phdr_info* info, const void* p) {
  const uintptr_t a = (uintptr_t)p;
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_LOAD) continue;
    const uintptr_t lo = info->dlpi_addr + ph.p_vaddr;
    if (a >= lo && a < lo + ph.p_memsz) return true;
  }
  return false;
}

inline int scan(dl_phdr_info* info, size_t, void* data) {
  Find* f = (Find*)data;
  if (!in_object(info, f->fn)) return 0;
  static const uint64_t sig[5] = {0, 0, 0x3ff0000000000000ull, 0, 0x3f7fffeaaaaeeeefull};
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_LOAD || !(ph.p_flags & PF_R) || (ph.p_flags & PF_W)) continue;
    const uintptr_t lo = (info->dlpi_addr + ph.p_vaddr + 7) & ~(uintptr_t)7;
    const uintptr_t hi = info->dlpi_addr + ph.p_vaddr + ph.p_filesz;
    for (uintptr_t p = lo; p + kSincosTableDoubles * sizeof(double) <= hi; p += 8) {
      if (std::memcmp((const void*)p, sig, sizeof(sig)) != 0) continue;
      f->found = (const double*)p;
      ++f->hits;
    }
  }
  return 1;
}
}  // namespace detail

// Copies the table into out[440]; false when it is not found exactly once or
// an entry is not sin/cos(k/128) split into hi + lo.
inline bool locate_sincos_table(double* out) {
  Dl_info di;
  void (*fn)(double, double*, double*) = &::sincos;
  if (!dladdr((const void*)fn, &di)) return false;
  detail::Find f{(const void*)fn, nullptr, 0};
  dl_iterate_phdr(detail::scan, &f);
  if (f.hits != 1) return false;
  std::memcpy(out, f.found, kSincosTableDoubles * sizeof(double));
  for (int k = 0; k < kSincosTableDoubles / 4; ++k) {
    const double x = k / 128.0;
    const double sn = out[4 * k], ssn = out[4 * k + 1], cs = out[4 * k + 2], ccs = out[4 * k + 3];
    const double s = std::sin(x), c = std::cos(x);
    if (std::fabs(sn - s) > 0x1p-52 * std::fabs(s) || std::fabs(cs - c) > 0x1p-52 * c) return false;
    if (std::fabs(ssn) > 0x1p-52 * std::fabs(sn) || std::fabs(ccs) > 0x1p-52 * cs) return false;
  }
  return true;
}

// The restatement with this table against the host's ::sincos on `n` seeded
// arguments spread over the restated domain, plus the branch boundaries.
// Returns the number of arguments whose sin or cos differ in any bit.
inline long long check_sincos(const double* tab, long long n, uint64_t seed) {
  long long bad = 0;
  auto one = [&](double x) {
    double s0, c0, s1, c1;
    ::sincos(x, &s0, &c0);
    libm::sincos(x, tab, &s1, &c1);
    if (ubits(s0) != ubits(s1) || ubits(c0) != ubits(c1)) ++bad;
  };
  static const uint32_t edges[] = {0x3e400000u, 0x3feb6000u, 0x400368fdu, 0x41991000u};
  for (uint32_t e : edges)
    for (int d = -64; d <= 64; ++d) {
      const double x = bits(((uint64_t)e << 32) + (uint64_t)(int64_t)d);
      one(x);
      one(-x);
    }
  std::mt19937_64 rng(seed);
  for (long long i = 0; i < n; ++i) {
    const uint64_t r = rng();
    double x;
    switch (r & 3) {
      case 0: x = std::ldexp((double)(r >> 11) * 0x1p-53, (int)((r >> 2) % 40) - 30); break;  // 2^-30..2^10
      case 1: x = ((double)(r >> 11) * 0x1p-53 - 0.5) * 16.0; break;                          // |x| < 8
      case 2: x = ((double)(r >> 11) * 0x1p-53 - 0.5) * 2.0e8; break;                         // up to 1e8
      default: x = (double)(int64_t)((r >> 11) % 4001 - 2000) * 0.0087266462599716477; break;  // degree grid
    }
    if ((r >> 10) & 1) x = -x;
    if (!sincos_device_ok(x)) continue;
    one(x);
  }
  return bad;
}

}  // namespace libm
}  // namespace csm
