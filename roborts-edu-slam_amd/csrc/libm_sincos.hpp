// libm_sincos.hpp — glibc 2.35's sincos() restated operation for operation,
// for the host and the device, so the angle rows of a window
// (AngleSearchLookUpTable::UpdateLookUpTable correlate_scan_matcher.h:171-172,
// whose cos/sin pair GCC merges into one sincos call, host_math.hpp) can be
// computed on the GPU bit-equal to the host's libm.
//
// Third-party algorithm: glibc 2.35 sysdeps/ieee754/dbl-64/s_sincos.c
// (__sincos) with do_sin/do_cos/TAYLOR_SIN/reduce_sincos from s_sin.c. On
// x86-64 `sincos` is not multi-versioned (no FMA variant; objdump -T shows a
// plain DF symbol), so every operation is a separately rounded binary64
// add/sub/mul — reproducible on any IEEE binary64 unit, including gfx950's
// v_fma-free v_add_f64/v_mul_f64, provided nothing is contracted into an FMA
// (the library is built with -ffp-contract=off) and subnormals are kept.
// The operation order below follows the shipped machine code of
// /lib/x86_64-linux-gnu/libm.so.6 (sincos at 0x2fa80), which agrees with
// the published source; commutations the compiler made are exact.
//
// The 110-entry table (__sincostab: sin and cos of k/128 as hi + lo pairs)
// is NOT restated: its low words are not the round-to-nearest remainders, so
// the table is taken from the libm mapped into this process
// (locate_sincos_table, csm_launch.cpp) and checked there.
//
// Domain: |x| < 105414350 (0x419921FB high word) and finite. Larger
// arguments take glibc's __branred (multi-word reduction), which is not
// restated; callers check the range (sincos_device_ok) and keep the host
// call outside it.
#pragma once

#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define CSM_SINCOS_HD __host__ __device__
#else
#define CSM_SINCOS_HD
#endif

namespace csm {
namespace libm {

constexpr int kSincosTableDoubles = 440;  // 110 × {sn, ssn, cs, ccs}

CSM_SINCOS_HD inline double bits(uint64_t u) {
  double d;
  std::memcpy(&d, &u, sizeof(d));
  return d;
}
CSM_SINCOS_HD inline uint64_t ubits(double d) {
  uint64_t u;
  std::memcpy(&u, &d, sizeof(u));
  return u;
}
CSM_SINCOS_HD inline double abs_(double d) { return bits(ubits(d) & 0x7fffffffffffffffull); }
CSM_SINCOS_HD inline double copysign_(double m, double s) {
  return bits((ubits(m) & 0x7fffffffffffffffull) | (ubits(s) & 0x8000000000000000ull));
}

// constants (usncs.h / s_sin.c), as stored in libm's .rodata
struct K {
  static CSM_SINCOS_HD double big() { return bits(0x42c8000000000000ull); }    // 0x1.8p45
  static CSM_SINCOS_HD double hp0() { return bits(0x3ff921fb54442d18ull); }    // pi/2 hi
  static CSM_SINCOS_HD double hp1() { return bits(0x3c91a62633145c07ull); }    // pi/2 lo
  static CSM_SINCOS_HD double hpinv() { return bits(0x3fe45f306dc9c883ull); }  // 2/pi
  static CSM_SINCOS_HD double toint() { return bits(0x4338000000000000ull); }  // 0x1.8p52
  static CSM_SINCOS_HD double mp1() { return bits(0x3ff921fb58000000ull); }
  static CSM_SINCOS_HD double mp2() { return bits(0xbe4dde973c000000ull); }
  static CSM_SINCOS_HD double pp3() { return bits(0xbc8cb3b398000000ull); }
  static CSM_SINCOS_HD double pp4() { return bits(0xbacd747f23e32ed7ull); }
  // TAYLOR_SIN polynomial: s1..s5
  static CSM_SINCOS_HD double s1() { return bits(0xbfc5555555555555ull); }
  static CSM_SINCOS_HD double s2() { return bits(0x3f81111111110eceull); }
  static CSM_SINCOS_HD double s3() { return bits(0xbf2a01a019db08b8ull); }
  static CSM_SINCOS_HD double s4() { return bits(0x3ec71de27b9a7ed9ull); }
  static CSM_SINCOS_HD double s5() { return bits(0xbe5addffc2fcdf59ull); }
  // table-based kernels: sn3, sn5, cs2, cs4, cs6
  static CSM_SINCOS_HD double sn3() { return bits(0xbfc5555555555515ull); }
  static CSM_SINCOS_HD double sn5() { return bits(0x3f811110e829872full); }
  static CSM_SINCOS_HD double cs2() { return bits(0x3fe0000000000000ull); }
  static CSM_SINCOS_HD double cs4() { return bits(0xbfa5555555555535ull); }
  static CSM_SINCOS_HD double cs6() { return bits(0x3f56c16bedd9e239ull); }
  static CSM_SINCOS_HD double taylor_max() { return bits(0x3fc020c49ba5e354ull); }  // 0.126
};

// s_sin.c do_cos(x, dx): cos(x + dx) for |x| < 0.855469 (table + polynomial)
CSM_SINCOS_HD inline double do_cos(double x, double dx, const double* tab) {
  if (x < 0) dx = -dx;
  const double ax = abs_(x);
  const double u = K::big() + ax;
  x = (ax - (u - K::big())) + dx;
  const double xx = x * x;
  const double s = x + (x * xx) * (K::sn3() + xx * K::sn5());
  const double c = xx * (K::cs2() + xx * (K::cs4() + xx * K::cs6()));
  const int k = (int)(uint32_t)ubits(u) << 2;
  const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
  const double cor = ((ccs - s * ssn) - cs * c) - sn * s;
  return cs + cor;
}

// s_sin.c TAYLOR_SIN(xx, a, da)
CSM_SINCOS_HD inline double taylor_sin(double xx, double a, double da) {
  const double poly = (((((K::s5() * xx + K::s4()) * xx + K::s3()) * xx + K::s2()) * xx) + K::s1());
  const double t = ((poly * a - 0.5 * da) * xx + da);
  return a + t;
}

// s_sin.c do_sin(x, dx): sin(x + dx) for |x| < 0.855469
CSM_SINCOS_HD inline double do_sin(double x, double dx, const double* tab) {
  const double xold = x;
  if (abs_(x) < K::taylor_max()) return taylor_sin(x * x, x, dx);
  if (x <= 0) dx = -dx;
  const double ax = abs_(x);
  const double u = K::big() + ax;
  x = ax - (u - K::big());
  const double xx = x * x;
  const double s = x + (dx + (x * xx) * (K::sn3() + xx * K::sn5()));
  const double c = x * dx + xx * (K::cs2() + xx * (K::cs4() + xx * K::cs6()));
  const int k = (int)(uint32_t)ubits(u) << 2;
  const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
  const double cor = ((ssn + s * ccs) - sn * c) + cs * s;
  return copysign_(sn + cor, xold);
}

// s_sin.c reduce_sincos: x = n·pi/2 + (a + da), |x| < 105414350
CSM_SINCOS_HD inline int reduce_sincos(double x, double* a, double* da) {
  const double t = x * K::hpinv() + K::toint();
  const double xn = t - K::toint();
  const double y = (x - xn * K::mp1()) - xn * K::mp2();
  const int n = (int)(ubits(t) & 3);
  double t1 = xn * K::pp3();
  const double t2 = y - t1;
  double db = (y - t2) - t1;
  t1 = xn * K::pp4();
  const double b = t2 - t1;
  db += (t2 - b) - t1;
  *a = b;
  *da = db;
  return n;
}

// The high word test that keeps x inside the restated domain.
CSM_SINCOS_HD inline bool sincos_device_ok(double x) {
  return (uint32_t)((ubits(x) >> 32) & 0x7fffffffu) < 0x419921FBu;
}

// s_sincos.c __sincos for |x| < 105414350 (sincos_device_ok)
CSM_SINCOS_HD inline void sincos(double x, const double* tab, double* sinx, double* cosx) {
  const uint32_t k = (uint32_t)((ubits(x) >> 32) & 0x7fffffffu);
  if (k < 0x400368fdu) {
    if (k < 0x3e400000u) {  // |x| < 2^-27
      *sinx = x;
      *cosx = 1.0;
      return;
    }
    if (k < 0x3feb6000u) {  // |x| < 0.855469
      *sinx = do_sin(x, 0.0, tab);
      *cosx = do_cos(x, 0.0, tab);
      return;
    }
    // |x| < 2.426265
    const double y = K::hp0() - abs_(x);
    const double a = y + K::hp1();
    const double da = (y - a) + K::hp1();
    *sinx = copysign_(do_cos(a, da, tab), x);
    *cosx = do_sin(a, da, tab);
    return;
  }
  double a, da;
  const int n = reduce_sincos(x, &a, &da) & 3;
  if (n == 1 || n == 2) {
    a = -a;
    da = -da;
  }
  double* so = sinx;
  double* co = cosx;
  if (n & 1) {
    so = cosx;
    co = sinx;
  }
  *so = do_sin(a, da, tab);
  const double xx = do_cos(a, da, tab);
  *co = (n & 2) ? -xx : xx;
}

}  // namespace libm
}  // namespace csm
