"""glibc sincos for the Python restatements.

The reference's GCC -O2 build turns cos(a)/sin(a) pairs into one glibc
sincos() call, which differs from separate cos and sin in the last bit for
about 0.14% of arguments (glibc 2.35). The C++ restatement and the product
call sincos explicitly (oracle/oracle_math.hpp, csrc/host_math.hpp); the
Python restatements use this binding so they compute the same pair.
"""
import ctypes as C
import ctypes.util

_m = C.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_m.sincos.restype = None
_m.sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]


def sincos(a: float):
    """(cos a, sin a) as glibc's sincos returns them."""
    s, c = C.c_double(), C.c_double()
    _m.sincos(float(a), C.byref(s), C.byref(c))
    return c.value, s.value
