// oracle_math.hpp — test infrastructure (see csm_oracle.cpp's header).
//
// The reference's GCC -O2 build merges cos(a) and sin(a) of one argument
// into one glibc sincos() call (GCC's cse_sincos pass), and glibc's sincos
// differs from separate cos/sin in the last bit for ~0.14% of arguments
// (glibc 2.35). Every cos/sin pair the restatement follows has that shape
// (correlate_scan_matcher.h:171-172,688-689; optimize_scan_matcher.h:96-97,
// 200-201; slam_processor.cpp:625-626; the sensor-pose rotations of the map
// updates), so the oracle calls sincos explicitly.
#pragma once

#include <cmath>

inline void ref_sincos(double a, double* s, double* c) { ::sincos(a, s, c); }
