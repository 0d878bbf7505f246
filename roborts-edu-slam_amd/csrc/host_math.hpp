// host_math.hpp — the host libm calls the reference's arithmetic depends on.
//
// The reference is built by GCC -O2 against glibc (CMakeLists.txt:5). GCC
// merges cos(a) and sin(a) of one argument into a single glibc sincos() call
// (its cse_sincos pass; no -ffast-math needed), and glibc's sincos does not
// always return what separate cos and sin return (about 0.14% of arguments
// on glibc 2.35 differ in the last bit). Every cos/sin pair of the
// reference's matcher and map code has that shape (AngleSearchLookUpTable
// correlate_scan_matcher.h:171-172, FindBestCandidate :688-689,
// BasedOptimizeScanMatch optimize_scan_matcher.h:96-97,200-201,
// UpdateMapByRange occu_grid_map.h:288-293, PredictPoseByOdom
// slam_processor.cpp:625-629), so the host calls sincos explicitly instead of
// leaving the choice to the optimiser.
#pragma once

#include <cmath>

namespace csm {

inline void host_sincos(double a, double* s, double* c) { ::sincos(a, s, c); }

}  // namespace csm
