// csm_pyramid.hpp — admissible multi-resolution branch-and-bound over large
// one-cell-step windows (loop closure, SURVEY.md 8e / BASELINE configs 3-4).
//
// The reference searches such windows exhaustively (MultiResolution...::
// ScanMatch, correlate_scan_matcher.h:516-603) or with its FAST matcher, whose
// bound is not admissible (the lowest level is scored on the raw grid,
// :333-393, so a pruned subtree can hold a better candidate). Here every
// level d >= 1 reads a max-pooled copy of the fixed-point grid whose cell
// (x, y) holds the maximum over the (2^d + 1)^2 cells [x, x + 2^d]^2, so the
// score of a node (all candidates j in [J 2^d, J 2^d + 2^d), k likewise, at
// one angle) is an upper bound of every candidate below it; depth 0 is the
// exact candidate score. Pruning keeps a node unless its bound is below the
// incumbent (or equal with a larger lowest index), so the result is the
// exhaustive search's argmax: max score, lowest (window, flat index).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>

#include "csm_internal.hpp"

namespace csm {

constexpr int kPyrMaxDepth = 10;

// One level of the pooled stack. Anchor cell (x, y) of grid g has logical
// column x' = x + shift and row y' = y + shift, valid in [0, width) x
// [0, height) (width = size_x + shift), zero (the outside value) elsewhere.
// Columns are stored phase-split: x' = qx * 2^lg + ph sits at column
// ph * q + qx (q = ceil(width / 2^lg)), so the anchors of nodes J, J+1, ...
// (2^lg cells apart) are adjacent in memory and a wave's gathers coalesce.
// Level 0 is the fixed-point grid itself (lg = 0, shift 0: plain rows,
// int32). Levels d >= 1 hold int16 values ceil(max / 2^qs) (qs = kPyrQuant):
// |fixed-point value| < 2^26 (csm_set_grid), so |max / 2^qs| <= 2^14, and
// 2^qs * ceil(max / 2^qs) >= max keeps every bound admissible while halving
// the bytes the node gathers pull through the caches.
constexpr int kPyrQuant = 12;
struct PyrGrid {
  const void* g;       // int32 (qs == 0) or int16 (qs > 0) cells
  int64_t stride;
  int32_t pitch;
  int32_t shift;
  int32_t width, height;
  int32_t lg, q;
  int32_t qs;          // 0: exact int32 level; kPyrQuant: int16 quantised level
  int32_t pad;
};

// Search nodes: window (20 bits) | angle (12) | J (16) | K (16).
__host__ __device__ constexpr uint64_t pyr_node(uint32_t w, uint32_t a, uint32_t J, uint32_t K) {
  return ((uint64_t)w << 44) | ((uint64_t)a << 32) | ((uint64_t)J << 16) | (uint64_t)K;
}
constexpr uint64_t kPyrNoNode = ~(uint64_t)0;

// Best of a list: value (bound or exact score), its lowest global candidate
// index (window * n_cand + flat), the node.
struct PyrPartial {
  double v;
  int64_t gflat;
  uint64_t node;
};

// Launchers (csm_pyramid.hip); all enqueue on `stream`.
// dst level d >= 1 from src level d - 1 (d = 1: src is the fixed-point grid).
hipError_t launch_pyr_pool(const PyrGrid& src, const PyrGrid& dst, int d, int32_t n_grids, hipStream_t stream);
// Top-level nodes [first, first + n) of the implicit list (window, angle, K, J), nj per axis
// (J fastest: a wave's nodes share window, angle and K, their anchors adjacent).
hipError_t launch_pyr_top(const LevelWork& L, int32_t nj, int64_t first, int64_t n, uint64_t* out,
                          hipStream_t stream);
// Node counts: n_dev (device, may be null) overrides n; `upper` (>= the
// count) sizes the grid, whose blocks stride over the list.
int pyr_blocks(int64_t upper);
// Block count of the bound kernel: the number of partials a bound launch
// writes (<= pyr_blocks's cap); the kernel spreads each node over up to a
// wave of lanes when the list is short.
int pyr_bound_blocks(int64_t upper, int32_t n_used);
// A search's start: *inc = {-DBL_MAX, INT64_MAX}, zero[0, n) = 0.
hipError_t launch_pyr_init(BestPartial* inc, unsigned long long* zero, int n, hipStream_t stream);
// Bounds (d >= 1) or exact scores (d = 0) of the nodes; one best per block
// into partials (pyr_bound_blocks(upper, n_used) entries); *scored (nullable) += the count. The windows share one scan: its
// n_used beams (stride step from pts) are staged in LDS.
hipError_t launch_pyr_bound(const LevelWork& L, const PyrGrid& lev, int d, const ScanWork* scans,
                            const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                            const uint64_t* nodes, int64_t n, const unsigned long long* n_dev, int64_t upper,
                            double* vals, PyrPartial* partials, unsigned long long* scored, hipStream_t stream);
// The whole top level in one launch (all windows, angles, J, K): nodes and
// bounds in list order, one best per block (pyr_top_blocks of them; -1 when
// the grid would not fit a launch).
int pyr_top_blocks(const LevelWork& L, int32_t nj, int32_t* ktiles, int32_t* kt, int32_t* col_blocks);
hipError_t launch_pyr_top_bound(const LevelWork& L, const PyrGrid& lev, int d, int32_t nj, const ScanWork* scans,
                                const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                                uint64_t* nodes, double* vals, PyrPartial* partials, hipStream_t stream);
// The top level as beam boxes (pyr_topbox_kernel): tb is level d in a padded
// phase-split int16 layout (8 * pyr_topbox_pieces(nj) zero cells past each
// phase's columns, 2^d * nj zero rows below); the host guarantees |t| < 2^24
// cells (the box test's rounding argument). Same outputs as
// launch_pyr_top_bound (the bounds as integer sums, the nodes implicit),
// one best per (window, angle) wave (n_scans * n_angles partials).
int pyr_topbox_pieces(int32_t nj);  // 16-byte pieces per node row (0: unsupported nj)
hipError_t launch_pyr_widen(const PyrGrid& src, const PyrGrid& dst, int32_t n_grids, hipStream_t stream);
// Writes each node's integer sum (level units) at its index of the implicit
// list ((window, angle, K, J), J fastest).
// With few (window, angle) pairs each one's beams are split over several
// waves (*split_out, nullable: how many) whose partial sums go to `slab`
// (kPyrTopMaxSplit ints per top node), then are added and bounded.
constexpr int kPyrTopMaxSplit = 16;
hipError_t launch_pyr_topbox(const LevelWork& L, const PyrGrid& tb, int d, int32_t nj, const ScanWork* scans,
                             const AngleEntry* angles, const double* pts, int32_t n_used, int32_t step,
                             int32_t* sums, int32_t* slab, PyrPartial* partials, hipStream_t stream,
                             int* split_out = nullptr);
// launch_pyr_expand for nodes [first, first + n) of that implicit list; every
// window must share one scan (divisor, beam count). thr: 2 int64 of device
// scratch (the incumbent as integer sums).
hipError_t launch_pyr_expand_top(const LevelWork& L, int d, int32_t nj, int qs, int32_t n_used, const ScanWork* scans,
                                 const int32_t* sums, int64_t first, int64_t n, const BestPartial* inc,
                                 int64_t* thr, uint64_t* out, unsigned long long* count, int64_t cap,
                                 hipStream_t stream);
// Reduce n partials. merge = true: fold the best into the incumbent *inc
// (better score, or equal with a lower index). merge = false: probe[i] =
// the best node of the i-th of n_probe equal segments of the partials, if it
// beats the incumbent (kPyrNoNode otherwise).
hipError_t launch_pyr_final(const PyrPartial* partials, int64_t n, bool merge, int n_probe, BestPartial* inc,
                            uint64_t* probe, hipStream_t stream);
// All 4^d leaves (depth 0 nodes) under each of probe[0, n_probe); invalid ones
// carry J or K beyond the window (scored as -inf).
hipError_t launch_pyr_probe(int d, int n_probe, const uint64_t* probe, uint64_t* out, hipStream_t stream);
// Children (depth d - 1) of the nodes whose bound survives the incumbent,
// appended at out[*count]; at most cap entries are written.
hipError_t launch_pyr_expand(const LevelWork& L, int d, const uint64_t* nodes, const double* bounds, int64_t n,
                             const unsigned long long* n_dev, int64_t upper, const BestPartial* inc, uint64_t* out,
                             unsigned long long* count, int64_t cap, hipStream_t stream);

struct PyrStats {
  int32_t depth = 0;
  int64_t nodes[kPyrMaxDepth + 1] = {};  // nodes bounded per depth (0: candidates scored exactly)
  int64_t probe_leaves = 0;              // candidates scored by incumbent probes
  int64_t slices = 0;                    // expand launches
  int64_t syncs = 0;                     // node counts read back by the host
  int32_t top_box = 0;                   // 1: the top level ran as beam boxes
  // PyrInputs::timed: the top-level kernel's time (HIP events around its
  // launch), its name as csm_kernel_stats reports it, and its algorithmic
  // bytes (one int16 pooled value per node and beam)
  double top_ms = 0.0, top_bytes = 0.0;
  char top_name[48] = {0};
  // PyrInputs::timed: the bound launches (pyr_bound_kernel, incumbent probes
  // excluded) per depth, HIP events around each: launches and summed ms
  int32_t bound_launches[kPyrMaxDepth + 1] = {};
  double bound_ms[kPyrMaxDepth + 1] = {};
  double build_ms = 0.0;                 // pooled levels built (0 when cached)
};

struct PyrInputs {
  hipStream_t stream;
  LevelWork L;              // n_angles, n_space, n_cand, n_scans (= windows), step_cells, penalty, fixed point
  PyrGrid level0;           // the fixed-point grid (shift 0, width size_x, height size_y)
  int32_t n_grids;
  uint64_t grid_gen;        // changes whenever the fixed-point grid does
  const ScanWork* scans;    // per window, device
  const AngleEntry* angles; // device
  const double* pts;        // device, the one scan's points
  int32_t n_used, step;
  int32_t depth;            // top depth
  int32_t top_mode;         // 0: beam boxes when eligible, 1: per-node gathers
  int32_t box_ok;           // every window's |t| < 2^24 cells (the box test's bound)
  int32_t one_scan;         // every window has the same divisor and beam count
  int32_t timed;            // time the top-level kernel (PyrStats::top_ms)
};

class PyramidSearch {
 public:
  PyramidSearch();
  ~PyramidSearch();
  PyramidSearch(const PyramidSearch&) = delete;
  PyramidSearch& operator=(const PyramidSearch&) = delete;
  // The best candidate over all windows (score, window * n_cand + flat).
  hipError_t run(const PyrInputs& in, BestPartial* best, PyrStats* stats, std::string* what);
  // Nodes per level list (0: 4M) and the smallest level that gets an
  // incumbent probe below the top (0: 4096).
  void configure(int64_t node_capacity, int probe_min_nodes);
  // Bytes one pooled level of the current geometry needs (all grids).
  static int64_t level_cells(int32_t sx, int32_t sy, int d);
  void release();

 private:
  struct Impl;
  Impl* p_;
};

}  // namespace csm
