// csm_search.cpp — host driver of the admissible multi-resolution search
// (csm_pyramid.hpp). The host walks the resolution levels; the device bounds
// every node of a level in one launch and compacts the survivors' children.
//
//   top depth D: every (window, angle, J, K) node, bounded on level D
//   probe: the best node's 4^d leaves are scored exactly, raising the
//          incumbent before the level is pruned (the first probe at the top
//          usually finds the answer; later ones tighten it)
//   expand: children of the nodes whose bound is not below the incumbent
//   depth 0: exact candidate scores, folded into the incumbent
//
// A level's child list is bounded by the node capacity: a parent list larger
// than capacity / 4 is expanded in slices, each descended before the next
// (depth-first over slices, level-synchronous inside one), so memory stays
// fixed whatever the pruning rate.
#include "csm_pyramid.hpp"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cstdio>
#include <vector>

namespace csm {

namespace {

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  ~Buf() { release(); }
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct PyramidSearch::Impl {
  // pooled levels 1..kPyrMaxDepth of the current fixed-point grid
  Buf level[kPyrMaxDepth + 1];
  PyrGrid lev[kPyrMaxDepth + 1]{};
  const void* key_g = nullptr;
  uint64_t key_gen = 0;
  int32_t key_sx = -1, key_sy = -1, key_grids = -1, built = 0;
  // the top level's box copy (pyr_topbox_kernel): depth and pieces it was built for
  Buf box;
  PyrGrid boxg{};
  int32_t box_depth = -1, box_npc = 0;
  // per-depth node lists, their values and counts (counts[d]: nodes[d]'s
  // length as the expand that filled it left it)
  Buf nodes[kPyrMaxDepth + 1], vals[kPyrMaxDepth + 1];
  Buf partials, probe_slot, probe_nodes, probe_vals;
  // device state of a search, set by one init launch: the incumbent, the
  // nodes scored per depth, and a pool of list counters (each expand appends
  // to a fresh, already zero counter: no memset per level). Once the fresh
  // slots are used up (many slices), list d counts in a slot of its own,
  // kCountPool + d, cleared before each expand into it: never the slot of the
  // parent list (depth d + 1) whose count that expand reads.
  static constexpr int kCountPool = 64;
  static constexpr int kCountSlots = kCountPool + kPyrMaxDepth + 1;
  Buf state;  // BestPartial inc | scored[kPyrMaxDepth + 1] | pool[kCountSlots]
  int cslot[kPyrMaxDepth + 1] = {};  // pool slot of list d's count (slot 0: never written, zero)
  int next_slot = 1;
  BestPartial* inc_dev() const { return (BestPartial*)state.p; }
  unsigned long long* scored_dev() const { return (unsigned long long*)((char*)state.p + sizeof(BestPartial)); }
  unsigned long long* pool_dev() const { return scored_dev() + kPyrMaxDepth + 1; }
  // the beam-box top level: integer sums of the implicit node list
  Buf top_sums, top_thr, top_slab;
  int top_implicit = -1;  // its depth while a search runs (-1: the top is a node list)
  int32_t top_nj = 0;
  // pinned: two counts read back, then the state's incumbent and scored
  // counts (pageable copies wait for the device: ~20-70 us each)
  unsigned long long* h_counts = nullptr;
  BestPartial* h_inc() const { return (BestPartial*)(h_counts + 2); }
  unsigned long long* h_scored() const { return (unsigned long long*)(h_inc() + 1); }
  hipEvent_t ev_top[2] = {nullptr, nullptr};  // PyrInputs::timed
  // PyrInputs::timed: an event pair around each bound launch (depth, pair)
  static constexpr int kBoundEvents = 256;
  std::vector<hipEvent_t> ev_bound;
  std::vector<int> ev_bound_depth;
  int n_ev_bound = 0;
  int64_t cap = (int64_t)1 << 25;
  // per level: the capacity of its node list, min(cap, the nodes the level
  // has at all), and that count; a level whose children always fit its list
  // is descended without reading a count back (no host round trip)
  int64_t capd[kPyrMaxDepth + 1] = {};
  int64_t possible[kPyrMaxDepth + 1] = {};
  void set_caps(const LevelWork& L, int D) {
    for (int d = 0; d <= D; ++d) {
      const double nj = (double)(((int64_t)L.n_space + (1 << d) - 1) >> d);
      const double all = (double)L.n_scans * (double)L.n_angles * nj * nj;
      possible[d] = all >= 9.0e18 ? INT64_MAX / 8 : (int64_t)all;
      capd[d] = std::max<int64_t>(4, std::min(cap, possible[d]));
    }
  }
  int probe_min = 4096;
  bool probes = true;  // false: no probe at any level, the top included (a test hook)
  static constexpr int kRoots = 8;  // probe roots per probe (best partials of distinct blocks)
  PyrInputs in{};
  PyrStats* st = nullptr;

  ~Impl() {
    if (h_counts) (void)hipHostFree(h_counts);
    for (hipEvent_t e : ev_top)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_bound)
      if (e) (void)hipEventDestroy(e);
  }
  hipError_t mark_top(int i, hipStream_t stream) {
    hipError_t e;
    if (!ev_top[i] && (e = hipEventCreate(&ev_top[i])) != hipSuccess) return e;
    return hipEventRecord(ev_top[i], stream);
  }

  hipError_t build(const PyrInputs& x) {
    const int32_t sx = x.level0.width, sy = x.level0.height;
    if (key_g != x.level0.g || key_gen != x.grid_gen || key_sx != sx || key_sy != sy || key_grids != x.n_grids) {
      built = 0;
      box_depth = -1;
      key_g = x.level0.g;
      key_gen = x.grid_gen;
      key_sx = sx;
      key_sy = sy;
      key_grids = x.n_grids;
    }
    lev[0] = x.level0;
    if (built >= x.depth) return hipSuccess;
    const double t0 = now_ms();
    hipError_t e;
    for (int d = built + 1; d <= x.depth; ++d) {
      PyrGrid& L = lev[d];
      L.shift = 1 << d;
      L.width = sx + L.shift;
      L.height = sy + L.shift;
      L.lg = d;
      L.q = (L.width + L.shift - 1) >> d;
      L.pitch = ((L.q << d) + 3) & ~3;
      L.stride = (int64_t)L.pitch * L.height;
      L.qs = kPyrQuant;
      if ((e = level[d].ensure((size_t)L.stride * (size_t)x.n_grids * sizeof(int16_t))) != hipSuccess) return e;
      L.g = level[d].p;
      if ((e = launch_pyr_pool(lev[d - 1], L, d, x.n_grids, x.stream)) != hipSuccess) return e;
    }
    if ((e = hipStreamSynchronize(x.stream)) != hipSuccess) return e;
    built = x.depth;
    if (st) st->build_ms = now_ms() - t0;
    return hipSuccess;
  }

  // Level D copied into the box layout (after build(x)): columns of each
  // phase padded by 8 * npc zeros, 2^D * nj zero rows below.
  hipError_t build_box(const PyrInputs& x, int D, int32_t nj, int npc) {
    if (box_depth == D && box_npc == npc &&
        boxg.height + (nj << D) <= (int32_t)(boxg.stride / boxg.pitch))
      return hipSuccess;
    const PyrGrid& src = lev[D];
    PyrGrid b = src;
    b.q = src.q + 8 * npc;
    b.pitch = b.q << D;
    const int64_t rows = (int64_t)src.height + ((int64_t)nj << D);
    b.stride = (int64_t)b.pitch * rows;
    if (b.stride * 2 >= INT32_MAX) return hipErrorInvalidValue;
    hipError_t e;
    const double t0 = now_ms();
    if ((e = box.ensure((size_t)b.stride * (size_t)x.n_grids * sizeof(int16_t))) != hipSuccess) return e;
    b.g = box.p;
    if ((e = launch_pyr_widen(src, b, x.n_grids, x.stream)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(x.stream)) != hipSuccess) return e;
    boxg = b;
    box_depth = D;
    box_npc = npc;
    if (st) st->build_ms += now_ms() - t0;
    return hipSuccess;
  }

  hipError_t ensure_lists(int D) {
    hipError_t e;
    for (int d = 0; d <= D; ++d) {
      if ((e = nodes[d].ensure((size_t)capd[d] * sizeof(uint64_t))) != hipSuccess) return e;
      if ((e = vals[d].ensure((size_t)capd[d] * sizeof(double))) != hipSuccess) return e;
    }
    const int64_t np = ((int64_t)1 << (2 * D)) * kRoots;
    if ((e = partials.ensure((size_t)pyr_blocks(INT64_MAX / 2) * sizeof(PyrPartial))) != hipSuccess) return e;
    if ((e = state.ensure(sizeof(BestPartial) + (kPyrMaxDepth + 1 + kCountSlots) * sizeof(unsigned long long))) !=
        hipSuccess)
      return e;
    if ((e = probe_slot.ensure(kRoots * sizeof(uint64_t))) != hipSuccess) return e;
    if ((e = probe_nodes.ensure((size_t)np * sizeof(uint64_t))) != hipSuccess) return e;
    if ((e = probe_vals.ensure((size_t)np * sizeof(double))) != hipSuccess) return e;
    if (!h_counts && (e = hipHostMalloc((void**)&h_counts,
                                        (2 + kPyrMaxDepth + 1) * sizeof(unsigned long long) + sizeof(BestPartial),
                                        hipHostMallocDefault)) != hipSuccess)
      return e;
    return hipSuccess;
  }

  unsigned long long* count_dev(int d) { return pool_dev() + cslot[d]; }

  // nodes (n on the host, or *n_dev), at most `upper` of them
  hipError_t bound(int d, const uint64_t* list, double* out, int64_t n, const unsigned long long* n_dev,
                   int64_t upper) {
    const bool timed = in.timed && n_ev_bound < kBoundEvents;
    hipError_t e;
    if (timed) {
      if (ev_bound.size() < (size_t)2 * kBoundEvents) ev_bound.resize((size_t)2 * kBoundEvents, nullptr);
      ev_bound_depth.resize(kBoundEvents);
      for (int k = 0; k < 2; ++k)
        if (!ev_bound[2 * n_ev_bound + k] && (e = hipEventCreate(&ev_bound[2 * n_ev_bound + k])) != hipSuccess)
          return e;
      if ((e = hipEventRecord(ev_bound[2 * n_ev_bound], in.stream)) != hipSuccess) return e;
    }
    if ((e = launch_pyr_bound(in.L, lev[d], d, in.scans, in.angles, in.pts, in.n_used, in.step, list, n, n_dev, upper,
                              out, (PyrPartial*)partials.p, scored_dev() + d, in.stream)) != hipSuccess)
      return e;
    if (timed) {
      if ((e = hipEventRecord(ev_bound[2 * n_ev_bound + 1], in.stream)) != hipSuccess) return e;
      ev_bound_depth[(size_t)n_ev_bound++] = d;
    }
    return hipSuccess;
  }

  // Score the leaves of the best nodes of n_partials block partials exactly
  // (the incumbent only ever rises).
  hipError_t probe(int d, int64_t n_partials) {
    hipError_t e;
    if ((e = launch_pyr_final((const PyrPartial*)partials.p, n_partials, false, kRoots, inc_dev(),
                              (uint64_t*)probe_slot.p, in.stream)) != hipSuccess)
      return e;
    if ((e = launch_pyr_probe(d, kRoots, (const uint64_t*)probe_slot.p, (uint64_t*)probe_nodes.p, in.stream)) !=
        hipSuccess)
      return e;
    const int64_t np = ((int64_t)1 << (2 * d)) * kRoots;
    if ((e = launch_pyr_bound(in.L, lev[0], 0, in.scans, in.angles, in.pts, in.n_used, in.step,
                              (const uint64_t*)probe_nodes.p, np, nullptr, np, (double*)probe_vals.p,
                              (PyrPartial*)partials.p, nullptr, in.stream)) != hipSuccess)
      return e;
    if ((e = launch_pyr_final((const PyrPartial*)partials.p, pyr_bound_blocks(np, in.n_used), true, 0, inc_dev(), nullptr,
                              in.stream)) != hipSuccess)
      return e;
    st->probe_leaves += np;
    return hipSuccess;
  }

  // Children of nodes[d][s, s + k) (k on the host, or *n_dev) into nodes[d-1].
  hipError_t expand(int d, int64_t s, int64_t k, const unsigned long long* n_dev, int64_t upper) {
    hipError_t e;
    if (next_slot < kCountPool) {
      cslot[d - 1] = next_slot++;  // zeroed by the search's init launch
    } else {  // fresh slots used up (many slices): list d - 1's own slot, cleared each time
      cslot[d - 1] = kCountPool + (d - 1);
      if ((e = hipMemsetAsync(count_dev(d - 1), 0, sizeof(unsigned long long), in.stream)) != hipSuccess) return e;
    }
    st->slices += 1;
    if (d == top_implicit)
      return launch_pyr_expand_top(in.L, d, top_nj, boxg.qs, in.n_used, in.scans, (const int32_t*)top_sums.p, s, k,
                                   inc_dev(), (int64_t*)top_thr.p, (uint64_t*)nodes[d - 1].p,
                                   count_dev(d - 1), capd[d - 1], in.stream);
    return launch_pyr_expand(in.L, d, (const uint64_t*)nodes[d].p + s, (const double*)vals[d].p + s, k, n_dev, upper,
                             inc_dev(), (uint64_t*)nodes[d - 1].p, count_dev(d - 1), capd[d - 1],
                             in.stream);
  }

  // counts[d - 1] and counts[d] to the host
  hipError_t read_counts(int d) {
    hipError_t e;
    if ((e = hipMemcpyAsync(h_counts, count_dev(d - 1), sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            in.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(h_counts + 1, count_dev(d), sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            in.stream)) != hipSuccess)
      return e;
    st->syncs += 1;
    return hipStreamSynchronize(in.stream);
  }

  // nodes[d] holds n nodes (n >= 0 known on the host; n < 0: counts[d]),
  // at most `upper`: bound them and descend. The host reads a count back
  // only when 4 * upper children might not fit the next list.
  hipError_t level_pass(int d, int64_t n, int64_t upper, bool top) {
    hipError_t e;
    const unsigned long long* nd = n >= 0 ? nullptr : count_dev(d);
    if ((e = bound(d, (const uint64_t*)nodes[d].p, (double*)vals[d].p, n, nd, upper)) != hipSuccess) return e;
    return descend(d, n, upper, top, pyr_bound_blocks(upper, in.n_used));
  }

  // nodes[d] and vals[d] are in place, the block bests in partials.
  hipError_t descend(int d, int64_t n, int64_t upper, bool top, int64_t n_partials) {
    hipError_t e;
    const unsigned long long* nd = n >= 0 ? nullptr : count_dev(d);
    if (d == 0)
      return launch_pyr_final((const PyrPartial*)partials.p, n_partials, true, 0, inc_dev(), nullptr,
                              in.stream);
    if (probes && (top || n >= probe_min) && (e = probe(d, n_partials)) != hipSuccess) return e;
    const int64_t child_upper = std::min(4 * upper, possible[d - 1]);
    if (child_upper <= capd[d - 1]) {
      if ((e = expand(d, 0, n, nd, upper)) != hipSuccess) return e;
      return level_pass(d - 1, -1, child_upper, false);
    }
    // optimistic: expand everything, then look at the count
    if ((e = expand(d, 0, n, nd, upper)) != hipSuccess) return e;
    if ((e = read_counts(d)) != hipSuccess) return e;
    const int64_t m = (int64_t)h_counts[0];
    if (n < 0) n = (int64_t)h_counts[1];
    if (m <= capd[d - 1]) return m > 0 ? level_pass(d - 1, m, m, false) : hipSuccess;
    // overflow (children dropped): slices of capacity / 4 parents, each descended
    const int64_t slice = std::max<int64_t>(1, capd[d - 1] / 4);
    for (int64_t s = 0; s < n; s += slice) {
      const int64_t k = std::min(slice, n - s);
      if ((e = expand(d, s, k, nullptr, k)) != hipSuccess) return e;
      if ((e = level_pass(d - 1, -1, 4 * k, false)) != hipSuccess) return e;
    }
    return hipSuccess;
  }
};

PyramidSearch::PyramidSearch() : p_(new Impl) {}
PyramidSearch::~PyramidSearch() { delete p_; }

void PyramidSearch::release() {
  delete p_;
  p_ = new Impl;
}

void PyramidSearch::configure(int64_t node_capacity, int probe_min_nodes) {
  p_->cap = node_capacity > 0 ? std::max<int64_t>(node_capacity, 4) : ((int64_t)1 << 25);
  p_->probe_min = probe_min_nodes > 0 ? probe_min_nodes : 4096;
  p_->probes = probe_min_nodes >= 0;
}

int64_t PyramidSearch::level_cells(int32_t sx, int32_t sy, int d) {
  const int32_t w = sx + (1 << d), h = sy + (1 << d);
  return (int64_t)((w + 3) & ~3) * h;
}

hipError_t PyramidSearch::run(const PyrInputs& x, BestPartial* best, PyrStats* stats, std::string* what) {
  Impl& I = *p_;
  PyrStats local;
  I.st = stats ? stats : &local;
  *I.st = PyrStats{};
  I.n_ev_bound = 0;
  I.st->depth = x.depth;
  I.in = x;
  hipError_t e;
  auto fail = [&](hipError_t err, const char* msg) {
    if (what) *what = msg;
    return err;
  };
  if (x.depth < 0 || x.depth > kPyrMaxDepth) return fail(hipErrorInvalidValue, "pyramid depth out of range");
  if ((e = I.build(x)) != hipSuccess) return fail(e, "pyramid levels");
  const int64_t nj = ((int64_t)x.L.n_space + (1 << x.depth) - 1) >> x.depth;
  const int64_t n_top = (int64_t)x.L.n_scans * x.L.n_angles * nj * nj;
  I.set_caps(x.L, x.depth);
  if ((e = I.ensure_lists(x.depth)) != hipSuccess) return fail(e, "pyramid node lists");
  for (int d = 0; d <= kPyrMaxDepth; ++d) I.cslot[d] = 0;
  I.next_slot = 1;
  if ((e = launch_pyr_init(I.inc_dev(), I.scored_dev(), kPyrMaxDepth + 1 + Impl::kCountSlots, x.stream)) != hipSuccess)
    return fail(e, "pyr_init_kernel");
  int32_t ktiles, kt, col_blocks;
  const int top_blocks = pyr_top_blocks(x.L, (int32_t)nj, &ktiles, &kt, &col_blocks);
  const int D = x.depth;
  int64_t top_scored = 0;
  // the top level as beam boxes: one-cell steps are given; the box test
  // needs |t| < 2^24 (box_ok), nj <= 32, a launch of n_scans * n_angles waves
  const int npc = pyr_topbox_pieces((int32_t)nj);
  const int64_t box_blocks = (int64_t)x.L.n_scans * x.L.n_angles;
  const bool use_box = D > 0 && x.top_mode == 0 && x.box_ok && x.one_scan && npc > 0 && box_blocks <= INT32_MAX &&
                       n_top <= ((int64_t)1 << 28) && x.n_used >= 1 && x.n_used <= 4096;
  if (use_box && (e = I.build_box(x, D, (int32_t)nj, npc)) == hipSuccess) {
    // the split waves' partial sums: only launches of few (window, angle)s split
    const size_t slab_ints = box_blocks < 4096 ? (size_t)n_top * kPyrTopMaxSplit : 0;  // launch_pyr_topbox's rule
    if ((e = I.top_sums.ensure((size_t)n_top * sizeof(int32_t))) != hipSuccess ||
        (e = I.top_thr.ensure(2 * sizeof(int64_t))) != hipSuccess ||
        (slab_ints && (e = I.top_slab.ensure(slab_ints * sizeof(int32_t))) != hipSuccess))
      return fail(e, "pyramid top level");
    if ((e = I.partials.ensure((size_t)std::max<int64_t>(box_blocks, pyr_blocks(INT64_MAX / 2)) *
                               sizeof(PyrPartial))) != hipSuccess)
      return fail(e, "pyramid partials");
    if (x.timed && (e = I.mark_top(0, x.stream)) != hipSuccess) return fail(e, "hipEventRecord");
    if ((e = launch_pyr_topbox(x.L, I.boxg, D, (int32_t)nj, x.scans, x.angles, x.pts, x.n_used, x.step,
                               (int32_t*)I.top_sums.p, slab_ints ? (int32_t*)I.top_slab.p : nullptr,
                               (PyrPartial*)I.partials.p, x.stream)) != hipSuccess)
      return fail(e, "pyr_topbox_kernel");
    if (x.timed) {
      if ((e = I.mark_top(1, x.stream)) != hipSuccess) return fail(e, "hipEventRecord");
      std::snprintf(I.st->top_name, sizeof(I.st->top_name), "pyr_topbox_kernel<%d,%d>", npc,
                    (int)((nj * npc + 63) / 64));
      I.st->top_bytes = (double)n_top * (double)x.n_used * 2.0;
    }
    top_scored = n_top;
    I.st->top_box = 1;
    I.top_implicit = D;
    I.top_nj = (int32_t)nj;
    e = I.descend(D, n_top, n_top, true, box_blocks);
    I.top_implicit = -1;
    if (e != hipSuccess) return fail(e, "pyramid level pass");
  } else if (use_box && e != hipErrorInvalidValue) {
    return fail(e, "pyramid box level");
  } else if (D > 0 && top_blocks > 0 && n_top <= ((int64_t)1 << 28)) {
    // the whole top level in one launch (column layout), then descend
    if ((e = I.nodes[D].ensure((size_t)n_top * sizeof(uint64_t))) != hipSuccess ||
        (e = I.vals[D].ensure((size_t)n_top * sizeof(double))) != hipSuccess)
      return fail(e, "pyramid top level");
    if ((e = I.partials.ensure((size_t)std::max<int64_t>(top_blocks, pyr_blocks(INT64_MAX / 2)) *
                               sizeof(PyrPartial))) != hipSuccess)
      return fail(e, "pyramid partials");
    if ((e = launch_pyr_top_bound(x.L, I.lev[D], D, (int32_t)nj, x.scans, x.angles, x.pts, x.n_used, x.step,
                                  (uint64_t*)I.nodes[D].p, (double*)I.vals[D].p, (PyrPartial*)I.partials.p,
                                  x.stream)) != hipSuccess)
      return fail(e, "pyr_top_bound_kernel");
    top_scored = n_top;
    if ((e = I.descend(D, n_top, n_top, true, top_blocks)) != hipSuccess) return fail(e, "pyramid level pass");
  } else {
    for (int64_t first = 0; first < n_top; first += I.capd[D]) {
      const int64_t m = std::min(I.capd[D], n_top - first);
      if ((e = launch_pyr_top(x.L, (int32_t)nj, first, m, (uint64_t*)I.nodes[D].p, x.stream)) != hipSuccess)
        return fail(e, "pyr_top_kernel");
      if ((e = I.level_pass(D, m, m, true)) != hipSuccess) return fail(e, "pyramid level pass");
    }
  }
  // the incumbent and the scored counts, one copy
  if ((e = hipMemcpyAsync(I.h_inc(), I.state.p, sizeof(BestPartial) + (kPyrMaxDepth + 1) * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, x.stream)) != hipSuccess)
    return fail(e, "incumbent copy");
  if ((e = hipStreamSynchronize(x.stream)) != hipSuccess) return fail(e, "pyramid search");
  unsigned long long* h_scored = I.h_scored();
  *best = I.h_inc()[0];
  for (int d = 0; d <= kPyrMaxDepth; ++d) I.st->nodes[d] = (int64_t)h_scored[d];
  if (x.timed && I.st->top_name[0]) {
    float ms = 0.f;
    if ((e = hipEventElapsedTime(&ms, I.ev_top[0], I.ev_top[1])) != hipSuccess) return fail(e, "hipEventElapsedTime");
    I.st->top_ms = ms;
  }
  for (int k = 0; k < I.n_ev_bound; ++k) {
    float ms = 0.f;
    if ((e = hipEventElapsedTime(&ms, I.ev_bound[2 * k], I.ev_bound[2 * k + 1])) != hipSuccess)
      return fail(e, "hipEventElapsedTime");
    const int d = I.ev_bound_depth[(size_t)k];
    I.st->bound_ms[d] += ms;
    I.st->bound_launches[d] += 1;
  }
  I.n_ev_bound = 0;
  I.st->nodes[D] += top_scored;
  return hipSuccess;
}

}  // namespace csm
