// csm_launch.cpp — a level's windows on the device: the window plan (the
// reference's angle LUT with host glibc sincos, AngleSearchLookUpTable
// :150-186, and the search start :538-548), the choice of scoring kernel, the
// launch with its device finish (run_windows, run_windows_small), the joins
// and the per-launch HIP-event accounting.
#include "csm_host.hpp"
#include "libm_sincos_table.hpp"

namespace csmh {

int window_dims(const csm_param& P, Dims& d) {
  if (!(P.search_angle_resolution > 0.0) || !(P.search_space_resolution > 0.0) ||
      !(P.search_angle_offset >= 0.0) || !(P.search_space_size >= 0.0))
    return CSM_ERR_INVALID_ARG;
  // serach_angle_size_ = offset*2 (:526); the LUT gets serach_angle_size_/2 (:536)
  const double half = (P.search_angle_offset * 2) / 2;
  const double na = std::floor(half * 2 / P.search_angle_resolution) + 1;
  const double ns = round_half_away(P.search_space_size / P.search_space_resolution) + 1;
  if (!(na >= 1.0 && na < 1e7 && ns >= 1.0 && ns < 1e7)) return CSM_ERR_INVALID_ARG;
  d.n_angles = (int32_t)na;
  d.n_space = (int32_t)ns;
  d.n_cand = (int64_t)d.n_angles * d.n_space * d.n_space;
  return CSM_OK;
}

// Beam subsampling (correlate_scan_matcher.h:561-566); false if the reference
// would divide by zero or loop forever (use_point_size <= 1 with n >= 2*U).
bool beam_rule(int n, int use_point_size, int& step, int& use, int& n_used) {
  use = use_point_size;
  if (n < 2 * use) {
    use = n;
    step = 1;
  } else {
    if (use - 1 <= 0) return false;
    step = n / (use - 1);
  }
  if (step <= 0) return false;
  n_used = (n + step - 1) / step;
  return true;
}

// Spin on the host flag the exact pass stores last (a launch + flag round
// trip measured 6 us on the GPU box against 12 us through an event,
// tools/ubench/roundtrip.hip). Every 256 spins the stream's event is
// polled: a launch that failed, or that completed without the flag, is an
// error instead of a hang.
int wait_flag(csm_ctx* c, const PendingRun& p, const int32_t* flag) {
  if (!flag) flag = p.host_flag;
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == p.flag_value) return CSM_OK;
    if ((spin & 255) == 0) {
      const hipError_t e = hipEventQuery(p.done);
      if (e == hipSuccess) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == p.flag_value) return CSM_OK;
        return c->fail(CSM_ERR_HIP, "finish: the level completed without its host signal");
      }
      if (e != hipErrorNotReady) return c->hip_fail(e, "hipEventQuery(level)");
    }
    __builtin_ia32_pause();
  }
}

int account_run(csm_ctx* c, const PendingRun& p);

int wait_run(csm_ctx* c, const PendingRun& p) {
  hipError_t e;
  if (p.host_flag) {
    const int st = wait_flag(c, p);
    if (st != CSM_OK) return st;
    if (p.timed && p.defer_timing) {
      c->deferred.push_back(p);
      return CSM_OK;
    }
    if (p.timed && (e = hipEventSynchronize(p.done)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize");
  } else if ((e = hipEventSynchronize(p.done)) != hipSuccess) {
    return c->hip_fail(e, "hipEventSynchronize");
  }
  return account_run(c, p);
}

// The timings of signalled launches, once their events have retired (before
// a launch records the events again, and before the stats are read).
int flush_deferred(csm_ctx* c) {
  int st = CSM_OK;
  for (const PendingRun& p : c->deferred) {
    const hipError_t e = hipEventSynchronize(p.done);
    if (e != hipSuccess) {
      st = c->hip_fail(e, "hipEventSynchronize(deferred)");
      break;
    }
    if ((st = account_run(c, p)) != CSM_OK) break;
  }
  c->deferred.clear();
  return st;
}

int account_run(csm_ctx* c, const PendingRun& p) {
  hipError_t e;
  if (p.timed) {
    float ms = 0.f;
    if ((e = hipEventElapsedTime(&ms, p.ev0, p.ev1)) != hipSuccess) return c->hip_fail(e, "hipEventElapsedTime");
    if (p.gap0) {  // two spans: the host's planning between them is not kernel time
      float g = 0.f;
      if ((e = hipEventElapsedTime(&g, p.gap0, p.gap1)) != hipSuccess) return c->hip_fail(e, "hipEventElapsedTime");
      ms -= g;
    }
    c->account(p.kname, ms, p.alg_bytes, p.scorings);
    if (p.gap0) {  // the same launch again under "span2:": two dispatches, each with its own ramp and tail
      char nm[48];  // (its bytes too: the one-dispatch launches' bytes per ms are then known)
      std::snprintf(nm, sizeof(nm), "span2:%.41s", p.kname);
      c->account(nm, ms, p.alg_bytes, 0.0);
    }
    if (p.device_finish) {
      if ((e = hipEventElapsedTime(&ms, p.ev1, p.ev2)) != hipSuccess) return c->hip_fail(e, "hipEventElapsedTime");
      c->account(p.fname, ms, p.finish_bytes, 0.0);
      if (p.ev_fast) {  // the same interval in its two passes: the fast one on the kernel stream, then
                        // the exact one on x_stream (it overlaps the other part's scoring)
        float mf = 0.f, mx = 0.f;
        if ((e = hipEventElapsedTime(&mf, p.ev1, p.ev_fast)) != hipSuccess ||
            (e = hipEventElapsedTime(&mx, p.ev_fast, p.ev2)) != hipSuccess)
          return c->hip_fail(e, "hipEventElapsedTime");
        const char* lt = std::strchr(p.fname, '<');
        char nm[48];
        std::snprintf(nm, sizeof(nm), "finish:fast%s", lt ? lt : "");
        c->account(nm, mf, 0.0, 0.0);
        std::snprintf(nm, sizeof(nm), "finish:exact%s", lt ? lt : "");
        c->account(nm, mx, 0.0, 0.0);
      }
      if (p.flags) {  // "scorings" of this entry = windows that took the exact sort
        int exact = 0;
        for (int i = 0; i < p.n_flags; ++i) exact += p.flags[i] != 0;
        c->account("finish:exact_windows", 0.f, 0.0, (double)exact);
        char nm[48];  // per level: "finish_kernel<n>" -> "finish:exact_windows<n>" (bytes = windows)
        const char* lt = std::strchr(p.fname, '<');
        std::snprintf(nm, sizeof(nm), "finish:exact_windows%s", lt ? lt : "");
        c->account(nm, 0.f, (double)p.n_flags, (double)exact);
      }
    }
  }
  return CSM_OK;
}

// Phase buckets of a sub-cell window step f (csm_phase.hip): candidate j of a
// beam with phase p = frac((lx + x0) + 0.5) reads column floor(p + j*f) past
// the beam's cell; that changes only where p + j*f crosses an integer, at the
// breakpoints ceil(j*f) - j*f. Breakpoints closer than 4 margins merge into
// one cluster; each gap between clusters, shrunk by the margin on both sides,
// is a bucket with fixed offsets ox[q][j]. Computed in long double, where
// j*f and the differences are exact (f has 53 bits, j < 2^11).
bool phase_table(double f, int ns, int margin_log2, csm::PhaseTable& T) {
  T = csm::PhaseTable{};
  if (!(f > 0.0 && f < 1.0) || ns < 1 || ns > csm::kPhaseMaxSpace) return false;
  const long double M = std::ldexp(1.0L, -margin_log2);
  std::vector<long double> bp = {0.0L, 1.0L};
  for (int j = 0; j < ns; ++j) {
    const long double jf = (long double)j * (long double)f;
    bp.push_back(std::ceil(jf) - jf);
  }
  std::sort(bp.begin(), bp.end());
  std::vector<std::pair<long double, long double>> cl;  // clusters [first, last]
  for (long double b : bp) {
    if (!cl.empty() && b - cl.back().second < 4 * M) cl.back().second = b;
    else cl.push_back({b, b});
  }
  int cells = 0;
  for (size_t i = 0; i + 1 < cl.size(); ++i) {
    const long double lo = cl[i].second + M, hi = cl[i + 1].first - M;
    if (!(hi > lo)) continue;
    if (T.nq == csm::kPhaseMaxBuckets) return false;
    const long double mid = (lo + hi) / 2;
    for (int j = 0; j < ns; ++j) {
      const long double o = std::floor(mid + (long double)j * (long double)f);
      if (o < 0 || o > 15) return false;
      T.ox[T.nq][j] = (int8_t)o;
      cells = std::max(cells, (int)o + 1);
    }
    // rounded inwards: a phase the device accepts lies inside [lo, hi]
    T.lo[T.nq] = std::nextafter((double)lo, 2.0);
    T.hi[T.nq] = std::nextafter((double)hi, -1.0);
    T.nq++;
  }
  T.cells = cells;
  if (T.nq > 0) {  // equal-width buckets: the fast form (PhaseTable::uniform)
    const long double n = (long double)T.nq;
    long double ulo = 0.0L, uhi = 1.0L;
    bool uni = true;
    for (int q = 0; q < T.nq && uni; ++q) {
      const long double a = (long double)T.lo[q] * n - q, b = (long double)T.hi[q] * n - q;
      uni = a > 0.0L && a < 0.25L && b > 0.75L && b < 1.0L;
      ulo = std::max(ulo, a);
      uhi = std::min(uhi, b);
    }
    // (phase * nq in fp64 is within 2^-50 of the real product: 1e-12 covers it)
    if (uni && uhi - ulo > 0.5L) {
      T.uniform = 1;
      T.ulo = std::nextafter((double)(ulo + 1e-12L), 2.0);
      T.uhi = std::nextafter((double)(uhi - 1e-12L), -1.0);
    }
  }
  return T.nq > 0;
}


// Exact fixed-point accumulation for one window: beams bounded, no offset
// wrap (every endpoint within 2^30 bytes of a row); the context's grid must
// be eligible too (c->int_ok).
bool int_mode_window_ok(const csm_ctx* c, const Dims& D, double f, const WindowPlan& W) {
  const double far = (double)(D.n_space - 1) * f;
  const double span = std::max(std::max(std::fabs(W.x0), std::fabs(W.x0 + far)),
                               std::max(std::fabs(W.y0), std::fabs(W.y0 + far)));
  const double R = c->pts_maxabs * (1.0 + 1e-9) + span + 2.0;
  if (!(R * 4.0 * (double)c->pitch < std::ldexp(1.0, 30))) return false;
  return !((double)W.n_used * c->int_max_abs * std::ldexp(1.0, c->int_exp) > std::ldexp(1.0, 53));
}

// ... for windows [i0, i1)
bool int_mode_ok(const csm_ctx* c, const Dims& D, double f, const std::vector<WindowPlan>& plans, size_t i0 = 0,
                 size_t i1 = SIZE_MAX) {
  if (!c->int_ok) return false;
  for (size_t i = i0; i < std::min(i1, plans.size()); ++i)
    if (!int_mode_window_ok(c, D, f, plans[i])) return false;
  return true;
}

void fill_scan_work_one(const Dims& D, const WindowPlan& W, int64_t pt_off, int32_t grid, size_t i, int64_t stride,
                        ScanWork& s) {
  s.pts_off = pt_off;
  s.angle_off = W.angle_off;
  s.out_off = (int64_t)i * (stride ? stride : D.n_cand);
  s.n_used = W.n_used;
  s.step = W.step;
  s.divisor = (double)(W.use - 0);
  s.x0 = W.x0;
  s.y0 = W.y0;
  s.cx = W.center[0];
  s.cy = W.center[1];
  s.ct = W.center[2];
  s.reserved = (int32_t)i;  // the window's index in its level (the fused finish's counters)
  s.grid_index = grid;
}

// stride: scores between consecutive windows (0: n_cand; the signalled device
// finish pads each window to whole 128-byte lines, score_stride)
void fill_scan_work(const Dims& D, const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                    const std::vector<int32_t>& grid_index, ScanWork* sw, size_t i0 = 0, size_t i1 = SIZE_MAX,
                    int64_t stride = 0) {
  for (size_t i = i0; i < std::min(i1, plans.size()); ++i)
    fill_scan_work_one(D, plans[i], pt_offsets[i], grid_index.empty() ? 0 : grid_index[i], i, stride, sw[i]);
}

bool signalled_finish(const csm_ctx* c, Finish mode) {
  return c->host_signal && mode == Finish::kDevice && c->fast_finish;
}

// Scores between consecutive windows of a launch: whole 128-byte lines per
// window with the host-signal device finish (the fused finish needs them: no
// line shared by two windows' finishers, csm_tail.hpp; the other signalled
// passes read through FinishArgs::score_stride), n_cand otherwise (the scores
// go to the host contiguous).
int64_t score_stride(const csm_ctx* c, const Dims& D, Finish mode) {
  return signalled_finish(c, mode) ? (D.n_cand + 15) / 16 * 16 : D.n_cand;
}

LevelWork make_level_work(const csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G, int nw,
                          bool use_int) {
  LevelWork L{};
  L.n_angles = D.n_angles;
  L.n_space = D.n_space;
  L.n_cand = D.n_cand;
  L.blocks_per_scan = D.n_angles;
  L.n_scans = nw;
  L.tile_ns = D.n_space;
  L.step_cells = P.search_space_resolution / G.mres;
  L.use_penalty = P.use_center_penalty ? 1 : 0;
  L.dist_gain = (P.type == CSM_COARSE) ? 0.4 : 0.2;  // :759-761
  L.size = P.search_space_size;
  L.mres = G.mres;
  L.grid = c->d_grid;
  L.grid_stride = (int64_t)c->info.size_x * c->info.size_y;
  L.size_x = c->info.size_x;
  L.size_y = c->info.size_y;
  L.outside = c->outside;
  L.int_mode = use_int ? 1 : 0;
  L.gridi = c->d_gridi;
  L.int_scale = std::ldexp(1.0, -c->int_exp);
  L.outside_i = c->outside_i;
  L.pitch = c->pitch;
  L.gridi_stride = (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows);
  return L;
}

// The reference's calling pattern, one scan and one level at a time
// (ScanMatchers::ScanMatch, scan_matchers.h:238-256), leaves the throughput
// kernels' one wave per (window, angle) on a few dozen waves; few windows go
// through the split kernel and a 16-wave fast finish instead.
bool small_launch(const csm_ctx* c, const Dims& D, int nw) {
  return c->small_path && c->fast_finish && nw <= c->small_max_windows && D.n_cand <= csm::kFinishMaxCand &&
         D.n_cand * (int64_t)nw <= INT32_MAX && csm::finish_lds_bytes(D.n_cand) <= 160 * 1024;
}

// Few-window launch: the split kernel (csm_split.hip) scores, the fast and
// exact finishes write each window's FinishOut straight into coherent pinned
// host memory, and the exact pass stores a fresh flag value last (wait_run
// spins on it). Everything on the context's stream; a single window with a
// small angle table travels in the kernel arguments, otherwise one H2D copy.
int run_windows_small(csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G,
                      const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                      const AngleEntry* angles, size_t n_angle_entries, const std::vector<int32_t>& grid_index,
                      bool device_finish, PendingRun* pend, int skip_lists) {
  const int nw = (int)plans.size();
  hipError_t e;
  // device carve: done counter (fixed place: zero between launches) | scans |
  // angles | need | list
  const size_t o_done = 0, o_scans = 64;
  const size_t o_ang = ((o_scans + (size_t)nw * sizeof(ScanWork)) + 15) & ~(size_t)15;
  const size_t o_need = (o_ang + n_angle_entries * sizeof(AngleEntry) + 15) & ~(size_t)15;
  const size_t o_list = (o_need + (size_t)nw * 4 + 7) & ~(size_t)7;  // {count, tag}: one 8-byte word
  const size_t dev_bytes = o_list + (size_t)(nw + 2) * 4;
  if (dev_bytes > c->small_dev.cap) {
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(small)");
    if ((e = c->small_dev.ensure(dev_bytes * 2)) != hipSuccess) return c->hip_fail(e, "hipMalloc(small)");
    if ((e = hipMemsetAsync(c->small_dev.p, 0, c->small_dev.cap, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemsetAsync(small)");
  }
  char* dv = (char*)c->small_dev.p;
  ScanWork* d_scans = (ScanWork*)(dv + o_scans);
  AngleEntry* d_angles = (AngleEntry*)(dv + o_ang);
  int32_t* d_need = (int32_t*)(dv + o_need);
  int32_t* d_list = (int32_t*)(dv + o_list);
  int32_t* d_done = (int32_t*)(dv + o_done);
  // host side: the windows' staging (laid out as the device carve from
  // o_scans on), and FinishOut[nw] + the flag (coherent)
  const size_t in_bytes = o_ang - o_scans + n_angle_entries * sizeof(AngleEntry);
  const size_t out_flag = ((size_t)nw * sizeof(csm::FinishOut) + 63) & ~(size_t)63;
  if ((e = c->h_small_in.ensure(in_bytes)) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(small in)");
  if (out_flag + 64 > c->h_small_out.cap) {
    if ((e = c->h_small_out.ensure(std::max<size_t>(out_flag + 64, 64 * 1024), hipHostMallocCoherent)) != hipSuccess)
      return c->hip_fail(e, "hipHostMalloc(small out)");
    std::memset(c->h_small_out.p, 0, c->h_small_out.cap);
  }
  csm::FinishOut* h_out = (csm::FinishOut*)c->h_small_out.p;
  int32_t* h_flag = (int32_t*)((char*)c->h_small_out.p + out_flag);
  ScanWork* sw = (ScanWork*)c->h_small_in.p;
  fill_scan_work(D, plans, pt_offsets, grid_index, sw);
  LevelWork L = make_level_work(c, P, D, G, nw, true);

  // splits: enough blocks to spread the level over the chip, at least
  // ceil(beams / kSplitMaxBeams) (int32 sums), at most one per 4 beams
  int max_used = 1;
  for (const WindowPlan& W : plans) max_used = std::max(max_used, W.n_used);
  const int64_t chunks = (D.n_cand + csm::kSplitThreads - 1) / csm::kSplitThreads;
  const int min_splits = (max_used + csm::kSplitMaxBeams - 1) / csm::kSplitMaxBeams;
  const int64_t want = (c->split_target_blocks + (int64_t)nw * chunks - 1) / ((int64_t)nw * chunks);
  const int splits = (int)std::max<int64_t>(min_splits, std::min<int64_t>(want, std::max(1, max_used / 4)));
  const size_t slab_bytes = (size_t)nw * (size_t)chunks * (size_t)splits * csm::kSplitThreads * sizeof(int32_t);
  const size_t arrive_bytes = (size_t)nw * (size_t)chunks * sizeof(int32_t);
  if ((e = c->split_slab.ensure(slab_bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(split slab)");
  if (arrive_bytes > c->split_arrive.cap) {  // counters start at zero; each launch leaves them at zero
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(split)");
    if ((e = c->split_arrive.ensure(arrive_bytes * 2)) != hipSuccess) return c->hip_fail(e, "hipMalloc(split arrive)");
    if ((e = hipMemsetAsync(c->split_arrive.p, 0, c->split_arrive.cap, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemsetAsync(split arrive)");
  }
  csm::SplitWork W{};
  W.splits = splits;
  W.chunks = (int32_t)chunks;
  W.slab = (int32_t*)c->split_slab.p;
  W.arrive = (int32_t*)c->split_arrive.p;
  W.clear_word = d_list;
  // the launch's flag value, also the tag its scoring kernel puts on the list
  int32_t flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
  if (flag_value == 0) flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
  W.clear_tag = flag_value;
  W.inline_window = (nw == 1 && D.n_angles <= csm::kSplitArgAngles && n_angle_entries == (size_t)D.n_angles) ? 1 : 0;
  if (W.inline_window) {
    W.sw = sw[0];
    W.sw.angle_off = 0;  // the copy block 0 stores for the finish starts the angle rows
    std::memcpy(W.ang, angles, (size_t)D.n_angles * sizeof(AngleEntry));
    W.scans_out = d_scans;
    W.angles_out = d_angles;
  } else {
    std::memcpy((char*)c->h_small_in.p + (o_ang - o_scans), angles, n_angle_entries * sizeof(AngleEntry));
    if ((e = hipMemcpyAsync(d_scans, c->h_small_in.p, in_bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(small windows)");
  }
  const size_t bytes = (size_t)nw * (size_t)D.n_cand * sizeof(double);
  if ((e = c->scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(scores)");
  if (c->profiling && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
  if ((e = csm::launch_score_split(L, W, d_scans, (const double*)c->pts.p, d_angles, (double*)c->scores.p,
                                   c->stream)) != hipSuccess)
    return c->hip_fail(e, "score_split_kernel");
  if (c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
  PendingRun local;
  PendingRun& p = pend ? *pend : local;
  p = PendingRun{};
  std::snprintf(p.kname, sizeof(p.kname), "score_split_kernel<%d,%d>", D.n_space, splits);
  double beams = 0.0;
  for (const WindowPlan& Wp : plans) beams += (double)Wp.n_used;
  p.alg_bytes = beams * (double)D.n_cand * 4.0;
  p.scorings = (double)nw * (double)D.n_cand;
  p.timed = c->profiling;
  p.ev0 = c->ev0;
  p.ev1 = c->ev1;
  p.ev2 = c->ev2;
  p.done = c->ev_done;
  if (!device_finish) {  // every score to the host (csm_score_window, host std::sort)
    if ((e = c->h_scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(scores)");
    if ((e = hipMemcpyAsync(c->h_scores.p, c->scores.p, bytes, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(scores)");
    if ((e = hipEventRecord(c->ev_done, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if (pend) return CSM_OK;
    return wait_run(c, p);
  }
  csm::FinishArgs A{};
  A.n_cand = D.n_cand;
  A.n_space = D.n_space;
  A.step_cells = L.step_cells;
  A.lin_tol = P.search_space_resolution / G.mres;
  A.skip_lists = skip_lists | own_lists_skip(P.type);
  A.need_exact = d_need;
  A.exact_list = d_list;
  A.done_ctr = d_done;
  A.host_flag = h_flag;
  A.wide_windows = c->fast_wide_windows;
  A.flag_value = flag_value;
  if ((e = csm::launch_finish(A, d_scans, d_angles, (const double*)c->scores.p, h_out, nw, c->stream)) != hipSuccess)
    return c->hip_fail(e, "finish_kernel");
  if (c->profiling && (e = hipEventRecord(c->ev2, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
  std::snprintf(p.fname, sizeof(p.fname), "finish_kernel<%lld>", (long long)D.n_cand);
  p.finish_bytes = (double)nw * (double)D.n_cand * 8.0;
  p.device_finish = true;
  p.fin_host = h_out;
  p.host_flag = h_flag;
  p.flag_value = A.flag_value;
  if ((e = hipEventRecord(c->ev_done, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
  if (pend) return CSM_OK;
  return wait_run(c, p);
}

// The fused fast finish (csm_tail.hpp); CSM_TAIL_FINISH=0 builds keep the
// separate fast-pass launch (A/B).
#ifndef CSM_TAIL_FINISH
#define CSM_TAIL_FINISH 1
#endif
constexpr bool kTailFinish = CSM_TAIL_FINISH != 0;
#ifndef CSM_TAIL_MAX_BEAMS
#define CSM_TAIL_MAX_BEAMS 512
#endif
constexpr int kTailMaxBeams = CSM_TAIL_MAX_BEAMS;  // levels summing more beams keep the separate fast pass

int run_windows(csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G,
                const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                const AngleEntry* angles, size_t n_angle_entries,
                const std::vector<int32_t>& grid_index, BestPartial* best_out,
                Finish mode, PendingRun* pend, int skip_lists, WinSpan sp) {
  if (best_out) mode = Finish::kBest;
  const int nw = (int)plans.size();
  if (nw == 0) return CSM_OK;
  const int w0 = sp.w1 < 0 ? 0 : sp.w0, w1 = sp.w1 < 0 ? nw : sp.w1;
  const int nr = w1 - w0;  // windows scored by this call
  const bool whole = w0 == 0 && w1 == nw && sp.score && sp.finish;
  const double tp0 = c->profiling ? now_ms() : 0.0;  // host cost of the launch before its inputs (host:launch:prep)
  if (!c->deferred.empty()) {  // the events below are recorded again
    const int fst = flush_deferred(c);
    if (fst != CSM_OK) return fst;
  }
  const double tp1 = c->profiling ? now_ms() : 0.0;  // (the deferred event reads are profiling's own cost)
  if (c->profiling) c->account("host:launch:flush_events", (float)(tp1 - tp0), 0.0, 0.0);
  if (!whole) {
    bool ok = mode == Finish::kDevice && (sp.score || sp.finish) && 0 <= w0 && w0 < w1 && w1 <= nw &&
              n_angle_entries == (size_t)nw * (size_t)D.n_angles;
    for (int w = w0; ok && w < w1; ++w) ok = plans[(size_t)w].angle_off == (int64_t)w * D.n_angles;
    if (!ok) return c->fail(CSM_ERR_INVALID_ARG, "run_windows: bad window span");
  }
  int st;
  if ((st = ensure_int_grid(c)) != CSM_OK) return st;
  // v2 column kernel: KT rows per lane, tiles balanced so at most a few rows idle
  const int ktiles = (D.n_space + 15) / 16;
  const int kt = (D.n_space + ktiles - 1) / ktiles;
  const int64_t n_cols = (int64_t)D.n_angles * D.n_space;
  const int64_t col_blocks = (n_cols + 63) / 64;
  if (n_cols >= INT32_MAX) return c->fail(CSM_ERR_UNSUPPORTED, "window too large for one launch");
  const double f = P.search_space_resolution / G.mres;
  // (sp.int_all: the plan pass found every window of the level in range)
  const bool use_int = (sp.int_all && c->int_ok) || int_mode_ok(c, D, f, plans, (size_t)w0, (size_t)w1);
  if (whole && mode != Finish::kBest && use_int && small_launch(c, D, nw))
    return run_windows_small(c, P, D, G, plans, pt_offsets, angles, n_angle_entries, grid_index,
                             mode == Finish::kDevice, pend, skip_lists);
  // v4 row-segment kernel: fixed-point grid and an instantiation whose row
  // segment covers the x-span of a group, (n_space-1)*f cells (+2 for the
  // truncations); the kernel re-checks and recomputes exactly if exceeded
  int rows_sq = 0;
  if (use_int && c->row_kernel && D.n_space <= 64) {
    const double span = (double)(D.n_space - 1) * f;
    // distinct columns of a group <= floor(span) + 2
    rows_sq = csm::rows_pick_sq(D.n_space, (int)std::floor(span * (1.0 + 1e-9) + 1e-9) + 2);
    if (c->info.size_x < 4 * rows_sq) rows_sq = 0;
  }
  // the box kernels' beam offsets are 24-bit products (BoxWave::point: the
  // point index and step * 16 each under 2^24). Over every window of the level,
  // not this call's span: the fused-finish decision below depends on it and must
  // be the same in every call of a level (level_ctr counts all of its windows).
  bool box_points_ok = true;
  for (const WindowPlan& W : plans) {
    box_points_ok = W.n_points < (1 << 24) && (int64_t)W.step * 16 < (1 << 24);
    if (!box_points_ok) break;
  }
  // v6 box kernel: whole-cell window step (use_int bounds |t| < 2^24 cells,
  // which its rounding margin needs)
  const bool box = use_int && box_points_ok && c->box_kernel && f == 1.0 && csm::box_supported(D.n_space) &&
                   c->pitch >= c->info.size_x + csm::kGridiPadCols;
  if (box) rows_sq = 0;
  // v11: the box read through the grid's palette (one byte per cell), pairs
  // of equal-count runs over the strip copies (palettes of <= 16 values);
  // otherwise the v6 kernel reads gridi
  bool box_pal = false;
  if (box && c->pair_kernel && csm::box_pair_supported(D.n_space)) {
    if ((st = ensure_palette(c)) != CSM_OK) return st;
    box_pal = c->pal_n > 0 && (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows) <= INT32_MAX;
  }
  const bool box_pair = box_pal && c->pal_strips_ok;
  // v6 over 16 x 16 tiles: the argmax of a one-cell-step window wider than 16
  // (loop-closure windows), in place of the column kernel's dword gathers
  const int tile_n = (D.n_space + 15) / 16;
  const bool box_tiled = !box && best_out && use_int && box_points_ok && c->box_kernel && f == 1.0 && D.n_space > 16 &&
                         c->pitch >= c->info.size_x + csm::kGridiPadCols &&
                         (int64_t)nw * tile_n * tile_n * D.n_angles <= INT32_MAX;
  if (box_tiled) rows_sq = 0;
  // v7 phase kernel: sub-cell window step with an instantiated bucket shape
  csm::PhaseTable PT{};
  const bool phase = !box && use_int && c->phase_kernel && f < 1.0 &&
                     phase_table(f, D.n_space, c->phase_margin_log2, PT) &&
                     csm::phase_supported(D.n_space, PT.cells, PT.nq) &&
                     c->pitch >= c->info.size_x + csm::kGridiPadCols;
  if (phase) rows_sq = 0;
  if (phase && c->phase_strips && (st = ensure_istrips(c)) != CSM_OK) return st;
  const bool phase_st = phase && c->phase_strips && c->istrips_ok;
  // v8 tiny-window kernel: a sub-cell step whose whole span is under one cell
  const bool tiny = !box && !phase && use_int && c->tiny_kernel && f < 1.0 && csm::tiny_supported(D.n_space, f) &&
                    c->pitch >= c->info.size_x + csm::kGridiPadCols &&
                    (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows) * 4 < INT32_MAX;
  if (tiny) rows_sq = 0;
  const int64_t rows_groups = rows_sq ? 64 / D.n_space : 1;
  const int64_t bps = box_tiled ? (int64_t)tile_n * tile_n * D.n_angles
                      : (box || phase || tiny) ? D.n_angles
                      : rows_sq ? (D.n_angles + rows_groups - 1) / rows_groups
                                : col_blocks * ktiles;
  if (bps * nr > INT32_MAX) return c->fail(CSM_ERR_UNSUPPORTED, "window too large for one launch");

  hipError_t e;
  if ((e = c->h_sw.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(scans)");
  ScanWork* sw = (ScanWork*)c->h_sw.p;  // pinned staging
  // Host-signal finish (the device finish with its fast pass): FinishOut goes
  // straight to coherent pinned memory and the pass that ends last sets a flag
  // the host spins on; the scoring kernel clears the flagged-window count.
  const bool sig = signalled_finish(c, mode);
  // The fused fast finish (csm_tail.hpp): the level's scoring launches finish
  // their windows themselves, no fast-pass launch. The same decision in every
  // call of a level (its spans and its finish-only call): every window in
  // fixed-point range and a kernel that carries the finish. Each window's
  // scores then start on a 128-byte line of their own (no line is shared by
  // two windows: a finisher's sc1 loads never find a line another window's
  // finisher brought into its L2 before that window's scores were stored).
  // Only for short scoring waves: each wave waits for its write-through score
  // stores before counting in, which at B = 1081 costs the scoring launches
  // as much as the separate fast pass costs (r05: +55 / +30 / +43 us on the
  // box / phase / tiny launches against -32 / -31 / -29 us of fast passes);
  // at B = 109 the host gets each level's signal ~50 us earlier and the step
  // shortens.
  int max_beams = 0;
  for (const WindowPlan& W : plans) max_beams = std::max(max_beams, (int)W.n_used);
  const bool tail = kTailFinish && sig && (box || phase || tiny) && max_beams <= kTailMaxBeams &&
                    (whole ? use_int : (sp.int_all && c->int_ok) || int_mode_ok(c, D, f, plans, 0, (size_t)nw));
  const int64_t stride = score_stride(c, D, mode);
  // the plan pass may have filled this call's ScanWork already (WinSpan::sw_ready:
  // level_plan_one, into this slot's staging, at this stride)
  if (sp.score && !(sp.sw_ready && sp.sw_stride == stride && (const void*)sp.sw_ready == (const void*)sw))
    fill_scan_work(D, plans, pt_offsets, grid_index, sw, (size_t)w0, (size_t)w1, stride);
  LevelWork L = make_level_work(c, P, D, G, nr, use_int);
  L.blocks_per_scan = box_tiled ? D.n_angles : (int32_t)bps;  // per (window, tile) when tiled
  L.max_n_used = max_beams;
  L.tile_n = box_tiled ? tile_n : 0;
  if (box_pair) {
    L.pal_n = c->pal_n;
    L.pal_grid = (const uint8_t*)c->pal_grid.p;
    L.pal_vals = (const int32_t*)c->pal_vals.p;
    L.pal_stride = (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows);
  }
  if (phase_st) {
    const csm::StripGeom SG = csm::istrip_geom(c->info.size_x, c->info.size_y);
    L.istrips = (const int32_t*)c->istrips.p;
    L.istrip_bytes = (int32_t)SG.strip_bytes;
    L.istrip_copy_bytes = (int32_t)SG.copy_bytes;
    L.istrip_grid_bytes = SG.grid_bytes;
  }
  if (box_pair) {
    const csm::StripGeom SG = csm::strip_geom(c->info.size_x, c->info.size_y);
    L.pal_strips = (const uint8_t*)c->pal_strips.p;
    L.strip_bytes = (int32_t)SG.strip_bytes;
    L.strip_copy_bytes = (int32_t)SG.copy_bytes;
    L.strip_grid_bytes = SG.grid_bytes;
  }
  L.n_cols = (int32_t)n_cols;
  L.ktiles = ktiles;
  L.col_blocks = (int32_t)col_blocks;

  int32_t *d_done = nullptr, *d_need = nullptr, *d_list = nullptr;
  int32_t sig_tag = 0;
  if (sig) {
    // done counter (0) | the fused finish's level counter (32) | need[nw] |
    // list {count, tag, windows[nw]}
    const size_t o_need = 64, o_list = (o_need + (size_t)nw * 4 + 7) & ~(size_t)7;  // {count, tag}: 8 bytes
    const size_t dbytes = o_list + (size_t)(nw + 2) * 4;
    if (dbytes > c->fin_sig.cap) {  // the counters start at zero; each launch leaves them at zero
      if ((e = c->fin_sig.ensure(dbytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(finish signal)");
      if ((e = hipMemsetAsync(c->fin_sig.p, 0, c->fin_sig.cap, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipMemsetAsync(finish signal)");
    }
    d_done = (int32_t*)c->fin_sig.p;
    d_need = (int32_t*)((char*)c->fin_sig.p + o_need);
    d_list = (int32_t*)((char*)c->fin_sig.p + o_list);
    // The level's first scoring call's block 0 clears the list to {0, tag}
    // (with the fused finish, the windows' finishers of every span append
    // after it, csm_tail.hpp)
    L.clear_word = (sp.score && w0 == 0) ? d_list : nullptr;
    // A fresh tag per level: its first scoring call draws it, later spans and
    // the finish (the level's last call, which may score nothing itself) use
    // the slot's latest one as their flag value. The slot's previous exact
    // pass (on x_stream) may still be queued when this level's scoring and
    // fast pass reuse the list: it had no windows (or the host would not have
    // gone on), and it finds another tag.
    if (sp.score && w0 == 0) {
      c->list_tag = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
      if (c->list_tag == 0) c->list_tag = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
    }
    sig_tag = c->list_tag;
    L.clear_tag = sig_tag;
  }
  // the signalled finish's arguments (the fused finish's and the finish call's)
  csm::FinishArgs SA{};
  csm::FinishOut* sig_out = nullptr;
  int32_t* sig_flag = nullptr;
  int32_t* sig_fast = nullptr;
  const int32_t* flags_h = nullptr;
  int n_flags = 0;
  if (sig) {
    SA.n_cand = D.n_cand;
    SA.score_stride = stride;
    SA.n_space = D.n_space;
    SA.step_cells = L.step_cells;
    SA.lin_tol = P.search_space_resolution / G.mres;
    SA.skip_lists = skip_lists | own_lists_skip(P.type);
    SA.need_exact = d_need;
    SA.exact_list = d_list;
    SA.done_ctr = d_done;
    SA.wide_windows = c->fast_wide_windows;
    // FinishOut[nw] | need[nw] (profiling: the flags the host counts) | flag
    const size_t out_need = ((size_t)nw * sizeof(csm::FinishOut) + 63) & ~(size_t)63;
    const size_t out_flag = (out_need + (size_t)nw * sizeof(int32_t) + 63) & ~(size_t)63;
    if (out_flag + 64 > c->h_fin_sig.cap) {
      if ((e = c->h_fin_sig.ensure(std::max<size_t>(out_flag + 64, 64 * 1024), hipHostMallocCoherent)) != hipSuccess)
        return c->hip_fail(e, "hipHostMalloc(finish signal)");
      std::memset(c->h_fin_sig.p, 0, c->h_fin_sig.cap);
    }
    sig_out = (csm::FinishOut*)c->h_fin_sig.p;
    sig_flag = (int32_t*)((char*)c->h_fin_sig.p + out_flag);
    if (c->profiling && !c->profile_first_level) {  // the fast pass's flags to the host: finish:exact_windows
      SA.need_exact = (int32_t*)((char*)c->h_fin_sig.p + out_need);
      flags_h = SA.need_exact;
      n_flags = nw;
    }
    SA.host_flag = sig_flag;
    SA.flag_value = sig_tag;
    SA.host_fast_flag = (c->early_complete && c->early_now) ? sig_flag + 8 : nullptr;  // same 64-byte slot
    sig_fast = SA.host_fast_flag;
  }
  if (tail) {
    L.tail.on = 1;
    L.tail.n_windows = nw;
    // the window counters: a buffer of their own, zeroed when it grows and
    // left at zero by every window's finisher (need and the list, whose
    // offsets move with nw, hold stale values)
    if ((size_t)nw * sizeof(int32_t) > c->win_ctr.cap) {
      if ((e = c->win_ctr.ensure((size_t)nw * sizeof(int32_t))) != hipSuccess)
        return c->hip_fail(e, "hipMalloc(window counters)");
      if ((e = hipMemsetAsync(c->win_ctr.p, 0, c->win_ctr.cap, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipMemsetAsync(window counters)");
    }
    L.tail.win_ctr = (int32_t*)c->win_ctr.p;
    L.tail.level_ctr = d_done + 8;
    L.tail.out = sig_out;
    L.tail.A = SA;
    if ((e = c->ang_max.ensure((size_t)nw * (size_t)D.n_angles * sizeof(double))) != hipSuccess)
      return c->hip_fail(e, "hipMalloc(angle maxima)");
    L.tail.ang_max = (double*)c->ang_max.p;
    if (sp.score && w0 == 0 && c->tail_open) {  // an earlier level of this slot stopped between spans
      if ((e = hipMemsetAsync(c->fin_sig.p, 0, c->fin_sig.cap, c->stream)) != hipSuccess ||
          (e = hipMemsetAsync(c->win_ctr.p, 0, c->win_ctr.cap, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipMemsetAsync(stale tail counters)");
      c->tail_open = false;
    }
  }

  if ((e = c->scans.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scans)");
  if ((e = c->angles.ensure(n_angle_entries * sizeof(AngleEntry))) != hipSuccess) return c->hip_fail(e, "hipMalloc(angles)");
  const double tl0 = c->profiling ? now_ms() : 0.0;  // host cost of the launch, by phase
  if (c->profiling) c->account("host:launch:prep", (float)(tl0 - tp1), 0.0, 0.0);
  if (sp.score) {  // this call's windows and angle rows
    const size_t a0 = whole ? 0 : (size_t)w0 * D.n_angles;
    const size_t na = whole ? n_angle_entries : (size_t)nr * D.n_angles;
    // (copied on the kernel stream itself instead, r03 A/B: 7.05-7.07 vs
    // 7.14-7.23 G scorings/s)
    hipStream_t is = c->h2d;
    if ((e = hipMemcpyAsync((ScanWork*)c->scans.p + w0, sw + w0, (size_t)nr * sizeof(ScanWork), hipMemcpyHostToDevice,
                            is)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(scans)");
    if (!(sp.dev_trig && sp.rows_gen) &&
        (e = hipMemcpyAsync((AngleEntry*)c->angles.p + a0, angles + a0, na * sizeof(AngleEntry), hipMemcpyHostToDevice,
                            is)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(angles)");
    if (sp.dev_trig) {  // the rows' cos/sin (the plan left them to the device)
      const double* tab = libm_sincos_table();
      if (!tab) return c->fail(CSM_ERR_UNSUPPORTED, "run_windows: device trig without the libm table");
      if (!c->trig_tab.p) {
        if ((e = c->trig_tab.ensure(csm::libm::kSincosTableDoubles * sizeof(double))) != hipSuccess)
          return c->hip_fail(e, "hipMalloc(sincos table)");
        if ((e = hipMemcpyAsync(c->trig_tab.p, tab, csm::libm::kSincosTableDoubles * sizeof(double),
                                hipMemcpyHostToDevice, is)) != hipSuccess)
          return c->hip_fail(e, "hipMemcpyAsync(sincos table)");
      }
      if (sp.rows_gen)  // the rows whole from the windows' ScanWork (copied above)
        e = csm::launch_angle_rows((const ScanWork*)c->scans.p + w0, nr, D.n_angles, (P.search_angle_offset * 2) / 2,
                                   P.search_angle_resolution, (AngleEntry*)c->angles.p, (const double*)c->trig_tab.p, is);
      else
        e = csm::launch_angle_trig((AngleEntry*)c->angles.p + a0, (int64_t)na, (const double*)c->trig_tab.p, is);
      if (e != hipSuccess) return c->hip_fail(e, "angle rows kernel");
      // launches: the launches with device rows; bytes: the rows' copy saved
      if (c->profiling) c->account(sp.rows_gen ? "host:trig_rows:gen" : "host:trig_rows", 0.0f,
                                   (double)na * sizeof(AngleEntry), 0.0);
    }
    if ((e = hipEventRecord(c->ev_in, c->h2d)) != hipSuccess || (e = hipStreamWaitEvent(c->stream, c->ev_in, 0)) != hipSuccess)
      return c->hip_fail(e, "inputs event");
  }

  // algorithmic traffic: one fp32 grid read per summed beam per candidate
  double beams = 0.0;
  for (const WindowPlan& W : plans) beams += (double)W.n_used;
  const double alg_bytes = beams * (double)D.n_cand * 4.0;
  const double scorings = (double)nw * (double)D.n_cand;
  char kname[48];
  if (box_pair)
    std::snprintf(kname, sizeof(kname), "score_box_pair_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (box)
    std::snprintf(kname, sizeof(kname), "score_box_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (box_tiled)
    std::snprintf(kname, sizeof(kname), "score_box_kernel<16,best,tiles>");
  else if (phase)
    std::snprintf(kname, sizeof(kname), "score_phase_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (tiny)
    std::snprintf(kname, sizeof(kname), "score_tiny_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (rows_sq)
    std::snprintf(kname, sizeof(kname), "score_rowsd_kernel<%d,%d,%s>", D.n_space, rows_sq,
                  best_out ? "best" : "all");
  else
    std::snprintf(kname, sizeof(kname), "score_cols_kernel<%d,%s,%s>", kt, use_int ? "int" : "f64",
                  best_out ? "best" : "all");
  const double tl1 = c->profiling ? now_ms() : 0.0;
  // (a signalled launch lets the host go on before its exact pass on
  // x_stream has retired; the list's tag, LevelWork::clear_tag, makes a stale
  // pass exit, so the slot's next scoring need not wait for it)
  // An event recorded on the kernel stream right before every scoring launch
  // (ev0 when it is timed): measured, not explained — without it an unprofiled
  // config-2 step took 2.33-2.43 ms against 2.17-2.20 ms with it (r05,
  // profiles/r05/experiments/ab_event_before_scoring.txt); the launch follows
  // the stream's wait on the inputs' copy event (ev_in).
  if (sp.score && c->score_marker && !(c->profiling && w0 == 0) &&
      (e = hipEventRecord(c->ev_k, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipEventRecord");
  if (c->profiling && sp.score && w0 == 0 && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipEventRecord");
  // a later span: the gap since the first one ends here (only the first gap is
  // taken out of the level's kernel time; later ones are short, spans overlap)
  if (c->profiling && sp.score && w0 > 0 && !c->span_gap) {
    if ((e = hipEventRecord(c->ev_g1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    c->span_gap = true;
  }

  // csm_set_profiling(ctx, 2) times the scoring kernel alone: the finish's
  // events on the kernel stream would add gaps to the value's region
  const bool time_fin = c->profiling && !c->profile_first_level;
  int32_t sig_value = 0;
  hipStream_t done_stream = c->d2h;
  double tl2 = 0.0;
  if (mode != Finish::kBest) {
    const size_t bytes = (size_t)nw * (size_t)D.n_cand * sizeof(double);
    if ((e = c->scores.ensure((size_t)nw * (size_t)stride * sizeof(double))) != hipSuccess)
      return c->hip_fail(e, "hipMalloc(scores)");
    const ScanWork* d_sw = (const ScanWork*)c->scans.p + w0;
    if (!sp.score)
      e = hipSuccess;  // scored by earlier calls
    else if (box_pair)
      e = csm::launch_score_box_pair(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                     (double*)c->scores.p, nullptr, D.n_space, c->stream);
    else if (box)
      e = csm::launch_score_box(L, d_sw, (const double*)c->pts.p,
                                (const AngleEntry*)c->angles.p, (double*)c->scores.p, nullptr, D.n_space,
                                c->stream);
    else if (phase)
      e = csm::launch_score_phase(L, PT, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                  (double*)c->scores.p, nullptr, D.n_space, c->stream);
    else if (tiny)
      e = csm::launch_score_tiny(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                 (double*)c->scores.p, nullptr, D.n_space, c->stream);
    else if (rows_sq)
      e = csm::launch_score_rows(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                 (double*)c->scores.p, nullptr, D.n_space, rows_sq, c->stream);
    else
      e = csm::launch_score_cols(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                 (double*)c->scores.p, nullptr, kt, c->stream);
    if (e != hipSuccess) return c->hip_fail(e, "score kernel");
    if (tail && sp.score) c->tail_open = w1 < nw;  // the level's last window is out: its counters close
    if (sp.score && c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipEventRecord");
    if (sp.score && !sp.finish && w0 == 0 && c->profiling && (e = hipEventRecord(c->ev_g0, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipEventRecord");  // the first span's end
    if (c->profiling) {
      c->account("host:launch:inputs", (float)(tl1 - tl0), 0.0, 0.0);
      c->account("host:launch:score", (float)(now_ms() - tl1), 0.0, 0.0);
    }
    if (!sp.finish) return CSM_OK;  // the finish comes with the level's last call
    tl2 = c->profiling ? now_ms() : 0.0;
    if (mode == Finish::kScoresToHost) {
      if ((e = c->h_scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(scores)");
      if ((e = hipEventRecord(c->ev_k, c->stream)) != hipSuccess || (e = hipStreamWaitEvent(c->d2h, c->ev_k, 0)) != hipSuccess)
        return c->hip_fail(e, "kernels event");
      if ((e = hipMemcpyAsync(c->h_scores.p, c->scores.p, bytes, hipMemcpyDeviceToHost, c->d2h)) != hipSuccess)
        return c->hip_fail(e, "hipMemcpyAsync(scores)");
    } else if (sig) {
      sig_value = SA.flag_value;
      done_stream = c->x_stream ? c->x_stream : c->stream;
      // with the fused finish the scoring launches did the fast pass's work:
      // only the exact pass is launched, after them
      if ((e = csm::launch_finish(SA, (const ScanWork*)c->scans.p, (const AngleEntry*)c->angles.p,
                                  (const double*)c->scores.p, sig_out, nw, c->stream, done_stream, c->ev_fast,
                                  tail)) != hipSuccess)
        return c->hip_fail(e, "finish_kernel");
      if (time_fin && done_stream != c->stream && (e = hipEventRecord(c->ev_ft, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipEventRecord");
      if (time_fin && (e = hipEventRecord(c->ev2, done_stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    } else {
      csm::FinishArgs A{};
      A.n_cand = D.n_cand;
      A.n_space = D.n_space;
      A.step_cells = L.step_cells;
      A.lin_tol = P.search_space_resolution / G.mres;
      A.skip_lists = skip_lists | own_lists_skip(P.type);
      const size_t fbytes = (size_t)nw * sizeof(csm::FinishOut);
      // + one "needs the exact sort" flag per window (fast finish, csm_finish.hip)
      // + the flags' compacted list (count, then windows)
      const size_t lbytes = ((size_t)nw * sizeof(int32_t) + 7) & ~(size_t)7;  // the list's {count, tag}: 8-aligned
      if ((e = c->fin.ensure(fbytes + lbytes + (size_t)(nw + 2) * sizeof(int32_t))) != hipSuccess)
        return c->hip_fail(e, "hipMalloc(finish)");
      A.need_exact = c->fast_finish ? (int32_t*)((char*)c->fin.p + fbytes) : nullptr;
      A.exact_list = c->fast_finish ? (int32_t*)((char*)c->fin.p + fbytes + lbytes) : nullptr;
      if ((e = c->h_fin.ensure(fbytes + (size_t)nw * sizeof(int32_t))) != hipSuccess)
        return c->hip_fail(e, "hipHostMalloc(finish)");
      // the exact pass on x_stream (when there is one and the fast pass runs first)
      hipStream_t fs = (c->x_stream && A.need_exact) ? c->x_stream : c->stream;
      if ((e = csm::launch_finish(A, (const ScanWork*)c->scans.p, (const AngleEntry*)c->angles.p,
                                  (const double*)c->scores.p, (csm::FinishOut*)c->fin.p, nw, c->stream, fs,
                                  c->ev_fast)) != hipSuccess)
        return c->hip_fail(e, "finish_kernel");
      if (time_fin && fs != c->stream && (e = hipEventRecord(c->ev_ft, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipEventRecord");
      if (time_fin && (e = hipEventRecord(c->ev2, fs)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
      // with profiling on, the flags come back too: how many windows needed the exact sort
      const size_t cbytes = fbytes + ((time_fin && A.need_exact) ? (size_t)nw * sizeof(int32_t) : 0);
      if ((e = hipEventRecord(c->ev_k, fs)) != hipSuccess || (e = hipStreamWaitEvent(c->d2h, c->ev_k, 0)) != hipSuccess)
        return c->hip_fail(e, "kernels event");
      if ((e = hipMemcpyAsync(c->h_fin.p, c->fin.p, cbytes, hipMemcpyDeviceToHost, c->d2h)) != hipSuccess)
        return c->hip_fail(e, "hipMemcpyAsync(finish)");
      if (cbytes > fbytes) {
        flags_h = (const int32_t*)((const char*)c->h_fin.p + fbytes);
        n_flags = nw;
      }
    }
  } else {
    const size_t pbytes = (size_t)nw * (size_t)bps * sizeof(BestPartial);
    if ((e = c->partials.ensure(pbytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(partials)");
    if ((e = c->best.ensure((size_t)nw * sizeof(BestPartial))) != hipSuccess) return c->hip_fail(e, "hipMalloc(best)");
    if (box_pair)
      e = csm::launch_score_box_pair(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                     (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                     D.n_space, c->stream);
    else if (box || box_tiled)
      e = csm::launch_score_box(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                box_tiled ? 16 : D.n_space, c->stream);
    else if (phase)
      e = csm::launch_score_phase(L, PT, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                  (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                  D.n_space, c->stream);
    else if (tiny)
      e = csm::launch_score_tiny(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                 (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p, D.n_space,
                                 c->stream);
    else if (rows_sq)
      e = csm::launch_score_rows(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                 (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                 D.n_space, rows_sq, c->stream);
    else
      e = csm::launch_score_cols(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                 (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                 kt, c->stream);
    if (e != hipSuccess) return c->hip_fail(e, "score kernel (best)");
    if (c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if (box_tiled) {  // (window, tile) over its angles, then window over its tiles: one
                      // block per window over ~10^5 partials took 0.13 ms on willow
      const int32_t tpw = tile_n * tile_n;
      if ((e = c->best_tiles.ensure((size_t)nw * tpw * sizeof(BestPartial))) != hipSuccess)
        return c->hip_fail(e, "hipMalloc(tile bests)");
      if ((e = csm::launch_reduce_best((const BestPartial*)c->partials.p, D.n_angles, nw * tpw,
                                       (BestPartial*)c->best_tiles.p, c->stream)) != hipSuccess ||
          (e = csm::launch_reduce_best((const BestPartial*)c->best_tiles.p, tpw, nw, (BestPartial*)c->best.p,
                                       c->stream)) != hipSuccess)
        return c->hip_fail(e, "reduce_best_kernel");
    } else if ((e = csm::launch_reduce_best((const BestPartial*)c->partials.p, (int32_t)bps, nw,
                                            (BestPartial*)c->best.p, c->stream)) != hipSuccess) {
      return c->hip_fail(e, "reduce_best_kernel");
    }
    if ((e = hipEventRecord(c->ev_k, c->stream)) != hipSuccess || (e = hipStreamWaitEvent(c->d2h, c->ev_k, 0)) != hipSuccess)
      return c->hip_fail(e, "kernels event");
    if ((e = hipMemcpyAsync(best_out, c->best.p, (size_t)nw * sizeof(BestPartial), hipMemcpyDeviceToHost, c->d2h)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(best)");
  }
  PendingRun local;
  PendingRun& p = pend ? *pend : local;
  p = PendingRun{};
  p.flags = flags_h;
  p.n_flags = n_flags;
  std::snprintf(p.kname, sizeof(p.kname), "%s", kname);
  std::snprintf(p.fname, sizeof(p.fname), "finish_kernel<%lld>", (long long)D.n_cand);
  p.alg_bytes = alg_bytes;
  p.scorings = scorings;
  p.finish_bytes = (double)nw * (double)D.n_cand * 8.0;
  p.device_finish = mode == Finish::kDevice && time_fin;
  p.timed = c->profiling;
  p.ev0 = c->ev0;
  p.ev1 = c->ev1;
  // (with the fused finish the fast interval is empty: the scoring time holds it)
  p.ev_fast = (time_fin && mode == Finish::kDevice && c->fast_finish && c->x_stream) ? c->ev_ft : nullptr;
  if (c->span_gap) {
    p.gap0 = c->ev_g0;
    p.gap1 = c->ev_g1;
    c->span_gap = false;
  }
  p.ev2 = c->ev2;
  p.done = c->ev_done;
  p.fin_host = sig_out;
  p.host_flag = sig_flag;
  p.fast_flag = sig_fast;
  p.flag_value = sig_value;
  p.defer_timing = sig;
  if ((e = hipEventRecord(c->ev_done, done_stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
  if (c->profiling && tl2 > 0.0) c->account("host:launch:finish", (float)(now_ms() - tl2), 0.0, 0.0);
  if (pend) return CSM_OK;
  return wait_run(c, p);
}

// Fill a WindowPlan + its AngleEntry rows (AngleSearchLookUpTable::UpdateLookUpTable
// :154-172 and ScanMatch :538-548) for a window centred at `center` (map coords).
// Writes D.n_angles rows at `out`; the caller sets W.angle_off.
bool plan_window_into(const csm_param& P, const Dims& D, const Geometry& G, int n_points,
                      const double center[3], AngleEntry* out, WindowPlan& W, bool host_trig) {
  W.center[0] = center[0];
  W.center[1] = center[1];
  W.center[2] = center[2];
  W.n_points = n_points;
  if (!beam_rule(n_points, P.use_point_size, W.step, W.use, W.n_used)) return false;
  const double ssize = P.search_space_size;
  W.x0 = center[0] - (ssize / G.mres) * 0.5;
  W.y0 = center[1] - (ssize / G.mres) * 0.5;
  if (!out) return true;  // angle rows shared with an earlier window of the same centre angle
  const double offset = (P.search_angle_offset * 2) / 2;
  const double start = center[2] - offset;
  for (int a = 0; a < D.n_angles; ++a) {
    AngleEntry& ae = out[a];
    ae.angle = start + a * P.search_angle_resolution;
    // (!host_trig: the launch's angle_trig_kernel writes cos/sin, except where
    // the restated sincos does not reach)
    if (host_trig || !csm::libm::sincos_device_ok(ae.angle)) csm::host_sincos(ae.angle, &ae.sine, &ae.cosine);
  }
  return true;
}

const double* libm_sincos_table() {
  struct Table {
    bool ok = false;
    double t[csm::libm::kSincosTableDoubles];
    Table() {
      ok = csm::libm::locate_sincos_table(t) && csm::libm::check_sincos(t, 4096, 0x7a61ull) == 0;
    }
  };
  static const Table tab;
  return tab.ok ? tab.t : nullptr;
}

bool plan_window(const csm_param& P, const Dims& D, const Geometry& G, int n_points,
                 const double center[3], std::vector<AngleEntry>& angles, WindowPlan& W) {
  const size_t base = angles.size();
  angles.resize(base + (size_t)D.n_angles);
  W.angle_off = (int64_t)base;
  return plan_window_into(P, D, G, n_points, center, angles.data() + base, W);
}

// Many windows of one scan (loop closure: one pose against many submaps share
// the centre angle): windows with an equal centre angle share their angle
// rows (the same host cos/sin, bit for bit), so the host computes and uploads
// them once.
bool plan_windows_shared(const csm_param& P, const Dims& D, const Geometry& G, int n_points, int n_windows,
                         const double* centers, std::vector<AngleEntry>& angles, std::vector<WindowPlan>& plans) {
  std::vector<std::pair<uint64_t, int64_t>> seen;
  for (int i = 0; i < n_windows; ++i) {
    const double* c = centers + 3 * i;
    uint64_t key;
    std::memcpy(&key, &c[2], sizeof(key));
    WindowPlan& W = plans[(size_t)i];
    int64_t off = -1;
    for (const auto& kv : seen)
      if (kv.first == key) off = kv.second;
    if (off >= 0) {
      W.angle_off = off;
      if (!plan_window_into(P, D, G, n_points, c, nullptr, W)) return false;
    } else {
      if (!plan_window(P, D, G, n_points, c, angles, W)) return false;
      if (seen.size() < 64) seen.push_back({key, W.angle_off});
    }
  }
  return true;
}

int upload_points(csm_ctx* c, const double* pts, int64_t n_total, void* pinned) {
  c->loaded_n = -1;  // the point buffer is shared with csm_load_scans
  const size_t nb = (size_t)std::max<int64_t>(n_total, 0) * 2 * sizeof(double);
  if (c->pts_cached && n_total > 0 && c->pts_host.size() * sizeof(double) == nb &&
      std::memcmp(c->pts_host.data(), pts, nb) == 0)
    return CSM_OK;  // the device buffer holds these points (and pts_maxabs is theirs)
  c->pts_cached = false;
  double m = 0.0;    // max |x| + |y| over the points: bounds every rotated endpoint
  for (int64_t i = 0; i < n_total; ++i) {
    const double a = std::fabs(pts[2 * i]) + std::fabs(pts[2 * i + 1]);
    m = (a > m || a != a) ? a : m;
  }
  c->pts_maxabs = m;
  const size_t bytes = (size_t)std::max<int64_t>(n_total, 1) * 2 * sizeof(double);
  hipError_t e;
  if ((e = c->pts.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(points)");
  // through pinned memory: a pageable source makes the copy wait for the device
  // (~20-70 us per call); small uploads (a scan, a few scans) use the context's
  // staging buffer once its last copy has finished, large ones copy directly
  const size_t nbytes = (size_t)n_total * 2 * sizeof(double);
  bool own = false;
  if (!pinned && n_total > 0 && nbytes <= ((size_t)4 << 20)) {
    if (c->ev_pts_used && (e = hipEventSynchronize(c->ev_pts)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize(points)");
    if ((e = c->h_pts.ensure(nbytes)) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(points)");
    pinned = c->h_pts.p;
    own = true;
  }
  if (pinned && n_total > 0) {
    std::memcpy(pinned, pts, nbytes);
    pts = (const double*)pinned;
  }
  if (n_total > 0 && (e = hipMemcpyAsync(c->pts.p, pts, nbytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(points)");
  if (own) {
    if ((e = hipEventRecord(c->ev_pts, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord(points)");
    c->ev_pts_used = true;
  }
  if (n_total > 0 && nbytes <= ((size_t)4 << 20)) {
    c->pts_host.assign(pts, pts + 2 * n_total);
    c->pts_cached = true;
  }
  return CSM_OK;
}

int check_points(csm_ctx* c, const double* pts, int64_t n_total) {
  if (n_total < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  if (n_total > 0 && pts == nullptr) return c->fail(CSM_ERR_INVALID_ARG, "null points");
  return CSM_OK;
}

int check_offsets(csm_ctx* c, int32_t n_scans, const int64_t* offsets) {
  if (n_scans < 0 || (n_scans > 0 && offsets == nullptr)) return c->fail(CSM_ERR_INVALID_ARG, "bad scan offsets");
  for (int s = 0; s < n_scans; ++s)
    if (offsets[s + 1] < offsets[s] || offsets[s + 1] - offsets[s] > INT32_MAX)
      return c->fail(CSM_ERR_INVALID_ARG, "scan offsets must be non-decreasing");
  return CSM_OK;
}

}  // namespace csmh
