// csm_driver.cpp — BasedCorrelationScanMatch::ScanMatch over batches of
// scans (correlate_scan_matcher.h:784-875) and the 3-level ScanMatchers
// driver (scan_matchers.h:179-289): levels planned, launched, joined and
// completed per part, with the parts of a resident batch in flight together.
#include "csm_host.hpp"
#include "libm_sincos.hpp"

namespace csmh {

// One level (BasedCorrelationScanMatch::ScanMatch) over a batch of scans,
// split in two so a pipelined caller can overlap the host work of one half
// with the device work of the other: level_begin plans the windows and
// enqueues them (nothing waits), level_end joins and completes them.
// Points must already be uploaded; offsets index them.
struct LevelRun {
  csm_param P{};
  Dims D;
  std::vector<int> scan_of;
  std::vector<WindowPlan> plans;
  std::vector<int64_t> pt_off;
  std::vector<int32_t> grid;             // resident grid of each window (empty: grid 0)
  const AngleEntry* angles = nullptr;    // pinned buffer of the slot that ran it
  AngleEntry* rows = nullptr;            // the same, writable while the level is planned
  const csm::FinishOut* fin = nullptr;   // ditto (device finish)
  const double* scores = nullptr;        // ditto (host finish)
  bool dev = false;
  int skip_lists = 0;  // live_lists
  PendingRun pend;
  int tag = -1;        // 3-level driver: level * 8 + part (per-phase host timings)
  // CSM_DEBUG_FIN: each window's FinishOut as completed, and how (1 settled
  // early, 2 owed by the exact pass, 3 joined)
  std::vector<csm::FinishOut>* snap = nullptr;
  std::vector<char>* how = nullptr;
  // a window's FinishOut never matched its seal (pinned host memory): 1
  mutable int err = 0;
  // the order its windows take the scans in (nullptr: scan order; the
  // 3-level driver's spatial order, window_order)
  const int32_t* order = nullptr;
  // the plan pass fills each window's ScanWork into the slot's pinned staging
  // at the launch's score stride (run_windows then skips its serial fill, ~15
  // us a 2048-window launch) and checks its fixed-point range (int_bad: some
  // window is out of range; int_known: every window has been planned)
  ScanWork* sw = nullptr;
  int64_t sw_stride = 0;
  int int_bad = 0;
  bool int_known = false;
  // the rows' cos/sin are left to the launch (csm_trig.hip): a device finish
  // (the host finish reads them), not the few-window path (its own copy)
  bool dev_trig = false;
  // some window has an angle outside the restated sincos's domain: its launch
  // copies the host's rows (the kernel fills the others in place)
  int trig_bad = 0;
  // back to a fresh run, the vectors' capacity kept
  void reset() {
    P = csm_param{};
    D = Dims{};
    scan_of.clear();
    // (plans keep their elements: level_alloc value-initialises them only for
    // a level launched in spans, whose unplanned windows the launch reads)
    pt_off.clear();
    grid.clear();
    angles = nullptr;
    rows = nullptr;
    fin = nullptr;
    scores = nullptr;
    dev = false;
    skip_lists = 0;
    pend = PendingRun{};
    tag = -1;
    snap = nullptr;
    how = nullptr;
    err = 0;
    order = nullptr;
    sw = nullptr;
    sw_stride = 0;
    int_bad = 0;
    int_known = false;
    dev_trig = false;
    trig_bad = 0;
  }
};

// Seals (csm_internal.hpp) are waited for at most this long: they land within
// microseconds of the flag; a seal that never matches is a failure, not a hang.
constexpr double kSealWaitMs = 2000.0;

// Window i's FinishOut from the pinned host memory the finish wrote, whole:
// spin until its seal names a final writer for this launch and the copy's
// pieces match it (the pieces can land after the launch's flag).
// Returns the writer (kSealFast / kSealExact), kSealPending when `pending_ok`
// and the fast pass left the window to the exact pass, 0 on a timeout.
uint32_t sealed_copy(const LevelRun& R, int i, csm::FinishOut& out, bool pending_ok) {
  const double t0 = now_ms();
  for (uint32_t spin = 1;; ++spin) {
    const uint32_t w = read_sealed(R.fin + i, R.pend.flag_value, out);
    if (w == csm::kSealFast || w == csm::kSealExact || (pending_ok && w == csm::kSealPending)) return w;
    if ((spin & 255) == 0 && now_ms() - t0 > kSealWaitMs) return 0u;
    __builtin_ia32_pause();
  }
}

// Which covariance lists of level l a caller of the 3-level driver can see,
// as the finish's skip mask (bit 0 positional, bit 1 angular: skipped).
// ComputePositionalCovariance resets the whole matrix (correlate_scan_matcher.h:891)
// and ComputeAngularCovariance writes (2,2) only (:1018), by type (:835-858); a
// later level that writes the same entries makes this level's value dead (the
// reference's coarse covariance is always overwritten by the fine level).
int live_lists(const csm_param* levels, int n_levels, int l) {
  auto pos = [](int t) { return t == CSM_COARSE || t == CSM_FAST || t == CSM_FINE; };
  auto ang = [](int t) { return t == CSM_COARSE || t == CSM_FAST || t == CSM_SUPER; };
  int skip = 0;
  for (int k = l + 1; k < n_levels; ++k) {
    if (pos(levels[k].type)) return 3;
    if (ang(levels[k].type)) skip |= 2;
  }
  return skip;
}

// Which scans of a level have windows, and its dimensions (no planning yet).
// `reset`: responses (and argmaxes) of the batch start at kMinResponse.
int level_prepare(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P, double* responses,
                  int64_t* argmax_flat, LevelRun& R, const int32_t* scan_grid, int skip_lists, bool reset) {
  R.P = P;
  R.skip_lists = skip_lists;
  R.scan_of.clear();
  R.grid.clear();
  int st = window_dims(P, R.D);
  if (st != CSM_OK) return c->fail(st, "invalid search window parameters");
  R.scan_of.reserve((size_t)n_scans);
  const bool ready = map_ready(c);
  int last_n = -1;  // the beam rule's verdict for the last point count (scans mostly share one)
  for (int k = 0; k < n_scans; ++k) {
    const int s = R.order ? R.order[k] : k;
    if (reset) {
      responses[s] = 0.0;  // kMinResponse (:1034)
      if (argmax_flat) argmax_flat[s] = -1;
    }
    const int n = (int)(offsets[s + 1] - offsets[s]);
    if (!ready || n == 0) continue;  // :792-795
    if (n != last_n) {
      int step, use, n_used;
      if (!beam_rule(n, P.use_point_size, step, use, n_used))
        return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
      last_n = n;
    }
    R.scan_of.push_back(s);
    if (scan_grid) R.grid.push_back(scan_grid[s]);
  }
  return CSM_OK;
}

// Device finish for the front-end windows (and enough of them to fill the
// chip); a handful of windows finish faster on the host's std::sort.
bool level_device_finish(const csm_ctx* c, const Dims& D, int nw) {
  return c->device_finish && D.n_cand <= csm::kFinishMaxCand && csm::finish_lds_bytes(D.n_cand) <= 160 * 1024 &&
         nw >= c->device_finish_min;
}

// Room for the level's plans and angle rows (pinned: uploaded by DMA).
// spans: the level goes out in spans, so its launches read window plans not
// planned yet (zeroed, as the kernel choice expects); otherwise every plan is
// written before the launch and the old ones are only resized (value-initialising
// 2048 plans cost ~20 us of the serial chain, r06).
int level_alloc(csm_ctx* c, const int64_t* offsets, LevelRun& R, HostBuf& rows, bool spans) {
  const int nw = (int)R.scan_of.size();
  if (spans)
    R.plans.assign((size_t)nw, WindowPlan{});
  else
    R.plans.resize((size_t)nw);
  R.pt_off.resize((size_t)nw);
  for (int i = 0; i < nw; ++i) R.pt_off[(size_t)i] = offsets[R.scan_of[(size_t)i]];
  hipError_t he = rows.ensure((size_t)nw * (size_t)R.D.n_angles * sizeof(AngleEntry));
  if (he != hipSuccess) return c->hip_fail(he, "hipHostMalloc(angles)");
  R.rows = (AngleEntry*)rows.p;
  R.angles = R.rows;
  // this slot's ScanWork staging (run_windows uploads it from c->h_sw; the
  // slot's previous launch has read it: its level was joined before this plan)
  if ((he = c->h_sw.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(he, "hipHostMalloc(scans)");
  R.sw = (ScanWork*)c->h_sw.p;
  const bool dev = level_device_finish(c, R.D, nw);
  R.sw_stride = score_stride(c, R.D, dev ? Finish::kDevice : Finish::kScoresToHost);
  R.int_bad = 0;
  R.int_known = false;
  R.dev_trig = c->device_trig && dev && !small_launch(c, R.D, nw) && libm_sincos_table() != nullptr;
  R.trig_bad = 0;
  return CSM_OK;
}

// Plan window i of a prepared level around the scan's current pose: host
// libm cos/sin per angle (AngleSearchLookUpTable::UpdateLookUpTable :154-172).
// Its ScanWork goes straight into the slot's staging, and its fixed-point
// range is checked (LevelRun::sw, int_bad).
void level_plan_one(const csm_ctx* c, LevelRun& R, const Geometry& G, const int64_t* offsets, const double* poses,
                    int i) {
  const int s = R.scan_of[(size_t)i];
  double center[3];
  G.to_map(poses + 3 * s, center);
  WindowPlan& W = R.plans[(size_t)i];
  AngleEntry* rows = R.rows + (size_t)i * (size_t)R.D.n_angles;
  plan_window_into(R.P, R.D, G, (int)(offsets[s + 1] - offsets[s]), center, rows, W, !R.dev_trig);
  // (the angles grow with their index: both ends inside the domain, all are)
  if (R.dev_trig && R.D.n_angles > 0 &&
      !(csm::libm::sincos_device_ok(rows[0].angle) && csm::libm::sincos_device_ok(rows[R.D.n_angles - 1].angle)))
    __atomic_store_n(&R.trig_bad, 1, __ATOMIC_RELAXED);
  W.angle_off = (int64_t)i * R.D.n_angles;
  if (R.sw)
    fill_scan_work_one(R.D, W, R.pt_off[(size_t)i], R.grid.empty() ? 0 : R.grid[(size_t)i], (size_t)i, R.sw_stride,
                       R.sw[i]);
  if (!int_mode_window_ok(c, R.D, R.P.search_space_resolution / G.mres, W))
    __atomic_store_n(&R.int_bad, 1, __ATOMIC_RELAXED);
}

// Enqueue a planned level, or a span of it (nothing waits).
int level_launch(csm_ctx* c, LevelRun& R, WinSpan sp = WinSpan{}) {
  const int nw = (int)R.scan_of.size();
  const Dims& D = R.D;
  const Geometry G(c->info);
  R.dev = level_device_finish(c, D, nw);
  sp.sw_ready = R.sw;
  sp.sw_stride = R.sw_stride;
  sp.int_all = R.int_known && !__atomic_load_n(&R.int_bad, __ATOMIC_RELAXED);
  sp.dev_trig = R.dev_trig;
  sp.rows_gen = R.dev_trig && !__atomic_load_n(&R.trig_bad, __ATOMIC_RELAXED);
  const int st = run_windows(c, R.P, D, G, R.plans, R.pt_off, R.angles, (size_t)nw * (size_t)D.n_angles, R.grid,
                             nullptr, R.dev ? Finish::kDevice : Finish::kScoresToHost, &R.pend, R.skip_lists, sp);
  if (st != CSM_OK || !sp.finish) return st;
  R.fin = R.pend.fin_host ? R.pend.fin_host : (const csm::FinishOut*)c->h_fin.p;
  R.scores = (const double*)c->h_scores.p;
  return CSM_OK;
}

int level_begin(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                const double* poses, double* responses, int64_t* argmax_flat, LevelRun& R,
                const int32_t* scan_grid, int skip_lists) {
  int st = level_prepare(c, n_scans, offsets, P, responses, argmax_flat, R, scan_grid, skip_lists, true);
  if (st != CSM_OK) return st;
  const int nw = (int)R.scan_of.size();
  if (nw == 0) return CSM_OK;
  const double t0 = now_ms();
  if ((st = level_alloc(c, offsets, R, c->h_angles, false)) != CSM_OK) return st;
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  if (c->profiling) c->account("host:plan:alloc", (float)(now_ms() - t0), 0.0, 0.0);
  c->parallel_for(nw, threads, [&](int i) { level_plan_one(c, R, G, offsets, poses, i); });
  R.int_known = true;
  if (threads > 1) c->account_pool("plan");
  const double t1 = now_ms();
  if ((st = level_launch(c, R)) != CSM_OK) return st;
  if (c->profiling) {  // per level (window size), and in all
    c->account("host:launch", (float)(now_ms() - t1), 0.0, 0.0);
    char nm[48];
    std::snprintf(nm, sizeof(nm), "host:plan<%lld>", (long long)R.D.n_cand);
    c->account("host:plan", (float)(t1 - t0), 0.0, 0.0);
    c->account(nm, (float)(t1 - t0), 0.0, 0.0);
  }
  return CSM_OK;
}

// level_begin with the plan in growing pieces: the pool plans the first
// `first` windows and their scoring goes out at once, then the next
// span_growth times as many while those score, and so on; the finish follows
// for all. For the 3-level driver's first part, where nothing else keeps the
// device busy while the host plans (a call's first ~0.3 ms with the whole
// level planned before one launch). The spans are whole-window
// ranges of one level: results are the one-launch level's.
int level_begin_split(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P, const double* poses,
                      double* responses, LevelRun& R, const int32_t* scan_grid, int skip_lists, int first) {
  const double t_in = now_ms();
  if (c->profiling && c->t_call > 0.0) c->account("host:first:entry->split", (float)(t_in - c->t_call), 0.0, 0.0);
  int st = level_prepare(c, n_scans, offsets, P, responses, nullptr, R, scan_grid, skip_lists, true);
  if (st != CSM_OK) return st;
  if (c->profiling) c->account("host:first:prepare", (float)(now_ms() - t_in), 0.0, 0.0);
  const int nw = (int)R.scan_of.size();
  if (first <= 0 || nw < 2 * first || !level_device_finish(c, R.D, nw))
    return level_begin(c, n_scans, offsets, P, poses, responses, nullptr, R, scan_grid, skip_lists);
  const double t0 = now_ms();
  if ((st = level_alloc(c, offsets, R, c->h_angles, true)) != CSM_OK) return st;
  const Geometry G(c->info);
  if (c->profiling) c->account("host:first:prepare+alloc", (float)(now_ms() - t_in), 0.0, 0.0);
  int w0 = 0;
  for (int64_t sz = first; w0 < nw; sz *= std::max(2, c->span_growth)) {
    // the last span takes the rest when it would leave less than a span behind
    const int w1 = (nw - w0 <= 2 * sz) ? nw : w0 + (int)sz;
    const double tp = now_ms();
    c->parallel_for(w1 - w0, c->host_threads, [&](int i) { level_plan_one(c, R, G, offsets, poses, w0 + i); });
    R.int_known = w1 == nw;
    c->account_pool("plan");
    if (c->profiling && w0 == 0) c->account("host:first:plan", (float)(now_ms() - tp), 0.0, 0.0);
    if ((st = level_launch(c, R, WinSpan{w0, w1, true, false})) != CSM_OK) return st;
    if (w0 == 0 && c->profiling && c->t_call > 0.0)
      c->account("host:entry->first_launch", (float)(now_ms() - c->t_call), 0.0, 0.0);
    w0 = w1;
  }
  if ((st = level_launch(c, R, WinSpan{0, nw, false, true})) != CSM_OK) return st;
  if (c->profiling) {
    char nm[48];
    std::snprintf(nm, sizeof(nm), "host:plan+launch<%lld,split>", (long long)R.D.n_cand);
    c->account(nm, (float)(now_ms() - t0), 0.0, 0.0);
  }
  return CSM_OK;
}

// Join a level's launch and check its device finish.
int level_join(csm_ctx* c, LevelRun& R) {
  const int nw = (int)R.scan_of.size();
  const double t1 = now_ms();
  const int st = wait_run(c, R.pend);
  if (st != CSM_OK) return st;
  if (c->profiling) {
    const float tw = (float)(now_ms() - t1);
    c->account("host:wait", tw, 0.0, 0.0);
    if (R.tag >= 0) {
      char nm[48];
      std::snprintf(nm, sizeof(nm), "host:wait<l%d,p%d>", R.tag / 8, R.tag % 8);
      c->account(nm, tw, 0.0, 0.0);
    }
  }
  if (R.dev && !R.pend.fin_host)  // (sealed windows are checked as they are completed)
    for (int i = 0; i < nw; ++i)
      if (R.fin[i].count < 0) return c->fail(CSM_ERR_HIP, "finish_kernel: work loop bound exceeded");
  return CSM_OK;
}

// After a level's windows are completed: a sealed window that never matched
// its seal (or carried the exact pass's overflow count) fails the call.
int level_check(csm_ctx* c, const LevelRun& R) {
  if (R.err) return c->fail(CSM_ERR_HIP, "finish: a window's FinishOut did not match its seal (or overflowed)");
  return CSM_OK;
}

// Complete window i of a joined level: pose, covariance and response
// (BasedCorrelationScanMatch::ScanMatch :815-869).
// defer (early completion): a window whose seal says the exact pass still owes
// it is not completed; returns false and the caller completes it after the join.
bool level_complete_one(const LevelRun& R, const Geometry& G, double* poses, double* covs, double* responses,
                        int64_t* argmax_flat, int i, bool defer = false) {
  thread_local std::vector<Entry> scratch;
  const Dims& D = R.D;
  const csm_param& P = R.P;
  const int s = R.scan_of[(size_t)i];
  const double f = P.search_space_resolution / G.mres;
  const CandGeom C{R.plans[(size_t)i], R.angles + R.plans[(size_t)i].angle_off, f, D.n_space,
                   (int64_t)D.n_space * D.n_space};
  csm::FinishOut local;
  const csm::FinishOut* o = nullptr;
  if (R.dev && R.pend.fin_host) {  // pinned host memory the finish wrote: a sealed copy
    const uint32_t w = sealed_copy(R, i, local, defer);
    if (w == csm::kSealPending) {
      if (R.how) (*R.how)[(size_t)i] = 2;
      return false;
    }
    if (w == 0 || local.count < 0) {
      __atomic_store_n(&R.err, 1, __ATOMIC_RELAXED);
      return true;
    }
    o = &local;
    if (R.snap) (*R.snap)[(size_t)i] = local;
    if (R.how && (*R.how)[(size_t)i] != 2) (*R.how)[(size_t)i] = 1;
  } else if (R.dev) {
    o = R.fin + i;
  } else {
    host_sort_finish(R.scores + (size_t)i * (size_t)D.n_cand, D, C, P, G, scratch, local);
    o = &local;
  }
  if (argmax_flat) argmax_flat[s] = o->front_idx;
  responses[s] = complete_window(*o, C, P, G, poses + 3 * s, covs + 9 * s, R.skip_lists);
  return true;
}

// A signalled level with the fast pass's early signal: wait for it. The
// windows it settled are then completed while the exact pass sorts the rest;
// which are which, each window's seal says (level_complete_one's defer).
int level_wait_fast(csm_ctx* c, const LevelRun& R) {
  const double t1 = now_ms();
  const int st = wait_flag(c, R.pend, R.pend.fast_flag);
  if (st != CSM_OK) return st;
  if (c->profiling) c->account("host:wait_fast", (float)(now_ms() - t1), 0.0, 0.0);
  return CSM_OK;
}

int level_end(csm_ctx* c, LevelRun& R, double* poses, double* covs, double* responses,
              int64_t* argmax_flat) {
  const int nw = (int)R.scan_of.size();
  if (nw == 0) return CSM_OK;
  int st;
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  double t2;
  if (R.dev && R.pend.fast_flag) {  // settled windows while the exact pass runs
    if ((st = level_wait_fast(c, R)) != CSM_OK) return st;
    t2 = now_ms();
    std::vector<int> owed((size_t)nw);
    int n_owed = 0;
    c->parallel_for(nw, threads, [&](int i) {
      if (!level_complete_one(R, G, poses, covs, responses, argmax_flat, i, true))
        owed[(size_t)__atomic_fetch_add(&n_owed, 1, __ATOMIC_RELAXED)] = i;
    });
    if ((st = level_join(c, R)) != CSM_OK) return st;
    c->parallel_for(n_owed, n_owed >= 32 ? threads : 1, [&](int k) {
      level_complete_one(R, G, poses, covs, responses, argmax_flat, owed[(size_t)k]);
    });
  } else {
    if ((st = level_join(c, R)) != CSM_OK) return st;
    t2 = now_ms();
    c->parallel_for(nw, threads, [&](int i) { level_complete_one(R, G, poses, covs, responses, argmax_flat, i); });
  }
  if ((st = level_check(c, R)) != CSM_OK) return st;
  if (threads > 1) c->account_pool("complete");
  if (c->profiling) {
    const float tc = (float)(now_ms() - t2);
    char nm[48];
    std::snprintf(nm, sizeof(nm), "host:complete<%lld>", (long long)R.D.n_cand);
    c->account("host:complete", tc, 0.0, 0.0);
    c->account(nm, tc, 0.0, 0.0);
  }
  return CSM_OK;
}

// level_end of R followed by level_begin of the next level N over the same
// scans, fused: one pass of the host pool completes window i (its new pose)
// and plans its next window right away, so the pool wakes once per level
// transition instead of twice and the next launch goes out one pool round
// trip earlier (the 3-level driver's critical path). `sum`
// accumulates each scan's response (ScanMatchers::ScanMatch :252-256) before
// the next level overwrites it. N's angle rows go to the other pinned buffer
// of the slot: R's rows are still being read.
// split: N goes out in two spans, its first half as soon as R's first half is
// completed (owed windows included, after the join), then the second half --
// for the hand-off nothing else on the device hides (the last part's
// fine -> super-fine: the device has only the other part's short super-fine
// level to run meanwhile).
int level_end_begin(csm_ctx* c, LevelRun& R, LevelRun& N, int32_t n_scans, const int64_t* offsets,
                    const csm_param& P, double* poses, double* covs, double* responses, double* sum,
                    const int32_t* scan_grid, int skip_lists, bool split = false) {
  const double tq = c->profiling ? now_ms() : 0.0;
  int st = level_prepare(c, n_scans, offsets, P, responses, nullptr, N, scan_grid, skip_lists, false);
  if (st != CSM_OK) return st;
  if (c->profiling) c->account("host:transition:prepare", (float)(now_ms() - tq), 0.0, 0.0);
  const int nw = (int)R.scan_of.size();
  if (N.scan_of != R.scan_of || nw == 0) {  // not the same windows: one after the other
    if ((st = level_end(c, R, poses, covs, responses, nullptr)) != CSM_OK) return st;
    for (int s = 0; s < n_scans; ++s) sum[s] += responses[s];
    return level_begin(c, n_scans, offsets, P, poses, responses, nullptr, N, scan_grid, skip_lists);
  }
  const bool early = R.dev && R.pend.fast_flag;
  if ((st = early ? level_wait_fast(c, R) : level_join(c, R)) != CSM_OK) return st;
  const double t2 = now_ms();
  std::swap(c->h_angles, c->h_angles_next);
  split = split && early && nw >= c->split_handoff_min && level_device_finish(c, N.D, nw);
  if ((st = level_alloc(c, offsets, N, c->h_angles, split)) != CSM_OK) return st;
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  auto one = [&](int i, bool defer) {
    if (!level_complete_one(R, G, poses, covs, responses, nullptr, i, defer)) return false;
    const int s = R.scan_of[(size_t)i];
    sum[s] += responses[s];
    level_plan_one(c, N, G, offsets, poses, i);
    return true;
  };
  if (split) {  // [0, h) completed, planned and scored while [h, nw) is completed and planned
    const int h = nw / 2;
    std::vector<int> owed((size_t)nw);
    int n_owed = 0;
    c->parallel_for(h, threads, [&](int i) {
      if (!one(i, true)) owed[(size_t)__atomic_fetch_add(&n_owed, 1, __ATOMIC_RELAXED)] = i;
    });
    if ((st = level_join(c, R)) != CSM_OK) return st;
    c->parallel_for(n_owed, n_owed >= 32 ? threads : 1, [&](int k) { one(owed[(size_t)k], false); });
    if ((st = level_check(c, R)) != CSM_OK) return st;
    if ((st = level_launch(c, N, WinSpan{0, h, true, false})) != CSM_OK) return st;
    c->parallel_for(nw - h, threads, [&](int i) { one(h + i, false); });
  } else if (early) {  // the settled windows while the exact pass runs, then the ones it owed
    std::vector<int> owed((size_t)nw);
    int n_owed = 0;
    c->parallel_for(nw, threads, [&](int i) {
      if (!one(i, true)) owed[(size_t)__atomic_fetch_add(&n_owed, 1, __ATOMIC_RELAXED)] = i;
    });
    if ((st = level_join(c, R)) != CSM_OK) return st;
    c->parallel_for(n_owed, n_owed >= 32 ? threads : 1, [&](int k) { one(owed[(size_t)k], false); });
  } else {
    c->parallel_for(nw, threads, [&](int i) { one(i, false); });
  }
  if ((st = level_check(c, R)) != CSM_OK) return st;
  N.int_known = true;  // every window of N planned
  if (threads > 1) c->account_pool("complete+plan");
  const double t3 = now_ms();
  if (split) {
    if ((st = level_launch(c, N, WinSpan{nw / 2, nw, true, false})) != CSM_OK ||
        (st = level_launch(c, N, WinSpan{0, nw, false, true})) != CSM_OK)
      return st;
  } else if ((st = level_launch(c, N)) != CSM_OK) {
    return st;
  }
  if (c->profiling) {
    c->account("host:launch", (float)(now_ms() - t3), 0.0, 0.0);
    c->account("host:complete+plan", (float)(t3 - t2), 0.0, 0.0);
    char nm[48];
    std::snprintf(nm, sizeof(nm), "host:complete+plan<l%d,p%d>", R.tag / 8, R.tag % 8);
    if (R.tag >= 0) c->account(nm, (float)(t3 - t2), 0.0, 0.0);
  }
  return CSM_OK;
}

int match_level(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                double* poses, double* covs, double* responses, int64_t* argmax_flat,
                const int32_t* scan_grid, int skip_lists) {
  if (P.type == CSM_FAST) return match_level_fast(c, n_scans, offsets, P, poses, covs, responses, argmax_flat);
  LevelRun R;
  int st = level_begin(c, n_scans, offsets, P, poses, responses, argmax_flat, R, scan_grid, skip_lists);
  if (st != CSM_OK) return st;
  return level_end(c, R, poses, covs, responses, argmax_flat);
}

// One batch through the 3-level driver (match_levels_pipelined). With
// csm_scan_matchers_submit the batch's last level is launched but its
// completion deferred: the next submitted batch's first launch goes out first
// (into the other half of the buffer slots), then the deferred completion runs
// while that one scores -- the device no longer idles between batches.
struct PipeJob {
  int K = 2, n_levels = 0, slot0 = 0;  // parts, levels, the parts' first buffer slot
  int first_windows = 0;                // the first part's first span (level_begin_split)
  int32_t n_scans = 0;
  const int64_t* offsets = nullptr;
  const int32_t* scan_grid = nullptr;
  csm_param levels[3]{};
  double *poses = nullptr, *covs = nullptr, *sum = nullptr;
  double* scores = nullptr;  // submitted: scores[s] = sum[s] / n_levels when complete
  std::vector<double> resp, own_sum;
  int32_t first[csm_ctx::kMaxParts]{}, count[csm_ctx::kMaxParts]{};
  // by level parity: level l's run and level l + 1's, per part. Reused across
  // batches: a fresh run's window plans (64 B each, 128 KB per 2048 windows)
  // came from mmap and paid ~40 us of page faults at every level start (r04).
  LevelRun R[2][csm_ctx::kMaxParts];
  bool pending = false;  // levels launched up to the last part's last hand-off; that and the completion deferred
  bool last_handoff_done = false;
  std::vector<int32_t> order[csm_ctx::kMaxParts];  // each part's scans in window order (window_order)
  std::vector<csm::FinishOut> snaps[csm_ctx::kMaxParts];  // CSM_DEBUG_FIN
  std::vector<char> hows[csm_ctx::kMaxParts];
};

struct PipeState {
  PipeJob job[2];
  int next = 0;  // the job slot the next submit takes (its parts: slots next * K ...)
};

PipeState& pipe_of(csm_ctx* c) {
  if (!c->pipe) c->pipe = new PipeState();
  return *static_cast<PipeState*>(c->pipe);
}

// part h of J with its buffer slot swapped in (slot 0 is the context's own)
template <typename F>
int with_slot(csm_ctx* c, const PipeJob& J, int h, F&& f) {
  const int sidx = J.slot0 + h;
  if (sidx > 0) c->swap_slot(sidx);
  const int st = f();
  if (sidx > 0) c->swap_slot(sidx);
  return st;
}

// The order a part's windows take its scans in. Consecutive windows go to
// one XCD (dev::xcd_remap: XCD x takes the x-th eighth of the launch), so the
// scans are ranked by the Morton code of their initial map cell (64-cell
// tiles) and rank m goes to launch position (m % 8) * n / 8 + m / 8: every
// XCD's share spans the whole map (the same work mix on every XCD), and at
// any moment the eight XCDs score windows that lie close together, which
// their L2s and the MALL share. r05 A/B: the pair kernel 0.637
// -> 0.613 ms, the phase kernel 0.252 -> 0.245; ranks in contiguous eighths
// (each XCD one region of the map) made the pair kernel 0.848 ms, the XCDs'
// regions holding unequal work. Scans are independent: no result changes.
#ifndef CSM_WINDOW_ORDER  // 0: scan order (A/B builds)
#define CSM_WINDOW_ORDER 1
#endif
// (ranked by a stable LSD radix sort of the 32-bit keys, ties in scan order:
// std::sort of 2 x 2048 (key, scan) pairs took ~0.1 ms of the submit's way to
// its first launch, r05)
void window_order(const Geometry& G, const double* poses, int32_t n, std::vector<int32_t>& out) {
  out.resize((size_t)n);
  thread_local std::vector<uint32_t> key, key2;
  thread_local std::vector<int32_t> idx2;
  key.resize((size_t)n);
  key2.resize((size_t)n);
  idx2.resize((size_t)n);
  auto spread = [](uint32_t v) {  // 16 bits -> every other bit
    v &= 0xFFFF;
    v = (v | (v << 8)) & 0x00FF00FFu;
    v = (v | (v << 4)) & 0x0F0F0F0Fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v;
  };
  for (int32_t s = 0; s < n; ++s) {
    double m[3];
    G.to_map(poses + 3 * (size_t)s, m);
    const double qx = std::floor(m[0] / 64.0), qy = std::floor(m[1] / 64.0);
    const uint32_t ix = (uint32_t)((int32_t)std::max(-32768.0, std::min(32767.0, qx)) + 32768);
    const uint32_t iy = (uint32_t)((int32_t)std::max(-32768.0, std::min(32767.0, qy)) + 32768);
    key[(size_t)s] = spread(ix) | (spread(iy) << 1);
  }
  // rank[] in `out` (as scratch) then by 8-bit digits, least significant first
  std::vector<int32_t>& idx = out;
  for (int32_t s = 0; s < n; ++s) idx[(size_t)s] = s;
  for (int shift = 0; shift < 32; shift += 8) {
    size_t cnt[257] = {0};
    for (int32_t i = 0; i < n; ++i) ++cnt[((key[(size_t)i] >> shift) & 0xFF) + 1];
    for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
    for (int32_t i = 0; i < n; ++i) {
      const size_t o = cnt[(key[(size_t)i] >> shift) & 0xFF]++;
      key2[o] = key[(size_t)i];
      idx2[o] = idx[(size_t)i];
    }
    key.swap(key2);
    idx.swap(idx2);
  }
  // idx holds the ranked scans (4 swaps: back in `out`); rank m -> position (m % 8) * n / 8 + m / 8
  if (CSM_WINDOW_ORDER == 2) return;  // (A/B: contiguous Morton ranges, each XCD one region)
  idx2.assign(idx.begin(), idx.end());
  int32_t pos = 0;
  for (int x = 0; x < 8; ++x)
    for (int32_t m = x; m < n; m += 8) out[(size_t)pos++] = idx2[(size_t)m];
}

void job_setup(csm_ctx* c, PipeJob& J, int32_t n_scans, const int64_t* offsets, const csm_param* levels,
               int n_levels, double* poses, double* covs, double* sum, const int32_t* scan_grid, int K, int slot0,
               bool submitted = false) {
  J.K = K;
  // submitted batches split their first span only when the coarse level sums
  // many beams: below that the step is host-bound and the extra launch costs
  // more than the shorter planning at the batch boundary (csm_host.hpp)
  J.first_windows = !submitted ? c->first_windows
                    : (n_levels > 0 && levels[0].use_point_size > c->first_windows_submit_min_use) ? c->first_windows_submit
                                                                                                   : 0;
  const int permille = submitted ? c->part0_permille_submit : c->part0_permille;
  J.n_levels = n_levels;
  J.slot0 = slot0;
  J.n_scans = n_scans;
  J.offsets = offsets;
  J.scan_grid = scan_grid;
  for (int l = 0; l < n_levels; ++l) J.levels[l] = levels[l];
  J.poses = poses;
  J.covs = covs;
  J.sum = sum;
  J.scores = nullptr;
  J.pending = false;
  J.last_handoff_done = false;
  // part 0 takes part0_permille of the scans, the others split the rest: a
  // larger first part shortens what nothing hides, the last part's
  // super-fine completion at the end of the call and its fine -> super-fine
  // hand-off (the device has only part 0's super-fine level to run meanwhile)
  const int64_t n0 = (K == 2 && permille > 0) ? (int64_t)n_scans * permille / 1000
                                                        : (int64_t)n_scans / K;
  for (int h = 0; h < K; ++h) {
    J.first[h] = h == 0 ? 0 : (int32_t)(n0 + (int64_t)(n_scans - n0) * (h - 1) / (K - 1));
    J.count[h] = (h == 0 ? (int32_t)n0 : (int32_t)(n0 + (int64_t)(n_scans - n0) * h / (K - 1))) - J.first[h];
  }
  J.resp.assign((size_t)n_scans, 0.0);
  for (auto& row : J.R)
    for (LevelRun& r : row) r.reset();
  for (int h = 0; h < K; ++h) J.order[h].clear();  // (job_begin ranks each part's windows)
}

int job_skip(const csm_ctx* c, const PipeJob& J, int l) {
  return c->skip_dead_lists ? live_lists(J.levels, J.n_levels, l) : 0;
}

// Level 0 of part h planned and launched (the first part in growing spans:
// the device waits for it).
int job_begin(csm_ctx* c, PipeJob& J, int h) {
  const int32_t s0 = J.first[h];
  J.R[0][h].tag = h;
  if (CSM_WINDOW_ORDER) {  // here, not in job_setup: part 0's launch goes out before the other parts are ranked
    window_order(Geometry(c->info), J.poses + 3 * (size_t)s0, J.count[h], J.order[h]);
    J.R[0][h].order = J.R[1][h].order = J.order[h].data();
  }
  return with_slot(c, J, h, [&] {
    const int32_t* g = J.scan_grid ? J.scan_grid + s0 : nullptr;
    if (h == 0)
      return level_begin_split(c, J.count[h], J.offsets + s0, J.levels[0], J.poses + 3 * (size_t)s0,
                               J.resp.data() + s0, J.R[0][h], g, job_skip(c, J, 0), J.first_windows);
    return level_begin(c, J.count[h], J.offsets + s0, J.levels[0], J.poses + 3 * (size_t)s0, J.resp.data() + s0,
                       nullptr, J.R[0][h], g, job_skip(c, J, 0));
  });
}

// The level transition (l -> l + 1) of part h.
int job_handoff(csm_ctx* c, PipeJob& J, int l, int h) {
  const int32_t s0 = J.first[h];
  J.R[(l + 1) & 1][h].tag = (l + 1) * 8 + h;
  // csm_set_profiling(ctx, 2): the later levels' launches go out without
  // timing events (their records cost ~50 us of kernel-stream gaps a config-2
  // step, profiles/r05/experiments/ab_profile_first_level.txt)
  const bool timed = c->profiling;
  c->profiling = timed && !c->profile_first_level;
  const int st = with_slot(c, J, h, [&] {
    return level_end_begin(c, J.R[l & 1][h], J.R[(l + 1) & 1][h], J.count[h], J.offsets + s0, J.levels[l + 1],
                           J.poses + 3 * (size_t)s0, J.covs + 9 * (size_t)s0, J.resp.data() + s0, J.sum + s0,
                           J.scan_grid ? J.scan_grid + s0 : nullptr, job_skip(c, J, l + 1),
                           c->split_last_handoff && h == J.K - 1 && l + 2 == J.n_levels);
  });
  c->profiling = timed;
  return st;
}

// Every level transition of J but the last part's last one, which is left to
// job_last_handoff (J.pending): when a submitted batch returns, the device
// still has the last part's previous level and the other parts' last level
// queued, enough to cover the host's way to the next batch's first launch.
int job_levels(csm_ctx* c, PipeJob& J) {
  const int K = J.K, n_levels = J.n_levels;
  int st;
  for (int l = 0; l + 1 < n_levels; ++l)
    for (int h = 0; h < K; ++h) {
      if (c->defer_last_handoff && l + 2 == n_levels && h == K - 1) continue;
      if ((st = job_handoff(c, J, l, h)) != CSM_OK) return st;
    }
  J.pending = true;
  J.last_handoff_done = n_levels < 2 || !c->defer_last_handoff;
  return CSM_OK;
}

// The last part's last level transition (the last launch of J).
int job_last_handoff(csm_ctx* c, PipeJob& J) {
  if (!J.pending || J.last_handoff_done) return CSM_OK;
  J.last_handoff_done = true;
  return job_handoff(c, J, J.n_levels - 2, J.K - 1);
}

// J's last level: every part's windows completed, responses summed (and the
// submitted batch's scores written).
int job_finish(csm_ctx* c, PipeJob& J) {
  if (!J.pending) return CSM_OK;
  int st;
  if ((st = job_last_handoff(c, J)) != CSM_OK) return st;
  J.pending = false;
  const int K = J.K, last = J.n_levels - 1;
  for (int h = 0; h < K; ++h) {
    const int32_t s0 = J.first[h];
    LevelRun& cur = J.R[last & 1][h];
    if (c->debug_fin) {
      J.snaps[h].assign(cur.scan_of.size(), csm::FinishOut{});
      J.hows[h].assign(cur.scan_of.size(), (char)3);
      cur.snap = &J.snaps[h];
      cur.how = &J.hows[h];
    }
    if ((st = level_end(c, cur, J.poses + 3 * (size_t)s0, J.covs + 9 * (size_t)s0, J.resp.data() + s0, nullptr)) !=
        CSM_OK)
      return st;
    for (int s = s0; s < s0 + J.count[h]; ++s) J.sum[(size_t)s] += J.resp[(size_t)s];
  }
  if (J.scores)
    for (int s = 0; s < J.n_scans; ++s) J.scores[s] = J.sum[(size_t)s] / J.n_levels;  // :281
  if (c->debug_fin) {  // the device idle: what the finish left against what was completed
    (void)hipDeviceSynchronize();
    for (int h = 0; h < K; ++h) {
      const LevelRun& L = J.R[last & 1][h];
      if (!L.dev || !L.fin) continue;
      for (size_t i = 0; i < J.snaps[h].size(); ++i) {
        const csm::FinishOut& a = J.snaps[h][i];
        const csm::FinishOut& b = L.fin[i];
        // the pieces the final seal names (the completed copy holds only those)
        const int lists = (int)(b.seal_tag_kind >> 34) & 3;
        bool same = a.seal_tag_kind == b.seal_tag_kind;
        for (int t = 0, n = csm::finish_n_pieces(lists); same && t < n; ++t) {
          const int pc = csm::finish_piece(t, lists);
          same = std::memcmp(reinterpret_cast<const char*>(&a) + 16 * pc, reinterpret_cast<const char*>(&b) + 16 * pc,
                             16) == 0;
        }
        if (same) continue;
        std::fprintf(stderr,
                     "csm debug_fin: part %d window %zu (scan %d) how %d: completed count %d n_pos %d n_ang %d front %d "
                     "ang0 %.17g | final count %d n_pos %d n_ang %d front %d ang0 %.17g\n",
                     h, i, J.first[h] + L.scan_of[i], (int)J.hows[h][i], a.count, a.n_pos, a.n_ang, a.front_idx,
                     a.ang_score[0], b.count, b.n_pos, b.n_ang, b.front_idx, b.ang_score[0]);
      }
    }
  }
  return CSM_OK;
}

// The driver's knobs for a pipelined batch: every part on the throughput
// kernels (parts in flight share no few-window buffers), early completion on.
struct PipeMode {
  csm_ctx* c;
  bool small_was;
  explicit PipeMode(csm_ctx* cc) : c(cc), small_was(cc->small_path) {
    c->small_path = false;
    c->early_now = true;
  }
  ~PipeMode() {
    c->small_path = small_was;
    c->early_now = false;
  }
};

// After a failure with a batch in flight: nothing stays pending, and nothing
// enqueued may still touch the buffers.
int pipe_abort(csm_ctx* c, int st) {
  if (c->pipe)
    for (PipeJob& J : static_cast<PipeState*>(c->pipe)->job) J.pending = false;
  (void)hipStreamSynchronize(c->stream);
  if (c->x_stream) (void)hipStreamSynchronize(c->x_stream);
  (void)hipStreamSynchronize(c->h2d);
  (void)hipStreamSynchronize(c->d2h);
  return st;
}

// A submitted batch whose last level is still pending is completed (every
// entry point but submit itself calls this first: the pending kernels read
// the loaded scans, the grid and the buffer slots).
int pipe_drain(csm_ctx* c) {
  if (!c->pipe) return CSM_OK;
  PipeState& PS = *static_cast<PipeState*>(c->pipe);
  for (PipeJob& J : PS.job)
    if (J.pending) {
      DeviceGuard g(c->device);
      PipeMode mode(c);  // its last hand-off launches as the rest of the batch did
      const int st = job_finish(c, J);
      if (st != CSM_OK) return pipe_abort(c, st);
    }
  return CSM_OK;
}

// Every launch of a pending batch made (its last part's last hand-off): the
// loaded points may change after this.
int pipe_last_launches(csm_ctx* c) {
  if (!c->pipe) return CSM_OK;
  for (PipeJob& J : static_cast<PipeState*>(c->pipe)->job)
    if (J.pending && !J.last_handoff_done) {
      PipeMode mode(c);
      const int st = job_last_handoff(c, J);
      if (st != CSM_OK) return pipe_abort(c, st);
    }
  return CSM_OK;
}

void pipe_free(csm_ctx* c) {
  delete static_cast<PipeState*>(c->pipe);
  c->pipe = nullptr;
}

// ScanMatchers::ScanMatch over a resident batch (scan_matchers.h:179-289),
// parts in flight: while the device runs one part's level, the host
// completes another part's previous level and plans its next one
// (level_end_begin). Scans are independent, so the split changes no result.
int match_levels_pipelined(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param* levels,
                           int n_levels, double* poses, double* covs, double* sum,
                           const int32_t* scan_grid = nullptr) {
  const int K = std::max(2, std::min(c->pipeline_parts, csm_ctx::kMaxParts));
  PipeMode mode(c);
  PipeJob& J = pipe_of(c).job[0];
  job_setup(c, J, n_scans, offsets, levels, n_levels, poses, covs, sum, scan_grid, K, 0);
  int st;
  for (int h = 0; h < K; ++h)
    if ((st = job_begin(c, J, h)) != CSM_OK) return pipe_abort(c, st);
  if ((st = job_levels(c, J)) != CSM_OK || (st = job_finish(c, J)) != CSM_OK) return pipe_abort(c, st);
  return CSM_OK;
}

// Batches queued with csm_load_scans_async are dropped (their uploads are
// waited for): a synchronous load names the batch the next match runs, so
// csm_scan_matchers / csm_scan_matchers_batch never match a queued batch
// into output arrays sized for their own scans.
int drop_staged(csm_ctx* c) {
  if (c->staged_count <= 0) return CSM_OK;
  hipError_t e;
  if (c->stage_stream && (e = hipStreamSynchronize(c->stage_stream)) != hipSuccess)
    return c->hip_fail(e, "hipStreamSynchronize(stage)");
  c->staged_count = 0;
  return CSM_OK;
}

// csm_load_scans once locked.
int load_scans_locked(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets) {
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
  int st;
  c->loaded_n = -1;
  c->loaded_grid.clear();
  if ((st = drop_staged(c)) != CSM_OK) return st;
  if ((st = check_offsets(c, n_scans, offsets)) != CSM_OK) return st;
  const int64_t n_total = n_scans > 0 ? offsets[n_scans] - offsets[0] : 0;
  if ((st = check_points(c, pts, n_total)) != CSM_OK) return st;
  c->loaded_off.assign(offsets, offsets + n_scans + 1);
  for (auto& o : c->loaded_off) o -= offsets[0];
  if ((st = upload_points(c, n_total > 0 ? pts + 2 * offsets[0] : pts, n_total)) != CSM_OK) return st;
  hipError_t e;
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(points)");
  c->loaded_n = n_scans;
  return CSM_OK;
}

}  // namespace csmh

using namespace csmh;

extern "C" {

int csm_scan_match_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                         const csm_param* param, double* poses, double* covs, double* responses,
                         int64_t* argmax_flat) {
  if (!c || !param || !poses || !covs || !responses) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
  int st;
  if ((st = check_offsets(c, n_scans, offsets)) != CSM_OK) return st;
  if (n_scans == 0) return CSM_OK;
  const int64_t n_total = offsets[n_scans] - offsets[0];
  if ((st = check_points(c, pts, n_total)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  std::vector<int64_t> off(offsets, offsets + n_scans + 1);
  for (auto& o : off) o -= offsets[0];
  if ((st = upload_points(c, pts + 2 * offsets[0], n_total)) != CSM_OK) return st;
  return match_level(c, n_scans, off.data(), *param, poses, covs, responses, argmax_flat);
}

int csm_scan_match(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                   double pose[3], double cov[9], double* response, int64_t* argmax_flat) {
  if (!c || !response) return CSM_ERR_INVALID_ARG;
  const int64_t off[2] = {0, n_points < 0 ? 0 : n_points};
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  return csm_scan_match_batch(c, 1, pts, off, param, pose, cov, response, argmax_flat);
}

int csm_load_scans(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return load_scans_locked(c, n_scans, pts, offsets);
}

int csm_load_scans_async(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st;
  if ((st = check_offsets(c, n_scans, offsets)) != CSM_OK) return st;
  const int64_t n_total = n_scans > 0 ? offsets[n_scans] - offsets[0] : 0;
  if ((st = check_points(c, pts, n_total)) != CSM_OK) return st;
  if (c->staged_count == 2) return c->fail(CSM_ERR_INVALID_ARG, "two batches already queued (csm_load_scans_async)");
  hipError_t e;
  if (!c->stage_stream && (e = hipStreamCreateWithFlags(&c->stage_stream, hipStreamNonBlocking)) != hipSuccess)
    return c->hip_fail(e, "hipStreamCreate(stage)");
  csm_ctx::Staged& S = c->staged[(c->staged_head + c->staged_count) % 2];
  if (!S.ready && (e = hipEventCreateWithFlags(&S.ready, hipEventDisableTiming)) != hipSuccess)
    return c->hip_fail(e, "hipEventCreate(stage)");
  if (!S.maxabs_h && (e = hipHostMalloc((void**)&S.maxabs_h, sizeof(unsigned long long), hipHostMallocDefault)) !=
                         hipSuccess)
    return c->hip_fail(e, "hipHostMalloc(stage)");
  const size_t bytes = (size_t)std::max<int64_t>(n_total, 1) * 2 * sizeof(double);
  if ((e = S.pts.ensure(bytes)) != hipSuccess || (e = S.maxabs_dev.ensure(sizeof(unsigned long long))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(stage)");
  // the buffer's previous batch was matched by a call that has returned, so
  // no kernel reads it any more
  if ((e = hipMemsetAsync(S.maxabs_dev.p, 0, sizeof(unsigned long long), c->stage_stream)) != hipSuccess ||
      (n_total > 0 && (e = hipMemcpyAsync(S.pts.p, pts + 2 * offsets[0], (size_t)n_total * 2 * sizeof(double),
                                          hipMemcpyHostToDevice, c->stage_stream)) != hipSuccess) ||
      (e = csm::launch_points_maxabs((const double*)S.pts.p, n_total, (unsigned long long*)S.maxabs_dev.p,
                                     c->stage_stream)) != hipSuccess ||
      (e = hipMemcpyAsync(S.maxabs_h, S.maxabs_dev.p, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          c->stage_stream)) != hipSuccess ||
      (e = hipEventRecord(S.ready, c->stage_stream)) != hipSuccess)
    return c->hip_fail(e, "csm_load_scans_async");
  S.off.assign(offsets, offsets + n_scans + 1);
  for (auto& o : S.off) o -= offsets[0];
  S.n = n_scans;
  c->staged_count++;
  return CSM_OK;
}

int csm_host_alloc(size_t bytes, void** out) {
  if (!out) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable) == hipSuccess ? CSM_OK : CSM_ERR_ALLOC;
}

int csm_host_free(void* p) { return (!p || hipHostFree(p) == hipSuccess) ? CSM_OK : CSM_ERR_INVALID_ARG; }

}  // extern "C"

namespace csmh {
// The oldest queued batch (csm_load_scans_async) becomes the loaded one.
int take_staged(csm_ctx* c) {
  if (c->staged_count <= 0) return CSM_OK;
  csm_ctx::Staged& S = c->staged[c->staged_head];
  hipError_t e;
  if ((e = hipEventSynchronize(S.ready)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize(stage)");
  std::swap(c->pts, S.pts);
  c->loaded_off.swap(S.off);
  c->loaded_n = S.n;
  c->loaded_grid.clear();
  double m;
  std::memcpy(&m, S.maxabs_h, sizeof(m));
  c->pts_maxabs = m;
  c->pts_cached = false;
  c->staged_head = (c->staged_head + 1) % 2;
  c->staged_count--;
  return CSM_OK;
}
}  // namespace csmh

extern "C" {

int csm_scan_matchers_submit(csm_ctx* c, const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                             double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st;
  // A queued batch (csm_load_scans_async) becomes the loaded one without
  // completing the pending batch: the swap parks the pending batch's points
  // in a staging slot, its last launch below borrows them back, and the next
  // upload into that slot comes after this call, which completes the pending
  // batch (its completion reads no points or offsets).
  // (checked before the swap: an early return after it would leave a pending
  // batch's last hand-off to launch on the new batch's points)
  if (c->staged_count == 0 && c->loaded_n < 0) return c->fail(CSM_ERR_INVALID_ARG, "no scans loaded (csm_load_scans)");
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  int parked = -1;
  double parked_maxabs = 0.0;
  if (c->staged_count > 0) {
    parked = c->staged_head;  // the slot take_staged swaps the current points into
    parked_maxabs = c->pts_maxabs;
    if ((st = take_staged(c)) != CSM_OK) return st;
  }
  // the pending batch's last launch (its last part's last hand-off), on its own points
  auto prior_last_launches = [&]() {
    if (parked >= 0) {
      std::swap(c->pts, c->staged[parked].pts);
      std::swap(c->pts_maxabs, parked_maxabs);
    }
    const int r = pipe_last_launches(c);
    if (parked >= 0) {
      std::swap(c->pts, c->staged[parked].pts);
      std::swap(c->pts_maxabs, parked_maxabs);
    }
    return r;
  };
  const int32_t n_scans = c->loaded_n;
  const int n_levels = use_fine ? 3 : 1;
  bool fast = false;
  for (int l = 0; l < n_levels; ++l) fast |= levels[l].type == CSM_FAST;
  const int32_t* grid = c->loaded_grid.empty() ? nullptr : c->loaded_grid.data();
  const int K = std::max(2, std::min(c->pipeline_parts, csm_ctx::kMaxParts));
  if (n_scans == 0 || fast || grid || n_scans < c->pipeline_min || 2 * K > csm_ctx::kMaxParts) {
    // nothing to overlap (or no second set of buffer slots): the batch completes here
    if ((st = prior_last_launches()) != CSM_OK || (st = pipe_drain(c)) != CSM_OK) return st;
    return matchers_loaded_locked(c, levels, use_fine, poses, covs, scores);
  }
  const double t_call = now_ms();
  c->t_call = t_call;
  PipeState& PS = pipe_of(c);
  PipeJob& J = PS.job[PS.next];
  PipeJob& P = PS.job[PS.next ^ 1];
  if (J.pending && ((st = prior_last_launches()) != CSM_OK || (st = pipe_drain(c)) != CSM_OK))
    return st;  // (cannot happen: submits alternate)
  PipeMode mode(c);
  job_setup(c, J, n_scans, c->loaded_off.data(), levels, n_levels, poses, covs, nullptr, nullptr, K, PS.next * K,
            true);
  J.own_sum.assign((size_t)n_scans, 0.0);
  J.sum = J.own_sum.data();
  J.scores = scores;
  // this batch's first part's first level, the previous batch's last launch
  // (its last part's last hand-off), this batch's other parts' first level,
  // then the previous batch's completion while those score, then the rest of
  // this batch up to its last part's last hand-off
  if ((st = job_begin(c, J, 0)) != CSM_OK) return pipe_abort(c, st);
  if ((st = prior_last_launches()) != CSM_OK) return pipe_abort(c, st);
  for (int h = 1; h < K; ++h)
    if ((st = job_begin(c, J, h)) != CSM_OK) return pipe_abort(c, st);
  if (P.pending && (st = job_finish(c, P)) != CSM_OK) return pipe_abort(c, st);
  if ((st = job_levels(c, J)) != CSM_OK) return pipe_abort(c, st);
  PS.next ^= 1;
  if (c->profiling) {
    c->t_exit = now_ms();
    c->account("host:submit", (float)(c->t_exit - t_call), 0.0, 0.0);
  }
  return CSM_OK;
}

int csm_scan_matchers_wait(csm_ctx* c) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return pipe_drain(c);
}

int csm_scan_matchers_loaded(csm_ctx* c, const csm_param levels[3], int32_t use_fine, double* poses,
                             double* covs, double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st0;
  if ((st0 = pipe_drain(c)) != CSM_OK || (st0 = take_staged(c)) != CSM_OK) return st0;
  return matchers_loaded_locked(c, levels, use_fine, poses, covs, scores);
}

}  // extern "C"

namespace csmh {
// csm_scan_matchers_loaded once locked, nothing pending, the staged batch taken.
int matchers_loaded_locked(csm_ctx* c, const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                           double* scores) {
  if (c->loaded_n < 0) return c->fail(CSM_ERR_INVALID_ARG, "no scans loaded (csm_load_scans)");
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  const int32_t n_scans = c->loaded_n;
  if (n_scans == 0) return CSM_OK;
  const double t_call = now_ms();
  c->t_call = t_call;
  if (c->profiling && c->t_exit > 0.0) c->account("host:between_calls", (float)(t_call - c->t_exit), 0.0, 0.0);
  // ScanMatchers::ScanMatch (scan_matchers.h:179-289), use_optimize = false:
  // coarse, then (use_fine) fine and super-fine, pose fed forward in place.
  std::vector<double> resp((size_t)n_scans, 0.0), sum((size_t)n_scans, 0.0);
  const int n_levels = use_fine ? 3 : 1;
  int st;
  bool fast = false;
  for (int l = 0; l < n_levels; ++l) fast |= levels[l].type == CSM_FAST;
  const int32_t* grid = c->loaded_grid.empty() ? nullptr : c->loaded_grid.data();
  for (int32_t s = 0; grid && s < n_scans; ++s)
    if (grid[s] < 0 || grid[s] >= c->n_grids) return c->fail(CSM_ERR_INVALID_ARG, "scan grid outside the resident stack");
  if (fast && grid) return c->fail(CSM_ERR_UNSUPPORTED, "FAST windows read grid 0 only");
  if (n_scans >= c->pipeline_min && !fast) {
    if ((st = match_levels_pipelined(c, n_scans, c->loaded_off.data(), levels, n_levels, poses, covs,
                                     sum.data(), grid)) != CSM_OK)
      return st;
  } else {
    for (int l = 0; l < n_levels; ++l) {
      if ((st = match_level(c, n_scans, c->loaded_off.data(), levels[l], poses, covs, resp.data(), nullptr,
                            grid, c->skip_dead_lists ? live_lists(levels, n_levels, l) : 0)) != CSM_OK)
        return st;
      for (int s = 0; s < n_scans; ++s) sum[(size_t)s] += resp[(size_t)s];
    }
  }
  for (int s = 0; s < n_scans; ++s) scores[s] = sum[(size_t)s] / n_levels;  // :281
  if (c->profiling) {
    c->t_exit = now_ms();
    c->account("host:call", (float)(c->t_exit - t_call), 0.0, 0.0);
  }
  return CSM_OK;
}
}  // namespace csmh

extern "C" {

int csm_scan_matchers_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                            const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                            double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int st = load_scans_locked(c, n_scans, pts, offsets);
  if (st != CSM_OK) return st;
  return matchers_loaded_locked(c, levels, use_fine, poses, covs, scores);
}

int csm_scan_matchers(csm_ctx* c, const double* pts, int32_t n_points, const csm_param levels[3],
                      int32_t use_fine, double pose[3], double cov[9], double* score) {
  if (!c || !score) return CSM_ERR_INVALID_ARG;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  const int64_t off[2] = {0, n_points};
  return csm_scan_matchers_batch(c, 1, pts, off, levels, use_fine, pose, cov, score);
}

int csm_load_scans_grids(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                         const int32_t* grid_index) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const int st = load_scans_locked(c, n_scans, pts, offsets);
  if (st != CSM_OK || !grid_index) return st;
  c->loaded_grid.assign(grid_index, grid_index + n_scans);
  return CSM_OK;
}

int csm_scan_matchers_batch_grids(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                                  const int32_t* grid_index, const csm_param levels[3], int32_t use_fine,
                                  double* poses, double* covs, double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st = load_scans_locked(c, n_scans, pts, offsets);
  if (st != CSM_OK) return st;
  if (grid_index) c->loaded_grid.assign(grid_index, grid_index + n_scans);
  return matchers_loaded_locked(c, levels, use_fine, poses, covs, scores);
}

}  // extern "C"
