// csm_api.cpp — host side of the C-ABI (include/csm.h).
//
// Owns the per-context HIP stream and device buffers, turns reference-style
// calls into batched device windows (csm_internal.hpp), and performs the
// reference's host finish: std::sort of the candidates, FindBestCandidate,
// covariance and the world-pose write-back
// (correlate_scan_matcher.h:606-611, 670-710, 784-1019).
//
// Compiled with g++ -O2 -ffp-contract=off (no -march), like the reference's
// Release build, so every host double expression rounds as the reference's
// does. The candidate sort is libstdc++'s std::sort on records compared by
// score only, fed in the reference's enumeration order: the permutation is a
// function of the comparison outcomes alone, so ties resolve exactly as in the
// reference (whose Candidate2D records are 40 bytes, ours 16).

#include "csm.h"
#include "csm_internal.hpp"
#include "csm_gridmap.h"
#include "csm_gridmap_internal.hpp"
#include "host_math.hpp"
#include "csm_pyramid.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using csm::AngleEntry;
using csm::BestPartial;
using csm::LevelWork;
using csm::ScanWork;

namespace {

constexpr double kMaxVariance = 500.0;      // util/slam_util.h:57
constexpr double kDoubleTolerance = 1e-06;  // util/slam_util.h:59
constexpr double kResponseFilterTolerance = 1e-2;  // correlate_scan_matcher.h:763
constexpr int kMaxVarianceUsePointSize = 20;       // correlate_scan_matcher.h:1033

inline bool double_equal(double a, double b, double tol = kDoubleTolerance) {
  // util::DoubleEqual (util/slam_util.h:70-73)
  const double d = a - b;
  return d < 0.0 ? d >= -std::fabs(tol) : d <= std::fabs(tol);
}

inline double round_half_away(double v) {  // util::Round (util/slam_util.h:75-77)
  return v >= 0.0 ? std::floor(v + 0.5) : std::ceil(v - 0.5);
}

// Map geometry as GridMapBase stores it (grid_map_base.h:47-71,307-309).
struct Geometry {
  double scale;   // scale_factor_ = 1.0 / resolution
  double tx, ty;  // translation of world_to_map_ = scale * offset
  double mres;    // GetCellLength() = 1 / scale_factor_
  double inv_a;   // diagonal of map_to_world_ (Eigen 2x2 inverse: s * (1 / (s*s)))
  explicit Geometry(const csm_map_info& m) {
    scale = 1.0 / m.resolution;
    tx = scale * m.offset_x;
    ty = scale * m.offset_y;
    mres = 1 / scale;
    const double det = scale * scale - 0.0 * 0.0;
    inv_a = scale * (1.0 / det);
  }
  // GetMapCoordsPose (grid_map_base.h:89-93)
  void to_map(const double w[3], double out[3]) const {
    out[0] = scale * w[0] + tx;
    out[1] = scale * w[1] + ty;
    out[2] = w[2];
  }
  // GetWorldCoordsPose (grid_map_base.h:83-87)
  void to_world(const double p[3], double out[3]) const {
    const double ntx = -(inv_a * tx), nty = -(inv_a * ty);
    out[0] = inv_a * p[0] + ntx;
    out[1] = inv_a * p[1] + nty;
    out[2] = p[2];
  }
};

struct DevBuf {
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
};

struct HostBuf {  // pinned staging for device->host score copies
  void* p = nullptr;
  size_t cap = 0;
  // flags: hipHostMallocCoherent for buffers kernels write straight into
  hipError_t ensure(size_t bytes, unsigned flags = hipHostMallocDefault) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, bytes, flags);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Window dimensions of one level (correlate_scan_matcher.h:154,538).
struct Dims {
  int32_t n_angles = 0, n_space = 0;
  int64_t n_cand = 0;
};

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

// Host plan of one window (a scan at one level, centred on its current pose).
struct WindowPlan {
  double center[3];
  int step = 1, use = 1, n_used = 0, n_points = 0;
  double x0 = 0, y0 = 0;
  int64_t angle_off = 0;
};

struct Entry {
  double score;
  int64_t idx;
};

// Candidate geometry of a window, rebuilt from its flat enumeration index
// exactly as the reference stored it in Candidate2D (:569,:572, angle :554).
struct CandGeom {
  const WindowPlan& W;
  const AngleEntry* angles;
  double f;
  int64_t ns, nss;
  double x(int64_t idx) const { return W.x0 + (int)((idx / ns) % ns) * f; }
  double y(int64_t idx) const { return W.y0 + (int)(idx % ns) * f; }
  const AngleEntry& a(int64_t idx) const { return angles[idx / nss]; }
};

// Host sort path: std::sort of the window's candidates and the three ordered
// scans, producing the same FinishOut the device finish kernel produces.
void host_sort_finish(const double* scores, const Dims& D, const CandGeom& C, const csm_param& P,
                      const Geometry& G, std::vector<Entry>& e, csm::FinishOut& o) {
  const int64_t n = D.n_cand;
  e.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) e[(size_t)i] = Entry{scores[i], i};
  std::sort(e.begin(), e.end(), [](const Entry& a, const Entry& b) { return a.score > b.score; });
  const double best = e[0].score;
  // FindBestCandidate (:670-710)
  double ax = 0.0, ay = 0.0, thx = 0.0, thy = 0.0, ssum = 0.0;
  int count = 0;
  for (size_t i = 0; i < e.size(); ++i) {
    const double sc = e[i].score;
    if (!double_equal(sc, best, kResponseFilterTolerance)) break;
    ax += C.x(e[i].idx) * sc;
    ay += C.y(e[i].idx) * sc;
    thx += C.a(e[i].idx).cosine * sc;  // cos(candidate.angle()), host libm
    thy += C.a(e[i].idx).sine * sc;
    ssum += sc;
    count++;
  }
  o.front_idx = (int32_t)e[0].idx;
  o.count = count;
  o.best_score = best;
  o.thx = thx;
  o.thy = thy;
  o.ssum = ssum;
  o.best_x = count > 1 ? ax / ssum : C.x(e[0].idx);
  o.best_y = count > 1 ? ay / ssum : C.y(e[0].idx);
  const double bound = std::min(best - 0.1, 0.5);
  // ComputePositionalCovariance's candidates (:915-928)
  o.n_pos = 0;
  for (size_t i = 0; i < e.size() && o.n_pos < csm::kCovPoints; ++i) {
    if (!(e[i].score > bound)) break;
    o.pos_idx[o.n_pos] = (int32_t)e[i].idx;
    o.pos_score[o.n_pos] = e[i].score;
    o.n_pos++;
  }
  // ComputeAngularCovariance's candidates (:990-1003)
  const double lin_tol = P.search_space_resolution / G.mres;
  o.n_ang = 0;
  for (size_t i = 0; i < e.size() && o.n_ang < csm::kCovPoints; ++i) {
    if (!(e[i].score >= bound)) break;  // sorted: nothing later qualifies
    const int64_t idx = e[i].idx;
    if (double_equal(C.x(idx), o.best_x, lin_tol) && double_equal(C.y(idx), o.best_y, lin_tol)) {
      o.ang_idx[o.n_ang] = (int32_t)idx;
      o.ang_score[o.n_ang] = e[i].score;
      o.n_ang++;
    }
  }
}

// Everything BasedCorrelationScanMatch::ScanMatch does once the sorted
// candidates are summarised in `o` (correlate_scan_matcher.h:700-707,
// 835-869, covariance :887-1019). Returns the response.
// skip_lists: covariances a later level overwrites (live_lists) are not
// computed; their lists were not filled.
double complete_window(const csm::FinishOut& o, const CandGeom& C, const csm_param& P,
                       const Geometry& G, double pose[3], double cov[9], int skip_lists = 0) {
  const double best_score = o.best_score;
  const double best_x = o.best_x, best_y = o.best_y;
  double best_a = C.a(o.front_idx).angle;
  if (o.count > 1) best_a = std::atan2(o.thy / o.ssum, o.thx / o.ssum);  // :702-706

  const double sres = P.search_space_resolution;
  const double max_ang_var = 4 * (P.search_angle_resolution * P.search_angle_resolution);  // :801

  auto positional = [&]() {  // ComputePositionalCovariance (:887-956)
    for (int i = 0; i < 9; ++i) cov[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (best_score < kDoubleTolerance) {
      cov[0] = kMaxVariance;
      cov[4] = kMaxVariance;
      cov[8] = max_ang_var;
      return;
    }
    double vxx = 0.0, vxy = 0.0, vyy = 0.0, norm = 0.0;
    for (int i = 0; i < o.n_pos; ++i) {
      const double sc = o.pos_score[i];
      const double dx = C.x(o.pos_idx[i]) - best_x, dy = C.y(o.pos_idx[i]) - best_y;
      norm += sc;
      vxx += (dx * dx * sc);
      vxy += (dx * dy * sc);
      vyy += (dy * dy * sc);
    }
    if (norm > kDoubleTolerance) {
      double xx = vxx / norm, xy = vxy / norm, yy = vyy / norm;
      const double r = sres / G.mres;
      const double minv = 0.1 * (r * r);
      xx = std::max<double>(xx, minv);
      yy = std::max<double>(yy, minv);
      const double m2 = G.mres * G.mres;
      cov[0] = (xx * m2) / best_score;
      cov[1] = (xy * m2) / best_score;
      cov[3] = (xy * m2) / best_score;
      cov[4] = (yy * m2) / best_score;
      cov[8] = max_ang_var;
    }
    if (double_equal(cov[0], 0.0)) cov[0] = kMaxVariance;
    if (double_equal(cov[4], 0.0)) cov[4] = kMaxVariance;
  };
  auto angular = [&]() {  // ComputeAngularCovariance (:965-1019)
    if (best_score < kDoubleTolerance) {
      cov[8] = max_ang_var;
      return;
    }
    double norm = 0.0, acc = 0.0;
    for (int i = 0; i < o.n_ang; ++i) {
      const double sc = o.ang_score[i];
      const double d = C.a(o.ang_idx[i]).angle - best_a;
      norm += sc;
      acc += (d * d * sc);
    }
    cov[8] = (norm > kDoubleTolerance) ? acc / norm : 200 * max_ang_var;
  };
  const bool pos = !(skip_lists & 1), ang = !(skip_lists & 2);
  switch (P.type) {
    case CSM_COARSE:
      if (pos) positional();
      if (ang) angular();
      break;
    case CSM_FINE:
      if (pos) positional();
      break;
    case CSM_SUPER:
      if (ang) angular();
      break;
    default:
      break;
  }
  const double response = best_score > 1.0 ? 1.0 : best_score;  // :861-863
  if (response > P.response_threshold) {                        // :866-869
    const double bp[3] = {best_x, best_y, best_a};
    G.to_world(bp, pose);
  }
  return response;
}

// Persistent worker pool for the per-window host work (angle tables before a
// launch, completion after it). Workers sleep on a condition variable between
// jobs; the calling thread works too and returns as soon as every item is done,
// without waiting for the workers to wake and check in: waking 15 sleeping
// threads costs ~0.1 ms on the GPU box's host, more than a level's whole plan
// (measured: plan of the 189-window fine level 0.14 ms with 16 threads when the
// caller waited for every worker, against 0.22 ms on one thread). Items are
// claimed with a compare-and-swap on (job epoch, next index), so a worker that
// wakes after its job ended finds a stale epoch (or no items left) and never
// touches the finished job.
class ThreadPool {
 public:
  ThreadPool(int threads, int spin_us) : n_threads_(std::max(1, threads)), spin_us_(std::max(0, spin_us)) {}
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  template <class F>
  void run(int n, int max_threads, F&& fn) {
    const int threads = std::min(std::min(n_threads_, max_threads), n);
    if (threads <= 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    start(threads - 1);
    std::function<void(int)> job = std::forward<F>(fn);
    // items are claimed in chunks: one shared counter bumped per item cost
    // more than the work itself at ~1 us per window (cache-line contention)
    const int chunk = std::max(1, n / (threads * 8));
    uint32_t ep;
    start_ns_ = now_ns();
    first_join_ns_.store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      n_items_ = n;
      chunk_ = chunk;
      ep = (uint32_t)(epoch_.load(std::memory_order_relaxed) + 1);
      done_.store(0, std::memory_order_relaxed);
      claim_.store((uint64_t)ep << 32, std::memory_order_release);
      epoch_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    const int mine = drain(job, n, chunk, ep, false);
    // chunks claimed by workers may still be running; they are short
    for (int spins = 0; done_.load(std::memory_order_acquire) < n; ++spins) {
      if (spins < 4096)
        __builtin_ia32_pause();
      else
        std::this_thread::yield();
    }
    last_caller_share_ = (double)mine / n;
    const int64_t j = first_join_ns_.load(std::memory_order_relaxed);
    last_join_us_ = j ? (double)(j - start_ns_) * 1e-3 : -1.0;
  }
  // the last job: the caller's share of the items, and when the first worker
  // joined it (us after the notify; -1: none did) — profiling only
  double last_caller_share() const { return last_caller_share_; }
  double last_join_us() const { return last_join_us_; }

 private:
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  int drain(const std::function<void(int)>& job, int n, int chunk, uint32_t ep, bool worker) {
    uint64_t c = claim_.load(std::memory_order_acquire);
    int ran = 0;
    for (;;) {
      if ((uint32_t)(c >> 32) != ep || (int64_t)(c & 0xffffffffu) >= n) return ran;
      if (!claim_.compare_exchange_weak(c, c + (uint64_t)chunk, std::memory_order_acq_rel)) continue;
      if (worker && ran == 0) {
        int64_t zero = 0;
        first_join_ns_.compare_exchange_strong(zero, now_ns(), std::memory_order_relaxed);
      }
      const int i0 = (int)(c & 0xffffffffu), i1 = std::min(n, i0 + chunk);
      for (int i = i0; i < i1; ++i) job(i);
      ran += i1 - i0;
      done_.fetch_add(i1 - i0, std::memory_order_release);
      c = claim_.load(std::memory_order_acquire);
    }
  }
  void start(int want) {
    std::lock_guard<std::mutex> lk(mu_);
    while ((int)workers_.size() < want) {
      const int id = (int)workers_.size();
      workers_.emplace_back([this, id] { loop(id); });
    }
    wanted_ = want;
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job = nullptr;
      int n = 0, chunk = 1;
      if (spin_us_ > 0) {  // optional: stay awake for the next job a while
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us_);
        for (int k = 1; epoch_.load(std::memory_order_acquire) == seen; ++k) {
          __builtin_ia32_pause();
          if ((k & 255) == 0 && std::chrono::steady_clock::now() > until) break;
        }
      }
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (epoch_.load() != seen && id < wanted_); });
        if (stop_) return;
        seen = epoch_.load();
        job = job_;
        n = n_items_;
        chunk = chunk_;
      }
      drain(*job, n, chunk, (uint32_t)seen, true);
    }
  }
  int n_threads_, spin_us_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  const std::function<void(int)>* job_ = nullptr;
  int n_items_ = 0, wanted_ = 0, chunk_ = 1;
  std::atomic<uint64_t> epoch_{0};
  std::atomic<uint64_t> claim_{0};
  std::atomic<int> done_{0};
  bool stop_ = false;
  int64_t start_ns_ = 0;
  std::atomic<int64_t> first_join_ns_{0};
  double last_caller_share_ = 0.0, last_join_us_ = -1.0;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int pick_cpl(int64_t n_cand) {
  if (n_cand >= 8192) return 4;
  if (n_cand >= 1024) return 2;
  return 1;
}

}  // namespace

// A launch left in flight by run_windows(..., pend): what wait_run needs to
// join it and account its kernels.
struct PendingRun {
  char kname[48] = {0};
  char fname[48] = {0};
  double alg_bytes = 0.0, scorings = 0.0, finish_bytes = 0.0;
  bool device_finish = false, timed = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, done = nullptr;
  hipEvent_t ev_fast = nullptr;  // after the fast finish pass, when the exact pass runs on x_stream
  const int32_t* flags = nullptr;  // need-exact flags on the host (profiling)
  int n_flags = 0;
  // few-window launches: the finish writes FinishOut here (host memory) and
  // stores flag_value at host_flag when the whole level is done
  const csm::FinishOut* fin_host = nullptr;
  const int32_t* host_flag = nullptr;
  int32_t flag_value = 0;
  // profiling with a host signal: read the launch's events later
  // (flush_deferred) instead of waiting for its last kernel to retire
  bool defer_timing = false;
};

struct csm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // kernels
  // Per-launch copies run on their own streams (DMA engines), ordered against
  // the kernels by events: a part's inputs go up while the other part's
  // kernels run, its results come down while the next kernels run.
  hipStream_t h2d = nullptr, d2h = nullptr;
  // The exact finish pass (a few latency-bound blocks per launch: the flagged
  // windows' sort chains) runs here, after the fast pass (ev_fast), so it
  // overlaps the other part's scoring on `stream`; the part's results go down
  // after it (ev_k on this stream). CSM_EXACT_STREAM=0: everything on `stream`.
  hipStream_t x_stream = nullptr;
  hipEvent_t ev_fast = nullptr;
  std::mutex mu;
  std::string err;
  float outside = 0.3f;  // kMapUnknownCellProb (slam/slam_processor.h:264)
  int host_threads = 1, pool_spin_us = 0;
  std::unique_ptr<ThreadPool> pool;
  template <class F>
  void parallel_for(int n, int threads, F&& fn) {
    if (!pool) pool.reset(new ThreadPool(host_threads, pool_spin_us));
    pool->run(n, threads, std::forward<F>(fn));
  }

  csm_map_info info{};
  bool has_grid = false;
  const float* d_grid = nullptr;  // owned (grid_buf) or borrowed
  DevBuf grid_buf;
  const void* key_cells = nullptr;
  int64_t key_stride = 0, key_version = -1;
  int32_t key_sx = -1, key_sy = -1;

  DevBuf pts, scans, angles, scores, partials, best, fin;
  DevBuf best_tiles;  // tiled box mode: one best per (window, tile) between the two reductions
  HostBuf h_search;   // csm_search_windows: pinned staging of the points and angle table
  bool staging_dirty = false;  // a search failed with copies out of its staging possibly in flight
  csm_gridmap* reader_map = nullptr;  // the map csm_set_grid_gridmap borrowed (its updates wait for this stream)
  HostBuf h_pts;      // upload_points: pinned staging of a scan's points (and small host arrays)
  hipEvent_t ev_pts = nullptr;  // the last copy out of h_pts
  bool ev_pts_used = false;
  HostBuf h_scores, h_fin, h_angles, h_sw;
  HostBuf h_angles_next;  // the next level's angle rows while this level's are still read (level_end_begin)
  // Host-signal device finish of the throughput path (CSM_HOST_SIGNAL=0: off):
  // the finish writes FinishOut straight into coherent pinned memory and the
  // pass that ends last stores a flag there (no D2H copy, no event round trip).
  // fin_sig: done counter | need[nw] | list[nw + 1]; h_fin_sig: FinishOut[nw] | flag.
  bool host_signal = true;
  DevBuf fin_sig;
  HostBuf h_fin_sig;
  bool device_finish = true;  // CSM_FINISH=host forces the host std::sort path
  bool fast_finish = true;    // CSM_FINISH=exact: always the full device std::sort emulation
  int device_finish_min = 1;  // fewest windows per launch that finish on the device
  bool column_kernel = true;  // CSM_KERNEL=v1 selects the lane-per-candidate kernels
  bool row_kernel = true;     // CSM_KERNEL=v2 (or v1) turns the row-segment kernels off
  bool row_dma = true;        // CSM_KERNEL=v3: register-staged row segments instead of LDS-DMA
  bool phase_kernel = true;   // v7 phase kernel for sub-cell window steps (CSM_KERNEL=v7 or unset)
  bool tiny_kernel = true;    // v8 tiny-window kernel, spans under one cell (CSM_KERNEL=v8 or unset)
  int phase_margin_log2 = 20; // CSM_PHASE_MARGIN_LOG2 (tests: a wider margin sends more beams to the exact path)
  bool box_kernel = true;     // v6 box kernel for one-cell window steps; any CSM_KERNEL other
                              // than v6 turns it off (CSM_KERNEL=v4: the LDS-DMA row kernel)
  // Few-window launches (run_windows_small): the split kernel's slab and
  // arrival counters, the device copy of the windows and the finish's scratch
  // (ScanWork[nw] | AngleEntry[..] | need[nw] | list[nw + 1] | done counter),
  // the windows' staging and the FinishOut the finish writes straight into
  // coherent pinned memory, followed by the flag the exact pass sets last.
  DevBuf split_slab, split_arrive, small_dev;
  HostBuf h_small_in, h_small_out;
  uint32_t flag_seq = 0;
  bool small_path = true;      // CSM_SMALL=0: few-window launches take the throughput kernels
  int small_max_windows = 32;  // CSM_SMALL_WINDOWS
  int split_target_blocks = 512;  // CSM_SPLIT_TARGET: blocks a split launch aims for
  int fast_wide_windows = 0;      // CSM_FAST_WIDE: fast finishes of <= this many windows on 1024 threads (0: 64; -1: never)
  HostBuf h_pack;  // pinned staging of packed grid rows / cell updates (grid uploads)
  hipEvent_t ev_pack = nullptr;  // the last copy out of h_pack (cell updates return before it ends)
  bool ev_pack_used = false;
  // the points last uploaded (upload_points skips an identical upload: the
  // reference's ScanMatchers calls each level with the same range data)
  std::vector<double> pts_host;
  bool pts_cached = false;
  DevBuf d_updates;  // csm_update_grid_cells entries on the device

  // Resident grids of other host maps. csm_set_grid keys a grid on the host
  // cells pointer (the map's identity); switching between maps (the front
  // end's fine map, the back end's maps) swaps the current grid with a parked
  // one instead of re-uploading it. The least recently used is evicted.
  struct GridSlot {
    csm_map_info info{};
    bool has_grid = false;
    const float* d_grid = nullptr;
    DevBuf grid_buf, gridi;
    const int32_t* d_gridi = nullptr;
    const void* key_cells = nullptr;
    int64_t key_stride = 0, key_version = -1;
    int32_t key_sx = -1, key_sy = -1;
    bool int_checked = false, int_ok = false;
    int int_exp = 0;
    int32_t pitch = 0, n_grids = 1, outside_i = 0;
    double int_max_abs = 0.0;
    uint64_t last_use = 0;
  };
  static constexpr int kParkedGrids = 3;
  GridSlot parked[kParkedGrids];
  uint64_t grid_clock = 0, cur_use = 0;
  void swap_grid(GridSlot& g) {
    std::swap(info, g.info);
    std::swap(has_grid, g.has_grid);
    std::swap(d_grid, g.d_grid);
    std::swap(grid_buf, g.grid_buf);
    std::swap(gridi, g.gridi);
    std::swap(d_gridi, g.d_gridi);
    std::swap(key_cells, g.key_cells);
    std::swap(key_stride, g.key_stride);
    std::swap(key_version, g.key_version);
    std::swap(key_sx, g.key_sx);
    std::swap(key_sy, g.key_sy);
    std::swap(int_checked, g.int_checked);
    std::swap(int_ok, g.int_ok);
    std::swap(int_exp, g.int_exp);
    std::swap(pitch, g.pitch);
    std::swap(n_grids, g.n_grids);
    std::swap(outside_i, g.outside_i);
    std::swap(int_max_abs, g.int_max_abs);
    std::swap(cur_use, g.last_use);
    grid_gen = ++gen_clock;
  }
  // The current grid is a host map's own copy (worth keeping when another
  // grid takes its place).
  bool owns_host_grid() const {
    return has_grid && key_cells != nullptr && d_grid == (const float*)grid_buf.p;
  }

  // Gauss-Newton matcher (csm_optimize_scan_match*): per-scan state up, sums down
  DevBuf opt_off, opt_scans, opt_sums;
  HostBuf h_opt_scans, h_opt_sums;

  // exact fixed-point copy of the grid (ensure_int_grid)
  DevBuf gridi, gstats;
  const int32_t* d_gridi = nullptr;  // the current fixed-point grid: gridi, or a map's mirror (borrowed)
  // Changes whenever the current fixed-point grid may have (rebuilt, cells or
  // rows refreshed, another grid swapped in): keys the pooled levels of the
  // multi-resolution search.
  uint64_t grid_gen = 0, gen_clock = 0;
  csm::PyramidSearch pyramid;
  bool int_checked = false, int_ok = false;
  int int_exp = 0;
  int32_t pitch = 0;  // gridi row pitch (cells)
  int32_t n_grids = 1;  // grids resident back to back (csm_set_grid_stack)
  double int_max_abs = 0.0;  // max |cell| (and |outside|) for the per-launch exactness bound
  int32_t outside_i = 0;
  double pts_maxabs = 0.0;   // max |x|+|y| of the resident points (NaN: unbounded)


  // scans made resident by csm_load_scans (offsets relative to pts)
  int32_t loaded_n = -1;
  std::vector<int64_t> loaded_off;
  std::vector<int32_t> loaded_grid;  // per loaded scan: the resident grid it is matched on (empty: grid 0)

  // per-kernel HIP-event timing (csm_set_profiling / csm_kernel_stats)
  bool profiling = false;
  bool stats_dump = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipEvent_t ev_ft = nullptr;    // profiling: the fast finish pass ended (timed; ev_fast is not)
  hipEvent_t ev_done = nullptr;  // end of a launch's work (async runs)
  hipEvent_t ev_in = nullptr;    // a launch's inputs are on the device
  hipEvent_t ev_k = nullptr;     // a launch's kernels are done

  // Second set of per-launch buffers: the 3-level driver keeps two halves of
  // a batch in flight (match_levels_pipelined); swap_slot() exchanges the
  // sets so run_windows works on whichever half is current. Every part uses
  // the one kernel stream: a stream per part measured slower (two concurrent
  // box-kernel launches contend for L2, 1.01 -> 1.57 ms each; profiles/r01).
  struct Slot {
    DevBuf scans, angles, scores, partials, best, fin;
    HostBuf h_scores, h_fin, h_angles, h_sw, h_angles_next, h_fin_sig;
    DevBuf fin_sig;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev_done = nullptr, ev_in = nullptr, ev_k = nullptr;
    hipEvent_t ev_ft = nullptr;
    hipEvent_t ev_fast = nullptr;
  };
  static constexpr int kMaxParts = 4;
  Slot alt[kMaxParts - 1];
  int pipeline_min = 512;    // fewest scans the 3-level driver splits into parts (CSM_PIPELINE)
  bool skip_dead_lists = true;  // live_lists (CSM_SKIP_DEAD_LISTS=0: every level fills both lists)
  int pipeline_parts = 2;    // parts in flight (CSM_PIPELINE_PARTS: 2..kMaxParts; 2 measured fastest)
  int first_windows = 64;    // level_begin_split: windows the first part's first launch takes (CSM_FIRST_WINDOWS; 0: one launch)
  void swap_slot(int i) {    // i >= 1: exchange the current buffer set with alt[i - 1]
    Slot& a = alt[i - 1];
    std::swap(scans, a.scans);
    std::swap(angles, a.angles);
    std::swap(scores, a.scores);
    std::swap(partials, a.partials);
    std::swap(best, a.best);
    std::swap(fin, a.fin);
    std::swap(h_scores, a.h_scores);
    std::swap(h_fin, a.h_fin);
    std::swap(h_angles, a.h_angles);
    std::swap(h_angles_next, a.h_angles_next);
    std::swap(h_fin_sig, a.h_fin_sig);
    std::swap(fin_sig, a.fin_sig);
    std::swap(h_sw, a.h_sw);
    std::swap(ev0, a.ev0);
    std::swap(ev1, a.ev1);
    std::swap(ev2, a.ev2);
    std::swap(ev_done, a.ev_done);
    std::swap(ev_in, a.ev_in);
    std::swap(ev_k, a.ev_k);
    std::swap(ev_fast, a.ev_fast);
    std::swap(ev_ft, a.ev_ft);
  }
  // profiling: the pool's last job, as "pool:<what>" (total_ms = the first
  // worker's join latency, algorithmic_bytes = the caller's share of the items)
  void account_pool(const char* what) {
    if (!profiling || !pool) return;
    char nm[48];
    std::snprintf(nm, sizeof(nm), "pool:%s", what);
    account(nm, (float)(std::max(0.0, pool->last_join_us()) * 1e-3), pool->last_caller_share(), 0.0);
  }
  std::vector<PendingRun> deferred;  // signalled launches whose timings are read later (flush_deferred)
  std::vector<csm_kernel_stat> stats;
  void account(const char* name, float ms, double bytes, double scorings) {
    for (auto& s : stats)
      if (std::strncmp(s.name, name, sizeof(s.name)) == 0) {
        s.launches += 1;
        s.total_ms += ms;
        s.algorithmic_bytes += bytes;
        s.scorings += scorings;
        return;
      }
    csm_kernel_stat s{};
    std::snprintf(s.name, sizeof(s.name), "%s", name);
    s.launches = 1;
    s.total_ms = ms;
    s.algorithmic_bytes = bytes;
    s.scorings = scorings;
    stats.push_back(s);
  }

  int fail(int code, const std::string& msg) {
    err = msg;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return CSM_ERR_HIP;
  }
};

namespace {

// Smallest power of two a float is an integer multiple of (0 for 0).
int float_granularity(float v, bool* zero) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u &= 0x7FFFFFFFu;
  *zero = (u == 0);
  if (*zero) return INT32_MAX;
  const uint32_t e = u >> 23, m = u & 0x7FFFFFu;
  const uint32_t mm = (e == 0) ? m : (m | 0x800000u);
  return ((e == 0) ? -149 : (int)e - 150) + __builtin_ctz(mm);
}

// Decide whether the grid (+ outside value) can be summed exactly in fixed
// point and build the shifted copy (value - outside) * 2^E on the device.
// Exact when every value is a multiple of 2^-E and the chunk sums fit:
// (max|v| + |outside|) * 2^E <= 2^26. Real scan-match grids (fp32 values in
// [0.3, 1]) give E = 25. A sum of B such values is exact in the reference's
// fp64 as long as B * max|v| * 2^E <= 2^53 (checked per launch).
int ensure_int_grid(csm_ctx* c) {
  if (c->int_checked) return CSM_OK;
  c->int_checked = true;
  c->int_ok = false;
  if (c->profiling) c->account("grid:analyze", 0.f, 0.0, 0.0);  // a whole-grid analysis + conversion
  const int64_t n = (int64_t)c->info.size_x * c->info.size_y * c->n_grids;
  hipError_t e;
  if ((e = c->gstats.ensure(sizeof(csm::GridStats) * (1 + csm::kAnalyzeBlocks))) != hipSuccess) return c->hip_fail(e, "hipMalloc(stats)");
  if ((e = csm::launch_analyze_grid(c->d_grid, n, (csm::GridStats*)c->gstats.p, c->stream)) != hipSuccess)
    return c->hip_fail(e, "analyze_grid_kernel");
  csm::GridStats st{};
  if ((e = hipMemcpyAsync(&st, c->gstats.p, sizeof(st), hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(stats)");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(stats)");
  if (st.nonfinite || !std::isfinite(c->outside)) return CSM_OK;
  bool ozero = false;
  const int og = float_granularity(c->outside, &ozero);
  const int min_g = std::min(st.min_gexp, og);
  float maxv;
  std::memcpy(&maxv, &st.max_abs_bits, 4);
  const double vmax = std::max((double)maxv, (double)std::fabs(c->outside));
  const int E = (min_g == INT32_MAX) ? 0 : std::max(0, -min_g);
  if (E > 60) return CSM_OK;
  const double scale = std::ldexp(1.0, E);
  // strict: |v - outside| * 2^E <= 2^26 - 1, so 32 of them fit an int32 chunk
  if (((double)maxv + std::fabs((double)c->outside)) * scale >= std::ldexp(1.0, 26)) return CSM_OK;
  const int32_t pitch = csm::gridi_pitch(c->info.size_x);  // 16-byte aligned rows, zero pad columns
  const int64_t ni = (int64_t)pitch * (c->info.size_y + csm::kGridiPadRows);  // + zero rows
  if (ni * 4 > 0x7F000000LL) return CSM_OK;  // buffer byte offsets (+ the kernels' bad offset) < 2^31
  if ((e = c->gridi.ensure((size_t)ni * (size_t)c->n_grids * sizeof(int32_t))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(gridi)");
  const int64_t cells1 = (int64_t)c->info.size_x * c->info.size_y;
  for (int gi = 0; gi < c->n_grids; ++gi)
    if ((e = csm::launch_fixed_point(c->d_grid + gi * cells1, c->info.size_x, c->info.size_y, pitch, c->outside, E,
                                     (int32_t*)c->gridi.p + gi * ni, c->stream)) != hipSuccess)
      return c->hip_fail(e, "fixed_point_kernel");
  // other parts' streams read gridi next (match_levels_pipelined)
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(gridi)");
  c->d_gridi = (const int32_t*)c->gridi.p;
  c->pitch = pitch;
  c->int_exp = E;
  c->int_max_abs = vmax;
  c->outside_i = (int32_t)((double)c->outside * scale);
  c->int_ok = true;
  c->grid_gen = ++c->gen_clock;
  return CSM_OK;
}

// The context stops reading a borrowed map: its later updates no longer wait
// for everything on this stream, only for the reads enqueued until now.
void release_map_reader(csm_ctx* c) {
  if (!c->reader_map) return;
  csm::gridmap_release_reader(c->reader_map, c->stream);
  c->reader_map = nullptr;
}

// Make the grid keyed on `cells` current: it is current already, or parked
// (swapped in), or new (the current host-map grid is parked first, evicting
// the least recently used slot). Returns true when the grid was found.
bool select_grid(csm_ctx* c, const void* cells) {
  release_map_reader(c);
  c->cur_use = ++c->grid_clock;
  if (c->owns_host_grid() && c->key_cells == cells) return true;
  for (auto& g : c->parked)
    if (g.has_grid && g.key_cells == cells) {
      if (c->owns_host_grid()) {
        c->swap_grid(g);
      } else {  // a borrowed or empty current grid is not kept
        csm_ctx::GridSlot tmp;
        c->swap_grid(tmp);
        c->swap_grid(g);
        std::swap(g, tmp);
        tmp.grid_buf.release();
        tmp.gridi.release();
      }
      c->cur_use = ++c->grid_clock;
      return true;
    }
  if (c->owns_host_grid()) {
    csm_ctx::GridSlot* v = &c->parked[0];
    for (auto& g : c->parked) {
      if (!g.has_grid) {
        v = &g;
        break;
      }
      if (g.last_use < v->last_use) v = &g;
    }
    v->grid_buf.release();
    v->gridi.release();
    *v = csm_ctx::GridSlot();
    c->swap_grid(*v);  // the current grid is parked; the empty slot becomes current
    c->cur_use = ++c->grid_clock;
  }
  c->has_grid = false;
  c->key_cells = nullptr;
  c->key_version = -1;
  return false;
}

// A borrowed device grid or a stack replaces the current grid: keep the
// current host-map grid parked so a later csm_set_grid of it is free.
void park_current(csm_ctx* c) {
  if (c->owns_host_grid()) select_grid(c, nullptr);
}

// Pack rows [y0, y1) of a strided host grid into dst (row-major fp32) on the
// context's host threads, and gather the values' fixed-point statistics
// (smallest power-of-two granularity, largest magnitude, non-finite).
struct PackStats {
  int min_g = INT32_MAX;
  float max_abs = 0.f;
  bool nonfinite = false;
};
PackStats pack_rows(csm_ctx* c, const void* cells, int64_t stride, int32_t sx, int32_t y0, int32_t y1, float* dst) {
  const int rows = y1 - y0;
  const int chunks = std::max(1, std::min(rows, c->host_threads * 4));
  std::vector<PackStats> part((size_t)chunks);
  c->parallel_for(chunks, c->host_threads, [&](int t) {
    const int r0 = y0 + (int)((int64_t)rows * t / chunks), r1 = y0 + (int)((int64_t)rows * (t + 1) / chunks);
    PackStats ps;
    for (int y = r0; y < r1; ++y) {
      const char* src = (const char*)cells + ((int64_t)y * sx) * stride;
      float* out = dst + (int64_t)(y - y0) * sx;
      if (stride == 4) {
        std::memcpy(out, src, (size_t)sx * 4);
      } else {
        for (int32_t x = 0; x < sx; ++x) std::memcpy(out + x, src + (int64_t)x * stride, 4);
      }
      for (int32_t x = 0; x < sx; ++x) {
        const float v = out[x];
        if (!std::isfinite(v)) ps.nonfinite = true;
        bool z;
        ps.min_g = std::min(ps.min_g, float_granularity(v, &z));
        ps.max_abs = std::max(ps.max_abs, std::fabs(v));
      }
    }
    part[(size_t)t] = ps;
  });
  PackStats all;
  for (const auto& p : part) {
    all.min_g = std::min(all.min_g, p.min_g);
    all.max_abs = std::max(all.max_abs, p.max_abs);
    all.nonfinite = all.nonfinite || p.nonfinite;
  }
  return all;
}

// New cell values keep the exact fixed-point copy valid when they are
// multiples of 2^-E and within its range (ensure_int_grid's conditions);
// otherwise the copy is rebuilt before the next match.
void note_new_values(csm_ctx* c, const PackStats& ps) {
  if (!c->int_checked || !c->int_ok) return;
  const double scale = std::ldexp(1.0, c->int_exp);
  if (ps.nonfinite || (ps.min_g != INT32_MAX && ps.min_g < -c->int_exp) ||
      ((double)ps.max_abs + std::fabs((double)c->outside)) * scale >= std::ldexp(1.0, 26)) {
    c->int_checked = false;
    return;
  }
  c->int_max_abs = std::max(c->int_max_abs, (double)ps.max_abs);
}

// Scores windows_n windows of one level on the device. plans[i] describes
// window i, pts_dev is the batch's points already resident. When best_out is
// null, every score is copied back into ctx->h_scores (window-major).
enum class Finish { kScoresToHost, kDevice, kBest };


// Spin on the host flag the exact pass stores last (a launch + flag round
// trip measured 6 us on the GPU box against 12 us through an event,
// tools/ubench/roundtrip.hip). Every 256 spins the stream's event is
// polled: a launch that failed, or that completed without the flag, is an
// error instead of a hang.
int wait_flag(csm_ctx* c, const PendingRun& p) {
  for (uint32_t spin = 1;; ++spin) {
    if (__atomic_load_n(p.host_flag, __ATOMIC_ACQUIRE) == p.flag_value) return CSM_OK;
    if ((spin & 255) == 0) {
      const hipError_t e = hipEventQuery(p.done);
      if (e == hipSuccess) {
        if (__atomic_load_n(p.host_flag, __ATOMIC_ACQUIRE) == p.flag_value) return CSM_OK;
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
    c->account(p.kname, ms, p.alg_bytes, p.scorings);
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
  return T.nq > 0;
}


// Exact fixed-point accumulation for these windows: grid eligible, beams
// bounded, no offset wrap (every endpoint within 2^30 bytes of a row).
bool int_mode_ok(const csm_ctx* c, const Dims& D, double f, const std::vector<WindowPlan>& plans, size_t i0 = 0,
                 size_t i1 = SIZE_MAX) {
  if (!c->int_ok) return false;
  for (size_t i = i0; i < std::min(i1, plans.size()); ++i) {
    const WindowPlan& W = plans[i];
    const double far = (double)(D.n_space - 1) * f;
    const double span = std::max(std::max(std::fabs(W.x0), std::fabs(W.x0 + far)),
                                 std::max(std::fabs(W.y0), std::fabs(W.y0 + far)));
    const double R = c->pts_maxabs * (1.0 + 1e-9) + span + 2.0;
    if (!(R * 4.0 * (double)c->pitch < std::ldexp(1.0, 30))) return false;
    if ((double)W.n_used * c->int_max_abs * std::ldexp(1.0, c->int_exp) > std::ldexp(1.0, 53)) return false;
  }
  return true;
}

void fill_scan_work(const Dims& D, const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                    const std::vector<int32_t>& grid_index, ScanWork* sw, size_t i0 = 0, size_t i1 = SIZE_MAX) {
  for (size_t i = i0; i < std::min(i1, plans.size()); ++i) {
    const WindowPlan& W = plans[i];
    ScanWork& s = sw[i];
    s.pts_off = pt_offsets[i];
    s.angle_off = W.angle_off;
    s.out_off = (int64_t)i * D.n_cand;
    s.n_used = W.n_used;
    s.step = W.step;
    s.divisor = (double)(W.use - 0);
    s.x0 = W.x0;
    s.y0 = W.y0;
    s.cx = W.center[0];
    s.cy = W.center[1];
    s.ct = W.center[2];
    s.reserved = 0;
    s.grid_index = grid_index.empty() ? 0 : grid_index[i];
  }
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
  const size_t o_list = o_need + (size_t)nw * 4;
  const size_t dev_bytes = o_list + (size_t)(nw + 1) * 4;
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
  A.skip_lists = skip_lists;
  A.need_exact = d_need;
  A.exact_list = d_list;
  A.done_ctr = d_done;
  A.host_flag = h_flag;
  A.wide_windows = c->fast_wide_windows;
  A.flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
  if (A.flag_value == 0) A.flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
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

// With pend == nullptr the call returns once results are on the host; with
// pend it returns as soon as the work is enqueued (join with wait_run).
// Part of a level's launch (the 3-level driver's chunked first plan): score
// windows [w0, w1) only, or only finish every window once all are scored.
// A part needs the device finish and window i's angle rows at i * n_angles.
struct WinSpan {
  int w0 = 0, w1 = -1;  // w1 < 0: every window
  bool score = true, finish = true;
};

int run_windows(csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G,
                const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                const AngleEntry* angles, size_t n_angle_entries,
                const std::vector<int32_t>& grid_index, BestPartial* best_out,
                Finish mode = Finish::kScoresToHost, PendingRun* pend = nullptr, int skip_lists = 0,
                WinSpan sp = WinSpan{}) {
  if (best_out) mode = Finish::kBest;
  const int nw = (int)plans.size();
  if (nw == 0) return CSM_OK;
  const int w0 = sp.w1 < 0 ? 0 : sp.w0, w1 = sp.w1 < 0 ? nw : sp.w1;
  const int nr = w1 - w0;  // windows scored by this call
  const bool whole = w0 == 0 && w1 == nw && sp.score && sp.finish;
  if (!c->deferred.empty()) {  // the events below are recorded again
    const int fst = flush_deferred(c);
    if (fst != CSM_OK) return fst;
  }
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
  const bool v2 = c->column_kernel && n_cols < INT32_MAX;
  const double f = P.search_space_resolution / G.mres;
  const bool use_int = v2 && int_mode_ok(c, D, f, plans, (size_t)w0, (size_t)w1);
  if (whole && mode != Finish::kBest && use_int && small_launch(c, D, nw))
    return run_windows_small(c, P, D, G, plans, pt_offsets, angles, n_angle_entries, grid_index,
                             mode == Finish::kDevice, pend, skip_lists);
  // v3 row-segment kernel: fixed-point grid and an instantiation whose row
  // segment covers the x-span of a group, (n_space-1)*f cells (+2 for the
  // truncations); the kernel re-checks and recomputes exactly if exceeded
  int rows_sq = 0;
  if (use_int && c->row_kernel && D.n_space <= 64) {
    const double span = (double)(D.n_space - 1) * f;
    // distinct columns of a group <= floor(span) + 2
    rows_sq = csm::rows_pick_sq(D.n_space, (int)std::floor(span * (1.0 + 1e-9) + 1e-9) + 2);
    if (c->info.size_x < 4 * rows_sq) rows_sq = 0;
  }
  // v6 box kernel: whole-cell window step (use_int bounds |t| < 2^24 cells,
  // which its rounding margin needs)
  const bool box = use_int && c->box_kernel && f == 1.0 && csm::box_supported(D.n_space) &&
                   c->pitch >= c->info.size_x + csm::kGridiPadCols;
  if (box) rows_sq = 0;
  // v6 over 16 x 16 tiles: the argmax of a one-cell-step window wider than 16
  // (loop-closure windows), in place of the column kernel's dword gathers
  const int tile_n = (D.n_space + 15) / 16;
  const bool box_tiled = !box && best_out && use_int && c->box_kernel && f == 1.0 && D.n_space > 16 &&
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
  // v8 tiny-window kernel: a sub-cell step whose whole span is under one cell
  const bool tiny = !box && !phase && use_int && c->tiny_kernel && f < 1.0 && csm::tiny_supported(D.n_space, f) &&
                    c->pitch >= c->info.size_x + csm::kGridiPadCols &&
                    (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows) * 4 < INT32_MAX;
  if (tiny) rows_sq = 0;
  const int cpl = pick_cpl(D.n_cand);
  const int64_t per_block = (int64_t)csm::kBlock * cpl;
  const int64_t rows_groups = rows_sq ? 64 / D.n_space : 1;
  const int64_t bps = box_tiled ? (int64_t)tile_n * tile_n * D.n_angles
                      : (box || phase || tiny) ? D.n_angles
                      : rows_sq ? (D.n_angles + rows_groups - 1) / rows_groups
                      : v2    ? col_blocks * ktiles
                              : (D.n_cand + per_block - 1) / per_block;
  if (bps * nr > INT32_MAX) return c->fail(CSM_ERR_UNSUPPORTED, "window too large for one launch");

  hipError_t e;
  if ((e = c->h_sw.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(scans)");
  ScanWork* sw = (ScanWork*)c->h_sw.p;  // pinned staging
  if (sp.score) fill_scan_work(D, plans, pt_offsets, grid_index, sw, (size_t)w0, (size_t)w1);
  LevelWork L = make_level_work(c, P, D, G, nr, use_int);
  L.blocks_per_scan = box_tiled ? D.n_angles : (int32_t)bps;  // per (window, tile) when tiled
  L.tile_n = box_tiled ? tile_n : 0;
  L.n_cols = (int32_t)n_cols;
  L.ktiles = ktiles;
  L.col_blocks = (int32_t)col_blocks;

  // Host-signal finish (the device finish with its fast pass): FinishOut goes
  // straight to coherent pinned memory and the pass that ends last sets a flag
  // the host spins on; the scoring kernel clears the flagged-window count.
  const bool sig = c->host_signal && mode == Finish::kDevice && c->fast_finish;
  int32_t *d_done = nullptr, *d_need = nullptr, *d_list = nullptr;
  if (sig) {
    const size_t o_need = 64, o_list = o_need + (size_t)nw * 4, dbytes = o_list + (size_t)(nw + 1) * 4;
    if (dbytes > c->fin_sig.cap) {  // the done counter starts at zero; each launch leaves it at zero
      if ((e = c->fin_sig.ensure(dbytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(finish signal)");
      if ((e = hipMemsetAsync(c->fin_sig.p, 0, c->fin_sig.cap, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipMemsetAsync(finish signal)");
    }
    d_done = (int32_t*)c->fin_sig.p;
    d_need = (int32_t*)((char*)c->fin_sig.p + o_need);
    d_list = (int32_t*)((char*)c->fin_sig.p + o_list);
    L.clear_word = d_list;
  }

  if ((e = c->scans.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scans)");
  if ((e = c->angles.ensure(n_angle_entries * sizeof(AngleEntry))) != hipSuccess) return c->hip_fail(e, "hipMalloc(angles)");
  const double tl0 = c->profiling ? now_ms() : 0.0;  // host cost of the launch, by phase
  if (sp.score) {  // this call's windows and angle rows
    const size_t a0 = whole ? 0 : (size_t)w0 * D.n_angles;
    const size_t na = whole ? n_angle_entries : (size_t)nr * D.n_angles;
    if ((e = hipMemcpyAsync((ScanWork*)c->scans.p + w0, sw + w0, (size_t)nr * sizeof(ScanWork), hipMemcpyHostToDevice,
                            c->h2d)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(scans)");
    if ((e = hipMemcpyAsync((AngleEntry*)c->angles.p + a0, angles + a0, na * sizeof(AngleEntry), hipMemcpyHostToDevice,
                            c->h2d)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(angles)");
    if ((e = hipEventRecord(c->ev_in, c->h2d)) != hipSuccess || (e = hipStreamWaitEvent(c->stream, c->ev_in, 0)) != hipSuccess)
      return c->hip_fail(e, "inputs event");
  }

  // algorithmic traffic: one fp32 grid read per summed beam per candidate
  double beams = 0.0;
  for (const WindowPlan& W : plans) beams += (double)W.n_used;
  const double alg_bytes = beams * (double)D.n_cand * 4.0;
  const double scorings = (double)nw * (double)D.n_cand;
  char kname[48];
  if (box)
    std::snprintf(kname, sizeof(kname), "score_box_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (box_tiled)
    std::snprintf(kname, sizeof(kname), "score_box_kernel<16,best,tiles>");
  else if (phase)
    std::snprintf(kname, sizeof(kname), "score_phase_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (tiny)
    std::snprintf(kname, sizeof(kname), "score_tiny_kernel<%d,%s>", D.n_space, best_out ? "best" : "all");
  else if (rows_sq)
    std::snprintf(kname, sizeof(kname), "%s<%d,%d,%s>", c->row_dma ? "score_rowsd_kernel" : "score_rows_kernel",
                  D.n_space, rows_sq, best_out ? "best" : "all");
  else if (v2)
    std::snprintf(kname, sizeof(kname), "score_cols_kernel<%d,%s,%s>", kt, use_int ? "int" : "f64",
                  best_out ? "best" : "all");
  else
    std::snprintf(kname, sizeof(kname), "%s<%d>", best_out ? "score_best_kernel" : "score_all_kernel", cpl);
  const double tl1 = c->profiling ? now_ms() : 0.0;
  // a signalled launch lets the host go on before its exact pass (on
  // x_stream) has retired: this slot's next scoring waits for it, so the
  // count it clears is no longer read
  if (sig && sp.score && (e = hipStreamWaitEvent(c->stream, c->ev_done, 0)) != hipSuccess)
    return c->hip_fail(e, "hipStreamWaitEvent(previous finish)");
  if (c->profiling && sp.score && w0 == 0 && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipEventRecord");

  const int32_t* flags_h = nullptr;
  int n_flags = 0;
  csm::FinishOut* sig_out = nullptr;
  int32_t* sig_flag = nullptr;
  int32_t sig_value = 0;
  hipStream_t done_stream = c->d2h;
  double tl2 = 0.0;
  if (mode != Finish::kBest) {
    const size_t bytes = (size_t)nw * (size_t)D.n_cand * sizeof(double);
    if ((e = c->scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(scores)");
    const ScanWork* d_sw = (const ScanWork*)c->scans.p + w0;
    if (!sp.score)
      e = hipSuccess;  // scored by earlier calls
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
                                 (double*)c->scores.p, nullptr, D.n_space, rows_sq, c->row_dma, c->stream);
    else if (v2)
      e = csm::launch_score_cols(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                 (double*)c->scores.p, nullptr, kt, c->stream);
    else
      e = csm::launch_score_all(L, d_sw, (const double*)c->pts.p, (const AngleEntry*)c->angles.p,
                                (double*)c->scores.p, cpl, c->stream);
    if (e != hipSuccess) return c->hip_fail(e, "score kernel");
    if (sp.score && c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipEventRecord");
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
      csm::FinishArgs A{};
      A.n_cand = D.n_cand;
      A.n_space = D.n_space;
      A.step_cells = L.step_cells;
      A.lin_tol = P.search_space_resolution / G.mres;
      A.skip_lists = skip_lists;
      A.need_exact = d_need;
      A.exact_list = d_list;
      A.done_ctr = d_done;
      A.wide_windows = c->fast_wide_windows;
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
      if (c->profiling) {  // the fast pass's flags to the host: finish:exact_windows
        A.need_exact = (int32_t*)((char*)c->h_fin_sig.p + out_need);
        flags_h = A.need_exact;
        n_flags = nw;
      }
      A.host_flag = sig_flag;
      A.flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
      if (A.flag_value == 0) A.flag_value = (int32_t)(++c->flag_seq & 0x7FFFFFFF);
      sig_value = A.flag_value;
      done_stream = c->x_stream ? c->x_stream : c->stream;
      if ((e = csm::launch_finish(A, (const ScanWork*)c->scans.p, (const AngleEntry*)c->angles.p,
                                  (const double*)c->scores.p, sig_out, nw, c->stream, done_stream, c->ev_fast)) !=
          hipSuccess)
        return c->hip_fail(e, "finish_kernel");
      if (c->profiling && done_stream != c->stream && (e = hipEventRecord(c->ev_ft, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipEventRecord");
      if (c->profiling && (e = hipEventRecord(c->ev2, done_stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    } else {
      csm::FinishArgs A{};
      A.n_cand = D.n_cand;
      A.n_space = D.n_space;
      A.step_cells = L.step_cells;
      A.lin_tol = P.search_space_resolution / G.mres;
      A.skip_lists = skip_lists;
      const size_t fbytes = (size_t)nw * sizeof(csm::FinishOut);
      // + one "needs the exact sort" flag per window (fast finish, csm_finish.hip)
      // + the flags' compacted list (count, then windows)
      if ((e = c->fin.ensure(fbytes + (size_t)(2 * nw + 1) * sizeof(int32_t))) != hipSuccess)
        return c->hip_fail(e, "hipMalloc(finish)");
      A.need_exact = c->fast_finish ? (int32_t*)((char*)c->fin.p + fbytes) : nullptr;
      A.exact_list = c->fast_finish ? A.need_exact + nw : nullptr;
      if ((e = c->h_fin.ensure(fbytes + (size_t)nw * sizeof(int32_t))) != hipSuccess)
        return c->hip_fail(e, "hipHostMalloc(finish)");
      // the exact pass on x_stream (when there is one and the fast pass runs first)
      hipStream_t fs = (c->x_stream && A.need_exact) ? c->x_stream : c->stream;
      if ((e = csm::launch_finish(A, (const ScanWork*)c->scans.p, (const AngleEntry*)c->angles.p,
                                  (const double*)c->scores.p, (csm::FinishOut*)c->fin.p, nw, c->stream, fs,
                                  c->ev_fast)) != hipSuccess)
        return c->hip_fail(e, "finish_kernel");
      if (c->profiling && fs != c->stream && (e = hipEventRecord(c->ev_ft, c->stream)) != hipSuccess)
        return c->hip_fail(e, "hipEventRecord");
      if (c->profiling && (e = hipEventRecord(c->ev2, fs)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
      // with profiling on, the flags come back too: how many windows needed the exact sort
      const size_t cbytes = fbytes + ((c->profiling && A.need_exact) ? (size_t)nw * sizeof(int32_t) : 0);
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
    if (box || box_tiled)
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
                                 D.n_space, rows_sq, c->row_dma, c->stream);
    else if (v2)
      e = csm::launch_score_cols(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                 (const AngleEntry*)c->angles.p, nullptr, (BestPartial*)c->partials.p,
                                 kt, c->stream);
    else
      e = csm::launch_score_best(L, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                 (const AngleEntry*)c->angles.p, (BestPartial*)c->partials.p, cpl,
                                 c->stream);
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
  p.device_finish = mode == Finish::kDevice;
  p.timed = c->profiling;
  p.ev0 = c->ev0;
  p.ev1 = c->ev1;
  p.ev_fast = (c->profiling && mode == Finish::kDevice && c->fast_finish && c->x_stream) ? c->ev_ft : nullptr;
  p.ev2 = c->ev2;
  p.done = c->ev_done;
  p.fin_host = sig_out;
  p.host_flag = sig_flag;
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
                      const double center[3], AngleEntry* out, WindowPlan& W) {
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
    csm::host_sincos(ae.angle, &ae.sine, &ae.cosine);
  }
  return true;
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

int upload_points(csm_ctx* c, const double* pts, int64_t n_total, void* pinned = nullptr) {
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

bool map_ready(const csm_ctx* c) { return c->has_grid && c->info.update_index >= 0; }

// ---- FAST (branch-and-bound) -------------------------------------------------
// BranchAndBoundCorrelateScanMatcher (correlate_scan_matcher.h:271-502). The
// device scores every node of the search tree (csm_bnb.hip); bnb_search then
// replays the reference's depth-first search over that table.

struct BCand {  // Candidate2D as the search uses it
  double score, x, y, angle;
  int a, i, j;  // angle index, node indices at its level
};
inline bool bcand_greater(const BCand& p, const BCand& q) { return p.score > q.score; }

struct TreeView {
  const double* s;  // one window's node scores
  int64_t per_angle;
  int64_t off[csm::kTreeMaxDepth + 1], m[csm::kTreeMaxDepth + 1];
  double score(int a, int level, int i, int j) const {
    return s[(int64_t)a * per_angle + off[level] + (int64_t)i * m[level] + j];
  }
};

// BranchAndBound (:434-476), recursion and all: the loop breaks on the
// caller's min_score, children are generated x-offset-major (:456-462), sorted
// by std::sort (:430; four elements: insertion sort) and searched with the
// best score so far; std::max keeps `best` unless best < sub.
BCand bnb_search(const TreeView& V, const std::vector<BCand>& list, int depth, double min_score,
                 const double* hw, const AngleEntry* ang) {
  if (depth == 0) return list.front();
  BCand best{min_score, 0.0, 0.0, 0.0, 0, 0, 0};  // Candidate2D(0, 0.0, 0.0, 0.0)
  std::vector<BCand> kids;
  for (const BCand& c : list) {
    if (c.score <= min_score) break;
    kids.clear();
    const double half_width = hw[depth];
    for (int ox = 0; ox < 2; ++ox) {
      for (int oy = 0; oy < 2; ++oy) {
        BCand k;
        k.x = c.x + (ox ? half_width : 0.0);
        k.y = c.y + (oy ? half_width : 0.0);
        k.angle = ang[c.a].angle;
        k.a = c.a;
        k.i = 2 * c.i + ox;
        k.j = 2 * c.j + oy;
        k.score = V.score(c.a, depth - 1, k.i, k.j);
        kids.push_back(k);
      }
    }
    std::sort(kids.begin(), kids.end(), bcand_greater);
    const BCand sub = bnb_search(V, std::vector<BCand>(kids), depth - 1, best.score, hw, ang);
    if (best.score < sub.score) best = sub;
  }
  return best;
}

// Positional + angular covariance over the sorted lowest-resolution list
// (:835-839 for FAST; :887-1019), pose write-back (:861-869).
double complete_fast(const std::vector<BCand>& cands, const BCand& best, const csm_param& P,
                     const Geometry& G, double pose[3], double cov[9]) {
  const double sres = P.search_space_resolution;
  const double max_ang_var = 4 * (P.search_angle_resolution * P.search_angle_resolution);
  const double bs = best.score;
  for (int i = 0; i < 9; ++i) cov[i] = (i % 4 == 0) ? 1.0 : 0.0;
  if (bs < kDoubleTolerance) {
    cov[0] = kMaxVariance;
    cov[4] = kMaxVariance;
    cov[8] = max_ang_var;
  } else {
    double vxx = 0.0, vxy = 0.0, vyy = 0.0, norm = 0.0;
    const double bound = std::min(bs - 0.1, 0.5);
    int counter = 0;
    for (const BCand& c : cands) {
      const double sc = c.score;
      if (!(sc > bound && counter < kMaxVarianceUsePointSize)) break;
      norm += sc;
      const double dx = c.x - best.x, dy = c.y - best.y;
      vxx += (dx * dx * sc);
      vxy += (dx * dy * sc);
      vyy += (dy * dy * sc);
      counter++;
    }
    if (norm > kDoubleTolerance) {
      double xx = vxx / norm, xy = vxy / norm, yy = vyy / norm;
      const double r = sres / G.mres;
      const double minv = 0.1 * (r * r);
      xx = std::max<double>(xx, minv);
      yy = std::max<double>(yy, minv);
      const double m2 = G.mres * G.mres;
      cov[0] = (xx * m2) / bs;
      cov[1] = (xy * m2) / bs;
      cov[3] = (xy * m2) / bs;
      cov[4] = (yy * m2) / bs;
      cov[8] = max_ang_var;
    }
    if (double_equal(cov[0], 0.0)) cov[0] = kMaxVariance;
    if (double_equal(cov[4], 0.0)) cov[4] = kMaxVariance;
  }
  if (bs < kDoubleTolerance) {
    cov[8] = max_ang_var;
  } else {
    const double lin_tol = sres / G.mres;
    const double bound = std::min(bs - 0.1, 0.5);
    double norm = 0.0, acc = 0.0;
    int counter = 0;
    for (const BCand& c : cands) {
      const double sc = c.score;
      if (sc >= bound && counter < kMaxVarianceUsePointSize) {
        if (double_equal(c.x, best.x, lin_tol) && double_equal(c.y, best.y, lin_tol)) {
          const double d = c.angle - best.angle;
          norm += sc;
          acc += (d * d * sc);
          counter++;
        }
      }
    }
    cov[8] = (norm > kDoubleTolerance) ? acc / norm : 200 * max_ang_var;
  }
  const double response = bs > 1.0 ? 1.0 : bs;
  if (response > P.response_threshold) {
    const double bp[3] = {best.x, best.y, best.angle};
    G.to_world(bp, pose);
  }
  return response;
}

int match_level_fast(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                     double* poses, double* covs, double* responses, int64_t* argmax_flat);

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
};

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
  for (int s = 0; s < n_scans; ++s) {
    if (reset) {
      responses[s] = 0.0;  // kMinResponse (:1034)
      if (argmax_flat) argmax_flat[s] = -1;
    }
    const int n = (int)(offsets[s + 1] - offsets[s]);
    if (!map_ready(c) || n == 0) continue;  // :792-795
    int step, use, n_used;
    if (!beam_rule(n, P.use_point_size, step, use, n_used))
      return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
    R.scan_of.push_back(s);
    if (scan_grid) R.grid.push_back(scan_grid[s]);
  }
  return CSM_OK;
}

// Room for the level's plans and angle rows (pinned: uploaded by DMA).
int level_alloc(csm_ctx* c, const int64_t* offsets, LevelRun& R, HostBuf& rows) {
  const int nw = (int)R.scan_of.size();
  R.plans.assign((size_t)nw, WindowPlan{});
  R.pt_off.resize((size_t)nw);
  for (int i = 0; i < nw; ++i) R.pt_off[(size_t)i] = offsets[R.scan_of[(size_t)i]];
  const hipError_t he = rows.ensure((size_t)nw * (size_t)R.D.n_angles * sizeof(AngleEntry));
  if (he != hipSuccess) return c->hip_fail(he, "hipHostMalloc(angles)");
  R.rows = (AngleEntry*)rows.p;
  R.angles = R.rows;
  return CSM_OK;
}

// Plan window i of a prepared level around the scan's current pose: host
// libm cos/sin per angle (AngleSearchLookUpTable::UpdateLookUpTable :154-172).
void level_plan_one(LevelRun& R, const Geometry& G, const int64_t* offsets, const double* poses, int i) {
  const int s = R.scan_of[(size_t)i];
  double center[3];
  G.to_map(poses + 3 * s, center);
  WindowPlan& W = R.plans[(size_t)i];
  plan_window_into(R.P, R.D, G, (int)(offsets[s + 1] - offsets[s]), center, R.rows + (size_t)i * (size_t)R.D.n_angles, W);
  W.angle_off = (int64_t)i * R.D.n_angles;
}

// Device finish for the front-end windows (and enough of them to fill the
// chip); a handful of windows finish faster on the host's std::sort.
bool level_device_finish(const csm_ctx* c, const Dims& D, int nw) {
  return c->device_finish && D.n_cand <= csm::kFinishMaxCand && csm::finish_lds_bytes(D.n_cand) <= 160 * 1024 &&
         nw >= c->device_finish_min;
}

// Enqueue a planned level, or a span of it (nothing waits).
int level_launch(csm_ctx* c, LevelRun& R, WinSpan sp = WinSpan{}) {
  const int nw = (int)R.scan_of.size();
  const Dims& D = R.D;
  const Geometry G(c->info);
  R.dev = level_device_finish(c, D, nw);
  const int st = run_windows(c, R.P, D, G, R.plans, R.pt_off, R.angles, (size_t)nw * (size_t)D.n_angles, R.grid,
                             nullptr, R.dev ? Finish::kDevice : Finish::kScoresToHost, &R.pend, R.skip_lists, sp);
  if (st != CSM_OK || !sp.finish) return st;
  R.fin = R.pend.fin_host ? R.pend.fin_host : (const csm::FinishOut*)c->h_fin.p;
  R.scores = (const double*)c->h_scores.p;
  return CSM_OK;
}

int level_begin(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                const double* poses, double* responses, int64_t* argmax_flat, LevelRun& R,
                const int32_t* scan_grid = nullptr, int skip_lists = 0) {
  int st = level_prepare(c, n_scans, offsets, P, responses, argmax_flat, R, scan_grid, skip_lists, true);
  if (st != CSM_OK) return st;
  const int nw = (int)R.scan_of.size();
  if (nw == 0) return CSM_OK;
  const double t0 = now_ms();
  if ((st = level_alloc(c, offsets, R, c->h_angles)) != CSM_OK) return st;
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  c->parallel_for(nw, threads, [&](int i) { level_plan_one(R, G, offsets, poses, i); });
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

// level_begin with the plan in two pieces: the first `first` windows are
// planned on the calling thread and their scoring goes out at once, the rest
// are planned on the pool while it runs, then the finish follows for all.
// For the 3-level driver's first part, where nothing else keeps the device
// busy while the host plans (a call's first ~0.15 ms).
int level_begin_split(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P, const double* poses,
                      double* responses, LevelRun& R, const int32_t* scan_grid, int skip_lists, int first) {
  int st = level_prepare(c, n_scans, offsets, P, responses, nullptr, R, scan_grid, skip_lists, true);
  if (st != CSM_OK) return st;
  const int nw = (int)R.scan_of.size();
  if (first <= 0 || nw < 2 * first || !level_device_finish(c, R.D, nw))
    return level_begin(c, n_scans, offsets, P, poses, responses, nullptr, R, scan_grid, skip_lists);
  const double t0 = now_ms();
  if ((st = level_alloc(c, offsets, R, c->h_angles)) != CSM_OK) return st;
  const Geometry G(c->info);
  for (int i = 0; i < first; ++i) level_plan_one(R, G, offsets, poses, i);
  if ((st = level_launch(c, R, WinSpan{0, first, true, false})) != CSM_OK) return st;
  c->parallel_for(nw - first, c->host_threads, [&](int i) { level_plan_one(R, G, offsets, poses, first + i); });
  c->account_pool("plan");
  if ((st = level_launch(c, R, WinSpan{first, nw, true, false})) != CSM_OK) return st;
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
  if (R.dev)
    for (int i = 0; i < nw; ++i)
      if (R.fin[i].count < 0) return c->fail(CSM_ERR_HIP, "finish_kernel: work loop bound exceeded");
  return CSM_OK;
}

// Complete window i of a joined level: pose, covariance and response
// (BasedCorrelationScanMatch::ScanMatch :815-869).
void level_complete_one(const LevelRun& R, const Geometry& G, double* poses, double* covs, double* responses,
                        int64_t* argmax_flat, int i) {
  thread_local std::vector<Entry> scratch;
  const Dims& D = R.D;
  const csm_param& P = R.P;
  const int s = R.scan_of[(size_t)i];
  const double f = P.search_space_resolution / G.mres;
  const CandGeom C{R.plans[(size_t)i], R.angles + R.plans[(size_t)i].angle_off, f, D.n_space,
                   (int64_t)D.n_space * D.n_space};
  csm::FinishOut local;
  const csm::FinishOut* o = nullptr;
  if (R.dev) {
    o = R.fin + i;
  } else {
    host_sort_finish(R.scores + (size_t)i * (size_t)D.n_cand, D, C, P, G, scratch, local);
    o = &local;
  }
  if (argmax_flat) argmax_flat[s] = o->front_idx;
  responses[s] = complete_window(*o, C, P, G, poses + 3 * s, covs + 9 * s, R.skip_lists);
}

int level_end(csm_ctx* c, LevelRun& R, double* poses, double* covs, double* responses,
              int64_t* argmax_flat) {
  const int nw = (int)R.scan_of.size();
  if (nw == 0) return CSM_OK;
  int st = level_join(c, R);
  if (st != CSM_OK) return st;
  const double t2 = now_ms();
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  c->parallel_for(nw, threads, [&](int i) { level_complete_one(R, G, poses, covs, responses, argmax_flat, i); });
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
int level_end_begin(csm_ctx* c, LevelRun& R, LevelRun& N, int32_t n_scans, const int64_t* offsets,
                    const csm_param& P, double* poses, double* covs, double* responses, double* sum,
                    const int32_t* scan_grid, int skip_lists) {
  int st = level_prepare(c, n_scans, offsets, P, responses, nullptr, N, scan_grid, skip_lists, false);
  if (st != CSM_OK) return st;
  const int nw = (int)R.scan_of.size();
  if (N.scan_of != R.scan_of || nw == 0) {  // not the same windows: one after the other
    if ((st = level_end(c, R, poses, covs, responses, nullptr)) != CSM_OK) return st;
    for (int s = 0; s < n_scans; ++s) sum[s] += responses[s];
    return level_begin(c, n_scans, offsets, P, poses, responses, nullptr, N, scan_grid, skip_lists);
  }
  if ((st = level_join(c, R)) != CSM_OK) return st;
  const double t2 = now_ms();
  std::swap(c->h_angles, c->h_angles_next);
  if ((st = level_alloc(c, offsets, N, c->h_angles)) != CSM_OK) return st;
  const Geometry G(c->info);
  const int threads = (nw >= 64) ? c->host_threads : 1;
  c->parallel_for(nw, threads, [&](int i) {
    level_complete_one(R, G, poses, covs, responses, nullptr, i);
    const int s = R.scan_of[(size_t)i];
    sum[s] += responses[s];
    level_plan_one(N, G, offsets, poses, i);
  });
  if (threads > 1) c->account_pool("complete+plan");
  const double t3 = now_ms();
  if ((st = level_launch(c, N)) != CSM_OK) return st;
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
                const int32_t* scan_grid = nullptr, int skip_lists = 0) {
  if (P.type == CSM_FAST) return match_level_fast(c, n_scans, offsets, P, poses, covs, responses, argmax_flat);
  LevelRun R;
  int st = level_begin(c, n_scans, offsets, P, poses, responses, argmax_flat, R, scan_grid, skip_lists);
  if (st != CSM_OK) return st;
  return level_end(c, R, poses, covs, responses, argmax_flat);
}

// ScanMatchers::ScanMatch over a resident batch (scan_matchers.h:179-289),
// parts in flight: while the device runs one part's level, the host
// completes another part's previous level and plans its next one
// (level_end_begin). Scans are independent, so the split changes no result.
int match_levels_pipelined(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param* levels,
                           int n_levels, double* poses, double* covs, double* sum,
                           const int32_t* scan_grid = nullptr) {
  const int K = std::max(2, std::min(c->pipeline_parts, csm_ctx::kMaxParts));
  // parts in flight share no few-window buffers: every part takes the
  // throughput kernels (a part is hundreds of windows at the default split)
  struct SmallOff {
    csm_ctx* c;
    bool was;
    ~SmallOff() { c->small_path = was; }
  } small_off{c, c->small_path};
  c->small_path = false;
  int32_t first[csm_ctx::kMaxParts], count[csm_ctx::kMaxParts];
  for (int h = 0; h < K; ++h) {
    first[h] = (int32_t)((int64_t)n_scans * h / K);
    count[h] = (int32_t)((int64_t)n_scans * (h + 1) / K) - first[h];
  }
  std::vector<double> resp((size_t)n_scans, 0.0);
  LevelRun R[2][csm_ctx::kMaxParts];  // by level parity: level l's run and level l + 1's
  auto skip = [&](int l) { return c->skip_dead_lists ? live_lists(levels, n_levels, l) : 0; };
  int st;
  for (int h = 0; h < K; ++h) {
    const int32_t s0 = first[h];
    R[0][h].tag = h;
    if (h > 0) c->swap_slot(h);
    if (h == 0)  // the device waits for this one
      st = level_begin_split(c, count[h], offsets + s0, levels[0], poses + 3 * (size_t)s0, resp.data() + s0, R[0][h],
                             scan_grid ? scan_grid + s0 : nullptr, skip(0), c->first_windows);
    else
      st = level_begin(c, count[h], offsets + s0, levels[0], poses + 3 * (size_t)s0, resp.data() + s0, nullptr,
                       R[0][h], scan_grid ? scan_grid + s0 : nullptr, skip(0));
    if (h > 0) c->swap_slot(h);
    if (st != CSM_OK) return st;
  }
  for (int l = 0; l < n_levels; ++l) {
    for (int h = 0; h < K; ++h) {
      const int32_t s0 = first[h];
      LevelRun& cur = R[l & 1][h];
      if (l + 1 < n_levels) {
        R[(l + 1) & 1][h].tag = (l + 1) * 8 + h;
        if (h > 0) c->swap_slot(h);
        st = level_end_begin(c, cur, R[(l + 1) & 1][h], count[h], offsets + s0, levels[l + 1],
                             poses + 3 * (size_t)s0, covs + 9 * (size_t)s0, resp.data() + s0, sum + s0,
                             scan_grid ? scan_grid + s0 : nullptr, skip(l + 1));
        if (h > 0) c->swap_slot(h);
      } else {
        st = level_end(c, cur, poses + 3 * (size_t)s0, covs + 9 * (size_t)s0, resp.data() + s0, nullptr);
        for (int s = s0; s < s0 + count[h]; ++s) sum[(size_t)s] += resp[(size_t)s];
      }
      if (st != CSM_OK) return st;
    }
  }
  return CSM_OK;
}

// FAST windows: tree scores on the device, the search and covariance on the
// host (BranchAndBoundCorrelateScanMatcher::ScanMatch :274-331, then
// BasedCorrelationScanMatch :815-869). Windows go in chunks bounded by the
// score table size.
int match_level_fast(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                     double* poses, double* covs, double* responses, int64_t* argmax_flat) {
  Dims D;  // the angle LUT is the multi-resolution matcher's (:297-300)
  if (window_dims(P, D) != CSM_OK) return c->fail(CSM_ERR_INVALID_ARG, "invalid search window parameters");
  const int depth = P.max_depth;
  if (depth < 0 || depth > csm::kTreeMaxDepth)
    return c->fail(CSM_ERR_UNSUPPORTED, "FAST: max_depth outside [0, 12]");
  const Geometry G(c->info);
  const double sres = P.search_space_resolution;
  const double lowest = (1 << depth) * sres;                                    // :308
  const double nl = round_half_away(P.search_space_size / lowest) + 1;          // :337
  if (!(nl >= 1.0 && nl < 4096.0)) return c->fail(CSM_ERR_INVALID_ARG, "FAST: bad lowest-resolution grid");
  csm::TreeWork T{};
  T.n_angles = D.n_angles;
  T.n_low = (int32_t)nl;
  T.depth = depth;
  T.f_low = lowest / G.mres;  // :347
  for (int d = 1; d <= depth; ++d) T.hw[d] = ((1 << (d - 1)) * sres) / G.mres;  // :454-455
  TreeView V{};
  V.per_angle = 0;
  for (int l = depth; l >= 0; --l) {
    V.m[l] = (int64_t)T.n_low << (depth - l);
    V.off[l] = V.per_angle;
    V.per_angle += V.m[l] * V.m[l];
  }
  T.nodes_per_angle = V.per_angle;
  T.grid = c->d_grid;
  T.size_x = c->info.size_x;
  T.size_y = c->info.size_y;
  T.outside = c->outside;
  const int64_t per_window = (int64_t)D.n_angles * V.per_angle;
  if (per_window > ((int64_t)1 << 31)) return c->fail(CSM_ERR_UNSUPPORTED, "FAST: search tree too large");

  std::vector<int> scan_of;
  for (int s = 0; s < n_scans; ++s) {
    responses[s] = 0.0;  // kMinResponse (:1034)
    if (argmax_flat) argmax_flat[s] = -1;  // no enumeration index for a tree node
    const int n = (int)(offsets[s + 1] - offsets[s]);
    if (!map_ready(c) || n == 0) continue;  // :792-795
    int step, use, n_used;
    if (!beam_rule(n, P.use_point_size, step, use, n_used))
      return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
    scan_of.push_back(s);
  }
  const int nw_all = (int)scan_of.size();
  const int chunk = (int)std::max<int64_t>(1, ((int64_t)256 << 20) / (per_window * 8));
  std::vector<WindowPlan> plans;
  std::vector<AngleEntry> angles;
  for (int w0 = 0; w0 < nw_all; w0 += chunk) {
    const int nw = std::min(chunk, nw_all - w0);
    plans.assign((size_t)nw, WindowPlan{});
    angles.clear();
    std::vector<ScanWork> sw((size_t)nw);
    for (int i = 0; i < nw; ++i) {
      const int s = scan_of[(size_t)(w0 + i)];
      double center[3];
      G.to_map(poses + 3 * s, center);  // :293
      plan_window(P, D, G, (int)(offsets[s + 1] - offsets[s]), center, angles, plans[(size_t)i]);
      const WindowPlan& W = plans[(size_t)i];
      ScanWork& q = sw[(size_t)i];
      q = ScanWork{};
      q.pts_off = offsets[s];
      q.angle_off = W.angle_off;
      q.out_off = (int64_t)i * per_window;
      q.n_used = W.n_used;
      q.step = W.step;
      q.divisor = (double)W.use;
      q.x0 = W.x0;  // search_space_start_x (:345-346)
      q.y0 = W.y0;
      q.cx = W.center[0];
      q.cy = W.center[1];
      q.ct = W.center[2];
    }
    T.n_windows = nw;
    hipError_t e;
    const size_t bytes = (size_t)nw * (size_t)per_window * sizeof(double);
    if ((e = c->scans.ensure(sw.size() * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scans)");
    if ((e = c->angles.ensure(angles.size() * sizeof(AngleEntry))) != hipSuccess) return c->hip_fail(e, "hipMalloc(angles)");
    if ((e = c->scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(tree scores)");
    if ((e = c->h_scores.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(tree scores)");
    if ((e = hipMemcpyAsync(c->scans.p, sw.data(), sw.size() * sizeof(ScanWork), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(scans)");
    if ((e = hipMemcpyAsync(c->angles.p, angles.data(), angles.size() * sizeof(AngleEntry), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(angles)");
    if (c->profiling && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = csm::launch_score_tree(T, (const ScanWork*)c->scans.p, (const double*)c->pts.p,
                                    (const AngleEntry*)c->angles.p, (double*)c->scores.p, c->stream)) != hipSuccess)
      return c->hip_fail(e, "score_tree_kernel");
    if (c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = hipMemcpyAsync(c->h_scores.p, c->scores.p, bytes, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(tree scores)");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize");
    if (c->profiling) {
      float ms = 0.f;
      if ((e = hipEventElapsedTime(&ms, c->ev0, c->ev1)) != hipSuccess) return c->hip_fail(e, "hipEventElapsedTime");
      double beams = 0.0;
      for (const WindowPlan& W : plans) beams += (double)W.n_used;
      c->account("score_tree_kernel", ms, beams * (double)per_window * 4.0, (double)nw * (double)per_window);
    }
    const int threads = (nw >= 8) ? c->host_threads : 1;
    c->parallel_for(nw, threads, [&](int i) {
      const int s = scan_of[(size_t)(w0 + i)];
      const WindowPlan& W = plans[(size_t)i];
      const AngleEntry* ang = angles.data() + W.angle_off;
      TreeView v = V;
      v.s = (const double*)c->h_scores.p + (size_t)i * (size_t)per_window;
      // ComputeLowestResolutionCandidates (:333-393): enumeration order, std::sort
      std::vector<BCand> low;
      low.reserve((size_t)D.n_angles * T.n_low * T.n_low);
      for (int a = 0; a < D.n_angles; ++a)
        for (int xi = 0; xi < T.n_low; ++xi)
          for (int yi = 0; yi < T.n_low; ++yi)
            low.push_back(BCand{v.score(a, depth, xi, yi), W.x0 + xi * T.f_low, W.y0 + yi * T.f_low,
                                ang[a].angle, a, xi, yi});
      std::sort(low.begin(), low.end(), bcand_greater);
      const BCand best = bnb_search(v, low, depth, low.front().score - 0.1, T.hw, ang);  // :316-318
      responses[s] = complete_fast(low, best, P, G, poses + 3 * s, covs + 9 * s);
    });
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

// Selects the context's device for a call and restores the caller's device
// on return (a host process calling in keeps its own current device).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// ---- Gauss-Newton scan matcher ------------------------------------------------
// BasedOptimizeScanMatch (optimize_scan_matcher.h:60-237; SURVEY.md 8f row
// f3). The device evaluates UpdateCost for every active scan per launch
// (csm_optimize.hip); the host keeps the reference's per-iteration control
// flow, glibc cos/sin, the 3x3 LDLT solve and UpdatePose.

constexpr double kOptCostPointSize = 1000;                // optimize_scan_matcher.h:234
constexpr double kOptMaxCost = 1.0 * kOptCostPointSize;   // :235

// util::MaxAbxLimit (util/slam_util.h:79-86)
double max_abs_limit(double value, double limit) {
  if (value > std::fabs(limit))
    value = std::fabs(limit);
  else if (value < -std::fabs(limit))
    value = -std::fabs(limit);
  return value;
}

// util::NormalizeAngle (util/slam_util.h:103-111)
double normalize_angle(double a) {
  double n = std::fmod(std::fmod(a, 2.0 * M_PI) + 2.0 * M_PI, 2.0 * M_PI);
  if (n > M_PI) n -= 2.0 * M_PI;
  return n;
}

// H_.ldlt().solve(b_) (optimize_scan_matcher.h:136-142): Eigen 3.3
// LDLT<Matrix3d, Lower>. Factor: diagonal pivoting on the trailing corner
// (first maximum wins), symmetric swaps through the lower triangle, then
// a_kk -= a_k. . (D a_k.)^T and the column below scaled by the pivot.
// Solve: P, unit-lower rows, D pseudo-inverse (|d| > DBL_MIN), unit-upper
// rows from the bottom, P^T. s = lower triangle of the symmetric H as
// {H00, H10, H11, H20, H21, H22}.
void ldlt_solve3(const double s[6], const double rhs[3], double out[3]) {
  double a[3][3] = {{s[0], s[1], s[3]}, {s[1], s[2], s[4]}, {s[3], s[4], s[5]}};
  int tr[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) {
    int big = k;
    double bv = std::fabs(a[k][k]);
    for (int i = k + 1; i < 3; ++i)
      if (std::fabs(a[i][i]) > bv) {
        bv = std::fabs(a[i][i]);
        big = i;
      }
    tr[k] = big;
    if (big != k) {
      for (int j = 0; j < k; ++j) std::swap(a[k][j], a[big][j]);
      for (int i = big + 1; i < 3; ++i) std::swap(a[i][k], a[i][big]);
      std::swap(a[k][k], a[big][big]);
      for (int i = k + 1; i < big; ++i) {
        const double t = a[i][k];
        a[i][k] = a[big][i];
        a[big][i] = t;
      }
    }
    if (k > 0) {
      double t[2];
      for (int i = 0; i < k; ++i) t[i] = a[i][i] * a[k][i];
      a[k][k] -= (k == 1) ? (a[k][0] * t[0]) : (a[k][0] * t[0] + a[k][1] * t[1]);
      if (k == 1) a[2][1] -= a[2][0] * t[0];
    }
    const double akk = a[k][k];
    const bool valid = std::fabs(akk) > 0.0;
    if (k == 0 && !valid) {
      tr[0] = 0;
      tr[1] = 1;
      tr[2] = 2;
      break;
    }
    if (k < 2 && valid)
      for (int r = k + 1; r < 3; ++r) a[r][k] /= akk;
  }
  double d[3] = {rhs[0], rhs[1], rhs[2]};
  for (int k = 0; k < 3; ++k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  d[1] -= a[1][0] * d[0];
  d[2] -= (a[2][0] * d[0] + a[2][1] * d[1]);
  for (int i = 0; i < 3; ++i) d[i] = (std::fabs(a[i][i]) > DBL_MIN) ? d[i] / a[i][i] : 0.0;
  d[1] -= a[2][1] * d[2];
  d[0] -= (a[1][0] * d[1] + a[2][0] * d[2]);
  for (int k = 2; k >= 0; --k)
    if (tr[k] != k) std::swap(d[k], d[tr[k]]);
  out[0] = d[0];
  out[1] = d[1];
  out[2] = d[2];
}

// n_scans scans whose points are resident in c->pts at offsets off (n+1,
// relative). poses world in/out, costs out; iters (nullable) = UpdateCost
// evaluations per scan.
int optimize_batch(csm_ctx* c, int32_t n_scans, const int64_t* off, const csm_optimize_param& P, double* poses,
                   double* costs, int32_t* iters) {
  const Geometry geo(c->info);
  const bool ready = map_ready(c);
  // per scan: kSkip = invalid input (pose untouched, kMaxCost), kRun =
  // iterating, kDone = converged or out of iterations, kNan = NaN step
  enum : uint8_t { kSkip = 0, kRun = 1, kDone = 2, kNan = 3 };
  std::vector<double> est((size_t)n_scans * 3), cost((size_t)n_scans, 0.0), last((size_t)n_scans, 0.0);
  std::vector<uint8_t> state((size_t)n_scans, kSkip);
  int n_active = 0;
  for (int32_t s = 0; s < n_scans; ++s) {
    if (iters) iters[s] = 0;
    if (!ready || off[s + 1] == off[s]) continue;  // :73-76
    geo.to_map(poses + 3 * s, &est[(size_t)3 * s]);  // GetMapCoordsPose (:79-80)
    // cost_ starts at 0.0 here; the reference returns its stale member when
    // iterate_max_times <= 0 (no iteration) — defined as 0.0
    state[(size_t)s] = (P.iterate_max_times > 0) ? kRun : kDone;
    n_active += state[(size_t)s] == kRun;
  }
  std::vector<uint8_t> active(state);
  for (auto& a : active) a = (a == kRun);
  hipError_t e;
  if ((e = c->opt_off.ensure(sizeof(int64_t) * (size_t)(n_scans + 1))) != hipSuccess ||
      (e = c->opt_scans.ensure(sizeof(csm::OptScan) * (size_t)n_scans)) != hipSuccess ||
      (e = c->opt_sums.ensure(sizeof(csm::OptSums) * (size_t)n_scans)) != hipSuccess ||
      (e = c->h_opt_scans.ensure(sizeof(csm::OptScan) * (size_t)n_scans)) != hipSuccess ||
      (e = c->h_opt_sums.ensure(sizeof(csm::OptSums) * (size_t)n_scans)) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(optimize)");
  if ((e = hipMemcpyAsync(c->opt_off.p, off, sizeof(int64_t) * (size_t)(n_scans + 1), hipMemcpyHostToDevice,
                          c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(optimize offsets)");
  csm::OptArgs A{};
  A.grid = c->d_grid;
  A.size_x = c->info.size_x;
  A.size_y = c->info.size_y;
  A.outside = c->outside;
  A.pts = (const double*)c->pts.p;
  A.offsets = (const int64_t*)c->opt_off.p;
  A.scans = (const csm::OptScan*)c->opt_scans.p;
  A.out = (csm::OptSums*)c->opt_sums.p;
  auto* hs = (csm::OptScan*)c->h_opt_scans.p;
  auto* hr = (const csm::OptSums*)c->h_opt_sums.p;
  const double mres = geo.mres;  // map_resolution_ = GetCellLength() (:82)
  for (int iter = 0; iter < P.iterate_max_times && n_active > 0; ++iter) {
    for (int32_t s = 0; s < n_scans; ++s) {
      csm::OptScan& o = hs[s];
      o.active = active[(size_t)s];
      if (!o.active) continue;
      const double* m = &est[(size_t)3 * s];
      csm::host_sincos(m[2], &o.s, &o.c);  // rotation (:96-97), de_s (:200-201)
      o.tx = m[0];
      o.ty = m[1];
    }
    if ((e = hipMemcpyAsync(c->opt_scans.p, hs, sizeof(csm::OptScan) * (size_t)n_scans, hipMemcpyHostToDevice,
                            c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(optimize state)");
    if (c->profiling && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = csm::launch_optimize_cost(A, n_scans, c->stream)) != hipSuccess)
      return c->hip_fail(e, "optimize_cost_kernel");
    if (c->profiling && (e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = hipMemcpyAsync(c->h_opt_sums.p, c->opt_sums.p, sizeof(csm::OptSums) * (size_t)n_scans,
                            hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(optimize sums)");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(optimize)");
    if (c->profiling) {
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
      double in_map = 0.0;
      for (int32_t s = 0; s < n_scans; ++s)
        if (active[(size_t)s]) in_map += hr[s].valid;
      c->account("optimize_cost_kernel", ms, 16.0 * in_map, 0.0);  // 4 fp32 corners per point in the map
    }
    for (int32_t s = 0; s < n_scans; ++s) {
      if (!active[(size_t)s]) continue;
      const csm::OptSums& r = hr[s];
      last[(size_t)s] = cost[(size_t)s];  // :88
      const int valid_point = 1 + r.valid;
      cost[(size_t)s] = r.v[0] * (kOptCostPointSize / valid_point);  // :220
      if (iters) iters[s] = iter + 1;
      double det[3];
      ldlt_solve3(&r.v[1], &r.v[7], det);  // CalculateDet (:101, :136-142)
      double* m = &est[(size_t)3 * s];
      const bool nan = std::isnan(det[0]) || std::isnan(det[1]) || std::isnan(det[2]);  // :103-106
      if (nan || (iter > 0 && (last[(size_t)s] - cost[(size_t)s] < P.cost_decrease_threshold ||
                               cost[(size_t)s] < P.cost_min_threshold))) {  // :112-118
        state[(size_t)s] = nan ? kNan : kDone;
        active[(size_t)s] = 0;
        --n_active;
        continue;
      }
      m[0] += max_abs_limit(det[0], P.max_update_distance / mres);  // UpdatePose (:144-152)
      m[1] += max_abs_limit(det[1], P.max_update_distance / mres);
      m[2] += max_abs_limit(det[2], P.max_update_angle);
    }
  }
  for (int32_t s = 0; s < n_scans; ++s) {
    if (state[(size_t)s] == kSkip || state[(size_t)s] == kNan) {
      costs[s] = kOptMaxCost;  // pose untouched
      continue;
    }
    double* m = &est[(size_t)3 * s];
    m[2] = normalize_angle(m[2]);    // :126
    geo.to_world(m, poses + 3 * s);  // GetWorldCoordsPose (:128)
    costs[s] = cost[(size_t)s];
  }
  return CSM_OK;
}

}  // namespace

extern "C" {

int csm_abi_version(void) { return CSM_ABI_VERSION; }

int csm_create(int device, csm_ctx** out) {
  if (!out) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return CSM_ERR_HIP;
  DeviceGuard dg(device);  // the caller's device is restored on return
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != device) return CSM_ERR_HIP;
  csm_ctx* c = new (std::nothrow) csm_ctx();
  if (!c) return CSM_ERR_ALLOC;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return CSM_ERR_HIP;
  }
  if (hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    if (c->h2d) (void)hipStreamDestroy(c->h2d);
    delete c;
    return CSM_ERR_HIP;
  }
  unsigned hw = std::thread::hardware_concurrency();
  int threads = (int)std::min<unsigned>(hw ? hw : 1, 16);
  if (const char* env = std::getenv("CSM_HOST_THREADS")) {
    const int v = std::atoi(env);
    if (v > 0) threads = v;
  }
  c->host_threads = threads;
  if (const char* env = std::getenv("CSM_POOL_SPIN_US")) c->pool_spin_us = std::atoi(env);
  if (const char* env = std::getenv("CSM_FIRST_WINDOWS")) c->first_windows = std::max(0, std::atoi(env));
  if (const char* env = std::getenv("CSM_HOST_SIGNAL")) c->host_signal = std::atoi(env) != 0;
  if (const char* env = std::getenv("CSM_FINISH")) {
    c->device_finish = std::strcmp(env, "host") != 0;
    c->fast_finish = std::strcmp(env, "exact") != 0;
    if (std::strcmp(env, "device") == 0) c->device_finish_min = 1;
  }
  if (const char* env = std::getenv("CSM_FINISH_MIN_WINDOWS")) c->device_finish_min = std::max(1, std::atoi(env));
  if (const char* env = std::getenv("CSM_KERNEL")) {
    c->column_kernel = std::strcmp(env, "v1") != 0;
    c->row_kernel = std::strcmp(env, "v1") != 0 && std::strcmp(env, "v2") != 0;
    c->row_dma = std::strcmp(env, "v3") != 0;
    c->box_kernel = std::strcmp(env, "v6") == 0 || std::strcmp(env, "v7") == 0;
    c->box_kernel = c->box_kernel || std::strcmp(env, "v8") == 0;
    c->phase_kernel = std::strcmp(env, "v7") == 0 || std::strcmp(env, "v8") == 0;
    c->tiny_kernel = std::strcmp(env, "v8") == 0;
  }
  if (const char* env = std::getenv("CSM_PHASE_MARGIN_LOG2"))
    c->phase_margin_log2 = std::max(2, std::min(std::atoi(env), 20));
  if (const char* env = std::getenv("CSM_PIPELINE")) {  // 0: never split the 3-level batch
    const int v = std::atoi(env);
    c->pipeline_min = v > 0 ? v : INT32_MAX;
  }
  if (const char* env = std::getenv("CSM_SKIP_DEAD_LISTS")) c->skip_dead_lists = std::atoi(env) != 0;
  if (const char* env = std::getenv("CSM_SMALL")) c->small_path = std::atoi(env) != 0;
  // CSM_STATS_DUMP=1: profiling on from the start, the per-kernel stats printed
  // to stderr by csm_destroy (C++ callers without a stats hook, tests/cpp)
  if (const char* env = std::getenv("CSM_STATS_DUMP")) c->stats_dump = std::atoi(env) != 0;
  if (const char* env = std::getenv("CSM_SMALL_WINDOWS")) c->small_max_windows = std::max(1, std::atoi(env));
  if (const char* env = std::getenv("CSM_SPLIT_TARGET")) c->split_target_blocks = std::max(1, std::atoi(env));
  if (const char* env = std::getenv("CSM_FAST_WIDE")) c->fast_wide_windows = std::atoi(env);
  if (const char* env = std::getenv("CSM_PIPELINE_PARTS"))
    c->pipeline_parts = std::max(2, std::min(std::atoi(env), csm_ctx::kMaxParts));
  bool ev_ok = true;
  for (hipEvent_t* ev : {&c->ev_done, &c->ev_in, &c->ev_k, &c->ev_fast, &c->ev_pts, &c->ev_pack})
    ev_ok = ev_ok && hipEventCreateWithFlags(ev, hipEventDisableTiming) == hipSuccess;
  for (auto& a : c->alt)
    for (hipEvent_t* ev : {&a.ev_done, &a.ev_in, &a.ev_k, &a.ev_fast})
      ev_ok = ev_ok && hipEventCreateWithFlags(ev, hipEventDisableTiming) == hipSuccess;
  const char* xs = std::getenv("CSM_EXACT_STREAM");
  if (!(xs && std::atoi(xs) == 0))
    ev_ok = ev_ok && hipStreamCreateWithFlags(&c->x_stream, hipStreamNonBlocking) == hipSuccess;
  if (!ev_ok) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return CSM_ERR_HIP;
  }
  *out = c;
  if (c->stats_dump) csm_set_profiling(c, 1);
  return CSM_OK;
}

int csm_destroy(csm_ctx* c) {
  if (!c) return CSM_OK;
  if (c->stats_dump)
    for (const auto& st : c->stats)
      std::fprintf(stderr, "csm stats: %-40s launches %8lld  avg_us %10.3f  total_ms %10.3f  alg_bytes %.6g\n",
                   st.name, (long long)st.launches, st.launches ? st.total_ms / st.launches * 1e3 : 0.0, st.total_ms,
                   st.algorithmic_bytes);
  {
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->h2d);
    (void)hipStreamSynchronize(c->d2h);
    if (c->x_stream) (void)hipStreamSynchronize(c->x_stream);
    csm::gridmap_drop_reader(c->stream);
    c->grid_buf.release();
    c->gridi.release();
    c->h_pack.release();
    c->h_pts.release();
    c->h_search.release();
    c->d_updates.release();
    for (auto& pg : c->parked) {
      pg.grid_buf.release();
      pg.gridi.release();
    }
    c->gstats.release();
    c->split_slab.release();
    c->split_arrive.release();
    c->small_dev.release();
    c->h_small_in.release();
    c->h_small_out.release();
    c->pts.release();
    c->scans.release();
    c->angles.release();
    c->scores.release();
    c->partials.release();
    c->best.release();
    c->fin.release();
    c->h_scores.release();
    c->h_fin.release();
    c->h_angles.release();
    c->h_angles_next.release();
    c->h_fin_sig.release();
    c->fin_sig.release();
    c->h_sw.release();
    c->opt_off.release();
    c->opt_scans.release();
    c->opt_sums.release();
    c->h_opt_scans.release();
    c->h_opt_sums.release();
    for (auto& a : c->alt) {
      a.scans.release();
      a.angles.release();
      a.scores.release();
      a.partials.release();
      a.best.release();
      a.fin.release();
      a.h_scores.release();
      a.h_fin.release();
      a.h_angles.release();
      a.h_angles_next.release();
      a.h_fin_sig.release();
      a.fin_sig.release();
      a.h_sw.release();
      for (hipEvent_t ev : {a.ev0, a.ev1, a.ev2, a.ev_done, a.ev_in, a.ev_k, a.ev_fast, a.ev_ft})
        if (ev) (void)hipEventDestroy(ev);
    }
    for (hipEvent_t ev : {c->ev0, c->ev1, c->ev2, c->ev_ft, c->ev_done, c->ev_in, c->ev_k, c->ev_fast, c->ev_pts,
                          c->ev_pack})
      if (ev) (void)hipEventDestroy(ev);
    if (c->x_stream) (void)hipStreamDestroy(c->x_stream);
    (void)hipStreamDestroy(c->h2d);
    (void)hipStreamDestroy(c->d2h);
    (void)hipStreamDestroy(c->stream);
  }
  delete c;
  return CSM_OK;
}

const char* csm_last_error(const csm_ctx* c) { return c ? c->err.c_str() : "null context"; }

int csm_set_outside_value(csm_ctx* c, float value) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  if (value != c->outside) {  // every fixed-point copy is shifted by it
    c->int_checked = false;
    for (auto& g : c->parked) g.int_checked = false;
  }
  c->outside = value;
  return CSM_OK;
}

int csm_window_dims(const csm_param* p, int32_t* n_angles, int32_t* n_space) {
  if (!p) return CSM_ERR_INVALID_ARG;
  Dims d;
  const int st = window_dims(*p, d);
  if (st != CSM_OK) return st;
  if (n_angles) *n_angles = d.n_angles;
  if (n_space) *n_space = d.n_space;
  return CSM_OK;
}

namespace {

int check_grid_args(csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info) {
  if (info->size_x <= 0 || info->size_y <= 0 || !(info->resolution > 0.0))
    return c->fail(CSM_ERR_INVALID_ARG, "grid size and resolution must be positive");
  if ((int64_t)info->size_x * info->size_y >= ((int64_t)1 << 31))
    return c->fail(CSM_ERR_INVALID_ARG, "grid larger than 2^31 cells");
  if (!cells || stride < 4 || stride % 4 != 0)
    return c->fail(CSM_ERR_INVALID_ARG, "cells must be non-null with a stride that is a multiple of 4 bytes");
  return CSM_OK;
}

// Whole-grid upload into the current slot (selected by the caller): rows are
// packed on the host threads into pinned staging, then one H2D copy.
int upload_grid(csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info, int64_t version) {
  const size_t ncell = (size_t)info->size_x * (size_t)info->size_y;
  hipError_t e;
  if (c->ev_pack_used && (e = hipEventSynchronize(c->ev_pack)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize(pack)");
  if ((e = c->grid_buf.ensure(ncell * sizeof(float))) != hipSuccess) return c->hip_fail(e, "hipMalloc(grid)");
  if ((e = c->h_pack.ensure(ncell * sizeof(float))) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(grid)");
  pack_rows(c, cells, stride, info->size_x, 0, info->size_y, (float*)c->h_pack.p);
  if ((e = hipMemcpyAsync(c->grid_buf.p, c->h_pack.p, ncell * sizeof(float), hipMemcpyHostToDevice, c->stream)) !=
      hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(grid)");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(grid)");
  if (c->profiling) c->account("grid:upload", 0.f, (double)(ncell * sizeof(float)), 0.0);
  c->info = *info;
  c->d_grid = (const float*)c->grid_buf.p;
  c->n_grids = 1;
  c->has_grid = true;
  c->int_checked = false;
  c->key_cells = cells;
  c->key_stride = stride;
  c->key_version = version;
  c->key_sx = info->size_x;
  c->key_sy = info->size_y;
  return CSM_OK;
}

// The current slot holds this map at this geometry (an incremental refresh
// applies); otherwise the caller uploads the whole grid.
bool same_geometry(const csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info) {
  return c->owns_host_grid() && c->n_grids == 1 && c->key_cells == cells && c->key_stride == stride &&
         c->key_sx == info->size_x && c->key_sy == info->size_y && c->info.resolution == info->resolution &&
         c->info.offset_x == info->offset_x && c->info.offset_y == info->offset_y;
}

}  // namespace

int csm_set_grid(csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info,
                 int64_t version) {
  if (!c || !info) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st = check_grid_args(c, cells, stride, info);
  if (st != CSM_OK) return st;
  select_grid(c, cells);
  if (version >= 0 && same_geometry(c, cells, stride, info) && version == c->key_version) {
    c->info = *info;
    return CSM_OK;
  }
  return upload_grid(c, cells, stride, info, version);
}

int csm_update_grid_rows(csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info, int64_t version,
                         int32_t row_begin, int32_t row_end) {
  if (!c || !info) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st = check_grid_args(c, cells, stride, info);
  if (st != CSM_OK) return st;
  if (row_begin < 0 || row_end > info->size_y || row_begin > row_end)
    return c->fail(CSM_ERR_INVALID_ARG, "row range outside the grid");
  select_grid(c, cells);
  if (!same_geometry(c, cells, stride, info)) return upload_grid(c, cells, stride, info, version);
  c->info = *info;
  c->key_version = version;
  if (row_begin == row_end) return CSM_OK;
  const int32_t sx = info->size_x;
  const size_t n = (size_t)(row_end - row_begin) * (size_t)sx;
  hipError_t e;
  if (c->ev_pack_used && (e = hipEventSynchronize(c->ev_pack)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize(pack)");
  if ((e = c->h_pack.ensure(n * sizeof(float))) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(rows)");
  const PackStats ps = pack_rows(c, cells, stride, sx, row_begin, row_end, (float*)c->h_pack.p);
  float* dst = (float*)c->grid_buf.p + (int64_t)row_begin * sx;
  if ((e = hipMemcpyAsync(dst, c->h_pack.p, n * sizeof(float), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(rows)");
  note_new_values(c, ps);
  if (c->int_checked && c->int_ok &&
      (e = csm::launch_fixed_point(dst, sx, row_end - row_begin, c->pitch, c->outside, c->int_exp,
                                   (int32_t*)c->gridi.p + (int64_t)row_begin * c->pitch, c->stream, false)) !=
          hipSuccess)
    return c->hip_fail(e, "fixed_point_kernel(rows)");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(rows)");
  c->grid_gen = ++c->gen_clock;
  if (c->profiling) c->account("grid:rows", 0.f, (double)(n * sizeof(float)), 0.0);
  return CSM_OK;
}

int csm_update_grid_cells(csm_ctx* c, const void* cells, int64_t stride, const csm_map_info* info, int64_t version,
                          const int32_t* cell_indices, int64_t n_indices) {
  if (!c || !info) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st = check_grid_args(c, cells, stride, info);
  if (st != CSM_OK) return st;
  if (n_indices < 0 || (n_indices > 0 && !cell_indices)) return c->fail(CSM_ERR_INVALID_ARG, "cell index list");
  select_grid(c, cells);
  if (!same_geometry(c, cells, stride, info)) return upload_grid(c, cells, stride, info, version);
  const int64_t ncell = (int64_t)info->size_x * info->size_y;
  hipError_t e;
  if (c->ev_pack_used && (e = hipEventSynchronize(c->ev_pack)) != hipSuccess) return c->hip_fail(e, "hipEventSynchronize(pack)");
  if ((e = c->h_pack.ensure((size_t)std::max<int64_t>(n_indices, 1) * sizeof(csm::CellUpdate))) != hipSuccess)
    return c->hip_fail(e, "hipHostMalloc(cell updates)");
  csm::CellUpdate* u = (csm::CellUpdate*)c->h_pack.p;
  const double t_pack0 = now_ms();
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(c->host_threads * 4, n_indices / 4096 + 1));
  std::vector<PackStats> part((size_t)chunks);
  std::atomic<bool> bad{false};
  c->parallel_for(chunks, c->host_threads, [&](int t) {
    const int64_t i0 = n_indices * t / chunks, i1 = n_indices * (t + 1) / chunks;
    PackStats ps;
    constexpr int64_t kAhead = 24;  // random reads of a large host map: keep misses in flight
    for (int64_t i = i0; i < std::min(i1, i0 + kAhead); ++i)
      __builtin_prefetch((const char*)cells + (int64_t)cell_indices[i] * stride);
    for (int64_t i = i0; i < i1; ++i) {
      if (i + kAhead < i1) __builtin_prefetch((const char*)cells + (int64_t)cell_indices[i + kAhead] * stride);
      const int32_t k = cell_indices[i];
      if (k < 0 || k >= ncell) {
        bad = true;
        return;
      }
      float v;
      std::memcpy(&v, (const char*)cells + (int64_t)k * stride, 4);
      u[i].index = k;
      u[i].value = v;
      if (!std::isfinite(v)) ps.nonfinite = true;
      bool z;
      ps.min_g = std::min(ps.min_g, float_granularity(v, &z));
      ps.max_abs = std::max(ps.max_abs, std::fabs(v));
    }
    part[(size_t)t] = ps;
  });
  if (bad) return c->fail(CSM_ERR_INVALID_ARG, "cell index outside the grid");
  if (c->profiling) c->account("host:cells_pack", (float)(now_ms() - t_pack0), 0.0, (double)n_indices);
  c->info = *info;
  c->key_version = version;
  if (n_indices == 0) return CSM_OK;
  PackStats all;
  for (const auto& p : part) {
    all.min_g = std::min(all.min_g, p.min_g);
    all.max_abs = std::max(all.max_abs, p.max_abs);
    all.nonfinite = all.nonfinite || p.nonfinite;
  }
  note_new_values(c, all);
  const size_t bytes = (size_t)n_indices * sizeof(csm::CellUpdate);
  if ((e = c->d_updates.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(cell updates)");
  if ((e = hipMemcpyAsync(c->d_updates.p, u, bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(cell updates)");
  const bool fixed = c->int_checked && c->int_ok;
  if ((e = csm::launch_update_cells((const csm::CellUpdate*)c->d_updates.p, n_indices, (float*)c->grid_buf.p,
                                    info->size_x, fixed ? (int32_t*)c->gridi.p : nullptr, c->pitch, c->outside,
                                    c->int_exp, c->stream)) != hipSuccess)
    return c->hip_fail(e, "update_cells_kernel");
  // no wait here: the matches that read the cells follow on the same stream;
  // the next writer of h_pack waits for this copy (ev_pack)
  if ((e = hipEventRecord(c->ev_pack, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord(pack)");
  c->ev_pack_used = true;
  c->grid_gen = ++c->gen_clock;
  if (c->profiling) c->account("grid:cells", 0.f, (double)bytes, 0.0);
  return CSM_OK;
}

namespace {
int set_grid_device_locked(csm_ctx* c, const float* dev, const csm_map_info* info) {
  if (!dev || info->size_x <= 0 || info->size_y <= 0 || !(info->resolution > 0.0))
    return c->fail(CSM_ERR_INVALID_ARG, "invalid device grid");
  if ((int64_t)info->size_x * info->size_y >= ((int64_t)1 << 31))
    return c->fail(CSM_ERR_INVALID_ARG, "grid larger than 2^31 cells");
  park_current(c);
  c->info = *info;
  c->d_grid = dev;
  c->n_grids = 1;
  c->has_grid = true;
  c->int_checked = false;
  c->key_cells = nullptr;
  c->key_version = -1;
  return CSM_OK;
}
}  // namespace

int csm_set_grid_device(csm_ctx* c, const float* dev, const csm_map_info* info) {
  if (!c || !info) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  release_map_reader(c);
  return set_grid_device_locked(c, dev, info);
}

int csm_set_grid_gridmap(csm_ctx* c, csm_gridmap* map) {
  if (!c || !map) return CSM_ERR_INVALID_ARG;
  float outside;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    outside = c->outside;
  }
  // the map's fixed-point mirror (kept by the map kernels from the cells each
  // update writes): no whole-grid analysis and conversion per borrow
  csm::GridMapFixed fx{};
  int st = csm::gridmap_fixed_point(map, outside, &fx);
  if (st != CSM_OK) return st;
  csm::GridMapView v{};
  if ((st = csm::gridmap_view(map, &v)) != CSM_OK) return st;
  if (v.device != c->device) return c->fail(CSM_ERR_INVALID_ARG, "map lives on another device");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  // the matcher's kernels run after the map's last update, and the map's
  // next update after the matcher's reads (csm::gridmap_add_reader)
  hipError_t e = hipStreamWaitEvent(c->stream, v.ready, 0);
  if (e != hipSuccess) return c->fail(CSM_ERR_HIP, hipGetErrorString(e));
  if (c->reader_map != map) release_map_reader(c);
  csm::gridmap_add_reader(map, c->stream);
  c->reader_map = map;
  csm_map_info info{};
  info.resolution = v.resolution;
  info.offset_x = v.offset_x;
  info.offset_y = v.offset_y;
  info.size_x = v.size_x;
  info.size_y = v.size_y;
  info.update_index = v.map_update_index;
  if ((st = set_grid_device_locked(c, v.prob, &info)) != CSM_OK) return st;
  if (fx.ok && fx.outside == c->outside) {  // ensure_int_grid's state, borrowed
    c->int_checked = true;
    c->int_ok = true;
    c->d_gridi = fx.fpm;
    c->pitch = fx.pitch;
    c->int_exp = fx.exp;
    c->int_max_abs = fx.max_abs;
    c->outside_i = (int32_t)((double)c->outside * std::ldexp(1.0, fx.exp));
    c->grid_gen = ++c->gen_clock;
    if (c->profiling) c->account("grid:mirror", 0.f, 0.0, 0.0);
  }
  return CSM_OK;
}

int csm_scan_match_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                         const csm_param* param, double* poses, double* covs, double* responses,
                         int64_t* argmax_flat) {
  if (!c || !param || !poses || !covs || !responses) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
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
  int st;
  c->loaded_n = -1;
  c->loaded_grid.clear();
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

int csm_scan_matchers_loaded(csm_ctx* c, const csm_param levels[3], int32_t use_fine, double* poses,
                             double* covs, double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (c->loaded_n < 0) return c->fail(CSM_ERR_INVALID_ARG, "no scans loaded (csm_load_scans)");
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  const int32_t n_scans = c->loaded_n;
  if (n_scans == 0) return CSM_OK;
  const double t_call = now_ms();
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
  if (c->profiling) c->account("host:call", (float)(now_ms() - t_call), 0.0, 0.0);
  return CSM_OK;
}

int csm_scan_matchers_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                            const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                            double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  const int st = csm_load_scans(c, n_scans, pts, offsets);
  if (st != CSM_OK) return st;
  return csm_scan_matchers_loaded(c, levels, use_fine, poses, covs, scores);
}

int csm_set_profiling(csm_ctx* c, int32_t on) {
  if (!c) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  hipError_t e;
  if (on && !c->ev0) {
    for (hipEvent_t* ev : {&c->ev0, &c->ev1, &c->ev2, &c->ev_ft})
      if ((e = hipEventCreate(ev)) != hipSuccess) return c->hip_fail(e, "hipEventCreate");
    for (auto& a : c->alt)
      for (hipEvent_t* ev : {&a.ev0, &a.ev1, &a.ev2, &a.ev_ft})
        if ((e = hipEventCreate(ev)) != hipSuccess) return c->hip_fail(e, "hipEventCreate");
  }
  (void)flush_deferred(c);  // timings of the earlier setting, dropped with the stats below
  c->profiling = on != 0;
  c->stats.clear();
  return CSM_OK;
}

int csm_kernel_stats(csm_ctx* c, csm_kernel_stat* out, int32_t capacity, int32_t* count) {
  if (!c || !count) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->deferred.empty()) {
    DeviceGuard g(c->device);
    const int st = flush_deferred(c);
    if (st != CSM_OK) return st;
  }
  *count = (int32_t)c->stats.size();
  for (int32_t i = 0; i < *count && i < capacity && out; ++i) out[i] = c->stats[(size_t)i];
  return CSM_OK;
}

int csm_scan_matchers(csm_ctx* c, const double* pts, int32_t n_points, const csm_param levels[3],
                      int32_t use_fine, double pose[3], double cov[9], double* score) {
  if (!c || !score) return CSM_ERR_INVALID_ARG;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  const int64_t off[2] = {0, n_points};
  return csm_scan_matchers_batch(c, 1, pts, off, levels, use_fine, pose, cov, score);
}

int csm_score_window(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                     const double center_map[3], double* scores_out, int64_t n_out) {
  if (!c || !param || !center_map || !scores_out) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  Dims D;
  int st = window_dims(*param, D);
  if (st != CSM_OK) return c->fail(st, "invalid search window parameters");
  if (n_out != D.n_cand) return c->fail(CSM_ERR_INVALID_ARG, "n_out must equal n_angles * n_space^2");
  if (n_points <= 0) return c->fail(CSM_ERR_INVALID_ARG, "no points");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  const Geometry G(c->info);
  std::vector<WindowPlan> plans(1);
  std::vector<AngleEntry> angles;
  if (!plan_window(*param, D, G, n_points, center_map, angles, plans[0]))
    return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
  if ((st = upload_points(c, pts, n_points)) != CSM_OK) return st;
  if ((st = run_windows(c, *param, D, G, plans, {0}, angles.data(), angles.size(), {}, nullptr)) != CSM_OK)
    return st;
  std::memcpy(scores_out, c->h_scores.p, (size_t)n_out * sizeof(double));
  return CSM_OK;
}

int csm_best_window(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                    const double center_map[3], csm_best* best) {
  if (!c || !param || !center_map || !best) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  Dims D;
  int st = window_dims(*param, D);
  if (st != CSM_OK) return c->fail(st, "invalid search window parameters");
  if (n_points <= 0) return c->fail(CSM_ERR_INVALID_ARG, "no points");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  const Geometry G(c->info);
  std::vector<WindowPlan> plans(1);
  std::vector<AngleEntry> angles;
  if (!plan_window(*param, D, G, n_points, center_map, angles, plans[0]))
    return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
  if ((st = upload_points(c, pts, n_points)) != CSM_OK) return st;
  BestPartial bp{};
  if ((st = run_windows(c, *param, D, G, plans, {0}, angles.data(), angles.size(), {}, &bp)) != CSM_OK)
    return st;
  const WindowPlan& W = plans[0];
  const int64_t ns = D.n_space, nss = ns * ns;
  best->score = bp.score;
  best->flat_index = bp.flat;
  best->x = W.x0 + (int)((bp.flat / ns) % ns) * (param->search_space_resolution / G.mres);
  best->y = W.y0 + (int)(bp.flat % ns) * (param->search_space_resolution / G.mres);
  best->angle = angles[(size_t)(bp.flat / nss)].angle;
  return CSM_OK;
}

int csm_best_windows(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                     int32_t n_windows, const int32_t* grid_index, const double* centers_map,
                     csm_best* best) {
  if (!c || !param || !centers_map || !best || n_windows < 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (n_windows == 0) return CSM_OK;
  Dims D;
  int st = window_dims(*param, D);
  if (st != CSM_OK) return c->fail(st, "invalid search window parameters");
  if (n_points <= 0) return c->fail(CSM_ERR_INVALID_ARG, "no points");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  std::vector<int32_t> gidx((size_t)n_windows, 0);
  for (int i = 0; i < n_windows; ++i) {
    gidx[(size_t)i] = grid_index ? grid_index[i] : 0;
    if (gidx[(size_t)i] < 0 || gidx[(size_t)i] >= c->n_grids)
      return c->fail(CSM_ERR_INVALID_ARG, "grid_index outside the resident grid stack");
  }
  const Geometry G(c->info);
  std::vector<WindowPlan> plans((size_t)n_windows);
  std::vector<AngleEntry> angles;
  if (!plan_windows_shared(*param, D, G, n_points, n_windows, centers_map, angles, plans))
    return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
  if ((st = upload_points(c, pts, n_points)) != CSM_OK) return st;
  std::vector<BestPartial> bp((size_t)n_windows);
  std::vector<int64_t> pt_off((size_t)n_windows, 0);
  if ((st = run_windows(c, *param, D, G, plans, pt_off, angles.data(), angles.size(), gidx, bp.data())) != CSM_OK)
    return st;
  const int64_t ns = D.n_space, nss = ns * ns;
  const double f = param->search_space_resolution / G.mres;
  for (int i = 0; i < n_windows; ++i) {
    const WindowPlan& W = plans[(size_t)i];
    best[i].score = bp[(size_t)i].score;
    best[i].flat_index = bp[(size_t)i].flat;
    best[i].x = W.x0 + (int)((bp[(size_t)i].flat / ns) % ns) * f;
    best[i].y = W.y0 + (int)(bp[(size_t)i].flat % ns) * f;
    best[i].angle = angles[(size_t)(W.angle_off + bp[(size_t)i].flat / nss)].angle;
  }
  return CSM_OK;
}

namespace {

// csm_search_windows' fallback: the exhaustive per-window argmax, reduced to
// the lowest (window, flat) among the best scores.
int search_exhaustive(csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G,
                      const std::vector<WindowPlan>& plans, const std::vector<AngleEntry>& angles,
                      const std::vector<int32_t>& gidx, BestPartial* out) {
  std::vector<BestPartial> bp(plans.size());
  std::vector<int64_t> pt_off(plans.size(), 0);
  int st = run_windows(c, P, D, G, plans, pt_off, angles.data(), angles.size(), gidx, bp.data());
  if (st != CSM_OK) return st;
  BestPartial b{-DBL_MAX, INT64_MAX};
  for (size_t i = 0; i < bp.size(); ++i) {
    const int64_t gf = (int64_t)i * D.n_cand + bp[i].flat;
    if (bp[i].score > b.score || (bp[i].score == b.score && gf < b.flat)) b = BestPartial{bp[i].score, gf};
  }
  *out = b;
  return CSM_OK;
}

}  // namespace

static int search_windows_locked(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                                 int32_t n_windows, const int32_t* grid_index, const double* centers_map,
                                 const csm_search_options* options, csm_best* best, int32_t* best_window,
                                 csm_search_stats* stats);

// The search stages its points, angle table and incumbent in pinned buffers
// that the next call rewrites; a call that fails after enqueuing a copy out of
// them leaves the stream marked, and the next call drains it first.
int csm_search_windows(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param, int32_t n_windows,
                       const int32_t* grid_index, const double* centers_map, const csm_search_options* options,
                       csm_best* best, int32_t* best_window, csm_search_stats* stats) {
  if (!c || !param || !centers_map || !best || !best_window || n_windows <= 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (c->staging_dirty) {
    (void)hipStreamSynchronize(c->stream);
    c->staging_dirty = false;
  }
  const int st = search_windows_locked(c, pts, n_points, param, n_windows, grid_index, centers_map, options, best,
                                       best_window, stats);
  c->staging_dirty = st != CSM_OK;
  return st;
}

static int search_windows_locked(csm_ctx* c, const double* pts, int32_t n_points, const csm_param* param,
                                 int32_t n_windows, const int32_t* grid_index, const double* centers_map,
                                 const csm_search_options* options, csm_best* best, int32_t* best_window,
                                 csm_search_stats* stats) {
  Dims D;
  int st = window_dims(*param, D);
  if (st != CSM_OK) return c->fail(st, "invalid search window parameters");
  if (n_points <= 0) return c->fail(CSM_ERR_INVALID_ARG, "no points");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  std::vector<int32_t> gidx((size_t)n_windows, 0);
  for (int i = 0; i < n_windows; ++i) {
    gidx[(size_t)i] = grid_index ? grid_index[i] : 0;
    if (gidx[(size_t)i] < 0 || gidx[(size_t)i] >= c->n_grids)
      return c->fail(CSM_ERR_INVALID_ARG, "grid_index outside the resident grid stack");
  }
  const Geometry G(c->info);
  std::vector<WindowPlan> plans((size_t)n_windows);
  std::vector<AngleEntry> angles;
  if (!plan_windows_shared(*param, D, G, n_points, n_windows, centers_map, angles, plans))
    return c->fail(CSM_ERR_INVALID_ARG, "use_point_size <= 1 with n_points >= 2*use_point_size");
  // the points, then the angle table, staged in pinned memory (the last call
  // on this context has synchronised, so the staging buffer is free)
  const size_t pts_bytes = ((size_t)n_points * 2 * sizeof(double) + 255) & ~(size_t)255;
  hipError_t e0;
  if ((e0 = c->h_search.ensure(pts_bytes + angles.size() * sizeof(AngleEntry))) != hipSuccess)
    return c->hip_fail(e0, "hipHostMalloc(search staging)");
  AngleEntry* h_ang = (AngleEntry*)((char*)c->h_search.p + pts_bytes);
  std::memcpy(h_ang, angles.data(), angles.size() * sizeof(AngleEntry));
  if ((st = upload_points(c, pts, n_points, c->h_search.p)) != CSM_OK) return st;
  if ((st = ensure_int_grid(c)) != CSM_OK) return st;
  csm_search_stats S{};
  S.candidates = (int64_t)n_windows * D.n_cand;
  const double f = param->search_space_resolution / G.mres;
  const WindowPlan& W0 = plans[0];
  // the pooled search: one-cell steps, the exact fixed-point grid, the beams
  // staged in LDS (64 KB), every index int-castable, node fields in range
  bool ok = f == 1.0 && c->int_ok && W0.n_used <= 4096 && n_windows < (1 << 20) && D.n_angles < 4096 &&
            D.n_space < 65536 &&
            (double)W0.n_used * c->int_max_abs * std::ldexp(1.0, c->int_exp) <= std::ldexp(1.0, 53);
  int depth = options ? options->max_depth : -1;
  if (depth < 0) {  // the shallowest top level with at most 32 x 32 nodes per angle (measured
                    // best on configs 3 and 4: profiles/r02/search_depth_sweep.txt)
    depth = 0;
    while (((D.n_space + (1 << depth) - 1) >> depth) > 32 && depth < csm::kPyrMaxDepth) ++depth;
  }
  depth = std::min(depth, csm::kPyrMaxDepth);
  bool box_ok = true;
  for (const WindowPlan& W : plans) {
    if (!ok) break;
    const double far = (double)(D.n_space - 1) * f;
    const double span = std::max(std::max(std::fabs(W.x0), std::fabs(W.x0 + far)),
                                 std::max(std::fabs(W.y0), std::fabs(W.y0 + far)));
    const double R = c->pts_maxabs * (1.0 + 1e-9) + span + 2.0 + (double)(1 << depth);
    if (!(R < std::ldexp(1.0, 29))) ok = false;
    // the top kernel's box test: every |t| < 2^24 cells (csm_pyramid.hip)
    if (!(R < std::ldexp(1.0, 23))) box_ok = false;
  }
  BestPartial b{};
  if (!ok) {
    S.exhaustive = 1;
    if ((st = search_exhaustive(c, *param, D, G, plans, angles, gidx, &b)) != CSM_OK) return st;
    S.nodes[0] = S.candidates;
    S.beam_reads = S.candidates * W0.n_used;
  } else {
    hipError_t e;
    const int nw = n_windows;
    if ((e = c->h_sw.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipHostMalloc(scans)");
    ScanWork* sw = (ScanWork*)c->h_sw.p;
    for (int i = 0; i < nw; ++i) {
      const WindowPlan& W = plans[(size_t)i];
      ScanWork& s = sw[i];
      s = ScanWork{};
      s.angle_off = W.angle_off;
      s.out_off = (int64_t)i * D.n_cand;
      s.n_used = W.n_used;
      s.step = W.step;
      s.divisor = (double)W.use;
      s.x0 = W.x0;
      s.y0 = W.y0;
      s.cx = W.center[0];
      s.cy = W.center[1];
      s.ct = W.center[2];
      s.grid_index = gidx[(size_t)i];
    }
    if ((e = c->scans.ensure((size_t)nw * sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scans)");
    if ((e = c->angles.ensure(angles.size() * sizeof(AngleEntry))) != hipSuccess) return c->hip_fail(e, "hipMalloc(angles)");
    if ((e = hipMemcpyAsync(c->scans.p, sw, (size_t)nw * sizeof(ScanWork), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(scans)");
    if ((e = hipMemcpyAsync(c->angles.p, h_ang, angles.size() * sizeof(AngleEntry), hipMemcpyHostToDevice,
                            c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(angles)");
    csm::PyrInputs in{};
    in.stream = c->stream;
    LevelWork& L = in.L;
    L.n_angles = D.n_angles;
    L.n_space = D.n_space;
    L.n_cand = D.n_cand;
    L.n_scans = nw;
    L.step_cells = f;
    L.use_penalty = param->use_center_penalty ? 1 : 0;
    L.dist_gain = (param->type == CSM_COARSE) ? 0.4 : 0.2;  // :759-761
    L.size = param->search_space_size;
    L.mres = G.mres;
    L.outside_i = c->outside_i;
    L.int_mode = 1;
    L.int_scale = std::ldexp(1.0, -c->int_exp);
    in.level0 = csm::PyrGrid{c->d_gridi,
                             (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows), c->pitch, 0,
                             c->info.size_x, c->info.size_y, 0, c->info.size_x, 0, 0};
    in.n_grids = c->n_grids;
    in.grid_gen = c->grid_gen;
    in.scans = (const ScanWork*)c->scans.p;
    in.angles = (const AngleEntry*)c->angles.p;
    in.pts = (const double*)c->pts.p;
    in.n_used = W0.n_used;
    in.step = W0.step;
    in.depth = depth;
    in.top_mode = options ? options->top_kernel : 0;
    in.box_ok = box_ok ? 1 : 0;
    in.timed = c->profiling ? 1 : 0;
    in.one_scan = 1;  // the windows share the one scan: check what the implicit top level relies on
    for (const WindowPlan& W : plans)
      if (W.use != W0.use || W.n_used != W0.n_used || W.step != W0.step) in.one_scan = 0;
    c->pyramid.configure(options ? options->node_capacity : 0, options ? options->probe_min_nodes : 0);
    csm::PyrStats ps;
    std::string what;
    float ms = 0.f;
    if (c->profiling && (e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return c->hip_fail(e, "hipEventRecord");
    if ((e = c->pyramid.run(in, &b, &ps, &what)) != hipSuccess) return c->hip_fail(e, what.c_str());
    if (c->profiling) {
      if ((e = hipEventRecord(c->ev1, c->stream)) != hipSuccess || (e = hipEventSynchronize(c->ev1)) != hipSuccess ||
          (e = hipEventElapsedTime(&ms, c->ev0, c->ev1)) != hipSuccess)
        return c->hip_fail(e, "pyramid timing");
    }
    S.depth = ps.depth;
    int64_t scored = ps.probe_leaves;
    for (int d = 0; d <= csm::kPyrMaxDepth; ++d) {
      S.nodes[d] = ps.nodes[d];
      scored += ps.nodes[d];
    }
    S.probe_leaves = ps.probe_leaves;
    S.beam_reads = scored * W0.n_used;
    S.build_ms = ps.build_ms;
    S.syncs = ps.syncs;
    S.top_box = ps.top_box;
    // one grid read per beam per scored node (the pooled levels included)
    if (c->profiling) {
      c->account("pyramid_search", ms, (double)S.beam_reads * 4.0, (double)S.candidates);
      if (ps.top_name[0]) c->account(ps.top_name, (float)ps.top_ms, ps.top_bytes, 0.0);
    }
  }
  if (b.flat == INT64_MAX) return c->fail(CSM_ERR_HIP, "search found no candidate");
  const int32_t w = (int32_t)(b.flat / D.n_cand);
  const int64_t flat = b.flat - (int64_t)w * D.n_cand;
  const int64_t ns = D.n_space, nss = ns * ns;
  const WindowPlan& W = plans[(size_t)w];
  best->score = b.score;
  best->flat_index = flat;
  best->x = W.x0 + (int)((flat / ns) % ns) * f;
  best->y = W.y0 + (int)(flat % ns) * f;
  best->angle = angles[(size_t)(W.angle_off + flat / nss)].angle;
  *best_window = w;
  if (stats) *stats = S;
  return CSM_OK;
}

int csm_set_grid_stack(csm_ctx* c, const float* cells, int32_t n_grids, const csm_map_info* info,
                       int64_t version) {
  if (!c || !info || !cells || n_grids <= 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  release_map_reader(c);
  if (info->size_x <= 0 || info->size_y <= 0 || !(info->resolution > 0.0))
    return c->fail(CSM_ERR_INVALID_ARG, "grid size and resolution must be positive");
  const int64_t ncell = (int64_t)info->size_x * info->size_y;
  if (ncell >= ((int64_t)1 << 31)) return c->fail(CSM_ERR_INVALID_ARG, "grid larger than 2^31 cells");
  select_grid(c, cells);
  const bool same = c->owns_host_grid() && version >= 0 && (const void*)cells == c->key_cells &&
                    c->key_stride == -n_grids && version == c->key_version && info->size_x == c->key_sx &&
                    info->size_y == c->key_sy;
  c->info = *info;
  if (same) return CSM_OK;
  const size_t bytes = (size_t)ncell * (size_t)n_grids * sizeof(float);
  hipError_t e;
  if ((e = c->grid_buf.ensure(bytes)) != hipSuccess) return c->hip_fail(e, "hipMalloc(grid stack)");
  if ((e = hipMemcpyAsync(c->grid_buf.p, cells, bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(grid stack)");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(grid stack)");
  c->d_grid = (const float*)c->grid_buf.p;
  c->n_grids = n_grids;
  c->has_grid = true;
  c->int_checked = false;
  c->key_cells = cells;
  c->key_stride = -n_grids;  // never equal to a csm_set_grid stride
  c->key_version = version;
  c->key_sx = info->size_x;
  c->key_sy = info->size_y;
  return CSM_OK;
}

int csm_phase_buckets(double step_cells, int32_t n_space, int32_t margin_log2, int32_t* n_buckets,
                      int32_t* cells, double* lo, double* hi, int8_t* ox) {
  if (!n_buckets || !cells || !lo || !hi || !ox || margin_log2 < 2 || margin_log2 > 40) return CSM_ERR_INVALID_ARG;
  csm::PhaseTable T{};
  if (!phase_table(step_cells, n_space, margin_log2, T)) return CSM_ERR_UNSUPPORTED;
  *n_buckets = T.nq;
  *cells = T.cells;
  for (int q = 0; q < csm::kPhaseMaxBuckets; ++q) {
    lo[q] = T.lo[q];
    hi[q] = T.hi[q];
    for (int j = 0; j < csm::kPhaseMaxSpace; ++j) ox[q * csm::kPhaseMaxSpace + j] = T.ox[q][j];
  }
  return CSM_OK;
}

int csm_sort_order(csm_ctx* c, const double* keys, int64_t n, int64_t* order) {
  if (!c || !keys || !order) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (n <= 0 || n > csm::kFinishMaxCand) return c->fail(CSM_ERR_INVALID_ARG, "n must be in [1, 10240]");
  // one dummy window whose "scores" are the keys: n_space = n keeps every
  // candidate on angle 0 for the scans that follow the sort
  ScanWork sw{};
  AngleEntry ae{0.0, 1.0, 0.0};
  hipError_t e;
  if ((e = c->scores.ensure((size_t)n * sizeof(double))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scores)");
  if ((e = c->scans.ensure(sizeof(ScanWork))) != hipSuccess) return c->hip_fail(e, "hipMalloc(scans)");
  if ((e = c->angles.ensure(sizeof(AngleEntry))) != hipSuccess) return c->hip_fail(e, "hipMalloc(angles)");
  if ((e = c->fin.ensure(sizeof(csm::FinishOut) + (size_t)n * sizeof(int32_t))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(finish)");
  if ((e = hipMemcpyAsync(c->scores.p, keys, (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(c->scans.p, &sw, sizeof(sw), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(c->angles.p, &ae, sizeof(ae), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(sort inputs)");
  csm::FinishArgs A{};
  A.n_cand = n;
  A.n_space = (int32_t)n;
  A.step_cells = 1.0;
  A.lin_tol = 1.0;
  int32_t* d_order = (int32_t*)((char*)c->fin.p + sizeof(csm::FinishOut));
  A.order_out = d_order;
  if ((e = csm::launch_finish(A, (const ScanWork*)c->scans.p, (const AngleEntry*)c->angles.p,
                              (const double*)c->scores.p, (csm::FinishOut*)c->fin.p, 1, c->stream)) != hipSuccess)
    return c->hip_fail(e, "finish_kernel");
  std::vector<int32_t> o((size_t)n);
  if ((e = hipMemcpyAsync(o.data(), d_order, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
    return c->hip_fail(e, "hipMemcpyAsync(order)");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize");
  for (int64_t i = 0; i < n; ++i) order[i] = o[(size_t)i];
  return CSM_OK;
}

int csm_optimize_scan_match_batch(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                                  const csm_optimize_param* param, double* poses, double* costs,
                                  int32_t* iterations) {
  if (!c || !param || (n_scans > 0 && (!poses || !costs))) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st;
  if ((st = check_offsets(c, n_scans, offsets)) != CSM_OK) return st;
  if (n_scans == 0) return CSM_OK;
  const int64_t n_total = offsets[n_scans] - offsets[0];
  if ((st = check_points(c, pts, n_total)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  std::vector<int64_t> off(offsets, offsets + n_scans + 1);
  for (auto& o : off) o -= offsets[0];
  if ((st = upload_points(c, pts + 2 * offsets[0], n_total)) != CSM_OK) return st;
  return optimize_batch(c, n_scans, off.data(), *param, poses, costs, iterations);
}

int csm_optimize_scan_match(csm_ctx* c, const double* pts, int32_t n_points, const csm_optimize_param* param,
                            double pose[3], double* cost) {
  if (!c || !cost || !pose) return CSM_ERR_INVALID_ARG;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  const int64_t off[2] = {0, n_points};
  return csm_optimize_scan_match_batch(c, 1, pts, off, param, pose, cost, nullptr);
}

int csm_optimize_update_cost(csm_ctx* c, const double* pts, int32_t n_points, const double est_map[3],
                             double* cost, double H[9], double b[3]) {
  if (!c || !est_map || !cost || !H || !b) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  int st;
  if (n_points < 0) return c->fail(CSM_ERR_INVALID_ARG, "negative point count");
  if ((st = check_points(c, pts, n_points)) != CSM_OK) return st;
  if (!c->has_grid) return c->fail(CSM_ERR_NO_GRID, "no grid set");
  if ((st = upload_points(c, pts, n_points)) != CSM_OK) return st;
  const int64_t off[2] = {0, n_points};
  hipError_t e;
  if ((e = c->opt_off.ensure(sizeof(off))) != hipSuccess || (e = c->opt_scans.ensure(sizeof(csm::OptScan))) != hipSuccess ||
      (e = c->opt_sums.ensure(sizeof(csm::OptSums))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(optimize)");
  csm::OptScan o{};
  csm::host_sincos(est_map[2], &o.s, &o.c);
  o.tx = est_map[0];
  o.ty = est_map[1];
  o.active = 1;
  csm::OptArgs A{};
  A.grid = c->d_grid;
  A.size_x = c->info.size_x;
  A.size_y = c->info.size_y;
  A.outside = c->outside;
  A.pts = (const double*)c->pts.p;
  A.offsets = (const int64_t*)c->opt_off.p;
  A.scans = (const csm::OptScan*)c->opt_scans.p;
  A.out = (csm::OptSums*)c->opt_sums.p;
  csm::OptSums r{};
  if ((e = hipMemcpyAsync(c->opt_off.p, off, sizeof(off), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(c->opt_scans.p, &o, sizeof(o), hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = csm::launch_optimize_cost(A, 1, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(&r, c->opt_sums.p, sizeof(r), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return c->hip_fail(e, "optimize_cost_kernel");
  *cost = r.v[0] * (kOptCostPointSize / (1 + r.valid));
  const double h[9] = {r.v[1], r.v[2], r.v[4], r.v[2], r.v[3], r.v[5], r.v[4], r.v[5], r.v[6]};
  std::memcpy(H, h, sizeof(h));
  b[0] = r.v[7];
  b[1] = r.v[8];
  b[2] = r.v[9];
  return CSM_OK;
}

int csm_load_scans_grids(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                         const int32_t* grid_index) {
  int st = csm_load_scans(c, n_scans, pts, offsets);
  if (st != CSM_OK || !grid_index) return st;
  std::lock_guard<std::mutex> lk(c->mu);
  c->loaded_grid.assign(grid_index, grid_index + n_scans);
  return CSM_OK;
}

int csm_scan_matchers_batch_grids(csm_ctx* c, int32_t n_scans, const double* pts, const int64_t* offsets,
                                  const int32_t* grid_index, const csm_param levels[3], int32_t use_fine,
                                  double* poses, double* covs, double* scores) {
  if (!c || !levels || !poses || !covs || !scores) return CSM_ERR_INVALID_ARG;
  const int st = csm_load_scans_grids(c, n_scans, pts, offsets, grid_index);
  if (st != CSM_OK) return st;
  return csm_scan_matchers_loaded(c, levels, use_fine, poses, covs, scores);
}

int csm_set_grid_stack_gridmaps(csm_ctx* c, csm_gridmap* const* maps, int32_t n_maps) {
  if (!c || !maps || n_maps <= 0) return CSM_ERR_INVALID_ARG;
  std::vector<csm::GridMapView> v((size_t)n_maps);
  for (int32_t i = 0; i < n_maps; ++i) {
    if (!maps[i]) return CSM_ERR_INVALID_ARG;
    const int st = csm::gridmap_view(maps[i], &v[(size_t)i]);
    if (st != CSM_OK) return st;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  release_map_reader(c);
  park_current(c);
  const csm::GridMapView& a = v[0];
  int32_t min_index = a.map_update_index;
  for (const auto& b : v) {
    if (b.device != c->device) return c->fail(CSM_ERR_INVALID_ARG, "map lives on another device");
    if (b.size_x != a.size_x || b.size_y != a.size_y || b.resolution != a.resolution || b.offset_x != a.offset_x ||
        b.offset_y != a.offset_y)
      return c->fail(CSM_ERR_INVALID_ARG, "stacked maps must share size, resolution and offset");
    min_index = std::min(min_index, b.map_update_index);
  }
  const int64_t ncell = (int64_t)a.size_x * a.size_y;
  if (ncell >= ((int64_t)1 << 31)) return c->fail(CSM_ERR_INVALID_ARG, "grid larger than 2^31 cells");
  hipError_t e;
  if ((e = c->grid_buf.ensure((size_t)ncell * (size_t)n_maps * sizeof(float))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(grid stack)");
  for (int32_t i = 0; i < n_maps; ++i) {  // after each map's last update, on the matcher's stream
    if ((e = hipStreamWaitEvent(c->stream, v[(size_t)i].ready, 0)) != hipSuccess ||
        (e = hipMemcpyAsync((float*)c->grid_buf.p + (size_t)i * (size_t)ncell, v[(size_t)i].prob,
                            (size_t)ncell * sizeof(float), hipMemcpyDeviceToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "hipMemcpyAsync(map stack)");
    csm::gridmap_add_read_fence(maps[i], c->stream);  // the map's next update after the copy (only)
  }
  c->info.resolution = a.resolution;
  c->info.offset_x = a.offset_x;
  c->info.offset_y = a.offset_y;
  c->info.size_x = a.size_x;
  c->info.size_y = a.size_y;
  c->info.update_index = min_index;
  c->d_grid = (const float*)c->grid_buf.p;
  c->n_grids = n_maps;
  c->has_grid = true;
  c->int_checked = false;
  c->key_cells = nullptr;
  c->key_version = -1;
  return CSM_OK;
}

}  // extern "C"
