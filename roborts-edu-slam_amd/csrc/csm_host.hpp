// csm_host.hpp — the host side of the C-ABI (include/csm.h), shared by its
// translation units: the context (csm_ctx), its buffers and worker pool, the
// window plan, and the functions one unit calls in another.
//
//   csm_api.cpp          context lifetime, profiling, raw window kernels, the search
//   csm_grid.cpp         resident grids: upload, refresh, stacks, borrowed maps
//   csm_launch.cpp       window plans and kernel launches (run_windows), joins
//   csm_driver.cpp       BasedCorrelationScanMatch / ScanMatchers batches, the
//                        pipelined 3-level driver
//   csm_host_finish.cpp  the host finish: std::sort, FindBest, covariance,
//                        the FAST (branch-and-bound) replay
//   csm_optimize_host.cpp the Gauss-Newton matcher's host loop
//
// Compiled with g++ -O2 -ffp-contract=off (no -march), like the reference's
// Release build, so every host double expression rounds as the reference's
// does. The candidate sort is libstdc++'s std::sort on records compared by
// score only, fed in the reference's enumeration order: the permutation is a
// function of the comparison outcomes alone, so ties resolve exactly as in the
// reference (whose Candidate2D records are 40 bytes, ours 16).
#pragma once

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

struct csm_ctx;

namespace csmh {
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
    const size_t want = csm::grow_bytes(bytes, cap);
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
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
    const size_t want = csm::grow_bytes(bytes, cap);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) cap = want;
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

// Window dimensions (csm_launch.cpp): n_angles, n_space (correlate_scan_matcher.h:154,538)
int window_dims(const csm_param& P, Dims& d);
// The reference's beam subsampling (:561-566)
bool beam_rule(int n, int use_point_size, int& step, int& use, int& n_used);

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

// csm_host_finish.cpp
void host_sort_finish(const double* scores, const Dims& D, const CandGeom& C, const csm_param& P,
                      const Geometry& G, std::vector<Entry>& e, csm::FinishOut& o);
int own_lists_skip(int type);
// A window's FinishOut that a finish wrote into pinned host memory, checked
// against its seal (csm_internal.hpp): copied to `out`, then kSealFast or
// kSealExact when the copy is whole for launch tag `tag`, kSealPending when the
// fast pass left the window to the exact pass, 0 when its pieces or its seal
// have not all landed yet.
uint32_t read_sealed(const csm::FinishOut* src, int32_t tag, csm::FinishOut& out);
// The writer the seal names for `tag`, from the seal's first word alone (0:
// not landed yet).
uint32_t seal_writer(const csm::FinishOut* src, int32_t tag);
double complete_window(const csm::FinishOut& o, const CandGeom& C, const csm_param& P,
                       const Geometry& G, double pose[3], double cov[9], int skip_lists = 0);

// csm_placement.cpp
void pin_to_plan(const csm_host_plan& p);
void context_host_plan(int device, int rank, int world, csm_host_plan* out);
int create_context(int device, int local_rank, int local_world, csm_ctx** out);

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
  // workers pinned to the plan's CPUs (csm_placement.cpp; the caller's thread is not)
  ThreadPool(int threads, const csm_host_plan& plan) : n_threads_(std::max(1, threads)), plan_(plan) {}
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
    const int chunk = std::max(1, n / (threads * chunk_div_));
    uint32_t ep;
    start_ns_ = now_ns();
    first_join_ns_.store(0, std::memory_order_relaxed);
    last_join_ns_.store(0, std::memory_order_relaxed);
    busy_ns_.store(0, std::memory_order_relaxed);
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
    const int64_t jl = last_join_ns_.load(std::memory_order_relaxed);
    last_last_join_us_ = jl ? (double)(jl - start_ns_) * 1e-3 : -1.0;
    last_wall_us_ = (double)(now_ns() - start_ns_) * 1e-3;
    last_busy_us_ = (double)busy_ns_.load(std::memory_order_relaxed) * 1e-3;
  }
  // the last job: the caller's share of the items, and when the first worker
  // joined it (us after the notify; -1: none did) — profiling only
  double last_caller_share() const { return last_caller_share_; }
  double last_join_us() const { return last_join_us_; }
  // profiling: when the last worker joined (us after the notify), the job's
  // wall time, and the time all threads spent inside items (summed)
  double last_last_join_us() const { return last_last_join_us_; }
  double last_wall_us() const { return last_wall_us_; }
  double last_busy_us() const { return last_busy_us_; }

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
      const int64_t tj = now_ns();
      if (worker && ran == 0) {
        int64_t zero = 0;
        first_join_ns_.compare_exchange_strong(zero, tj, std::memory_order_relaxed);
        last_join_ns_.store(tj, std::memory_order_relaxed);  // (racy max: profiling only)
      }
      const int i0 = (int)(c & 0xffffffffu), i1 = std::min(n, i0 + chunk);
      for (int i = i0; i < i1; ++i) job(i);
      busy_ns_.fetch_add(now_ns() - tj, std::memory_order_relaxed);
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
    pin_to_plan(plan_);
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job = nullptr;
      int n = 0, chunk = 1;
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
  int n_threads_;
  csm_host_plan plan_;
  static constexpr int chunk_div_ = 8;  // chunks per thread and job
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
  std::atomic<int64_t> first_join_ns_{0}, last_join_ns_{0}, busy_ns_{0};
  double last_caller_share_ = 0.0, last_join_us_ = -1.0, last_last_join_us_ = -1.0, last_wall_us_ = 0.0,
         last_busy_us_ = 0.0;
};

inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}


// A launch left in flight by run_windows(..., pend): what wait_run needs to
// join it and account its kernels.
struct PendingRun {
  char kname[48] = {0};
  char fname[48] = {0};
  double alg_bytes = 0.0, scorings = 0.0, finish_bytes = 0.0;
  bool device_finish = false, timed = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, done = nullptr;
  hipEvent_t ev_fast = nullptr;  // after the fast finish pass, when the exact pass runs on x_stream
  hipEvent_t gap0 = nullptr, gap1 = nullptr;  // a two-span level: not kernel time between these
  const int32_t* flags = nullptr;  // need-exact flags on the host (profiling)
  int n_flags = 0;
  // few-window launches: the finish writes FinishOut here (host memory) and
  // stores flag_value at host_flag when the whole level is done
  const csm::FinishOut* fin_host = nullptr;
  const int32_t* host_flag = nullptr;
  int32_t flag_value = 0;
  // the fast pass's early signal (FinishArgs::host_fast_flag), or null
  const int32_t* fast_flag = nullptr;
  // profiling with a host signal: read the launch's events later
  // (flush_deferred) instead of waiting for its last kernel to retire
  bool defer_timing = false;
};

}  // namespace csmh

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
  // after it (ev_k on this stream).
  hipStream_t x_stream = nullptr;
  hipEvent_t ev_fast = nullptr;
  // Signalled levels of the 3-level driver: the host completes (and plans the
  // next level of) the windows the fast pass settled while the exact pass
  // sorts the flagged ones (FinishArgs::host_fast_flag).
  bool early_complete = true;
  bool early_now = false;  // set by match_levels_pipelined
  // CSM_DEBUG_FIN builds: the 3-level driver snapshots the last level's FinishOut
  // as each window is completed and, once the device is idle, compares it with
  // what the finish finally left in host memory (stderr; diagnostics of the
  // host-signal paths)
  bool debug_fin = false;
  std::mutex mu;
  std::string err;
  float outside = 0.3f;  // kMapUnknownCellProb (slam/slam_processor.h:264)
  int host_threads = 1;
  csm_host_plan host_plan{};  // where the pool runs (csm_placement.cpp)
  bool score_marker = true;   // the event recorded before each scoring launch (CSM_SCORE_MARKER=0: A/B)
  // The 3-level driver's angle rows: cos/sin on the device (csm_trig.hip,
  // glibc's sincos restated; CSM_DEVICE_TRIG=0: the host's ::sincos), when
  // the host's libm passed libm_sincos_table()'s checks
  bool device_trig = true;
  csmh::DevBuf trig_tab;      // libm's sincos table on this device (uploaded on first use)
  std::unique_ptr<csmh::ThreadPool> pool;
  template <class F>
  void parallel_for(int n, int threads, F&& fn) {
    if (!pool) pool.reset(new csmh::ThreadPool(host_threads, host_plan));
    pool->run(n, threads, std::forward<F>(fn));
  }

  csm_map_info info{};
  bool has_grid = false;
  const float* d_grid = nullptr;  // owned (grid_buf) or borrowed
  csmh::DevBuf grid_buf;
  const void* key_cells = nullptr;
  int64_t key_stride = 0, key_version = -1;
  int32_t key_sx = -1, key_sy = -1;

  csmh::DevBuf pts, scans, angles, scores, partials, best, fin;
  csmh::DevBuf ang_max;  // the fused fast finish: per (window, angle) max score (csm_tail.hpp)
  csmh::DevBuf win_ctr;  // ... and per window the waves arrived (zero between launches)
  csmh::DevBuf best_tiles;  // tiled box mode: one best per (window, tile) between the two reductions
  csmh::HostBuf h_search;   // csm_search_windows: pinned staging of the points and angle table
  bool staging_dirty = false;  // a search failed with copies out of its staging possibly in flight
  csm_gridmap* reader_map = nullptr;  // the map csm_set_grid_gridmap borrowed (its updates wait for this stream)
  csmh::HostBuf h_pts;      // upload_points: pinned staging of a scan's points (and small host arrays)
  hipEvent_t ev_pts = nullptr;  // the last copy out of h_pts
  bool ev_pts_used = false;
  csmh::HostBuf h_scores, h_fin, h_angles, h_sw;
  csmh::HostBuf h_angles_next;  // the next level's angle rows while this level's are still read (level_end_begin)
  // Host-signal device finish of the throughput path (CSM_HOST_SIGNAL=0: off):
  // the finish writes FinishOut straight into coherent pinned memory and the
  // pass that ends last stores a flag there (no D2H copy, no event round trip).
  // fin_sig: done counter | need[nw] | list {count, tag, windows[nw]}; h_fin_sig: FinishOut[nw] | flag.
  bool host_signal = true;
  double t_call = 0.0, t_exit = 0.0;  // profiling: the 3-level call's entry and the previous call's exit (now_ms)
  csmh::DevBuf fin_sig;
  csmh::HostBuf h_fin_sig;
  bool device_finish = true;  // CSM_FINISH=host forces the host std::sort path
  bool fast_finish = true;    // CSM_FINISH=exact: always the full device std::sort emulation
  int device_finish_min = 1;  // fewest windows per launch that finish on the device
  bool row_kernel = true;     // CSM_KERNEL=v2 turns the row-segment kernel (v4) off: column kernel only
  bool phase_kernel = true;   // v7 phase kernel for sub-cell window steps (CSM_KERNEL=v7 or unset)
  bool tiny_kernel = true;    // v8 tiny-window kernel, spans under one cell (CSM_KERNEL=v8 or unset)
  int phase_margin_log2 = 20; // CSM_PHASE_MARGIN_LOG2 (tests: a wider margin sends more beams to the exact path)
  // the grid's palette: the byte copy of gridi (palette indices) and the
  // palette, rebuilt when grid_gen moves on (the pair box kernel's source)
  csmh::DevBuf pal_grid, pal_vals, pal_scratch;
  csmh::DevBuf pal_strips;     // strip copies of pal_grid (v11 pair kernel; palettes of <= kPairMaxPal values)
  bool pal_strips_ok = false;
  bool pair_kernel = true;     // v11 pair box kernel where the grid has a palette (CSM_KERNEL set: off)
  csmh::DevBuf istrips;        // strip copies of gridi (the phase kernel's strip form)
  uint64_t istrips_gen = 0;    // grid_gen they were built for
  const int32_t* istrips_src = nullptr;
  bool istrips_ok = false;
  bool phase_strips = true;    // CSM_PHASE_STRIPS=0: the phase kernel reads gridi row-major
  int32_t pal_n = 0;           // palette size (0: none, e.g. more than kPalMax values)
  uint64_t pal_gen = 0;        // grid_gen the palette was built for
  const int32_t* pal_src = nullptr;  // ... and the gridi it was built from
  bool box_kernel = true;     // v6 box kernel for one-cell window steps; any CSM_KERNEL other
                              // than v6 turns it off (CSM_KERNEL=v4: the LDS-DMA row kernel)
  // Few-window launches (run_windows_small): the split kernel's slab and
  // arrival counters, the device copy of the windows and the finish's scratch
  // (ScanWork[nw] | AngleEntry[..] | need[nw] | list[nw + 1] | done counter),
  // the windows' staging and the FinishOut the finish writes straight into
  // coherent pinned memory, followed by the flag the exact pass sets last.
  csmh::DevBuf split_slab, split_arrive, small_dev;
  csmh::HostBuf h_small_in, h_small_out;
  uint32_t flag_seq = 0;
  bool small_path = true;      // CSM_SMALL=0: few-window launches take the throughput kernels
  int small_max_windows = 32;  // launches of at most this many windows take the few-window path
  int split_target_blocks = 512;  // blocks a split launch aims for
  int fast_wide_windows = 0;      // fast finishes of <= this many windows on 1024 threads (0: 64)
  csmh::HostBuf h_pack;  // pinned staging of packed grid rows / cell updates (grid uploads)
  hipEvent_t ev_pack = nullptr;  // the last copy out of h_pack (cell updates return before it ends)
  bool ev_pack_used = false;
  // the points last uploaded (upload_points skips an identical upload: the
  // reference's ScanMatchers calls each level with the same range data)
  std::vector<double> pts_host;
  bool pts_cached = false;
  csmh::DevBuf d_updates;  // csm_update_grid_cells entries on the device

  // Resident grids of other host maps. csm_set_grid keys a grid on the host
  // cells pointer (the map's identity); switching between maps (the front
  // end's fine map, the back end's maps) swaps the current grid with a parked
  // one instead of re-uploading it. The least recently used is evicted.
  struct GridSlot {
    csm_map_info info{};
    bool has_grid = false;
    const float* d_grid = nullptr;
    csmh::DevBuf grid_buf, gridi;
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
  csmh::DevBuf opt_off, opt_scans, opt_sums;
  csmh::HostBuf h_opt_scans, h_opt_sums;

  // exact fixed-point copy of the grid (ensure_int_grid)
  csmh::DevBuf gridi, gstats;
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


  // Batches queued by csm_load_scans_async: uploaded on stage_stream (not on
  // h2d, whose per-launch input copies would queue behind a batch), their
  // max |x| + |y| found on the device; csm_scan_matchers_loaded swaps the
  // oldest into `pts` (the old buffer takes the next batch).
  struct Staged {
    csmh::DevBuf pts, maxabs_dev;
    std::vector<int64_t> off;
    int32_t n = -1;
    hipEvent_t ready = nullptr;
    unsigned long long* maxabs_h = nullptr;  // pinned
  };
  hipStream_t stage_stream = nullptr;
  Staged staged[2];
  int staged_head = 0, staged_count = 0;

  // scans made resident by csm_load_scans (offsets relative to pts)
  int32_t loaded_n = -1;
  std::vector<int64_t> loaded_off;
  std::vector<int32_t> loaded_grid;  // per loaded scan: the resident grid it is matched on (empty: grid 0)

  // per-kernel HIP-event timing (csm_set_profiling / csm_kernel_stats)
  bool profiling = false;
  bool profile_first_level = false;  // csm_set_profiling(ctx, 2): the 3-level driver times its first level only
  bool stats_dump = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipEvent_t ev_ft = nullptr;    // profiling: the fast finish pass ended (timed; ev_fast is not)
  // profiling a level scored in two spans (level_begin_split): the first span's
  // end and the second's start, so the host's planning between them is not
  // counted as kernel time
  hipEvent_t ev_g0 = nullptr, ev_g1 = nullptr;
  bool span_gap = false;
  int32_t list_tag = 0;  // host signal: the tag of the slot's latest scoring call (run_windows)
  // the fused finish: a level's first span is out but its last window's span
  // is not (a level that failed on the host between them leaves level_ctr and
  // the window counters part-counted; the slot's next tail level zeroes them)
  bool tail_open = false;
  hipEvent_t ev_done = nullptr;  // end of a launch's work (async runs)
  hipEvent_t ev_in = nullptr;    // a launch's inputs are on the device
  hipEvent_t ev_k = nullptr;     // a launch's kernels are done

  // Second set of per-launch buffers: the 3-level driver keeps two halves of
  // a batch in flight (match_levels_pipelined); swap_slot() exchanges the
  // sets so run_windows works on whichever half is current. Every part uses
  // the one kernel stream: a stream per part measured slower (two concurrent
  // box-kernel launches contend for L2, 1.01 -> 1.57 ms each; profiles/r01).
  struct Slot {
    csmh::DevBuf scans, angles, scores, partials, best, fin, ang_max, win_ctr;
    csmh::HostBuf h_scores, h_fin, h_angles, h_sw, h_angles_next, h_fin_sig;
    csmh::DevBuf fin_sig;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev_done = nullptr, ev_in = nullptr, ev_k = nullptr;
    hipEvent_t ev_ft = nullptr, ev_g0 = nullptr, ev_g1 = nullptr;
    hipEvent_t ev_fast = nullptr;
    bool span_gap = false;
    int32_t list_tag = 0;
    bool tail_open = false;
  };
  static constexpr int kMaxParts = 4;
  Slot alt[kMaxParts - 1];
  int pipeline_min = 512;    // fewest scans the 3-level driver splits into parts (CSM_PIPELINE)
  bool skip_dead_lists = true;  // live_lists (CSM_SKIP_DEAD_LISTS=0: every level fills both lists)
  int pipeline_parts = 2;    // parts in flight (CSM_PIPELINE_PARTS: 2..kMaxParts; 2 measured fastest)
  int first_windows = 128;   // level_begin_split: windows the first part's first launch takes (CSM_FIRST_WINDOWS; 0: one launch)
  // submitted batches (the device has the previous batch's work queued): a
  // 512-window first span, so the batch boundary's host planning covers 512
  // windows instead of the whole part (r05 A/B, 3 interleaved rounds, config-2
  // ms/step: 0 2.165 / 2.185 / 2.170, 512 2.090 / 2.107 / 2.112, 768 2.105 /
  // 2.111 / 2.115; r04's 128 was slower than one launch). Only for coarse
  // levels of use_point_size > 512: B = 109 (use_point_size 100) is host-bound
  // and measured 1.468 ms one launch against 1.495 split (6 rounds each).
  int first_windows_submit = 512;  // (CSM_FIRST_WINDOWS sets both, CSM_FIRST_WINDOWS_SUBMIT this one)
  int first_windows_submit_min_use = 512;
  int span_growth = 4;       // ... and each later span's growth
  void* pipe = nullptr;  // csm_driver.cpp PipeState: submitted batches (csm_scan_matchers_submit)
  bool split_last_handoff = true;  // the last part's hand-off to the last level in two spans
  int split_handoff_min = 256;     // ... for parts of at least this many windows (CSM_SPLIT_HANDOFF_MIN)
  bool defer_last_handoff = true;  // a submitted batch leaves its last part's last hand-off to the next call (CSM_DEFER_HANDOFF)
  int part0_permille = 550;  // two parts: the first one's share of the scans (
                             // r04 A/B, 2 runs each: 500 9.40, 550 9.61, 600 9.56, 650 9.47 G scorings/s)
  int part0_permille_submit = 500;  // ... for submitted batches (r04 A/B with
                                    // the deferred hand-off: 500 10.45 / 10.48, 550 10.39 / 10.41 G)
  void swap_slot(int i) {    // i >= 1: exchange the current buffer set with alt[i - 1]
    Slot& a = alt[i - 1];
    std::swap(scans, a.scans);
    std::swap(angles, a.angles);
    std::swap(scores, a.scores);
    std::swap(partials, a.partials);
    std::swap(best, a.best);
    std::swap(fin, a.fin);
    std::swap(ang_max, a.ang_max);
    std::swap(win_ctr, a.win_ctr);
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
    std::swap(ev_g0, a.ev_g0);
    std::swap(ev_g1, a.ev_g1);
    std::swap(span_gap, a.span_gap);
    std::swap(list_tag, a.list_tag);
    std::swap(tail_open, a.tail_open);
  }
  // profiling: the pool's last job, as "pool:<what>" (total_ms = the first
  // worker's join latency, algorithmic_bytes = the caller's share of the items)
  void account_pool(const char* what) {
    if (!profiling || !pool) return;
    char nm[48];
    std::snprintf(nm, sizeof(nm), "pool:%s", what);
    account(nm, (float)(std::max(0.0, pool->last_join_us()) * 1e-3), pool->last_caller_share(), 0.0);
    // wall time of the job (total_ms), the last worker's join (bytes, us), the
    // items' time summed over threads (scorings, us)
    std::snprintf(nm, sizeof(nm), "pool:%s:wall", what);
    account(nm, (float)(pool->last_wall_us() * 1e-3), std::max(0.0, pool->last_last_join_us()), pool->last_busy_us());
  }
  std::vector<csmh::PendingRun> deferred;  // signalled launches whose timings are read later (flush_deferred)
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

namespace csmh {

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

// Scores windows_n windows of one level on the device. plans[i] describes
// window i, pts_dev is the batch's points already resident. When best_out is
// null, every score is copied back into ctx->h_scores (window-major).
enum class Finish { kScoresToHost, kDevice, kBest };


// With pend == nullptr the call returns once results are on the host; with
// pend it returns as soon as the work is enqueued (join with wait_run).
// Part of a level's launch (the 3-level driver's chunked first plan): score
// windows [w0, w1) only, or only finish every window once all are scored.
// A part needs the device finish and window i's angle rows at i * n_angles.
struct WinSpan {
  int w0 = 0, w1 = -1;  // w1 < 0: every window
  bool score = true, finish = true;
  // the caller's plan pass filled the windows' ScanWork into the slot's
  // staging (c->h_sw, this pointer) at sw_stride, and found every window of
  // the level in fixed-point range (int_all): run_windows skips both loops
  const ScanWork* sw_ready = nullptr;
  int64_t sw_stride = 0;
  bool int_all = false;
  // the plan left the rows' cos/sin to the device (plan_window_into host_trig
  // false): the launch computes them after the rows' copy (csm_trig.hip)
  bool dev_trig = false;
  // ... and every window of the span has its angles inside the restated
  // domain: the device builds the rows whole from the ScanWork, no rows' copy
  bool rows_gen = false;
};

// glibc's sincos table from this process's libm, or nullptr when it was not
// found or the restated sincos did not equal ::sincos on the check's
// arguments (csm_launch.cpp; libm_sincos_table.hpp). Located once.
const double* libm_sincos_table();

bool signalled_finish(const csm_ctx* c, Finish mode);
int64_t score_stride(const csm_ctx* c, const Dims& D, Finish mode);
bool small_launch(const csm_ctx* c, const Dims& D, int nw);
bool int_mode_window_ok(const csm_ctx* c, const Dims& D, double f, const WindowPlan& W);
void fill_scan_work_one(const Dims& D, const WindowPlan& W, int64_t pt_off, int32_t grid, size_t i, int64_t stride,
                        ScanWork& s);

// csm_grid.cpp
int ensure_int_grid(csm_ctx* c);
void release_map_reader(csm_ctx* c);

// csm_grid.cpp: the strip copies of gridi for the phase kernel (c->istrips_ok)
int ensure_istrips(csm_ctx* c);
// csm_grid.cpp: the palette copy of gridi for the v10 box kernel (c->pal_n = 0: none)
int ensure_palette(csm_ctx* c);

// csm_launch.cpp
int wait_flag(csm_ctx* c, const PendingRun& p, const int32_t* flag = nullptr);
int wait_run(csm_ctx* c, const PendingRun& p);
int flush_deferred(csm_ctx* c);
bool phase_table(double f, int ns, int margin_log2, csm::PhaseTable& T);
int run_windows(csm_ctx* c, const csm_param& P, const Dims& D, const Geometry& G,
                const std::vector<WindowPlan>& plans, const std::vector<int64_t>& pt_offsets,
                const AngleEntry* angles, size_t n_angle_entries,
                const std::vector<int32_t>& grid_index, BestPartial* best_out,
                Finish mode = Finish::kScoresToHost, PendingRun* pend = nullptr, int skip_lists = 0,
                WinSpan sp = WinSpan{});
bool plan_window_into(const csm_param& P, const Dims& D, const Geometry& G, int n_points,
                      const double center[3], AngleEntry* out, WindowPlan& W, bool host_trig = true);
bool plan_window(const csm_param& P, const Dims& D, const Geometry& G, int n_points,
                 const double center[3], std::vector<AngleEntry>& angles, WindowPlan& W);
bool plan_windows_shared(const csm_param& P, const Dims& D, const Geometry& G, int n_points, int n_windows,
                         const double* centers, std::vector<AngleEntry>& angles, std::vector<WindowPlan>& plans);
int upload_points(csm_ctx* c, const double* pts, int64_t n_total, void* pinned = nullptr);
int check_points(csm_ctx* c, const double* pts, int64_t n_total);
int check_offsets(csm_ctx* c, int32_t n_scans, const int64_t* offsets);

// csm_host_finish.cpp: FAST windows (the reference's branch and bound)
int match_level_fast(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                     double* poses, double* covs, double* responses, int64_t* argmax_flat);

// csm_driver.cpp
int match_level(csm_ctx* c, int32_t n_scans, const int64_t* offsets, const csm_param& P,
                double* poses, double* covs, double* responses, int64_t* argmax_flat,
                const int32_t* scan_grid = nullptr, int skip_lists = 0);

// csm_optimize_host.cpp
constexpr double kOptCostPointSize = 1000;                // optimize_scan_matcher.h:234
constexpr double kOptMaxCost = 1.0 * kOptCostPointSize;   // :235

inline bool map_ready(const csm_ctx* c) { return c->has_grid && c->info.update_index >= 0; }

// csm_driver.cpp: a submitted batch still pending is completed (every entry
// point but csm_scan_matchers_submit calls it first); the state's release
int pipe_drain(csm_ctx* c);
void pipe_free(csm_ctx* c);
int take_staged(csm_ctx* c);
int matchers_loaded_locked(csm_ctx* c, const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                           double* scores);

}  // namespace csmh
