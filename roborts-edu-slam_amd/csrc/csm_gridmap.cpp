// csm_gridmap.cpp — host side and C ABI of the device-resident occupancy-grid
// maps (include/csm_gridmap.h).
//
// The reference's per-scan bookkeeping runs here, on the host, with its own
// arithmetic (g++ -O2 -ffp-contract=off, like the reference build): the
// world->map pose, the scan's transform and endpoint cells, the bound boxes
// and map growth of UpdateBound/ExtendSize, the update counters. It is O(beams)
// per scan. Everything O(cells) — the Bresenham lines, the blur splats, the cell
// updates, resets, the growth copy and the map check's ray walks — runs in the
// kernels of csm_gridmap.hip. There is no CPU fallback: without a device
// csm_gridmap_create fails.
//
// Paths cited are relative to the reference root.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "csm_gridmap.h"
#include "csm_gridmap_internal.hpp"
#include "csm_internal.hpp"
#include "host_math.hpp"

namespace {

using csm::GmCells;
using csm::GmEnd;
using csm::GmOps;

constexpr float kDefaultCellProb = 0.5f;  // grid_map_cell.h:30

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = csm::grow_bytes(bytes, cap);
    release();
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Box {  // BoundBox<double> (util/boundbox.h:35-143); default max FLT_MIN
  double minx = (double)FLT_MAX, miny = (double)FLT_MAX;
  double maxx = (double)FLT_MIN, maxy = (double)FLT_MIN;
  void add(double x, double y) {
    if (x < minx) minx = x;
    if (y < miny) miny = y;
    if (x > maxx) maxx = x;
    if (y > maxy) maxy = y;
  }
  void add_box(const Box& b) {
    add(b.minx, b.miny);
    add(b.maxx, b.maxy);
  }
  void extend(double e) {
    minx -= e;
    miny -= e;
    maxx += e;
    maxy += e;
  }
  bool in(double x, double y) const { return x > minx && x < maxx && y > miny && y < maxy; }
  int size_x() const { return (int)(std::ceil(maxx) - std::floor(minx)); }
  int size_y() const { return (int)(std::ceil(maxy) - std::floor(miny)); }
};

// Affine2d(Translation2d(t) * Rotation2Dd(th)) * p (Eigen: translation plus the
// product linear * p, linear = [c -s; s c]).
inline void pose_apply(double c, double s, double tx, double ty, double px, double py, double& ox, double& oy) {
  ox = (c * px + (-s) * py) + tx;
  oy = (s * px + c * py) + ty;
}

}  // namespace

struct csm_gridmap {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ready = nullptr;       // after the last enqueued update
  hipEvent_t staged = nullptr;      // the last H2D copy out of h_ends has been consumed
  hipEvent_t read_done = nullptr;   // reader streams' work so far (wait_readers)
  std::mutex mu;
  std::string err;

  int kind = csm::kGmProbability;
  // GridMapBase
  double scale_factor = 1.0;
  int size_x = 0, size_y = 0, row = 0;
  double off_x = 0.0, off_y = 0.0;
  Box bound;
  double extend_factor = 1.0;
  float default_prob = kDefaultCellProb;
  int map_update_index = -1;
  // GaussianBlur
  bool blur_states = false;
  int half_kernel = 0;
  std::vector<double> kernel;
  // OccuGridMap
  bool auto_resize = true, just_update_occu = false;
  int cur_update_index = 0, cur_mark_occu = -1, cur_mark_free = -1;
  double occu_offset = 0.72;
  GmOps ops{};
  uint32_t seq = 0;  // scans drawn with lines (line event keys)

  DBuf prob, pass, hit, uidx, touched, fkey, oseq, ends, ktab, count;
  // Fixed-point mirror of prob for the scan matcher (gridmap_fixed_point):
  // kept equal to (prob - fpm_outside) * 2^fpm_exp by every kernel that writes
  // prob while fpm_valid; a growth or an incompatible value drops it.
  DBuf fpm;
  bool fpm_valid = false;
  float fpm_outside = 0.f;
  int fpm_exp = 0;
  int32_t fpm_pitch = 0;
  // A superset of the values the cells can hold, known while every write is
  // a host-known value (fresh cells, resets, blur splats of the kernel table);
  // lost for good once an occupied or line update computes values on the device.
  bool vals_known = true;
  int vals_min_g = INT32_MAX;  // every nonzero value is a multiple of 2^vals_min_g
  float vals_max = 0.f;        // max |value|
  void* h_ends = nullptr;
  size_t h_cap = 0;
  bool ktab_dirty = true;
  std::vector<GmEnd> pending;  // blur endpoints not yet drawn (order-free, batched)

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return CSM_ERR_HIP;
  }
  int64_t ncells() const { return (int64_t)row * size_y; }
  GmCells cells() const {
    GmCells C;
    C.prob = prob.as<float>();
    C.pass = kind == csm::kGmCount ? pass.as<float>() : nullptr;
    C.hit = kind == csm::kGmCount ? hit.as<float>() : nullptr;
    C.uidx = uidx.as<int32_t>();
    C.touched = touched.as<uint8_t>();
    C.row = row;
    C.size_x = size_x;
    C.size_y = size_y;
    C.fpm = fpm_valid ? fpm.as<int32_t>() : nullptr;
    C.fpm_pitch = fpm_pitch;
    C.fpm_outside = fpm_outside;
    C.fpm_scale = std::ldexp(1.0, fpm_exp);
    return C;
  }
  // (max |v| + |outside|) * 2^E below 2^26: the matcher's int32 chunk sums
  bool fpm_fits(int min_g, float vmax, float outside, int E) const {
    return (min_g == INT32_MAX || min_g >= -E) && ((double)vmax + std::fabs((double)outside)) * std::ldexp(1.0, E) <
                                                      std::ldexp(1.0, 26);
  }
  // A value the cells may now hold (before the kernel that writes it).
  void note_value(float v);
  void note_unknown() {
    vals_known = false;
    fpm_valid = false;
  }
};

namespace {
// Smallest power of two a float is an integer multiple of (INT32_MAX for 0).
int float_granularity(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u &= 0x7FFFFFFFu;
  if (u == 0) return INT32_MAX;
  const uint32_t e = u >> 23, mant = u & 0x7FFFFFu;
  const uint32_t mm = (e == 0) ? mant : (mant | 0x800000u);
  return ((e == 0) ? -149 : (int)e - 150) + __builtin_ctz(mm);
}
}  // namespace

void csm_gridmap::note_value(float v) {
  if (!std::isfinite(v)) {
    note_unknown();
    return;
  }
  vals_min_g = std::min(vals_min_g, float_granularity(v));
  vals_max = std::max(vals_max, std::fabs(v));
  if (fpm_valid && !fpm_fits(vals_min_g, vals_max, fpm_outside, fpm_exp)) fpm_valid = false;
}

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define GM_HIP(expr)                                 \
  do {                                               \
    hipError_t e_ = (expr);                          \
    if (e_ != hipSuccess) return m->hip_fail(e_, #expr); \
  } while (0)

int alloc_cells(csm_gridmap* m, int64_t n, DBuf& p, DBuf& ps, DBuf& h, DBuf& u, DBuf& t) {
  GM_HIP(p.ensure((size_t)n * 4));
  if (m->kind == csm::kGmCount) {
    GM_HIP(ps.ensure((size_t)n * 4));
    GM_HIP(h.ensure((size_t)n * 4));
  }
  GM_HIP(u.ensure((size_t)n * 4));
  GM_HIP(t.ensure((size_t)n));
  return CSM_OK;
}

// Host staging -> device ends buffer, on the map's stream.
int upload_ends(csm_gridmap* m, const std::vector<GmEnd>& v) {
  if (v.empty()) return CSM_OK;
  const size_t bytes = v.size() * sizeof(GmEnd);
  GM_HIP(hipEventSynchronize(m->staged));
  if (bytes > m->h_cap) {
    const size_t want = csm::grow_bytes(bytes, m->h_cap);
    if (m->h_ends) (void)hipHostFree(m->h_ends);
    m->h_ends = nullptr;
    m->h_cap = 0;
    GM_HIP(hipHostMalloc(&m->h_ends, want, hipHostMallocDefault));
    m->h_cap = want;
  }
  if (bytes > m->ends.cap) {
    GM_HIP(hipStreamSynchronize(m->stream));  // the old buffer may still be read
    GM_HIP(m->ends.ensure(bytes));
  }
  std::memcpy(m->h_ends, v.data(), bytes);
  GM_HIP(hipMemcpyAsync(m->ends.p, m->h_ends, bytes, hipMemcpyHostToDevice, m->stream));
  GM_HIP(hipEventRecord(m->staged, m->stream));
  return CSM_OK;
}

int upload_ktab(csm_gridmap* m) {
  if (!m->ktab_dirty) return CSM_OK;
  const int k2 = (int)m->kernel.size();
  std::vector<float> t((size_t)k2);
  // SetGridProbability(cell, kernel_value[k] * cell_occu_prob_offset_): the
  // double product narrowed to the float parameter (occu_grid_map.h:567).
  for (int k = 0; k < k2; ++k) t[(size_t)k] = (float)(m->kernel[(size_t)k] * m->occu_offset);
  m->note_value(1.0f);  // the splat's centre
  for (float v : t)
    if (v <= 1.0f) m->note_value(v);  // the values blur_splat_kernel writes
  GM_HIP(hipStreamSynchronize(m->stream));
  GM_HIP(m->ktab.ensure((size_t)(k2 > 0 ? k2 : 1) * 4));
  if (k2 > 0) GM_HIP(hipMemcpy(m->ktab.p, t.data(), (size_t)k2 * 4, hipMemcpyHostToDevice));
  m->ktab_dirty = false;
  return CSM_OK;
}

int flush_pending(csm_gridmap* m) {
  if (m->pending.empty()) return CSM_OK;
  int st;
  if ((st = upload_ktab(m)) != CSM_OK) return st;
  if ((st = upload_ends(m, m->pending)) != CSM_OK) return st;
  GM_HIP(csm::gm_launch_blur(m->ends.as<GmEnd>(), (int)m->pending.size(), m->cells(), m->half_kernel,
                             m->ktab.as<float>(), m->half_kernel + 1, m->stream));
  m->pending.clear();
  return CSM_OK;
}

// ExtendSize(EXTEND_PARTLY) (grid_map_base.h:182-244): host geometry, device copy.
int extend_size(csm_gridmap* m) {
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;
  Box t;
  t.add_box(m->bound);
  const double map_max_x = (double)m->size_x, map_max_y = (double)m->size_y;
  t.add(0.0, 0.0);
  t.add(map_max_x, map_max_y);
  double min_x = t.minx, min_y = t.miny, max_x = t.maxx, max_y = t.maxy;
  if (m->bound.minx <= 0.0) min_x -= (double)t.size_x() * m->extend_factor;
  if (m->bound.miny <= 0.0) min_y -= (double)t.size_y() * m->extend_factor;
  if (m->bound.maxx >= map_max_x) max_x += (double)t.size_x() * m->extend_factor;
  if (m->bound.maxy >= map_max_y) max_y += (double)t.size_y() * m->extend_factor;
  t.add(min_x, min_y);
  t.add(max_x, max_y);
  const double fx = std::floor(t.minx), fy = std::floor(t.miny);
  const int gx = -(int)fx, gy = -(int)fy;
  const int nsx = t.size_x(), nsy = t.size_y();
  const int64_t n = (int64_t)nsx * nsy;
  if (nsx <= 0 || nsy <= 0 || n >= ((int64_t)1 << 31))
    return m->fail(CSM_ERR_ALLOC, "map growth beyond 2^31 cells");
  DBuf np, nps, nh, nu, nt;
  if ((st = alloc_cells(m, n, np, nps, nh, nu, nt)) != CSM_OK) return st;
  GmCells N;
  N.prob = np.as<float>();
  N.pass = m->kind == csm::kGmCount ? nps.as<float>() : nullptr;
  N.hit = m->kind == csm::kGmCount ? nh.as<float>() : nullptr;
  N.uidx = nu.as<int32_t>();
  N.touched = nt.as<uint8_t>();
  N.row = nsx;
  N.size_x = nsx;
  N.size_y = nsy;
  N.fpm = nullptr;  // the mirror is rebuilt at the new size on the matcher's next request
  N.fpm_pitch = 0;
  N.fpm_outside = 0.f;
  N.fpm_scale = 1.0;
  m->fpm_valid = false;
  m->note_value(m->default_prob);  // fresh cells (fresh_kernel)
  m->note_value(kDefaultCellProb);
  GM_HIP(csm::gm_launch_fresh(N, n, m->default_prob, m->stream));
  GM_HIP(csm::gm_launch_extend_copy(m->cells(), N, gx, gy, m->stream));
  GM_HIP(hipStreamSynchronize(m->stream));
  std::swap(m->prob, np);
  std::swap(m->pass, nps);
  std::swap(m->hit, nh);
  std::swap(m->uidx, nu);
  std::swap(m->touched, nt);
  np.release();
  nps.release();
  nh.release();
  nu.release();
  nt.release();
  m->fkey.release();  // per-scan line scratch: rebuilt at the new size
  m->oseq.release();
  m->off_x -= fx / m->scale_factor;
  m->off_y -= fy / m->scale_factor;
  m->row = nsx;
  m->size_x = nsx;
  m->size_y = nsy;
  Box nb;
  nb.minx = m->bound.minx - t.minx;
  nb.miny = m->bound.miny - t.miny;
  nb.maxx = m->bound.maxx - t.minx;
  nb.maxy = m->bound.maxy - t.miny;
  m->bound = nb;
  return CSM_OK;
}

bool point_in_map(const csm_gridmap* m, double x, double y, double tol = 0.0) {  // :344-352
  return x > tol && x < m->size_x - tol && y > tol && y < m->size_y - tol;
}

// UpdateBound (grid_map_base.h:247-264). *grown = the map was extended.
int update_bound(csm_gridmap* m, const Box& b, bool* grown) {
  *grown = false;
  if (m->bound.in(b.minx, b.miny) && m->bound.in(b.maxx, b.maxy)) return CSM_OK;
  m->bound.add_box(b);
  if (!point_in_map(m, m->bound.minx, m->bound.miny) || !point_in_map(m, m->bound.maxx, m->bound.maxy)) {
    *grown = true;
    return extend_size(m);
  }
  return CSM_OK;
}

enum Mode { kBlur = 0, kOccupied = 1, kLines = 2 };

int scan_mode(const csm_gridmap* m, bool use_blur, int* mode) {
  if (!m->blur_states) use_blur = false;  // :265-267
  if (m->just_update_occu)
    *mode = use_blur ? kBlur : kOccupied;
  else if (use_blur)
    return CSM_ERR_UNSUPPORTED;
  else
    *mode = kLines;
  if (*mode == kBlur && m->kind == csm::kGmCount) return CSM_ERR_UNSUPPORTED;
  return CSM_OK;
}

int ensure_line_scratch(csm_gridmap* m) {
  const int64_t n = m->ncells();
  if (m->fkey.cap >= (size_t)n * 8 && m->oseq.cap >= (size_t)n * 4) return CSM_OK;
  GM_HIP(hipStreamSynchronize(m->stream));
  GM_HIP(m->fkey.ensure((size_t)n * 8));
  GM_HIP(m->oseq.ensure((size_t)n * 4));
  GM_HIP(hipMemsetAsync(m->fkey.p, 0, (size_t)n * 8, m->stream));
  GM_HIP(hipMemsetAsync(m->oseq.p, 0, (size_t)n * 4, m->stream));
  m->seq = 0;
  return CSM_OK;
}

// UpdateMapByRange (occu_grid_map.h:258-329).
int update_by_range(csm_gridmap* m, const double* pts, int n, const double origin[2], const double pose[3],
                    bool use_blur, bool* updated) {
  int mode = 0, st;
  if ((st = scan_mode(m, use_blur, &mode)) != CSM_OK)
    return m->fail(st, "update mode not supported (full update with blur, or blur on CountCell)");
  if (!m->blur_states) use_blur = false;
  m->cur_mark_free = m->cur_update_index + 1;
  m->cur_mark_occu = m->cur_update_index + 2;
  // GetMapCoordsPose (grid_map_base.h:89-93)
  const double s = m->scale_factor;
  const double pmx = s * pose[0] + s * m->off_x, pmy = s * pose[1] + s * m->off_y, pth = pose[2];
  double c, sn;
  csm::host_sincos(pth, &sn, &c);
  std::vector<double> tp((size_t)2 * n);
  for (int i = 0; i < n; ++i) pose_apply(c, sn, pmx, pmy, pts[2 * i], pts[2 * i + 1], tp[2 * i], tp[2 * i + 1]);
  if (m->auto_resize && n > 0) {
    Box b;
    for (int i = 0; i < n; ++i) b.add(tp[2 * i], tp[2 * i + 1]);
    if (use_blur) b.extend((double)m->half_kernel);
    bool grown = false;
    if ((st = update_bound(m, b, &grown)) != CSM_OK) return st;
    if (grown) {
      m->cur_update_index += 3;
      *updated = false;
      return CSM_OK;
    }
  }
  double sx, sy;
  pose_apply(c, sn, pmx, pmy, origin[0], origin[1], sx, sy);
  const int x0 = (int)(sx + 0.5), y0 = (int)(sy + 0.5);
  std::vector<GmEnd> ends;
  ends.reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    const int x1 = (int)(tp[2 * i] + 0.5), y1 = (int)(tp[2 * i + 1] + 0.5);
    if (x0 != x1 || y0 != y1) ends.push_back(GmEnd{x1, y1, m->cur_mark_free, m->cur_mark_occu});
  }
  const int tol = m->half_kernel + 1;
  if (mode == kBlur) {
    m->pending.insert(m->pending.end(), ends.begin(), ends.end());
  } else {
    if ((st = flush_pending(m)) != CSM_OK) return st;
    if ((st = upload_ends(m, ends)) != CSM_OK) return st;
    m->note_unknown();  // cell values computed on the device from here on
    if (mode == kOccupied) {
      GM_HIP(csm::gm_launch_occupied(m->ends.as<GmEnd>(), (int)ends.size(), m->cells(), m->ops, tol, m->stream));
    } else {
      if ((st = ensure_line_scratch(m)) != CSM_OK) return st;
      if (m->seq == 0xFFFFFFFFu) {  // key space exhausted: clear the scratch
        GM_HIP(hipMemsetAsync(m->fkey.p, 0, m->fkey.cap, m->stream));
        GM_HIP(hipMemsetAsync(m->oseq.p, 0, m->oseq.cap, m->stream));
        m->seq = 0;
      }
      ++m->seq;
      GM_HIP(csm::gm_launch_lines(m->ends.as<GmEnd>(), (int)ends.size(), x0, y0, m->cells(), m->ops,
                                  m->fkey.as<uint64_t>(), m->oseq.as<uint32_t>(), m->seq, tol, m->stream));
    }
  }
  m->map_update_index++;  // SetUpdated
  m->cur_update_index += 3;
  *updated = true;
  return CSM_OK;
}

int finish(csm_gridmap* m) {
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;
  GM_HIP(hipEventRecord(m->ready, m->stream));
  return CSM_OK;
}

}  // namespace

namespace {
// Matcher streams that read a map's cells (csm_set_grid_gridmap borrows them
// until the next set_grid; csm_set_grid_stack_gridmaps copies them on its
// stream). A map update first waits for the work already enqueued on those
// streams, so an update issued after a set_grid* call can never overwrite
// cells a pending match or copy still reads.
std::mutex g_readers_mu;
std::map<const csm_gridmap*, std::vector<hipStream_t>> g_readers;
// One-shot read fences: events recorded on a reader stream once its reads of
// the map were all enqueued (a stack copy, or a matcher that moved on to
// another grid). An update waits for each once; completed ones are dropped.
std::map<const csm_gridmap*, std::vector<hipEvent_t>> g_fences;

int wait_readers(csm_gridmap* m) {
  std::lock_guard<std::mutex> lk(g_readers_mu);
  auto it = g_readers.find(m);
  if (it != g_readers.end())
    for (hipStream_t s : it->second) {
      GM_HIP(hipEventRecord(m->read_done, s));
      GM_HIP(hipStreamWaitEvent(m->stream, m->read_done, 0));
    }
  auto f = g_fences.find(m);
  if (f != g_fences.end()) {
    std::vector<hipEvent_t> keep;
    for (hipEvent_t ev : f->second) {
      if (hipEventQuery(ev) == hipSuccess) {  // done (and waited for by an earlier update, or now moot)
        (void)hipEventDestroy(ev);
        continue;
      }
      GM_HIP(hipStreamWaitEvent(m->stream, ev, 0));
      keep.push_back(ev);
    }
    f->second.swap(keep);
  }
  return CSM_OK;
}

// The map's next update waits for the reads enqueued on s so far. The event
// is created on the map's device (the reader's stream lives there: a borrow
// from another device is refused). If it cannot be created or recorded, the
// reads are waited for here instead: a fence is never silently dropped.
void add_fence_locked(const csm_gridmap* m, hipStream_t s) {
  DeviceGuard g(m->device);
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamSynchronize(s);
    return;
  }
  if (hipEventRecord(ev, s) != hipSuccess) {
    (void)hipEventDestroy(ev);
    (void)hipStreamSynchronize(s);
    return;
  }
  g_fences[m].push_back(ev);
}
}  // namespace

namespace csm {
void gridmap_add_reader(csm_gridmap* m, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_readers_mu);
  auto& v = g_readers[m];
  if (std::find(v.begin(), v.end(), s) == v.end()) v.push_back(s);
}
void gridmap_drop_reader(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_readers_mu);
  for (auto& kv : g_readers) {
    auto& v = kv.second;
    if (std::find(v.begin(), v.end(), s) == v.end()) continue;
    add_fence_locked(kv.first, s);  // the reads already enqueued still order the map's next update
    v.erase(std::remove(v.begin(), v.end(), s), v.end());
  }
}
void gridmap_release_reader(csm_gridmap* m, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_readers_mu);
  auto it = g_readers.find(m);
  if (it == g_readers.end()) return;
  auto& v = it->second;
  if (std::find(v.begin(), v.end(), s) == v.end()) return;
  add_fence_locked(m, s);
  v.erase(std::remove(v.begin(), v.end(), s), v.end());
}
void gridmap_add_read_fence(csm_gridmap* m, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_readers_mu);
  add_fence_locked(m, s);
}

int gridmap_fixed_point(csm_gridmap* m, float outside, GridMapFixed* f) {
  if (!m || !f) return CSM_ERR_INVALID_ARG;
  *f = GridMapFixed{};
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;  // pending splats first (they keep a valid mirror)
  if (!m->vals_known || m->kind != kGmProbability || !std::isfinite(outside)) return CSM_OK;
  // E: every value and `outside` multiples of 2^-E (ensure_int_grid's rule, on
  // the host-known value set instead of a scan of the cells)
  const int min_g = std::min(m->vals_min_g, float_granularity(outside));
  const int E = (min_g == INT32_MAX) ? 0 : std::max(0, -min_g);
  if (E > 60 || !m->fpm_fits(min_g, m->vals_max, outside, E)) return CSM_OK;
  const int32_t pitch = gridi_pitch(m->size_x);
  const int64_t ni = (int64_t)pitch * (m->size_y + kGridiPadRows);
  if (ni * 4 > 0x7F000000LL) return CSM_OK;
  if (!(m->fpm_valid && m->fpm_outside == outside && m->fpm_exp == E && m->fpm_pitch == pitch)) {
    if ((size_t)ni * 4 > m->fpm.cap) GM_HIP(hipStreamSynchronize(m->stream));  // the old buffer may still be read
    GM_HIP(m->fpm.ensure((size_t)ni * 4));
    GM_HIP(launch_fixed_point(m->prob.as<float>(), m->size_x, m->size_y, pitch, outside, E, m->fpm.as<int32_t>(),
                              m->stream, true));
    m->fpm_valid = true;
    m->fpm_outside = outside;
    m->fpm_exp = E;
    m->fpm_pitch = pitch;
    GM_HIP(hipEventRecord(m->ready, m->stream));
  }
  f->ok = true;
  f->fpm = m->fpm.as<int32_t>();
  f->pitch = pitch;
  f->exp = E;
  f->max_abs = std::max((double)m->vals_max, std::fabs((double)outside));
  f->outside = outside;
  return CSM_OK;
}

int gridmap_view(csm_gridmap* m, GridMapView* v) {
  if (!m || !v) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  v->prob = m->prob.as<float>();
  v->size_x = m->size_x;
  v->size_y = m->size_y;
  v->resolution = 1 / m->scale_factor;
  v->offset_x = m->off_x;
  v->offset_y = m->off_y;
  v->map_update_index = m->map_update_index;
  v->ready = m->ready;
  v->device = m->device;
  return CSM_OK;
}
}  // namespace csm

extern "C" {

int csm_gridmap_create(int device, int32_t kind, double resolution, int32_t size_x, int32_t size_y, double offset_x,
                       double offset_y, double deviation, float default_cell_prob, csm_gridmap** out) {
  if (!out) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  if ((kind != CSM_PROBABILITY_CELL && kind != CSM_COUNT_CELL) || !(resolution > 0.0) || size_x <= 0 ||
      size_y <= 0 || (int64_t)size_x * size_y >= ((int64_t)1 << 31))
    return CSM_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return CSM_ERR_HIP;
  auto* m = new csm_gridmap();
  m->device = device;
  DeviceGuard g(device);
  if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&m->ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->read_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->staged, hipEventDisableTiming) != hipSuccess) {
    csm_gridmap_destroy(m);
    return CSM_ERR_HIP;
  }
  m->kind = kind;
  m->scale_factor = 1.0 / resolution;  // grid_map_base.h:50
  m->off_x = offset_x;
  m->off_y = offset_y;
  m->default_prob = default_cell_prob;
  m->size_x = size_x;
  m->size_y = size_y;
  m->row = size_x;
  // cell functions' constructors (grid_map_cell.h:86-92, 334-337)
  if (kind == CSM_COUNT_CELL)
    m->ops = GmOps{kind, 0.0f, 0.0f, 0.5f, 2.0f};
  else
    m->ops = GmOps{kind, 0.5f, 0.2f, 0.5f, 2.0f};
  // GaussianBlur (occu_grid_map.h:40-105)
  if (deviation > 0.5 * resolution && deviation < 10 * resolution && resolution > 0) {
    m->blur_states = true;
    m->half_kernel = (int)((deviation / resolution) * std::sqrt(std::log(2)));
    const int ks = 2 * m->half_kernel + 1;
    m->kernel.assign((size_t)ks * ks, 0.0);
    for (int i = -m->half_kernel; i <= m->half_kernel; ++i)
      for (int j = -m->half_kernel; j <= m->half_kernel; ++j) {
        const double d = std::hypot(i * resolution, j * resolution);
        const double q = d / deviation;
        m->kernel[(size_t)((i + m->half_kernel) + ks * (j + m->half_kernel))] = std::exp(-0.5 * (q * q));
      }
  }
  const int64_t n = (int64_t)size_x * size_y;
  m->note_value(default_cell_prob);  // fresh_kernel: element 0, then kDefaultCellProb
  m->note_value(kDefaultCellProb);
  int st = alloc_cells(m, n, m->prob, m->pass, m->hit, m->uidx, m->touched);
  if (st == CSM_OK && (csm::gm_launch_fresh(m->cells(), n, default_cell_prob, m->stream) != hipSuccess ||
                       m->count.ensure(64) != hipSuccess || hipEventRecord(m->staged, m->stream) != hipSuccess ||
                       hipEventRecord(m->ready, m->stream) != hipSuccess))
    st = CSM_ERR_HIP;
  if (st != CSM_OK) {
    csm_gridmap_destroy(m);
    return st;
  }
  *out = m;
  return CSM_OK;
}

int csm_gridmap_destroy(csm_gridmap* m) {
  if (!m) return CSM_OK;
  {
    DeviceGuard g(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    for (DBuf* b : {&m->prob, &m->pass, &m->hit, &m->uidx, &m->touched, &m->fkey, &m->oseq, &m->ends, &m->ktab,
                    &m->count, &m->fpm})
      b->release();
    if (m->h_ends) (void)hipHostFree(m->h_ends);
    {
      std::lock_guard<std::mutex> lk(g_readers_mu);
      g_readers.erase(m);
      auto f = g_fences.find(m);
      if (f != g_fences.end()) {
        for (hipEvent_t ev : f->second) (void)hipEventDestroy(ev);
        g_fences.erase(f);
      }
    }
    if (m->ready) (void)hipEventDestroy(m->ready);
    if (m->staged) (void)hipEventDestroy(m->staged);
    if (m->read_done) (void)hipEventDestroy(m->read_done);
    if (m->stream) (void)hipStreamDestroy(m->stream);
  }
  delete m;
  return CSM_OK;
}

const char* csm_gridmap_last_error(const csm_gridmap* m) { return m ? m->err.c_str() : "null map"; }

int csm_gridmap_set_options(csm_gridmap* m, int32_t auto_resize, int32_t just_update_occu, double occu_offset,
                            double extend_factor) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  m->auto_resize = auto_resize != 0;
  m->just_update_occu = just_update_occu != 0;
  if (occu_offset != m->occu_offset) {
    DeviceGuard g(m->device);
    int st = flush_pending(m);  // drawn with the old offset's kernel values
    if (st != CSM_OK) return st;
    m->occu_offset = occu_offset;
    m->ktab_dirty = true;
  }
  if (extend_factor > 0) m->extend_factor = extend_factor;
  return CSM_OK;
}

int csm_gridmap_set_cell_params(csm_gridmap* m, float free_factor, float occu_factor, float occu_threshold,
                                float min_pass) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  m->ops.free_factor = free_factor;
  m->ops.occu_factor = occu_factor;
  if (m->kind == CSM_COUNT_CELL) {
    m->ops.occu_threshold = occu_threshold;
    m->ops.min_pass = min_pass;
  }
  return CSM_OK;
}

int csm_gridmap_set_map_offset(csm_gridmap* m, double ox, double oy) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  m->off_x = ox;
  m->off_y = oy;
  return CSM_OK;
}

int csm_gridmap_reset(csm_gridmap* m) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  if (int rst = wait_readers(m)) return rst;
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;
  // Reset (grid_map_base.h:95-103) leaves map_update_point_ as it is.
  m->note_value(m->default_prob);
  GM_HIP(csm::gm_launch_reset(m->cells(), m->ncells(), m->default_prob, false, false, m->stream));
  return finish(m);
}

int csm_gridmap_update_bound(csm_gridmap* m, double min_x, double min_y, double max_x, double max_y,
                             int32_t* inside) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  if (int rst = wait_readers(m)) return rst;
  Box b;
  b.minx = min_x;
  b.miny = min_y;
  b.maxx = max_x;
  b.maxy = max_y;
  bool grown = false;
  int st = update_bound(m, b, &grown);
  if (st != CSM_OK) return st;
  if (inside) *inside = grown ? 0 : 1;
  return finish(m);
}

int csm_gridmap_update_by_range(csm_gridmap* m, const double* pts, int32_t n, const double origin[2],
                                const double pose[3], int32_t use_blur, int32_t* updated) {
  if (!m || !pose || (n > 0 && !pts) || n < 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  if (int rst = wait_readers(m)) return rst;
  const double zero[2] = {0.0, 0.0};
  bool up = false;
  int st = update_by_range(m, pts, n, origin ? origin : zero, pose, use_blur != 0, &up);
  if (st != CSM_OK) return st;
  if (updated) *updated = up ? 1 : 0;
  return finish(m);
}

int csm_gridmap_init_with_range_vec(csm_gridmap* m, int32_t n_scans, const double* pts, const int64_t* offsets,
                                    const double* origins, const double* poses, int32_t use_blur,
                                    int32_t speedup) {
  if (!m || n_scans < 0 || (n_scans > 0 && (!offsets || !poses))) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  if (int rst = wait_readers(m)) return rst;
  for (int k = 0; k < n_scans; ++k)
    if (offsets[k + 1] < offsets[k] || (offsets[k + 1] > offsets[k] && !pts)) return CSM_ERR_INVALID_ARG;
  int mode = 0, st;
  if (n_scans > 0 && (st = scan_mode(m, use_blur != 0, &mode)) != CSM_OK)
    return m->fail(st, "update mode not supported (full update with blur, or blur on CountCell)");
  if ((st = flush_pending(m)) != CSM_OK) return st;
  // speedup: ResetValueSpeedup(map_update_point_); else Reset(); then the list is cleared
  m->note_value(m->default_prob);
  GM_HIP(csm::gm_launch_reset(m->cells(), m->ncells(), m->default_prob, speedup != 0, true, m->stream));
  m->cur_update_index = 0;
  m->cur_mark_occu = -1;
  m->cur_mark_free = -1;
  const double zero[2] = {0.0, 0.0};
  for (int k = 0; k < n_scans; ++k) {
    int tries = 5;  // :240-244: the call, then up to 5 retries
    for (;;) {
      bool up = false;
      st = update_by_range(m, pts + 2 * offsets[k], (int)(offsets[k + 1] - offsets[k]),
                           origins ? origins + 2 * k : zero, poses + 3 * k, use_blur != 0, &up);
      if (st != CSM_OK) return st;
      if (up || !tries) break;
      tries--;
    }
  }
  if (!m->auto_resize) {  // UpdateBoundAdaptMap (grid_map_base.h:266-273)
    m->bound.minx = 0.0;
    m->bound.miny = 0.0;
    m->bound.maxx = (double)(m->size_x + 1);
    m->bound.maxy = (double)(m->size_y + 1);
  }
  return finish(m);
}

int csm_gridmap_feedback_penalty(csm_gridmap* m, const double* pts, int32_t n, const double origin[2],
                                 const double best_pose[3], int32_t check_point_num, double bound_tolerance,
                                 double penalty_gain, int32_t use_blur, double* coeff) {
  if (!m || !best_pose || !coeff || n < 0 || (n > 0 && !pts)) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  // MapFeedbackResponsePenalty (occu_grid_map.h:331-392)
  if (bound_tolerance < 0 || check_point_num <= 0 || penalty_gain <= 0.0 || penalty_gain >= 1.0) {
    *coeff = 1.0;
    return CSM_OK;
  }
  const double s = m->scale_factor;
  const double pmx = s * best_pose[0] + s * m->off_x, pmy = s * best_pose[1] + s * m->off_y;
  if (!point_in_map(m, pmx, pmy)) {
    *coeff = 0.0;
    return CSM_OK;
  }
  double c, sn;
  csm::host_sincos(best_pose[2], &sn, &c);
  const double zero[2] = {0.0, 0.0};
  const double* o = origin ? origin : zero;
  double sx, sy;
  pose_apply(c, sn, pmx, pmy, o[0], o[1], sx, sy);
  const int x0 = (int)(sx + 0.5), y0 = (int)(sy + 0.5);
  int step = 1;
  if (n < 2 * check_point_num)
    step = 1;
  else
    step = n / (check_point_num - 1);
  std::vector<GmEnd> rays;
  for (int i = 0; i < n; i += step) {
    double ex, ey;
    pose_apply(c, sn, pmx, pmy, pts[2 * i], pts[2 * i + 1], ex, ey);
    const int x1 = (int)(ex + 0.5), y1 = (int)(ey + 0.5);
    if ((x0 == x1 && y0 == y1) || !point_in_map(m, x1, y1)) continue;
    rays.push_back(GmEnd{x1, y1, 0, 0});
  }
  // smallest integer d2 with sqrt(d2) > bound_tolerance (util::EuclideanDistance2d,
  // slam_util.h:94-96; sqrt is monotonic, so the test is d2 >= min_d2)
  int64_t min_d2 = INT64_MAX;  // NaN or huge tolerance: no cell is ever far enough
  if (bound_tolerance < 1e9) {
    const double t0 = std::floor(bound_tolerance * bound_tolerance) - 2.0;
    min_d2 = t0 > 0.0 ? (int64_t)t0 : 0;
    while (!(std::sqrt((double)min_d2) > bound_tolerance)) ++min_d2;
  }
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;
  int count = 0;
  if (!rays.empty()) {
    if ((st = upload_ends(m, rays)) != CSM_OK) return st;
    GM_HIP(hipMemsetAsync(m->count.p, 0, 4, m->stream));
    GM_HIP(csm::gm_launch_feedback(m->ends.as<GmEnd>(), (int)rays.size(), x0, y0, m->cells(), m->ops,
                                   use_blur ? 1 : 0, m->occu_offset, min_d2, m->count.as<int>(), m->stream));
    GM_HIP(hipMemcpyAsync(&count, m->count.p, 4, hipMemcpyDeviceToHost, m->stream));
    GM_HIP(hipStreamSynchronize(m->stream));
  }
  double penalty = 0;
  for (int i = 0; i < count; ++i) penalty += 1.0;
  penalty *= penalty_gain;
  *coeff = std::max((1.0 + 2 * penalty_gain - penalty), 0.1);
  return CSM_OK;
}

int csm_gridmap_get_state(csm_gridmap* m, csm_gridmap_state* o) {
  if (!m || !o) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  o->resolution = 1 / m->scale_factor;
  o->offset_x = m->off_x;
  o->offset_y = m->off_y;
  o->bound_min_x = m->bound.minx;
  o->bound_min_y = m->bound.miny;
  o->bound_max_x = m->bound.maxx;
  o->bound_max_y = m->bound.maxy;
  o->size_x = m->size_x;
  o->size_y = m->size_y;
  o->map_update_index = m->map_update_index;
  o->cur_update_index = m->cur_update_index;
  o->half_kernel = m->half_kernel;
  o->blur_states = m->blur_states ? 1 : 0;
  o->kind = m->kind;
  o->reserved = 0;
  o->scale_factor = m->scale_factor;
  return CSM_OK;
}

int csm_gridmap_download(csm_gridmap* m, float* prob, float* pass, float* hit, int32_t* uidx, uint8_t* touched) {
  if (!m) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  int st;
  if ((st = flush_pending(m)) != CSM_OK) return st;
  const size_t n = (size_t)m->ncells();
  if (prob) GM_HIP(hipMemcpyAsync(prob, m->prob.p, n * 4, hipMemcpyDeviceToHost, m->stream));
  if (pass) {
    if (m->kind == CSM_COUNT_CELL)
      GM_HIP(hipMemcpyAsync(pass, m->pass.p, n * 4, hipMemcpyDeviceToHost, m->stream));
    else
      std::memset(pass, 0, n * 4);
  }
  if (hit) {
    if (m->kind == CSM_COUNT_CELL)
      GM_HIP(hipMemcpyAsync(hit, m->hit.p, n * 4, hipMemcpyDeviceToHost, m->stream));
    else
      std::memset(hit, 0, n * 4);
  }
  if (uidx) GM_HIP(hipMemcpyAsync(uidx, m->uidx.p, n * 4, hipMemcpyDeviceToHost, m->stream));
  if (touched) GM_HIP(hipMemcpyAsync(touched, m->touched.p, n, hipMemcpyDeviceToHost, m->stream));
  GM_HIP(hipStreamSynchronize(m->stream));
  return CSM_OK;
}

int csm_gridmap_device_prob(csm_gridmap* m, const float** p) {
  if (!m || !p) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  DeviceGuard g(m->device);
  int st = finish(m);
  if (st != CSM_OK) return st;
  *p = m->prob.as<float>();
  return CSM_OK;
}

}  // extern "C"
