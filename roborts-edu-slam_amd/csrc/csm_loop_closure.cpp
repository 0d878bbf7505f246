// csm_loop_closure.cpp — the sharded loop-closure search behind a C-ABI
// (include/csm_loop_closure.h; reference TryCloseLoop,
// pose_graph/range_scan_pose_graph.cpp:299-355). One process drives every
// device: a matcher context per device holds its shard of the submaps, the
// shards are searched concurrently from host threads, and one RCCL
// communicator per device (ncclCommInitAll) agrees on the answer.
#include "csm_loop_closure.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cfloat>
#include <cstddef>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <memory>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "csm_exchange.hpp"

namespace {

// RCCL, resolved from a privately loaded librccl (RTLD_LOCAL): the matcher
// library has no link-time dependency on it, and a host process that
// carries its own RCCL (PyTorch) keeps it.
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool load(std::string& err) {
    if (h) return true;
    for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      err = std::string("cannot load librccl.so.1: ") + dlerror();
      return false;
    }
    CommInitAll = (decltype(CommInitAll))dlsym(h, "ncclCommInitAll");
    CommDestroy = (decltype(CommDestroy))dlsym(h, "ncclCommDestroy");
    AllReduce = (decltype(AllReduce))dlsym(h, "ncclAllReduce");
    GroupStart = (decltype(GroupStart))dlsym(h, "ncclGroupStart");
    GroupEnd = (decltype(GroupEnd))dlsym(h, "ncclGroupEnd");
    GetErrorString = (decltype(GetErrorString))dlsym(h, "ncclGetErrorString");
    if (!CommInitAll || !CommDestroy || !AllReduce || !GroupStart || !GroupEnd || !GetErrorString) {
      err = "librccl.so.1 lacks an NCCL entry point";
      dlclose(h);
      h = nullptr;
      return false;
    }
    return true;
  }
};

Rccl& rccl() {
  static Rccl r;
  return r;
}

// The caller's current device is restored on every return: a host process
// (PyTorch, a ROS node) calling in must not be left on another GPU.
struct DeviceRestore {
  int prev = -1;
  DeviceRestore() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceRestore() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
std::mutex& rccl_mu() {
  static std::mutex m;
  return m;
}

// submaps [lo, hi) of `rank` (contiguous, sizes differ by at most one;
// roborts_csm/loop_closure.py shard_range)
void shard_range(int32_t n, int rank, int world, int32_t* lo, int32_t* hi) {
  const int32_t q = n / world, r = n % world;
  *lo = rank * q + (rank < r ? rank : r);
  *hi = *lo + q + (rank < r ? 1 : 0);
}

// One persistent host thread per device but the first (the caller's thread
// searches device 0's shard): a query wakes them instead of creating and
// joining G - 1 threads (tens of us against a ~0.3 ms query at 8 devices).
class ShardWorkers {
 public:
  explicit ShardWorkers(int n) {
    for (int r = 1; r < n; ++r) th_.emplace_back([this, r] { loop(r); });
  }
  ~ShardWorkers() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(r) for every r in [0, n): r = 0 on the calling thread
  void run(const std::function<void(int)>& fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      pending_ = (int)th_.size();
      ++epoch_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int r) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || epoch_ != seen; });
        if (stop_) return;
        seen = epoch_;
        job = job_;
      }
      (*job)(r);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t epoch_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

}  // namespace

namespace csmh {
int create_context(int device, int local_rank, int local_world, csm_ctx** out);  // csm_api.cpp
}

struct csm_loop_closure {
  std::mutex mu;
  std::string err;
  std::vector<int> devices;
  std::vector<csm_ctx*> ctx;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<csm::LcExchange*> xbuf;  // device, one per device
  csm::LcExchange* h_x = nullptr;      // pinned host staging, one per device
  int32_t n_submaps = 0;
  // A failure after the exchange's first collective was enqueued leaves the
  // communicators out of step: the handle refuses further matches.
  bool broken = false;
  double resolution = 0.0;
  std::vector<double> offsets;
  std::vector<int32_t> lo, hi;
  std::unique_ptr<ShardWorkers> workers;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return CSM_ERR_HIP;
  }
  int nccl_fail(ncclResult_t r, const char* what) {
    err = std::string(what) + ": " + rccl().GetErrorString(r);
    return CSM_ERR_HIP;
  }
};

extern "C" {

int csm_loop_closure_destroy(csm_loop_closure* lc) {
  if (!lc) return CSM_ERR_INVALID_ARG;
  DeviceRestore restore;
  for (size_t r = 0; r < lc->comms.size(); ++r)
    if (lc->comms[r]) (void)rccl().CommDestroy(lc->comms[r]);
  for (size_t r = 0; r < lc->devices.size(); ++r) {
    (void)hipSetDevice(lc->devices[r]);
    if (r < lc->xbuf.size() && lc->xbuf[r]) (void)hipFree(lc->xbuf[r]);
    if (r < lc->streams.size() && lc->streams[r]) (void)hipStreamDestroy(lc->streams[r]);
  }
  lc->workers.reset();
  if (lc->h_x) (void)hipHostFree(lc->h_x);
  for (csm_ctx* c : lc->ctx)
    if (c) csm_destroy(c);
  delete lc;
  return CSM_OK;
}

int csm_loop_closure_create(int32_t n_devices, const int32_t* devices, csm_loop_closure** out) {
  if (!out || n_devices <= 0) return CSM_ERR_INVALID_ARG;
  *out = nullptr;
  DeviceRestore restore;
  csm_loop_closure* lc = new csm_loop_closure();
  for (int r = 0; r < n_devices; ++r) lc->devices.push_back(devices ? devices[r] : r);
  int st;
  {
    std::lock_guard<std::mutex> lk(rccl_mu());
    if (!rccl().load(lc->err)) {
      *out = lc;  // the caller reads csm_loop_closure_last_error, then destroys
      return CSM_ERR_UNSUPPORTED;
    }
  }
  for (int r = 0; r < n_devices; ++r) {
    csm_ctx* c = nullptr;
    // the G contexts share this process's CPUs: host plan of rank r of G
    if ((st = csmh::create_context(lc->devices[r], r, n_devices, &c)) != CSM_OK) {
      lc->err = "csm_create on device " + std::to_string(lc->devices[r]) + " failed";
      *out = lc;
      return st;
    }
    lc->ctx.push_back(c);
    hipError_t e;
    hipStream_t s = nullptr;
    void* x = nullptr;
    if ((e = hipSetDevice(lc->devices[r])) != hipSuccess || (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&x, sizeof(csm::LcExchange))) != hipSuccess) {
      *out = lc;
      return lc->hip_fail(e, "exchange buffers");
    }
    lc->streams.push_back(s);
    lc->xbuf.push_back((csm::LcExchange*)x);
  }
  hipError_t e;
  if ((e = hipHostMalloc((void**)&lc->h_x, sizeof(csm::LcExchange) * n_devices, hipHostMallocDefault)) != hipSuccess) {
    *out = lc;
    return lc->hip_fail(e, "hipHostMalloc(exchange)");
  }
  lc->comms.assign((size_t)n_devices, nullptr);
  ncclResult_t nr = rccl().CommInitAll(lc->comms.data(), n_devices, lc->devices.data());
  if (nr != ncclSuccess) {
    lc->comms.assign((size_t)n_devices, nullptr);
    *out = lc;
    return lc->nccl_fail(nr, "ncclCommInitAll");
  }
  *out = lc;
  return CSM_OK;
}

const char* csm_loop_closure_last_error(const csm_loop_closure* lc) { return lc ? lc->err.c_str() : "null handle"; }

int csm_loop_closure_set_submaps(csm_loop_closure* lc, const float* cells, int32_t n_submaps, const csm_map_info* info,
                                 const double* offsets, int64_t version) {
  if (!lc || !cells || !info || !offsets || n_submaps <= 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(lc->mu);
  DeviceRestore restore;
  const int G = (int)lc->devices.size();
  const int64_t per = (int64_t)info->size_x * info->size_y;
  // the new shard ranges are committed only once every shard is resident: a
  // failed upload leaves no submaps (match then fails with CSM_ERR_NO_GRID)
  // instead of a mix of old and new stacks under the old ranges
  std::vector<int32_t> lo((size_t)G, 0), hi((size_t)G, 0);
  lc->n_submaps = 0;
  for (int r = 0; r < G; ++r) {
    shard_range(n_submaps, r, G, &lo[(size_t)r], &hi[(size_t)r]);
    const int32_t n = hi[(size_t)r] - lo[(size_t)r];
    if (n == 0) continue;
    int st = csm_set_grid_stack(lc->ctx[(size_t)r], cells + lo[(size_t)r] * per, n, info, version);
    if (st != CSM_OK) return lc->fail(st, std::string("device ") + std::to_string(lc->devices[(size_t)r]) + ": " +
                                              csm_last_error(lc->ctx[(size_t)r]));
  }
  lc->lo.swap(lo);
  lc->hi.swap(hi);
  lc->resolution = info->resolution;
  lc->offsets.assign(offsets, offsets + 2 * (size_t)n_submaps);
  lc->n_submaps = n_submaps;
  return CSM_OK;
}

int csm_loop_closure_match(csm_loop_closure* lc, const double* pts, int32_t n_points, const csm_param* param,
                           const double pose_world[3], int32_t search, csm_loop_closure_result* res) {
  if (!lc || !pts || !param || !pose_world || !res) return CSM_ERR_INVALID_ARG;
  if (search != CSM_LC_PYRAMID && search != CSM_LC_EXHAUSTIVE) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(lc->mu);
  DeviceRestore restore;
  if (lc->broken) return lc->fail(CSM_ERR_HIP, "an earlier exchange failed part-way: the communicators are out of step");
  if (lc->n_submaps == 0) return lc->fail(CSM_ERR_NO_GRID, "no submaps set");
  int32_t na = 0, ns = 0;
  if (csm_window_dims(param, &na, &ns) != CSM_OK) return lc->fail(CSM_ERR_INVALID_ARG, "invalid window parameters");
  const int64_t n_cand = (int64_t)na * ns * ns;
  const int G = (int)lc->devices.size();
  // GetMapCoordsPose of the query pose in every submap (grid_map_base.h:68-69,89-93:
  // Scaling(1 / resolution) * Translation(offset), in Eigen's order)
  const double s = 1.0 / lc->resolution;
  std::vector<double> centers(3 * (size_t)lc->n_submaps);
  for (int32_t i = 0; i < lc->n_submaps; ++i) {
    centers[3 * (size_t)i] = s * pose_world[0] + s * lc->offsets[2 * (size_t)i];
    centers[3 * (size_t)i + 1] = s * pose_world[1] + s * lc->offsets[2 * (size_t)i + 1];
    centers[3 * (size_t)i + 2] = pose_world[2];
  }
  using clock = std::chrono::steady_clock;
  const auto ms_since = [](clock::time_point t) {
    return std::chrono::duration<double, std::milli>(clock::now() - t).count();
  };
  const clock::time_point t_search = clock::now();
  // per device: its shard's best, searched concurrently
  std::vector<int> status((size_t)G, CSM_OK);
  std::vector<std::string> errs((size_t)G);
  auto run = [&](int r) {
    csm::LcExchange& x = lc->h_x[r];
    x = csm::LcExchange{};
    x.local_score = -DBL_MAX;
    x.local_idx = -1;
    const int32_t lo = lc->lo[(size_t)r], n = lc->hi[(size_t)r] - lo;
    if (n > 0) {
      std::vector<int32_t> gi((size_t)n);
      for (int32_t i = 0; i < n; ++i) gi[(size_t)i] = i;
      const double* c = centers.data() + 3 * (size_t)lo;
      csm_best b{};
      int32_t w = -1;
      int st;
      if (search == CSM_LC_PYRAMID) {
        st = csm_search_windows(lc->ctx[(size_t)r], pts, n_points, param, n, gi.data(), c, nullptr, &b, &w, nullptr);
      } else {
        std::vector<csm_best> all((size_t)n);
        st = csm_best_windows(lc->ctx[(size_t)r], pts, n_points, param, n, gi.data(), c, all.data());
        for (int32_t i = 0; st == CSM_OK && i < n; ++i) {
          const csm_best& q = all[(size_t)i];
          if (w < 0 || q.score > b.score || (q.score == b.score && (int64_t)i * n_cand + q.flat_index <
                                                                      (int64_t)w * n_cand + b.flat_index)) {
            b = q;
            w = i;
          }
        }
      }
      if (st != CSM_OK) {
        status[(size_t)r] = st;
        errs[(size_t)r] = csm_last_error(lc->ctx[(size_t)r]);
        return;
      }
      x.local_score = b.score;
      x.local_idx = (int64_t)(lo + w) * n_cand + b.flat_index;
      x.local_row[0] = (double)(lo + w);
      x.local_row[1] = b.x;
      x.local_row[2] = b.y;
      x.local_row[3] = b.angle;
    }
    x.score = x.local_score;
  };
  if (!lc->workers) lc->workers.reset(new ShardWorkers(G));
  lc->workers->run(run);
  for (int r = 0; r < G; ++r)
    if (status[(size_t)r] != CSM_OK)
      return lc->fail(status[(size_t)r], "device " + std::to_string(lc->devices[(size_t)r]) + ": " + errs[(size_t)r]);

  const double search_ms = ms_since(t_search);
  const clock::time_point t_exchange = clock::now();
  // the exchange: MAX score -> pick -> MIN index -> row -> SUM row, all enqueued
  hipError_t e;
  ncclResult_t nr;
  Rccl& R = rccl();
  for (int r = 0; r < G; ++r) {
    if ((e = hipSetDevice(lc->devices[(size_t)r])) != hipSuccess) return lc->hip_fail(e, "hipSetDevice");
    if ((e = hipMemcpyAsync(lc->xbuf[(size_t)r], &lc->h_x[r], offsetof(csm::LcExchange, score_max),
                            hipMemcpyHostToDevice, lc->streams[(size_t)r])) != hipSuccess)
      return lc->hip_fail(e, "hipMemcpyAsync(exchange)");
  }
  auto all_reduce = [&](size_t off_in, size_t off_out, size_t count, ncclDataType_t t, ncclRedOp_t op) -> int {
    if ((nr = R.GroupStart()) != ncclSuccess) return lc->nccl_fail(nr, "ncclGroupStart");
    for (int r = 0; r < G; ++r) {
      char* b = (char*)lc->xbuf[(size_t)r];
      if ((nr = R.AllReduce(b + off_in, b + off_out, count, t, op, lc->comms[(size_t)r], lc->streams[(size_t)r])) !=
          ncclSuccess) {
        (void)R.GroupEnd();
        return lc->nccl_fail(nr, "ncclAllReduce");
      }
    }
    if ((nr = R.GroupEnd()) != ncclSuccess) return lc->nccl_fail(nr, "ncclGroupEnd");
    return CSM_OK;
  };
  // From the first collective on, a failure on one device leaves collectives
  // in flight on the others: every stream is drained (best effort; the staging
  // h_x stays untouched until then) and the handle refuses later matches.
  auto abandon = [&](int st) {
    lc->broken = true;
    for (int r = 0; r < G; ++r)
      if (hipSetDevice(lc->devices[(size_t)r]) == hipSuccess) (void)hipStreamSynchronize(lc->streams[(size_t)r]);
    return st;
  };
  int st;
  if ((st = all_reduce(offsetof(csm::LcExchange, score), offsetof(csm::LcExchange, score_max), 1, ncclFloat64,
                       ncclMax)) != CSM_OK)
    return abandon(st);
  for (int r = 0; r < G; ++r) {
    if ((e = hipSetDevice(lc->devices[(size_t)r])) != hipSuccess ||
        (e = csm::launch_lc_pick(lc->xbuf[(size_t)r], lc->streams[(size_t)r])) != hipSuccess)
      return abandon(lc->hip_fail(e, "lc_pick_kernel"));
  }
  if ((st = all_reduce(offsetof(csm::LcExchange, idx), offsetof(csm::LcExchange, idx_min), 1, ncclInt64, ncclMin)) !=
      CSM_OK)
    return abandon(st);
  for (int r = 0; r < G; ++r) {
    if ((e = hipSetDevice(lc->devices[(size_t)r])) != hipSuccess ||
        (e = csm::launch_lc_row(lc->xbuf[(size_t)r], lc->streams[(size_t)r])) != hipSuccess)
      return abandon(lc->hip_fail(e, "lc_row_kernel"));
  }
  if ((st = all_reduce(offsetof(csm::LcExchange, row), offsetof(csm::LcExchange, row_sum), 4, ncclFloat64,
                       ncclSum)) != CSM_OK)
    return abandon(st);
  csm::LcExchange* out = &lc->h_x[0];
  if ((e = hipSetDevice(lc->devices[0])) != hipSuccess ||
      (e = hipMemcpyAsync(out, lc->xbuf[0], sizeof(csm::LcExchange), hipMemcpyDeviceToHost, lc->streams[0])) !=
          hipSuccess)
    return abandon(lc->hip_fail(e, "hipMemcpyAsync(exchange result)"));
  for (int r = 0; r < G; ++r) {
    if ((e = hipSetDevice(lc->devices[(size_t)r])) != hipSuccess ||
        (e = hipStreamSynchronize(lc->streams[(size_t)r])) != hipSuccess)
      return abandon(lc->hip_fail(e, "exchange"));
  }
  res->search_ms = search_ms;
  res->exchange_ms = ms_since(t_exchange);
  res->n_devices = G;
  res->score = out->score_max;
  const bool none = out->idx_min == INT64_MAX;
  res->global_index = none ? -1 : out->idx_min;
  res->submap = none ? -1 : (int32_t)out->row_sum[0];
  res->x = out->row_sum[1];
  res->y = out->row_sum[2];
  res->angle = out->row_sum[3];
  // GetWorldCoordsPose of the winner in its submap (grid_map_base.h:83-87; csm_api.cpp Geometry)
  if (!none) {
    const double tx = s * lc->offsets[2 * (size_t)res->submap], ty = s * lc->offsets[2 * (size_t)res->submap + 1];
    const double inv_a = s * (1.0 / (s * s - 0.0 * 0.0));
    const double ntx = -(inv_a * tx), nty = -(inv_a * ty);
    res->pose_world[0] = inv_a * res->x + ntx;
    res->pose_world[1] = inv_a * res->y + nty;
    res->pose_world[2] = res->angle;
  }
  return CSM_OK;
}

}  // extern "C"
