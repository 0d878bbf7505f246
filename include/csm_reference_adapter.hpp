// csm_reference_adapter.hpp — drop-in replacement for the reference's
// BasedCorrelationScanMatch (src/scan_match/correlate_scan_matcher.h:766-1036)
// on top of the C-ABI in csm.h. Header-only C++14, no dependency beyond what
// the reference already has (Eigen, its map and range-data types).
//
// The class keeps the reference's exact entry-point signature
//   double ScanMatch(std::shared_ptr<ScanMatchMap>, std::shared_ptr<RangeDataContainer2d>,
//                    std::shared_ptr<CorrelationScanMatchParam>, Eigen::Vector3d&, Eigen::Matrix3d&)
// (correlate_scan_matcher.h:784-788), so ScanMatchers (scan_matchers.h:238,249,256),
// SlamProcessor and the pose-graph back-end stay untouched.
//
// Error convention (correlate_scan_matcher.h:790-795): the reference never
// throws here; on an invalid map or scan it logs a warning and returns
// kMinResponse = 0.0 with the pose and covariance untouched. The adapter does
// the same for every library failure (no device, HIP error): it logs through
// the adapter's log hook (default: stderr; point it at glog's LOG(WARNING)) and
// returns 0.0, pose and covariance untouched. Nothing here throws.
//
// Map residency:
//  * The grid is read through GetCellData() with the reference's 8-byte
//    ProbabilityCell stride; the library keeps up to four maps resident,
//    keyed on that pointer, so the front end's fine map and the back end's
//    maps (ScanMatchInterface) do not evict each other.
//  * A map that also exposes GetCellGeneration() (an integer the reference
//    side bumps whenever the cell buffer is allocated: AllocateGridCell and
//    ExtendSize, grid_map_base.h:152-166,186-254) is keyed on (cell pointer,
//    size, generation): a freed buffer reused at the same address by another
//    map is then never refreshed incrementally against the old map's device
//    copy. Without it the key is (cell pointer, size), and a reuse at the same
//    address and size is detected only through the update list and reset count.
//  * When the map also exposes GetUpdatePoints() (the reference's
//    map_update_point_, occu_grid_map.h:589: every cell UpdateMapByRange
//    writes is appended, :509,528,571) and GetResetCount() (bumped by
//    Reset / ResetValueSpeedup, grid_map_base.h:95-120), only the cells
//    appended since the previous call are re-read (csm_update_grid_cells).
//    A reset, a new cell buffer or a new size (ExtendSize, :186-254)
//    re-uploads the whole grid.
//  * Without those accessors the grid is re-uploaded whenever
//    map_update_index() changes (csm_set_grid; packed on the library's host
//    threads).
//
// Template parameters keep this header free of the reference's own headers:
//   MapT   : GetSizeX(), GetSizeY(), GetCellLength(), map_update_index(),
//            GetCellData(); optionally GetUpdatePoints() -> const std::vector<int>&
//            and GetResetCount() -> integer. The map offset comes through
//            OffsetFn (GridMapBase's map_offset_).
//   RangeT : GetSize(), GetDataPoint(i) -> Eigen::Vector2d-like (x(), y()).
//   ParamT : CorrelationScanMatchParam's getters.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "csm.h"

namespace roborts_csm {

template <class ParamT>
inline csm_param to_csm_param(const ParamT& p) {
  csm_param c;
  c.search_space_size = p.search_space_size();
  c.search_space_resolution = p.search_space_resolution();
  c.search_angle_offset = p.search_angle_offset();
  c.search_angle_resolution = p.search_angle_resolution();
  c.response_threshold = p.response_threshold();
  c.use_point_size = p.use_point_size();
  c.max_depth = p.max_depth();
  c.use_center_penalty = p.use_center_penalty() ? 1 : 0;
  c.type = static_cast<int32_t>(p.correlation_scan_match_type());
  return c;
}

// Log hook for warnings (the reference logs with glog's LOG(WARNING)).
using LogFn = void (*)(const char* message);
inline void default_log(const char* message) { std::fprintf(stderr, "[roborts_csm] WARNING: %s\n", message); }

// One library context (one HIP stream and its device buffers) on one GPU.
// Construction never throws: ok() is false when the device is unusable, and
// every match through it then logs and returns 0.0.
class DeviceContext {
 public:
  explicit DeviceContext(int device = 0) {
    status_ = csm_create(device, &ctx_);
    if (status_ != CSM_OK) ctx_ = nullptr;
  }
  ~DeviceContext() {
    if (ctx_) csm_destroy(ctx_);
  }
  DeviceContext(const DeviceContext&) = delete;
  DeviceContext& operator=(const DeviceContext&) = delete;
  bool ok() const { return ctx_ != nullptr; }
  csm_ctx* get() const { return ctx_; }
  std::string last_error() const {
    return ctx_ ? std::string(csm_last_error(ctx_))
                : "csm_create failed (status " + std::to_string(status_) + "): no usable MI355X device";
  }

 private:
  csm_ctx* ctx_ = nullptr;
  int status_ = CSM_OK;
};

namespace detail {
template <class...>
struct voider {
  using type = void;
};
template <class M, class = void>
struct has_update_points : std::false_type {};
template <class M>
struct has_update_points<M, typename voider<decltype(std::declval<const M&>().GetUpdatePoints()),
                                            decltype(std::declval<const M&>().GetResetCount())>::type>
    : std::true_type {};
template <class M, class = void>
struct has_cell_generation : std::false_type {};
template <class M>
struct has_cell_generation<M, typename voider<decltype(std::declval<const M&>().GetCellGeneration())>::type>
    : std::true_type {};
template <class M>
int64_t cell_generation(const M& m, std::true_type) {
  return static_cast<int64_t>(m.GetCellGeneration());
}
template <class M>
int64_t cell_generation(const M&, std::false_type) {
  return -1;
}
}  // namespace detail

// Drop-in for roborts_slam::BasedCorrelationScanMatch.
template <class MapT, class RangeT, class ParamT, class Vec3, class Mat3, class OffsetFn>
class BasedCorrelationScanMatchGpu {
 public:
  BasedCorrelationScanMatchGpu(std::shared_ptr<DeviceContext> device, OffsetFn map_offset, LogFn log = default_log)
      : dev_(std::move(device)), map_offset_(map_offset), log_(log ? log : default_log) {}

  double ScanMatch(std::shared_ptr<MapT> map, std::shared_ptr<RangeT> range_data,
                   std::shared_ptr<ParamT> scan_match_param, Vec3& current_pose, Mat3& cov_matrix) {
    if (!dev_ || !dev_->ok()) return warn(dev_ ? dev_->last_error() : std::string("no device context"));
    if (!map || !range_data || !scan_match_param) return warn("null map, range data or parameters");
    const int n = range_data->GetSize();
    points_.resize(static_cast<size_t>(n) * 2);
    for (int i = 0; i < n; ++i) {
      const auto& p = range_data->GetDataPoint(i);
      points_[2 * i] = p.x();
      points_[2 * i + 1] = p.y();
    }
    if (!refresh_grid(*map)) return warn(dev_->last_error());
    double pose[3] = {current_pose[0], current_pose[1], current_pose[2]};
    double cov[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) cov[3 * r + c] = cov_matrix(r, c);
    const csm_param p = to_csm_param(*scan_match_param);
    double response = 0.0;
    if (csm_scan_match(dev_->get(), points_.data(), n, &p, pose, cov, &response, nullptr) != CSM_OK)
      return warn(dev_->last_error());
    current_pose[0] = pose[0];
    current_pose[1] = pose[1];
    current_pose[2] = pose[2];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) cov_matrix(r, c) = cov[3 * r + c];
    return response;
  }

  // Cells re-read by the last refresh (-1: whole grid, 0: none); for tests.
  int64_t last_refresh_cells() const { return last_refresh_; }

 private:
  struct MapState {
    int32_t size_x = -1, size_y = -1;
    int64_t reset_count = -1;
    int64_t generation = -1;  // GetCellGeneration(), or -1 without the accessor
    size_t points_seen = 0;
    int32_t update_index = -1;
  };

  double warn(const std::string& what) {
    const std::string m = "correlative scan match on the device failed: " + what + "; returning 0.0";
    log_(m.c_str());
    return 0.0;  // kMinResponse (correlate_scan_matcher.h:1034), pose and covariance untouched
  }

  csm_map_info info_of(const MapT& map) const {
    csm_map_info info;
    info.resolution = map.GetCellLength();
    const auto off = map_offset_(map);
    info.offset_x = off[0];
    info.offset_y = off[1];
    info.size_x = map.GetSizeX();
    info.size_y = map.GetSizeY();
    info.update_index = map.map_update_index();
    info.reserved = 0;
    return info;
  }

  // ProbabilityCell {float prob_value_; int update_index_;} (grid_map_cell.h:301-328)
  bool refresh_grid(const MapT& map) { return refresh_grid(map, detail::has_update_points<MapT>()); }

  bool refresh_grid(const MapT& map, std::false_type) {
    const csm_map_info info = info_of(map);
    const void* cells = static_cast<const void*>(map.GetCellData());
    last_refresh_ = -1;
    return csm_set_grid(dev_->get(), cells, 8, &info, map.map_update_index()) == CSM_OK;
  }

  bool refresh_grid(const MapT& map, std::true_type) {
    const csm_map_info info = info_of(map);
    const void* cells = static_cast<const void*>(map.GetCellData());
    const std::vector<int>& pts = map.GetUpdatePoints();
    const int64_t resets = static_cast<int64_t>(map.GetResetCount());
    const int64_t gen = detail::cell_generation(map, detail::has_cell_generation<MapT>());
    MapState& s = maps_[cells];
    int st;
    if (s.size_x == info.size_x && s.size_y == info.size_y && s.reset_count == resets && s.generation == gen &&
        pts.size() >= s.points_seen) {
      if (s.update_index == info.update_index && pts.size() == s.points_seen) {
        last_refresh_ = 0;
        st = csm_set_grid(dev_->get(), cells, 8, &info, info.update_index);  // resident: no copy
      } else {
        const int64_t fresh = static_cast<int64_t>(pts.size() - s.points_seen);
        last_refresh_ = fresh;
        st = csm_update_grid_cells(dev_->get(), cells, 8, &info, info.update_index,
                                   reinterpret_cast<const int32_t*>(pts.data()) + s.points_seen, fresh);
      }
    } else {
      last_refresh_ = -1;
      st = csm_set_grid(dev_->get(), cells, 8, &info, -1);
    }
    if (st != CSM_OK) {
      maps_.erase(cells);
      return false;
    }
    s.size_x = info.size_x;
    s.size_y = info.size_y;
    s.reset_count = resets;
    s.generation = gen;
    s.points_seen = pts.size();
    s.update_index = info.update_index;
    if (maps_.size() > 8) {  // forget maps that are gone (ExtendSize frees the old buffer)
      auto keep = std::move(s);
      maps_.clear();
      maps_[cells] = keep;
    }
    return true;
  }

  std::shared_ptr<DeviceContext> dev_;
  OffsetFn map_offset_;
  LogFn log_;
  std::vector<double> points_;
  std::map<const void*, MapState> maps_;
  int64_t last_refresh_ = 0;
};

}  // namespace roborts_csm
