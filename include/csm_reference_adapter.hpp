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
// Map access: the adapter uploads the grid through csm_set_grid with the
// reference's 8-byte ProbabilityCell stride. GridMapBase keeps grid_cell_
// private (grid_map_base.h:383), so the maintainer adds one accessor there:
//     const CellType* GetCellData() const { return grid_cell_; }
// The device copy is keyed on (cell pointer, size, map_update_index()): a map
// updated in place must bump map_update_index() (SetUpdated, :369) — which
// the reference does after every UpdateMap — and an ExtendSize reallocation
// changes the pointer and size, so both force a re-upload.
//
// Template parameters keep this header free of the reference's own headers:
//   MapT   : GetSizeX(), GetSizeY(), GetCellLength(), IsMapInit(),
//            map_update_index(), GetCellData(), GetMapCoordsPose(), plus the
//            map offset through MapOffset(map) (a free function the maintainer
//            defines from GridMapBase's map_offset_).
//   RangeT : GetSize(), GetDataPoint(i) -> Eigen::Vector2d-like (x(), y()).
//   ParamT : CorrelationScanMatchParam's getters.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>
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

class DeviceContext {
 public:
  explicit DeviceContext(int device = 0) {
    if (csm_create(device, &ctx_) != CSM_OK) throw std::runtime_error("csm_create failed");
  }
  ~DeviceContext() { csm_destroy(ctx_); }
  DeviceContext(const DeviceContext&) = delete;
  DeviceContext& operator=(const DeviceContext&) = delete;
  csm_ctx* get() const { return ctx_; }
  std::string last_error() const { return csm_last_error(ctx_); }

 private:
  csm_ctx* ctx_ = nullptr;
};

// Drop-in for roborts_slam::BasedCorrelationScanMatch.
template <class MapT, class RangeT, class ParamT, class Vec3, class Mat3, class OffsetFn>
class BasedCorrelationScanMatchGpu {
 public:
  BasedCorrelationScanMatchGpu(std::shared_ptr<DeviceContext> device, OffsetFn map_offset)
      : dev_(std::move(device)), map_offset_(map_offset) {}

  double ScanMatch(std::shared_ptr<MapT> map, std::shared_ptr<RangeT> range_data,
                   std::shared_ptr<ParamT> scan_match_param, Vec3& current_pose, Mat3& cov_matrix) {
    const int n = range_data->GetSize();
    points_.resize(static_cast<size_t>(n) * 2);
    for (int i = 0; i < n; ++i) {
      const auto& p = range_data->GetDataPoint(i);
      points_[2 * i] = p.x();
      points_[2 * i + 1] = p.y();
    }
    csm_map_info info;
    info.resolution = map->GetCellLength();
    const auto off = map_offset_(*map);
    info.offset_x = off[0];
    info.offset_y = off[1];
    info.size_x = map->GetSizeX();
    info.size_y = map->GetSizeY();
    info.update_index = map->map_update_index();
    info.reserved = 0;
    // ProbabilityCell {float prob_value_; int update_index_;} (grid_map_cell.h:301-328)
    const void* cells = static_cast<const void*>(map->GetCellData());
    if (csm_set_grid(dev_->get(), cells, 8, &info, map->map_update_index()) != CSM_OK)
      throw std::runtime_error(dev_->last_error());
    double pose[3] = {current_pose[0], current_pose[1], current_pose[2]};
    double cov[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) cov[3 * r + c] = cov_matrix(r, c);
    const csm_param p = to_csm_param(*scan_match_param);
    double response = 0.0;
    if (csm_scan_match(dev_->get(), points_.data(), n, &p, pose, cov, &response, nullptr) != CSM_OK)
      throw std::runtime_error(dev_->last_error());
    current_pose[0] = pose[0];
    current_pose[1] = pose[1];
    current_pose[2] = pose[2];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) cov_matrix(r, c) = cov[3 * r + c];
    return response;
  }

 private:
  std::shared_ptr<DeviceContext> dev_;
  OffsetFn map_offset_;
  std::vector<double> points_;
};

}  // namespace roborts_csm
