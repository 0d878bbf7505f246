// Compile check of include/csm_reference_adapter.hpp against minimal stand-ins
// for the reference-side types it is templated on (our own test types, not the
// reference's headers).
#include <array>
#include <memory>
#include "csm_reference_adapter.hpp"

struct Vec2 { double a[2]; double x() const { return a[0]; } double y() const { return a[1]; } };
struct Vec3 { double a[3]; double& operator[](int i) { return a[i]; } };
struct Mat3 { double a[9]; double& operator()(int r, int c) { return a[3 * r + c]; } };
struct Cell { float prob_value_; int update_index_; };
struct Map {
  std::vector<Cell> cells = std::vector<Cell>(16, Cell{0.3f, -1});
  int GetSizeX() const { return 4; }
  int GetSizeY() const { return 4; }
  double GetCellLength() const { return 0.05; }
  bool IsMapInit() const { return true; }
  int map_update_index() const { return 0; }
  const Cell* GetCellData() const { return cells.data(); }
};
struct Range {
  std::vector<Vec2> pts;
  int GetSize() const { return (int)pts.size(); }
  const Vec2& GetDataPoint(int i) const { return pts[(size_t)i]; }
};
enum Type { COARSE = 0 };
struct Param {
  double search_space_size() const { return 0.6; }
  double search_space_resolution() const { return 0.05; }
  double search_angle_offset() const { return 0.523; }
  double search_angle_resolution() const { return 0.0349; }
  double response_threshold() const { return 0.6; }
  int use_point_size() const { return 100; }
  int max_depth() const { return 0; }
  bool use_center_penalty() const { return true; }
  Type correlation_scan_match_type() const { return COARSE; }
};

int main() {
  auto off = [](const Map&) { return std::array<double, 2>{0.0, 0.0}; };
  using M = roborts_csm::BasedCorrelationScanMatchGpu<Map, Range, Param, Vec3, Mat3, decltype(off)>;
  M* m = nullptr;  // construction needs a GPU; this file only has to compile
  (void)m;
  csm_param p = roborts_csm::to_csm_param(Param());
  return p.use_point_size == 100 ? 0 : 1;
}
