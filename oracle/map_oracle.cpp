// map_oracle.cpp — CPU restatement of RoboRTS-Edu-SLAM's occupancy-grid map
// building and of the post-match map check (row f4).
//
// *** TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT. ***
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library (oracle/build/liboracle.so), as the checker / CPU
// baseline. The product (libroborts_csm.so) never links, loads or calls it.
//
// PARITY UNPINNED by the reference: it ships no tests for map building and
// cannot be compiled here (Eigen3, glog, boost, ROS absent).
// This file is a sequential, call-for-call restatement of
//   map/occu_grid_map.h      GaussianBlur :38-115, LineVisitor (Bresenham) :119-192,
//                            InitMapWithRangeVec :222-255, UpdateMapByRange :258-329,
//                            MapFeedbackResponsePenalty :331-392, CellUpdate and the
//                            Set* cell updates :474-576
//   map/grid_map_cell.h      ProbabilityCell(+Functions) :301-388, CountCell(+Functions) :42-161
//   map/grid_map_base.h      Reset/ResetValueSpeedup :95-112, AllocateGridCell :152-166,
//                            ExtendSize :182-244, UpdateBound :247-264, UpdateBoundAdaptMap
//                            :266-273, set_map_offset :275-279, PointInMap :336-352
//   util/boundbox.h          BoundBox :35-143
//   slam/sensor_data_manager.h  CreateFrom / TransformLocalToMap :99-175
// with the reference's evaluation order (g++ -O2 -ffp-contract=off, no FMA),
// and it is cross-checked against an independent Python restatement
// (tests/map_pyref.py) in the CPU tests.
//
// Reference behaviour kept on purpose (it changes results):
//  * `new CellType[n]{default_cell_prob_}` (grid_map_base.h:160,214) initialises
//    only element 0 from default_cell_prob_; every other element is
//    value-initialised by the default constructor, i.e. kDefaultCellProb = 0.5f
//    (grid_map_cell.h:30). Maps that are never Reset() keep that pattern.
//  * map_update_point_ holds linear indices; ExtendSize does not remap them, so a
//    later ResetValueSpeedup resets the cells now at those indices.
//  * UpdateMapByRange returns false (nothing drawn) when the scan forced a resize.
// Definitions where the reference is undefined:
//  * An empty scan with auto-resize on: the reference would grow the map to a
//    FLT_MAX box (UB); here the bound step is skipped.
//  * MapFeedbackResponsePenalty reading a line cell outside the grid (possible
//    only when the start cell rounds onto the map's far edge): such a cell is
//    not occupied.

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>

#include "oracle_math.hpp"

namespace {

constexpr float kDefaultCellProb = 0.5f;  // grid_map_cell.h:30

enum CellKind { kProbabilityCell = 0, kCountCell = 1 };
enum UpdateType { kSetFree = 0, kSetOccupied = 1, kSetOccupiedBlur = 2 };  // occu_grid_map.h:32-36
enum GridState { kUnknown = -1, kOccupied = 100, kFree = 0 };              // grid_map_cell.h:32-37

// Superset of ProbabilityCell {prob, update_index} and CountCell
// {pass, hit, prob, update_index}; ProbabilityCell leaves pass/hit at 0.
struct Cell {
  float prob = kDefaultCellProb;
  float pass = 0.0f;
  float hit = 0.0f;
  int32_t uidx = -1;
};

// BoundBox<double> (util/boundbox.h:35-143). Default max is FLT_MIN (the
// smallest positive normal float), as in the reference.
struct Box {
  double minx = (double)FLT_MAX, miny = (double)FLT_MAX;
  double maxx = (double)FLT_MIN, maxy = (double)FLT_MIN;
  void reset() { *this = Box(); }
  void add(double x, double y) {  // AddPoint :100-106
    if (x < minx) minx = x;
    if (y < miny) miny = y;
    if (x > maxx) maxx = x;
    if (y > maxy) maxy = y;
  }
  void add_box(const Box& b) {  // AddBoundBox :120-124
    add(b.minx, b.miny);
    add(b.maxx, b.maxy);
  }
  void extend(double e) {  // ExtendBoundBox :126-129
    minx -= e;
    miny -= e;
    maxx += e;
    maxy += e;
  }
  bool in(double x, double y) const {  // IsInBounds :131-135
    return x > minx && x < maxx && y > miny && y < maxy;
  }
  int size_x() const { return (int)(std::ceil(maxx) - std::floor(minx)); }  // GetBoxSize :78-83
  int size_y() const { return (int)(std::ceil(maxy) - std::floor(miny)); }
};

struct OMap {
  int kind = kProbabilityCell;
  // GridMapBase
  double scale_factor = 1.0;
  int size_x = 0, size_y = 0;  // map_size_
  int row = 0;                 // size_x_ (row length used by GetCell)
  double off_x = 0.0, off_y = 0.0;
  Box bound;
  double extend_factor = 1.0;
  float default_prob = kDefaultCellProb;
  int map_update_index = -1;
  std::vector<Cell> cells;
  // GaussianBlur (occu_grid_map.h:38-115)
  bool blur_states = false;
  int half_kernel = 0, kernel_size = 0;
  std::vector<double> kernel;
  // OccuGridMap
  bool use_blur = false;
  bool auto_resize = true;
  bool just_update_occu = false;
  int cur_update_index = 0, cur_mark_occu = -1, cur_mark_free = -1;
  double occu_offset = 0.72;  // cell_occu_prob_offset_ (:601)
  std::vector<int> update_points;
  double bound_tolerance = 0.0;
  int cur_end_x = 0, cur_end_y = 0;
  // cell functions (grid_map_cell.h:82-92, 207-214, 330-337)
  float occu_factor = 0.5f, free_factor = 0.2f, occu_threshold = 0.5f, min_pass = 2.0f;
};

Cell fresh_cell(const OMap& m, int64_t i) {  // `new CellType[n]{default}` (grid_map_base.h:160,214)
  Cell c;
  c.prob = i == 0 ? m.default_prob : kDefaultCellProb;
  return c;
}

void reset_cell(const OMap& m, Cell& c) {  // ResetGridCell (grid_map_cell.h:64-69, 318-322)
  c.prob = m.default_prob;
  c.pass = 0.0f;
  c.hit = 0.0f;
  c.uidx = -1;
}

// ---- cell functions ----------------------------------------------------------
void set_occupied(const OMap& m, Cell& c) {
  if (m.kind == kCountCell) {  // CountCellFunctions::UpdateSetOccupied :94-101
    c.hit += (1.0f + m.occu_factor);
    c.pass += (1.0f + m.free_factor);
    c.prob = c.hit / c.pass;
    if (c.prob > 1.0f) c.prob = 1.0f;
  } else {  // ProbabilityCellFunctions::UpdateSetOccupied :339-343
    float v = c.prob + m.occu_factor;
    if (v > 1.0f) v = 1.0f;
    c.prob = v;
  }
}
void set_free(const OMap& m, Cell& c) {
  if (m.kind == kCountCell) {  // :103-106
    c.pass += (1.0f + m.free_factor);
    c.prob = c.hit / c.pass;
  } else {  // :345-349
    float v = c.prob - m.free_factor;
    if (v < 0.0f) v = 0.0f;
    c.prob = v;
  }
}
void unset_free(const OMap& m, Cell& c) {
  if (m.kind == kCountCell) {  // :108-111
    c.pass -= (1.0f + m.free_factor);
    c.prob = c.hit / c.pass;
  } else {  // :351-355
    float v = c.prob + m.free_factor;
    if (v > 1.0f) v = 1.0f;
    c.prob = v;
  }
}
void set_probability(const OMap& m, Cell& c, float p) {
  if (m.kind == kCountCell) {  // :117-123
    if (c.prob < p) {
      c.prob = p;
      c.hit = p * c.pass;
    }
  } else if (c.prob < p && p <= 1.0f) {  // :361-365
    c.prob = p;
  }
}
int grid_state(const OMap& m, const Cell& c) {
  if (m.kind == kCountCell) {  // :125-136
    if (c.pass >= m.min_pass) return c.prob < m.occu_threshold ? kFree : kOccupied;
    return kUnknown;
  }
  if (c.prob < 0.5f) return kFree;  // :367-375
  if (c.prob > 0.5f) return kOccupied;
  return kUnknown;
}

// ---- GridMapBase -----------------------------------------------------------------
Cell& cell_at(OMap& m, int x, int y) { return m.cells[(size_t)((int64_t)y * m.row + x)]; }
int grid_index(const OMap& m, int x, int y) { return y * m.row + x; }

bool point_in_map(const OMap& m, double x, double y, double tol = 0.0) {  // :344-352
  return x > tol && x < m.size_x - tol && y > tol && y < m.size_y - tol;
}

void allocate(OMap& m, int sx, int sy) {  // AllocateGridCell :152-166
  const int64_t n = (int64_t)sx * sy;
  m.cells.resize(n > 0 ? (size_t)n : 0);
  for (int64_t i = 0; i < n; ++i) m.cells[(size_t)i] = fresh_cell(m, i);
  m.size_x = sx;
  m.size_y = sy;
}

void extend_size(OMap& m) {  // ExtendSize(EXTEND_PARTLY) :182-244
  Box t;
  t.add_box(m.bound);
  const double map_min_x = 0.0, map_min_y = 0.0;
  const double map_max_x = (double)m.size_x, map_max_y = (double)m.size_y;
  t.add(map_min_x, map_min_y);
  t.add(map_max_x, map_max_y);
  double min_x = t.minx, min_y = t.miny, max_x = t.maxx, max_y = t.maxy;
  if (m.bound.minx <= map_min_x) min_x -= (double)t.size_x() * m.extend_factor;
  if (m.bound.miny <= map_min_y) min_y -= (double)t.size_y() * m.extend_factor;
  if (m.bound.maxx >= map_max_x) max_x += (double)t.size_x() * m.extend_factor;
  if (m.bound.maxy >= map_max_y) max_y += (double)t.size_y() * m.extend_factor;
  t.add(min_x, min_y);
  t.add(max_x, max_y);
  const double fx = std::floor(t.minx), fy = std::floor(t.miny);
  m.off_x -= fx / m.scale_factor;
  m.off_y -= fy / m.scale_factor;
  const int gx = -(int)fx, gy = -(int)fy;
  const int pre_row = m.row, pre_sy = m.size_y;
  const int nsx = t.size_x(), nsy = t.size_y();
  std::vector<Cell> old;
  old.swap(m.cells);
  m.row = nsx;
  const int64_t n = (int64_t)nsx * nsy;
  m.cells.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) m.cells[(size_t)i] = fresh_cell(m, i);
  for (int r = 0; r < pre_sy; ++r)
    std::memcpy(&m.cells[(size_t)((int64_t)(gy + r) * nsx + gx)], &old[(size_t)((int64_t)r * pre_row)],
                sizeof(Cell) * (size_t)pre_row);
  m.size_x = nsx;
  m.size_y = nsy;
  Box nb;
  nb.minx = m.bound.minx - t.minx;
  nb.miny = m.bound.miny - t.miny;
  nb.maxx = m.bound.maxx - t.minx;
  nb.maxy = m.bound.maxy - t.miny;
  m.bound = nb;
}

bool update_bound(OMap& m, const Box& b) {  // UpdateBound :247-264
  if (m.bound.in(b.minx, b.miny) && m.bound.in(b.maxx, b.maxy)) return true;
  m.bound.add_box(b);
  if (!point_in_map(m, m.bound.minx, m.bound.miny) || !point_in_map(m, m.bound.maxx, m.bound.maxy)) {
    extend_size(m);
    return false;
  }
  return true;
}

// GetMapCoordsPose (grid_map_base.h:89-93): Scaling(s) * Translation(o).
void world_to_map(const OMap& m, const double w[3], double out[3]) {
  const double s = m.scale_factor;
  out[0] = s * w[0] + s * m.off_x;
  out[1] = s * w[1] + s * m.off_y;
  out[2] = w[2];
}

// ---- OccuGridMap --------------------------------------------------------------------
void init_kernel(OMap& m, double sigma, double res) {  // GaussianBlur :40-105
  if (sigma > 0.5 * res && sigma < 10 * res && res > 0) {
    m.blur_states = true;
    m.half_kernel = (int)((sigma / res) * std::sqrt(std::log(2)));
    m.kernel_size = m.half_kernel * 2 + 1;
    m.kernel.assign((size_t)m.kernel_size * m.kernel_size, 0.0);
    for (int i = -m.half_kernel; i <= m.half_kernel; ++i)
      for (int j = -m.half_kernel; j <= m.half_kernel; ++j) {
        const double d = std::hypot(i * res, j * res);
        const double q = d / sigma;
        m.kernel[(size_t)((i + m.half_kernel) + m.kernel_size * (j + m.half_kernel))] = std::exp(-0.5 * (q * q));
      }
  } else {
    m.blur_states = false;
    m.half_kernel = 0;
    m.kernel_size = 0;
  }
}

void set_cell_free(OMap& m, int x, int y) {  // :499-510
  Cell& c = cell_at(m, x, y);
  if (c.uidx < m.cur_mark_free) {
    set_free(m, c);
    c.uidx = m.cur_mark_free;
  }
  m.update_points.push_back(grid_index(m, x, y));
}

void set_cell_occu(OMap& m, int x, int y) {  // :512-529
  Cell& c = cell_at(m, x, y);
  if (c.uidx < m.cur_mark_occu) {
    if (c.uidx == m.cur_mark_free) unset_free(m, c);
    set_occupied(m, c);
    c.uidx = m.cur_mark_occu;
  }
  m.update_points.push_back(grid_index(m, x, y));
}

void set_cell_occu_blur(OMap& m, int x, int y) {  // :531-576
  Cell& center = cell_at(m, x, y);
  if (center.uidx < m.cur_mark_occu) {
    if (!m.just_update_occu) {
      if (center.uidx == m.cur_mark_free) unset_free(m, center);
      set_occupied(m, center);
      center.uidx = m.cur_mark_occu;
    } else {
      set_probability(m, center, 1.0f);
    }
    const int hk = m.half_kernel, ks = m.kernel_size;
    for (int j = -hk; j <= hk; ++j)
      for (int i = -hk; i <= hk; ++i) {
        const int k = (i + hk) + ks * (j + hk);
        set_probability(m, cell_at(m, x + i, y + j), (float)(m.kernel[(size_t)k] * m.occu_offset));
        m.update_points.push_back(grid_index(m, x + i, y + j));
      }
  }
}

void cell_update(OMap& m, int x, int y, int type) {  // CellUpdate :474-497
  if (!point_in_map(m, x, y, m.half_kernel + 1)) return;
  if (type == kSetFree)
    set_cell_free(m, x, y);
  else if (type == kSetOccupied)
    set_cell_occu(m, x, y);
  else
    set_cell_occu_blur(m, x, y);
}

// LineVisitor::ErgodLineBresenhami (occu_grid_map.h:125-188): visit(x, y)
// for each cell in the reference's order.
template <class F>
void bresenham(int x0, int y0, int x1, int y1, F&& visit) {
  const bool steep = std::abs(y1 - y0) > std::abs(x1 - x0);
  if (steep) {
    std::swap(x0, y0);
    std::swap(x1, y1);
  }
  if (x0 > x1) {
    std::swap(x0, x1);
    std::swap(y0, y1);
  }
  const int dx = x1 - x0, dy = std::abs(y1 - y0);
  int err = 0, y = y0;
  const int ystep = y0 < y1 ? 1 : -1;
  for (int x = x0; x <= x1; ++x) {
    if (steep)
      visit(y, x);
    else
      visit(x, y);
    err += dy;
    if (2 * err >= dx) {
      y += ystep;
      err -= dx;
    }
  }
}

// Affine2d(Translation2d(t) * Rotation2Dd(th)) applied to p: linear * p + t with
// linear = [c -s; s c] (Rotation2D::toRotationMatrix), Eigen's
// translation-then-add-product order.
inline void pose_apply(double c, double s, double tx, double ty, double px, double py, double& ox, double& oy) {
  ox = (c * px + (-s) * py) + tx;
  oy = (s * px + c * py) + ty;
}

bool update_by_range(OMap& m, const double* pts, int n, const double origin[2], const double pose[3],
                     bool use_blur) {  // UpdateMapByRange :258-329
  if (!m.blur_states) use_blur = false;
  m.use_blur = use_blur;
  m.cur_mark_free = m.cur_update_index + 1;
  m.cur_mark_occu = m.cur_update_index + 2;
  double pm[3];
  world_to_map(m, pose, pm);
  double c, s;
  ref_sincos(pm[2], &s, &c);
  std::vector<double> tp((size_t)2 * (n > 0 ? n : 0));
  for (int i = 0; i < n; ++i) pose_apply(c, s, pm[0], pm[1], pts[2 * i], pts[2 * i + 1], tp[2 * i], tp[2 * i + 1]);
  if (m.auto_resize && n > 0) {
    Box b;
    for (int i = 0; i < n; ++i) b.add(tp[2 * i], tp[2 * i + 1]);
    if (use_blur) b.extend((double)m.half_kernel);
    if (!update_bound(m, b)) {
      m.cur_update_index += 3;
      return false;
    }
  }
  double sx, sy;
  pose_apply(c, s, pm[0], pm[1], origin[0], origin[1], sx, sy);
  const int x0 = (int)(sx + 0.5), y0 = (int)(sy + 0.5);
  for (int i = 0; i < n; ++i) {
    const int x1 = (int)(tp[2 * i] + 0.5), y1 = (int)(tp[2 * i + 1] + 0.5);
    if (x0 != x1 || y0 != y1) {
      if (!m.just_update_occu) bresenham(x0, y0, x1, y1, [&](int x, int y) { cell_update(m, x, y, kSetFree); });
      cell_update(m, x1, y1, use_blur ? kSetOccupiedBlur : kSetOccupied);
    }
  }
  m.map_update_index++;
  m.cur_update_index += 3;
  return true;
}

void reset_all(OMap& m) {  // Reset :95-103
  for (auto& c : m.cells) reset_cell(m, c);
}

void init_with_range_vec(OMap& m, const double* pts, const int64_t* offsets, int n_scans, const double* origins,
                         const double* poses, bool use_blur, bool speedup) {  // InitMapWithRangeVec :222-255
  if (speedup) {
    for (int idx : m.update_points) reset_cell(m, m.cells[(size_t)idx]);  // ResetValueSpeedup :112-117
  } else {
    reset_all(m);
  }
  m.cur_update_index = 0;
  m.cur_mark_occu = -1;
  m.cur_mark_free = -1;
  m.update_points.clear();
  for (int k = 0; k < n_scans; ++k) {
    int tries = 5;
    while (!update_by_range(m, pts + 2 * offsets[k], (int)(offsets[k + 1] - offsets[k]), origins + 2 * k,
                            poses + 3 * k, use_blur) &&
           tries)
      tries--;
  }
  if (!m.auto_resize) {  // UpdateBoundAdaptMap :266-273
    m.bound.minx = 0.0;
    m.bound.miny = 0.0;
    m.bound.maxx = (double)(m.size_x + 1);
    m.bound.maxy = (double)(m.size_y + 1);
  }
}

double feedback_penalty(OMap& m, const double* pts, int n, const double origin[2], const double best_pose[3],
                        int check_point_num, double bound_tolerance, double penalty_gain,
                        bool use_blur) {  // MapFeedbackResponsePenalty :331-392
  if (bound_tolerance < 0 || check_point_num <= 0 || penalty_gain <= 0.0 || penalty_gain >= 1.0) return 1.0;
  m.use_blur = use_blur;
  m.bound_tolerance = bound_tolerance;
  double pm[3];
  world_to_map(m, best_pose, pm);
  if (!point_in_map(m, pm[0], pm[1])) return 0.0;
  double c, s;
  ref_sincos(pm[2], &s, &c);
  double sx, sy;
  pose_apply(c, s, pm[0], pm[1], origin[0], origin[1], sx, sy);
  const int x0 = (int)(sx + 0.5), y0 = (int)(sy + 0.5);
  int step = 1;
  if (n < 2 * check_point_num)
    step = 1;
  else
    step = n / (check_point_num - 1);
  double penalty = 0;
  for (int i = 0; i < n; i += step) {
    double ex, ey;
    pose_apply(c, s, pm[0], pm[1], pts[2 * i], pts[2 * i + 1], ex, ey);
    const int x1 = (int)(ex + 0.5), y1 = (int)(ey + 0.5);
    if ((x0 == x1 && y0 == y1) || !point_in_map(m, x1, y1)) continue;
    m.cur_end_x = x1;
    m.cur_end_y = y1;
    double res = 0.0;
    bresenham(x0, y0, x1, y1, [&](int x, int y) {  // CheckOccuLineVisitorCallback :447-471
      double sum = 0.0;
      bool occ = false;
      if (x >= 0 && y >= 0 && x < m.size_x && y < m.size_y) {
        const Cell& cell = cell_at(m, x, y);
        occ = m.use_blur ? ((double)cell.prob > m.occu_offset) : (grid_state(m, cell) == kOccupied);
      }
      if (occ) {
        const double dx = (double)m.cur_end_x - (double)x, dy = (double)m.cur_end_y - (double)y;
        if (std::sqrt(dx * dx + dy * dy) > m.bound_tolerance) sum += 1.0;
      }
      if (res < 1.0) res += sum;
    });
    penalty += res;
  }
  penalty *= penalty_gain;
  return std::max((1.0 + 2 * penalty_gain - penalty), 0.1);
}

}  // namespace

extern "C" {

// OccuGridMap(resolution, size, offset, deviation, default_cell_prob)
// (occu_grid_map.h:201-217) with the cell functions' constructor factors.
void* oracle_gridmap_create(int kind, double resolution, int size_x, int size_y, double off_x, double off_y,
                            double deviation, float default_prob) {
  auto m = std::make_unique<OMap>();
  m->kind = kind;
  m->scale_factor = 1.0 / resolution;
  m->off_x = off_x;
  m->off_y = off_y;
  m->default_prob = default_prob;
  if (kind == kCountCell) {
    m->free_factor = 0.0f;
    m->occu_factor = 0.0f;
    m->occu_threshold = 0.5f;
    m->min_pass = 2.0f;
  }
  allocate(*m, size_x, size_y);
  m->row = m->size_x;
  init_kernel(*m, deviation, resolution);
  return m.release();
}

void oracle_gridmap_destroy(void* h) { delete static_cast<OMap*>(h); }

// set_use_auto_map_resize / set_just_update_occu / set_cell_occu_prob_offset /
// set_extend_factor (occu_grid_map.h:429-439, grid_map_base.h:175-179).
void oracle_gridmap_set_options(void* h, int auto_resize, int just_update_occu, double occu_offset,
                                double extend_factor) {
  OMap& m = *static_cast<OMap*>(h);
  m.auto_resize = auto_resize != 0;
  m.just_update_occu = just_update_occu != 0;
  m.occu_offset = occu_offset;
  if (extend_factor > 0) m.extend_factor = extend_factor;
}

// SetUpdateFreeFactor / SetUpdateOccupiedFactor / SetOccuThreshold / SetMinPassThrough
void oracle_gridmap_set_cell_params(void* h, float free_factor, float occu_factor, float occu_threshold,
                                    float min_pass) {
  OMap& m = *static_cast<OMap*>(h);
  m.free_factor = free_factor;
  m.occu_factor = occu_factor;
  if (m.kind == kCountCell) {
    m.occu_threshold = occu_threshold;
    m.min_pass = min_pass;
  }
}

void oracle_gridmap_set_map_offset(void* h, double ox, double oy) {
  OMap& m = *static_cast<OMap*>(h);
  m.off_x = ox;
  m.off_y = oy;
}

void oracle_gridmap_reset(void* h) { reset_all(*static_cast<OMap*>(h)); }

int oracle_gridmap_update_by_range(void* h, const double* pts, int n, const double origin[2], const double pose[3],
                                   int use_blur) {
  return update_by_range(*static_cast<OMap*>(h), pts, n, origin, pose, use_blur != 0) ? 1 : 0;
}

void oracle_gridmap_init_with_range_vec(void* h, const double* pts, const int64_t* offsets, int n_scans,
                                        const double* origins, const double* poses, int use_blur, int speedup) {
  init_with_range_vec(*static_cast<OMap*>(h), pts, offsets, n_scans, origins, poses, use_blur != 0, speedup != 0);
}

double oracle_gridmap_feedback_penalty(void* h, const double* pts, int n, const double origin[2],
                                       const double best_pose[3], int check_point_num, double bound_tolerance,
                                       double penalty_gain, int use_blur) {
  return feedback_penalty(*static_cast<OMap*>(h), pts, n, origin, best_pose, check_point_num, bound_tolerance,
                          penalty_gain, use_blur != 0);
}

// Geometry and counters: ints[0..7] = size_x, size_y, map_update_index,
// cur_update_index, half_kernel, n_update_points, blur_states, kind;
// dbl[0..6] = resolution, off_x, off_y, bound min x/y, max x/y.
void oracle_gridmap_info(void* h, int32_t* ints, double* dbl) {
  const OMap& m = *static_cast<OMap*>(h);
  ints[0] = m.size_x;
  ints[1] = m.size_y;
  ints[2] = m.map_update_index;
  ints[3] = m.cur_update_index;
  ints[4] = m.half_kernel;
  ints[5] = (int32_t)m.update_points.size();
  ints[6] = m.blur_states ? 1 : 0;
  ints[7] = m.kind;
  dbl[0] = 1 / m.scale_factor;
  dbl[1] = m.off_x;
  dbl[2] = m.off_y;
  dbl[3] = m.bound.minx;
  dbl[4] = m.bound.miny;
  dbl[5] = m.bound.maxx;
  dbl[6] = m.bound.maxy;
}

// Cells as separate arrays (size_y * size_x each; any pointer may be null).
void oracle_gridmap_cells(void* h, float* prob, float* pass, float* hit, int32_t* uidx) {
  const OMap& m = *static_cast<OMap*>(h);
  for (size_t i = 0; i < m.cells.size(); ++i) {
    if (prob) prob[i] = m.cells[i].prob;
    if (pass) pass[i] = m.cells[i].pass;
    if (hit) hit[i] = m.cells[i].hit;
    if (uidx) uidx[i] = m.cells[i].uidx;
  }
}

// map_update_point_ as a set: flags[i] = 1 if linear index i is in the list.
void oracle_gridmap_touched(void* h, uint8_t* flags) {
  const OMap& m = *static_cast<OMap*>(h);
  std::memset(flags, 0, m.cells.size());
  for (int idx : m.update_points) flags[idx] = 1;
}

// Blur kernel values (kernel_size^2, index (i+hk) + ks*(j+hk)).
int oracle_gridmap_kernel(void* h, double* out, int cap) {
  const OMap& m = *static_cast<OMap*>(h);
  const int n = (int)m.kernel.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = m.kernel[(size_t)i];
  return n;
}

// The reference's Bresenham visit order (test hook): writes up to cap cells
// as (x, y) pairs, returns the count.
int oracle_bresenham(int x0, int y0, int x1, int y1, int32_t* out, int cap) {
  int k = 0;
  bresenham(x0, y0, x1, y1, [&](int x, int y) {
    if (k < cap) {
      out[2 * k] = x;
      out[2 * k + 1] = y;
    }
    ++k;
  });
  return k;
}

}  // extern "C"

// ---- SlamProcessor::process front-end (slam/slam_processor.cpp:65-248) ---------
// Test-infrastructure restatement of the loop include/csm_frontend.h runs on
// the device; the matcher is this library's oracle_scan_matchers
// (csm_oracle.cpp) reading the fine map's cells.

extern "C" {
struct oracle_map_c {
  const float* cells;
  int64_t stride_floats;
  int32_t size_x, size_y;
  double resolution;
  double offset_x, offset_y;
  int32_t update_index;
  float outside_value;
};
double oracle_scan_matchers(const oracle_map_c* mc, const double* pts, int n, const void* levels3, int use_fine,
                            double pose[3], double cov[9]);
double oracle_scan_match(const oracle_map_c* mc, const double* pts, int n, const void* param, double pose[3],
                         double cov[9], int64_t* argmax_flat, int64_t* n_scored);
double oracle_optimize_scan_match(const oracle_map_c* mc, const double* pts, int n, const void* param,
                                  double pose[3], int* iterations);
}

namespace {

struct FeParam {  // layout of csm_frontend_param (include/csm_frontend.h)
  double range_max, init_map_size, map_offset_x, map_offset_y, map_extend_factor, gaussian_blur_offset;
  double map_resolution, map_update_free_factor, map_update_occu_factor, map_occu_threshold, map_min_passthrough;
  double coarse_map_resolution, coarse_map_deviation, fine_map_resolution, fine_map_deviation;
  int32_t coarse_map_use_blur, fine_map_use_blur, use_odometry, use_map_check_feedback, map_check_point_num,
      use_map_update_move_check;
  double map_check_bound_tolerance, map_check_penalty_gain;
  double map_update_score_threshold, map_update_distance_threshold, map_update_angle_threshold;
  struct Level {
    double size, res, aoff, ares, thr;
    int32_t use_point_size, max_depth, use_center_penalty, type;
  } levels[3];
  int32_t use_optimize_scan_match, reserved;
  double optimize_failed_cost;
  struct Opt {  // csm_optimize_param
    int32_t iterate_max_times, reserved;
    double cost_decrease_threshold, cost_min_threshold, max_update_distance, max_update_angle;
  } optimize;
};

struct FeResult {  // layout of csm_frontend_result
  double pose[3], match_pose[3], cov[9], score, map_penalty, optimize_cost;
  int32_t data_index, matched, map_updated, pose_accepted;
};

struct OFrontEnd {
  FeParam p;
  std::unique_ptr<OMap> maps[3];
  int data_index = 0;
  double cur[3] = {0, 0, 0}, last_odom[3] = {0, 0, 0}, last_update[3] = {0, 0, 0};
  double score = 0.0;
  int penalize_times = 0;
  // the kept scans (SensorDataManager's range data of the maps, :216-221):
  // sensor-frame points (m) and the pose each was drawn at
  std::vector<double> kept_pts;
  std::vector<int64_t> kept_off{0};
  std::vector<double> kept_pose;
};

double norm_angle(double a) {  // util::NormalizeAngle (util/slam_util.h:103-111)
  double n = std::fmod(std::fmod(a, 2.0 * M_PI) + 2.0 * M_PI, 2.0 * M_PI);
  if (n > M_PI) n -= 2.0 * M_PI;
  return n;
}

std::unique_ptr<OMap> make_map(int kind, double res, int sz, double ox, double oy, double dev, float dflt) {
  auto m = std::make_unique<OMap>();
  m->kind = kind;
  m->scale_factor = 1.0 / res;
  m->off_x = ox;
  m->off_y = oy;
  m->default_prob = dflt;
  if (kind == kCountCell) {
    m->free_factor = 0.0f;
    m->occu_factor = 0.0f;
    m->occu_threshold = 0.5f;
    m->min_pass = 2.0f;
  }
  allocate(*m, sz, sz);
  m->row = m->size_x;
  init_kernel(*m, dev, res);
  return m;
}

oracle_map_c map_view(const OMap& m) {  // what oracle_scan_match* read of a ScanMatchMap
  oracle_map_c mc;
  mc.cells = &m.cells[0].prob;
  mc.stride_floats = (int64_t)(sizeof(Cell) / sizeof(float));
  mc.size_x = m.size_x;
  mc.size_y = m.size_y;
  mc.resolution = 1 / m.scale_factor;
  mc.offset_x = m.off_x;
  mc.offset_y = m.off_y;
  mc.update_index = m.map_update_index;
  mc.outside_value = 0.3f;
  return mc;
}

// ScanMatchers::MapSizeCheck (scan_matchers.h:365-390) for one map.
void map_size_check(OMap& m, const double pose[3], double range_max, double offset) {
  double pm[3];
  world_to_map(m, pose, pm);
  const double mres = 1 / m.scale_factor;
  const double max_size = (range_max + offset) / mres;
  Box b;
  b.minx = pm[0] - max_size;
  b.miny = pm[1] - max_size;
  b.maxx = pm[0] + max_size;
  b.maxy = pm[1] + max_size;
  update_bound(m, b);
}

// ScanMatchers::ScanMatch (scan_matchers.h:179-289) on a coarse and a fine
// ScanMatchMap: MapSizeCheck on both, the optional Gauss-Newton matcher on the
// coarse map, the correlative coarse level when it is off, failed or
// !use_fine, then fine and super-fine on the fine map. Returns the mean.
double matchers_on_maps(OMap& coarse, OMap& fine, const double* cp, const double* fp, int n,
                        const FeParam::Level* levels, int use_opt, double failed, const FeParam::Opt& opt,
                        double range_max, int use_fine, double pose[3], double cov[9], double* opt_cost) {
  map_size_check(coarse, pose, range_max, levels[0].size);
  map_size_check(fine, pose, range_max, levels[0].size);
  const oracle_map_c mc = map_view(fine);
  *opt_cost = 0.0;
  if (!use_opt) return oracle_scan_matchers(&mc, fp, n, levels, use_fine, pose, cov);
  const oracle_map_c cmc = map_view(coarse);
  double proc[3] = {pose[0], pose[1], pose[2]};
  const double cost = oracle_optimize_scan_match(&cmc, cp, n, &opt, proc, nullptr);
  *opt_cost = cost;
  double sum = failed / (cost + failed);
  int times = 1;
  if (!use_fine || cost > failed) {
    sum = 0.0;
    times--;
    std::memcpy(proc, pose, sizeof(proc));
    sum += oracle_scan_match(&mc, fp, n, &levels[0], proc, cov, nullptr, nullptr);
    times++;
  }
  if (use_fine) {
    for (int k = 1; k <= 2; ++k) {
      sum += oracle_scan_match(&mc, fp, n, &levels[k], proc, cov, nullptr, nullptr);
      times++;
    }
  }
  std::memcpy(pose, proc, sizeof(proc));
  return sum / times;
}

}  // namespace

extern "C" {

void* oracle_frontend_create(const void* param) {
  auto* f = new OFrontEnd();
  std::memcpy(&f->p, param, sizeof(FeParam));
  return f;
}
void oracle_frontend_destroy(void* h) { delete static_cast<OFrontEnd*>(h); }
int oracle_frontend_param_size(void) { return (int)sizeof(FeParam); }
int oracle_frontend_result_size(void) { return (int)sizeof(FeResult); }
void* oracle_frontend_map(void* h, int which) { return static_cast<OFrontEnd*>(h)->maps[which].get(); }

int oracle_frontend_process(void* h, const double* pts, int n, const double odom[3], void* result) {
  OFrontEnd& f = *static_cast<OFrontEnd*>(h);
  const FeParam& p = f.p;
  FeResult r;
  std::memset(&r, 0, sizeof(r));
  const bool first = f.data_index == 0;
  if (first) {  // CreateAllMap (:464-527)
    const double rm = p.range_max;
    const double ims = (p.init_map_size < 3.0) ? (3.0 * rm) : (p.init_map_size * rm);
    const double ox = ims * p.map_offset_x, oy = ims * p.map_offset_y;
    f.maps[0] = make_map(kCountCell, p.map_resolution, (int)(ims / p.map_resolution), ox, oy, 0.0, 0.5f);
    f.maps[1] = make_map(kProbabilityCell, p.coarse_map_resolution, (int)(ims / p.coarse_map_resolution), ox, oy,
                         p.coarse_map_deviation, 0.3f);
    f.maps[2] = make_map(kProbabilityCell, p.fine_map_resolution, (int)(ims / p.fine_map_resolution), ox, oy,
                         p.fine_map_deviation, 0.3f);
    for (int k = 0; k < 3; ++k) {
      if (p.map_extend_factor > 0) f.maps[k]->extend_factor = p.map_extend_factor;
      f.maps[k]->auto_resize = true;
      if (k > 0) {
        f.maps[k]->occu_offset = p.gaussian_blur_offset;
        f.maps[k]->just_update_occu = true;
      }
    }
    f.cur[0] = f.cur[1] = f.cur[2] = 0.0;
  }
  double predict[3] = {f.cur[0], f.cur[1], f.cur[2]};
  std::vector<double> pp((size_t)2 * n), cp((size_t)2 * n), fp((size_t)2 * n);
  const double fpub = 1 / p.map_resolution, fco = 1 / p.coarse_map_resolution, ffi = 1 / p.fine_map_resolution;
  for (int i = 0; i < 2 * n; ++i) {
    pp[(size_t)i] = pts[i] * fpub;
    cp[(size_t)i] = pts[i] * fco;
    fp[(size_t)i] = pts[i] * ffi;
  }
  double cov[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  r.map_penalty = 1.0;
  if (!first) {
    if (p.use_odometry) {  // PredictPoseByOdom (:618-635)
      const double a = f.cur[2] - f.last_odom[2];
      double c, s;
      ref_sincos(a, &s, &c);
      const double tx = f.cur[0] - (c * f.last_odom[0] + (-s) * f.last_odom[1]);
      const double ty = f.cur[1] - (s * f.last_odom[0] + c * f.last_odom[1]);
      predict[0] = (c * odom[0] + (-s) * odom[1]) + tx;
      predict[1] = (s * odom[0] + c * odom[1]) + ty;
      predict[2] = a + odom[2];
    }
    double pose[3] = {predict[0], predict[1], predict[2]};
    double opt_cost = 0.0;
    double score = matchers_on_maps(*f.maps[1], *f.maps[2], cp.data(), fp.data(), n, p.levels, p.use_optimize_scan_match,
                                    p.optimize_failed_cost, p.optimize, p.range_max, 1, pose, cov, &opt_cost);
    r.optimize_cost = opt_cost;
    std::memcpy(r.match_pose, pose, sizeof(pose));
    double penalty = 1.0;
    if (p.use_map_check_feedback)  // MapCheckPenalize (:573-595)
      penalty = feedback_penalty(*f.maps[0], pp.data(), n, (const double[2]){0.0, 0.0}, pose, p.map_check_point_num,
                                 p.map_check_bound_tolerance, p.map_check_penalty_gain, false);
    r.map_penalty = penalty;
    if (f.penalize_times < 5) {
      score *= penalty;
      score = (score > 1.0) ? (1.0) : (score);
      if (penalty < 0.7)
        f.penalize_times++;
      else
        f.penalize_times = 0;
    } else {
      f.penalize_times = 0;
    }
    if (score > std::max(0.5, p.map_update_score_threshold)) {
      std::memcpy(f.cur, pose, sizeof(pose));
      r.pose_accepted = 1;
    }
    f.score = score;
    r.matched = 1;
  }
  bool updated = false;
  const double dx = f.cur[0] - f.last_update[0], dy = f.cur[1] - f.last_update[1];
  const bool moved = std::sqrt(dx * dx + dy * dy) >= p.map_update_distance_threshold ||
                     std::fabs(norm_angle(f.cur[2] - f.last_update[2])) >= p.map_update_angle_threshold;
  if ((f.score > p.map_update_score_threshold && (moved || !p.use_map_update_move_check)) || f.data_index < 1) {
    OMap& pub = *f.maps[0];  // UpdateMap (:529-571)
    if (first) {
      pub.occu_threshold = 0.5f;
      pub.min_pass = 1.0f;
      pub.free_factor = (float)p.map_min_passthrough;
      pub.occu_factor = (float)(p.map_min_passthrough * 2);
    } else {
      pub.occu_threshold = (float)p.map_occu_threshold;
      pub.min_pass = (float)p.map_min_passthrough;
      pub.free_factor = (float)p.map_update_free_factor;
      pub.occu_factor = (float)p.map_update_occu_factor;
    }
    const double org[2] = {0.0, 0.0};
    update_by_range(pub, pp.data(), n, org, f.cur, false);
    update_by_range(*f.maps[1], cp.data(), n, org, f.cur, p.coarse_map_use_blur != 0);
    update_by_range(*f.maps[2], fp.data(), n, org, f.cur, p.fine_map_use_blur != 0);
    std::memcpy(f.last_update, f.cur, sizeof(f.cur));
    updated = true;
  }
  r.data_index = f.data_index;
  if (updated) {
    f.data_index++;
    std::memcpy(f.last_odom, odom, sizeof(f.last_odom));
    f.kept_pts.insert(f.kept_pts.end(), pts, pts + 2 * (size_t)n);
    f.kept_off.push_back((int64_t)(f.kept_pts.size() / 2));
    f.kept_pose.insert(f.kept_pose.end(), f.cur, f.cur + 3);
  }
  std::memcpy(r.pose, f.cur, sizeof(r.pose));
  std::memcpy(r.cov, cov, sizeof(cov));
  r.score = f.score;
  r.map_updated = updated ? 1 : 0;
  std::memcpy(result, &r, sizeof(r));
  return 0;
}

// SlamProcessor::CorrectPoseAndMap (slam/slam_processor.cpp:329-370): the
// corrected poses replace the kept scans' poses (UpdateRangeData :597-602),
// then each map is rebuilt from every kept scan (InitMapWithRangeVec): the
// PubMap from ids 0..last plus map_min_passthrough_ more copies of scan 0,
// the scan-match maps with their blur settings. Returns 1 on an id beyond the
// kept scans (the reference's CHECK_LE aborts).
int oracle_frontend_correct(void* h, int n, const int32_t* ids, const double* poses) {
  OFrontEnd& f = *static_cast<OFrontEnd*>(h);
  const FeParam& p = f.p;
  const int kept = (int)f.kept_off.size() - 1;
  for (int i = 0; i < n; ++i)
    if (ids[i] < 0 || ids[i] >= kept) return 1;
  if (kept == 0) return 0;
  for (int i = 0; i < n; ++i) std::memcpy(&f.kept_pose[3 * (size_t)ids[i]], poses + 3 * i, 3 * sizeof(double));
  std::vector<int> pub_ids;
  for (int i = 0; i < kept; ++i) pub_ids.push_back(i);
  for (int i = 0; i < p.map_min_passthrough; ++i) pub_ids.push_back(0);
  const double res[3] = {p.map_resolution, p.coarse_map_resolution, p.fine_map_resolution};
  const bool blur[3] = {false, p.coarse_map_use_blur != 0, p.fine_map_use_blur != 0};
  for (int k = 0; k < 3; ++k) {
    std::vector<int> use = pub_ids;
    if (k > 0) use.resize((size_t)kept);
    const double factor = 1 / res[k];  // CreateFrom (sensor_data_manager.h:99-115)
    std::vector<double> pts, ps;
    std::vector<int64_t> off{0};
    for (int id : use) {
      for (int64_t j = 2 * f.kept_off[(size_t)id]; j < 2 * f.kept_off[(size_t)id + 1]; ++j)
        pts.push_back(f.kept_pts[(size_t)j] * factor);
      off.push_back((int64_t)(pts.size() / 2));
      ps.insert(ps.end(), &f.kept_pose[3 * (size_t)id], &f.kept_pose[3 * (size_t)id] + 3);
    }
    std::vector<double> org(2 * use.size(), 0.0);
    init_with_range_vec(*f.maps[k], pts.data(), off.data(), (int)use.size(), org.data(), ps.data(), blur[k], false);
  }
  return 0;
}

}  // extern "C"

// ---- SlamProcessor::ScanMatchInterface (slam/slam_processor.cpp:250-326) -----
// Test-infrastructure restatement of the calls include/csm_backend.h runs on
// the device; job j of a call rebuilds and reads map pair j, in job order.

namespace {

struct BeParam {  // layout of csm_backend_param (include/csm_backend.h)
  double range_max, gaussian_blur_offset, map_resolution;
  double coarse_map_resolution, coarse_map_deviation, fine_map_resolution, fine_map_deviation;
  int32_t coarse_map_use_blur, fine_map_use_blur, use_map_check_feedback, map_check_point_num;
  double map_check_bound_tolerance, map_check_penalty_gain;
  FeParam::Level levels[3];
  int32_t use_optimize_scan_match, reserved;
  double optimize_failed_cost;
  FeParam::Opt optimize;
};

struct BeJob {  // layout of csm_backend_job
  const double* points_m;
  int32_t n_points, n_chain;
  const int32_t* chain_ids;
  int32_t use_fine_scan_match, reserved;
  double pose[3], cov[9], score, map_penalty, optimize_cost;
};

struct OKept {
  std::vector<double> coarse, fine;
  double pose[3];
};

struct OBackEnd {
  BeParam p;
  std::vector<OKept> scans;
  std::vector<std::unique_ptr<OMap>> maps[2];  // coarse, fine per job slot
};

std::vector<double> scaled(const double* pts, int n, double factor) {  // CreateFrom (:99-115)
  std::vector<double> v((size_t)2 * n);
  for (int i = 0; i < 2 * n; ++i) v[(size_t)i] = pts[i] * factor;
  return v;
}

}  // namespace

extern "C" {

void* oracle_backend_create(const void* param) {
  auto* b = new OBackEnd();
  std::memcpy(&b->p, param, sizeof(BeParam));
  return b;
}
void oracle_backend_destroy(void* h) { delete static_cast<OBackEnd*>(h); }
int oracle_backend_param_size(void) { return (int)sizeof(BeParam); }
int oracle_backend_job_size(void) { return (int)sizeof(BeJob); }
void* oracle_backend_map(void* h, int slot, int which) {
  OBackEnd& b = *static_cast<OBackEnd*>(h);
  return slot < (int)b.maps[which].size() ? b.maps[which][(size_t)slot].get() : nullptr;
}

int oracle_backend_add_scan(void* h, const double* pts, int n, const double pose[3]) {
  OBackEnd& b = *static_cast<OBackEnd*>(h);
  OKept k;
  k.coarse = scaled(pts, n, 1 / b.p.coarse_map_resolution);
  k.fine = scaled(pts, n, 1 / b.p.fine_map_resolution);
  std::memcpy(k.pose, pose, sizeof(k.pose));
  b.scans.push_back(std::move(k));
  return (int)b.scans.size() - 1;
}

void oracle_backend_set_scan_pose(void* h, int id, const double pose[3]) {
  std::memcpy(static_cast<OBackEnd*>(h)->scans[(size_t)id].pose, pose, sizeof(double) * 3);
}

int oracle_backend_scan_match(void* h, void* pub_map, const double cur[3], void* jobs_v, int n_jobs) {
  OBackEnd& b = *static_cast<OBackEnd*>(h);
  const BeParam& p = b.p;
  BeJob* jobs = static_cast<BeJob*>(jobs_v);
  for (int j = 0; j < n_jobs; ++j) {
    BeJob& jb = jobs[j];
    // the back-end maps (CreateScanMatchMapWithRangeVec :428-446); first contents wiped by the first reset
    const double ims = (p.range_max + 2.0) * 2;
    const double res[2] = {p.coarse_map_resolution, p.fine_map_resolution};
    const double dev[2] = {p.coarse_map_deviation, p.fine_map_deviation};
    for (int k = 0; k < 2; ++k) {
      while ((int)b.maps[k].size() <= j)
        b.maps[k].push_back(make_map(kProbabilityCell, res[k], (int)(ims / res[k]), 0.0, 0.0, dev[k], 0.3f));
      OMap& m = *b.maps[k][(size_t)j];
      // ResetScanMatchMapWithRangeVec (:448-462)
      const double resolution = 1 / m.scale_factor;
      m.off_x = -(cur[0] - 0.5 * m.size_x * resolution);
      m.off_y = -(cur[1] - 0.5 * m.size_y * resolution);
      m.auto_resize = false;
      m.just_update_occu = true;
      m.occu_offset = p.gaussian_blur_offset;
      std::vector<double> pts, poses;
      std::vector<int64_t> off(1, 0);
      for (int c = 0; c < jb.n_chain; ++c) {
        const OKept& ks = b.scans[(size_t)jb.chain_ids[c]];
        const std::vector<double>& v = k ? ks.fine : ks.coarse;
        pts.insert(pts.end(), v.begin(), v.end());
        off.push_back(off.back() + (int64_t)(v.size() / 2));
        poses.insert(poses.end(), ks.pose, ks.pose + 3);
      }
      std::vector<double> origins((size_t)2 * jb.n_chain, 0.0);
      init_with_range_vec(m, pts.data(), off.data(), jb.n_chain, origins.data(), poses.data(),
                          (k ? p.fine_map_use_blur : p.coarse_map_use_blur) != 0, true);
    }
    const std::vector<double> cp = scaled(jb.points_m, jb.n_points, 1 / p.coarse_map_resolution);  // :268-272
    const std::vector<double> fp = scaled(jb.points_m, jb.n_points, 1 / p.fine_map_resolution);
    const double eye[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    std::memcpy(jb.cov, eye, sizeof(eye));
    jb.score = matchers_on_maps(*b.maps[0][(size_t)j], *b.maps[1][(size_t)j], cp.data(), fp.data(), jb.n_points,
                                p.levels, p.use_optimize_scan_match, p.optimize_failed_cost, p.optimize, p.range_max,
                                jb.use_fine_scan_match, jb.pose, jb.cov, &jb.optimize_cost);
    jb.map_penalty = 1.0;
    if (pub_map && p.use_map_check_feedback) {  // MapCheckPenalize(..., true) (:315-317, :573-595)
      const std::vector<double> pp = scaled(jb.points_m, jb.n_points, 1 / p.map_resolution);
      const double zero[2] = {0.0, 0.0};
      const double penalty = feedback_penalty(*static_cast<OMap*>(pub_map), pp.data(), jb.n_points, zero, jb.pose,
                                              p.map_check_point_num, p.map_check_bound_tolerance,
                                              p.map_check_penalty_gain, false);
      jb.map_penalty = (1 / (1 + std::exp(-10 * (penalty - 0.4))));
    }
    jb.score *= jb.map_penalty;
    jb.score = (jb.score > 1.0) ? (1.0) : (jb.score);
  }
  return 0;
}

}  // extern "C"
