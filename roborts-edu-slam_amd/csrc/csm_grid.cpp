// csm_grid.cpp — the matcher's resident grids (include/csm.h grid entry
// points): the reference's AoS ProbabilityCell map uploaded and kept keyed on
// (cells pointer, stride, size, map_update_index) (grid_map_cell.h:301-328,
// grid_map_base.h:352-354), incremental row / cell refreshes, grid stacks,
// borrowed device maps (csm_gridmap), and the exact fixed-point copy every
// integer-mode kernel reads.
#include "csm_host.hpp"

namespace csmh {

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

// The palette copy of the current gridi (csm_palette.hip), built once per
// grid generation: the grid's distinct fixed-point values and a byte per cell
// holding its value's index, read by the v10 palette box kernel. A grid with
// more than csm::kPalMax values gets none (pal_n = 0).
int ensure_palette(csm_ctx* c) {
  if (!c->int_ok || !c->d_gridi) {
    c->pal_n = 0;
    return CSM_OK;
  }
  if (c->pal_gen == c->grid_gen && c->pal_src == c->d_gridi) return CSM_OK;
  const int64_t n = (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows) * c->n_grids;
  hipError_t e;
  if ((e = c->pal_grid.ensure((size_t)n)) != hipSuccess) return c->hip_fail(e, "hipMalloc(palette grid)");
  if ((e = c->pal_vals.ensure((csm::kPalMax + 4) * sizeof(int32_t))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(palette)");
  if ((e = c->pal_scratch.ensure((size_t)csm::pal_scratch_ints(n) * sizeof(int32_t))) != hipSuccess)
    return c->hip_fail(e, "hipMalloc(palette scratch)");
  int32_t* vals = (int32_t*)c->pal_vals.p;
  if ((e = csm::launch_build_palette(c->d_gridi, n, (int32_t*)c->pal_scratch.p, vals, vals + csm::kPalMax,
                                     (uint8_t*)c->pal_grid.p, c->stream)) != hipSuccess)
    return c->hip_fail(e, "palette kernels");
  int32_t m = 0;
  if ((e = hipMemcpyAsync(&m, vals + csm::kPalMax, sizeof(m), hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return c->hip_fail(e, "palette size");
  c->pal_n = (m >= 1 && m <= csm::kPalMax) ? m : 0;
  c->pal_strips_ok = false;
  const csm::StripGeom SG = csm::strip_geom(c->info.size_x, c->info.size_y);
  // (the pair kernel's strip offsets are 24-bit products: strips under 2^24 bytes)
  if (c->pair_kernel && c->pal_n >= 1 && c->pal_n <= csm::kPairMaxPal && SG.grid_bytes <= INT32_MAX &&
      SG.strip_bytes < (1 << 24)) {
    if ((e = c->pal_strips.ensure((size_t)SG.grid_bytes * (size_t)c->n_grids)) != hipSuccess)
      return c->hip_fail(e, "hipMalloc(palette strips)");
    const int64_t idx_stride = (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows);
    if ((e = csm::launch_build_strips((const uint8_t*)c->pal_grid.p, c->pitch, c->info.size_x, c->info.size_y,
                                      idx_stride, c->n_grids, (uint8_t*)c->pal_strips.p, c->stream)) != hipSuccess)
      return c->hip_fail(e, "pal_strips_kernel");
    // other parts' streams read the strips next (like gridi)
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(strips)");
    c->pal_strips_ok = true;
  }
  c->pal_gen = c->grid_gen;
  c->pal_src = c->d_gridi;
  if (c->profiling) c->account("grid:palette", 0.f, (double)n, (double)c->pal_n);
  return CSM_OK;
}

// The strip copies of the current gridi for the phase kernel, once per grid
// generation (istrips_ok = false: none, the kernel reads gridi row-major).
int ensure_istrips(csm_ctx* c) {
  if (!c->int_ok || !c->d_gridi) {
    c->istrips_ok = false;
    return CSM_OK;
  }
  if (c->istrips_gen == c->grid_gen && c->istrips_src == c->d_gridi) return CSM_OK;
  c->istrips_ok = false;
  const csm::StripGeom SG = csm::istrip_geom(c->info.size_x, c->info.size_y);
  if (SG.grid_bytes <= INT32_MAX) {
    hipError_t e;
    if ((e = c->istrips.ensure((size_t)SG.grid_bytes * (size_t)c->n_grids)) != hipSuccess)
      return c->hip_fail(e, "hipMalloc(gridi strips)");
    const int64_t stride = (int64_t)c->pitch * (c->info.size_y + csm::kGridiPadRows);
    if ((e = csm::launch_build_istrips(c->d_gridi, c->pitch, c->info.size_x, c->info.size_y, stride, c->n_grids,
                                       (int32_t*)c->istrips.p, c->stream)) != hipSuccess)
      return c->hip_fail(e, "istrips_kernel");
    // other parts' streams read the strips next (like gridi)
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize(istrips)");
    c->istrips_ok = true;
    if (c->profiling) c->account("grid:istrips", 0.f, (double)SG.grid_bytes * c->n_grids, 0.0);
  }
  c->istrips_gen = c->grid_gen;
  c->istrips_src = c->d_gridi;
  return CSM_OK;
}

}  // namespace csmh

using namespace csmh;

extern "C" {

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
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
  DeviceGuard g(c->device);  // the read fence is created and recorded on the context's device
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
  release_map_reader(c);
  return set_grid_device_locked(c, dev, info);
}

int csm_set_grid_gridmap(csm_ctx* c, csm_gridmap* map) {
  if (!c || !map) return CSM_ERR_INVALID_ARG;
  float outside;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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

int csm_set_grid_stack(csm_ctx* c, const float* cells, int32_t n_grids, const csm_map_info* info,
                       int64_t version) {
  if (!c || !info || !cells || n_grids <= 0) return CSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
  if (const int dst = pipe_drain(c)) return dst;  // a submitted batch still reads the context
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
