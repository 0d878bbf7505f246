// csm_host_finish.cpp — the reference's host finish of a window once its
// candidates are scored: std::sort + FindBestCandidate (host path), the
// covariances and the world-pose write-back (correlate_scan_matcher.h:606-611,
// 670-710, 784-1019), and the FAST matcher's depth-first search replayed over
// the device's node table (BranchAndBoundCorrelateScanMatcher, :271-502).
#include "csm_host.hpp"

#include <cstddef>
#include <cstring>

namespace csmh {

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

// Covariance lists a level's own type never reads, as the finish's skip mask:
// ComputePositionalCovariance runs for COARSE/FAST/FINE, ComputeAngularCovariance
// for COARSE/FAST/SUPER (correlate_scan_matcher.h:835-858, complete_window).
// The fast finish then neither builds nor stores them, and ties inside an
// unread list no longer send a window to the exact pass.
int own_lists_skip(int type) {
  switch (type) {
    case CSM_COARSE:
    case CSM_FAST: return 0;
    case CSM_FINE: return 2;
    case CSM_SUPER: return 1;
    default: return 3;
  }
}

// Everything BasedCorrelationScanMatch::ScanMatch does once the sorted
// candidates are summarised in `o` (correlate_scan_matcher.h:700-707,
// 835-869, covariance :887-1019). Returns the response.
// skip_lists: covariances a later level overwrites (live_lists) are not
// computed; their lists were not filled.
uint32_t seal_writer(const csm::FinishOut* src, int32_t tag) {
  const uint64_t tk = __atomic_load_n(&src->seal_tag_kind, __ATOMIC_ACQUIRE);
  return (uint32_t)tk == (uint32_t)tag ? (uint32_t)(tk >> 32) & 3u : 0u;
}

// Only the pieces the seal names are copied (and hashed): the GPU wrote them
// into memory no CPU cache holds, so every line read is a memory round trip
// (a coarse window's header is 2 of the structure's 9 lines).
uint32_t read_sealed(const csm::FinishOut* src, int32_t tag, csm::FinishOut& out) {
  const uint64_t tk = __atomic_load_n(&src->seal_tag_kind, __ATOMIC_ACQUIRE);
  if ((uint32_t)tk != (uint32_t)tag) return 0u;
  const uint32_t kind = (uint32_t)(tk >> 32), writer = kind & 3u;
  if (writer == csm::kSealPending) return writer;
  const int lists = (int)(kind >> 2) & 3;
  const uint64_t chk = __atomic_load_n(&src->seal_chk, __ATOMIC_RELAXED);
  const char* in = reinterpret_cast<const char*>(src);
  char* o = reinterpret_cast<char*>(&out);
  std::memcpy(o, in, 64);                                              // header, pieces 0-3
  if (lists & 1) {
    std::memcpy(o + offsetof(csm::FinishOut, pos_idx), in + offsetof(csm::FinishOut, pos_idx), 80);
    std::memcpy(o + offsetof(csm::FinishOut, pos_score), in + offsetof(csm::FinishOut, pos_score), 160);
  }
  if (lists & 2) {
    std::memcpy(o + offsetof(csm::FinishOut, ang_idx), in + offsetof(csm::FinishOut, ang_idx), 80);
    std::memcpy(o + offsetof(csm::FinishOut, ang_score), in + offsetof(csm::FinishOut, ang_score), 160);
  }
  out.seal_tag_kind = tk;
  out.seal_chk = chk;
  uint64_t h = csm::finish_seal_share(tk);
  const uint32_t* words = reinterpret_cast<const uint32_t*>(&out);
  for (int t = 0, n = csm::finish_n_pieces(lists); t < n; ++t) {
    const int pc = csm::finish_piece(t, lists);
    h += csm::finish_piece_hash(pc, words[4 * pc], words[4 * pc + 1], words[4 * pc + 2], words[4 * pc + 3]);
  }
  return h == chk ? writer : 0u;
}

double complete_window(const csm::FinishOut& o, const CandGeom& C, const csm_param& P,
                       const Geometry& G, double pose[3], double cov[9], int skip_lists) {
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

}  // namespace csmh
