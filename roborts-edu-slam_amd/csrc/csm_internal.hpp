// csm_internal.hpp — types shared by the HIP kernels (csm_kernels.hip) and the
// host side of the C-ABI (csm_api.cpp). Not installed; include/csm.h is the
// public boundary.
#pragma once

#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace csm {

// One window to search: a scan (its points) at one level, centred on one pose.
// Everything a lane needs to rebuild its candidate's (x, y, theta) exactly as
// MultiResolutionCorrelateScanMatcher::ScanMatch does
// (correlate_scan_matcher.h:536-572) is precomputed on the host.
struct ScanWork {
  int64_t pts_off;      // first point of this scan in the batch point array
  int64_t angle_off;    // first AngleEntry of this window
  int64_t out_off;      // first output slot (all-scores mode)
  int32_t n_used;       // B = ceil(N / step): beams summed
  int32_t step;         // beam stride (:561-566)
  double divisor;       // use_point_size after the :561 rule
  double x0, y0;        // search_space_start_x/y (:546-547), map cells
  double cx, cy, ct;    // window centre (map cells, rad)
  int32_t reserved;
  int32_t grid_index;   // which resident grid (submap) this window reads
};

// Per-angle data of a window: theta_i = start + i*ares and the host libm
// cos/sin of it (AngleSearchLookUpTable::UpdateLookUpTable :161-172).
struct AngleEntry {
  double angle, cosine, sine;
};

// ---- device finish (csm_finish.hip) -------------------------------------
constexpr int kCovPoints = 20;          // kMaxVarianceUsePointSize (:1033)
constexpr int64_t kFinishMaxCand = 10240;  // windows above this finish on the host (LDS: 160 KB)

struct FinishArgs {
  int64_t n_cand;
  int64_t score_stride;  // scores between consecutive windows (0: n_cand)
  int32_t n_space;
  // Covariance lists nobody reads (bit 0: positional, bit 1: angular). In the
  // 3-level driver a later level overwrites them (csm_api.cpp live_lists);
  // the finish then decides and fills only FindBest's prefix and the rest.
  int32_t skip_lists;
  double step_cells;   // res / map_resolution
  double lin_tol;      // search_space_resolution / map_resolution (:840,:852)
  int32_t* order_out;  // optional: the sorted permutation, n_cand per window
  int32_t* need_exact; // per window: 1 = the fast finish saw a tie that matters (device scratch)
  int32_t* exact_list; // [0] = count, [1] = tag (flag_value), then the flagged windows (device
                       // scratch, 8-byte aligned, n_windows + 2)
  // Host signal (nullable, listed exact pass only): the pass's last block to
  // finish stores flag_value at host_flag with system scope once every
  // FinishOut is written (done_ctr: a device counter, zero between launches).
  int32_t* done_ctr;
  int32_t* host_flag;
  int32_t flag_value;
  // fast finishes of at most this many windows run 1024 threads per window
  // (256 otherwise); 0 selects kFinishWideWindows
  int32_t wide_windows;
  // Early host signal (nullable, with host_flag): the fast pass's last block
  // stores flag_value here once every window is sealed -- a flagged window's
  // seal says pending (kSealPending) -- so the host completes the settled
  // windows while the exact pass sorts the rest.
  int32_t* host_fast_flag;
};
constexpr int kFinishWideWindows = 64;

// What the host needs to complete BasedCorrelationScanMatch::ScanMatch for
// one window after the device sorted its candidates.
struct FinishOut {
  int32_t front_idx;   // flat index std::sort put first (the argmax)
  int32_t count;       // FindBestCandidate tied-prefix length
  int32_t n_pos, n_ang;
  double best_score;
  double best_x, best_y;   // averaged (count > 1) or front (map cells)
  double thx, thy, ssum;   // sums for atan2(thy/ssum, thx/ssum) (host libm)
  int32_t pos_idx[kCovPoints];
  int32_t ang_idx[kCovPoints];
  double pos_score[kCovPoints];
  double ang_score[kCovPoints];
  // The seal (r04). The finishes write FinishOut into pinned host memory and
  // the host spins on a flag; the pieces of a window can land after that flag
  // (tools/stress_ties.py + CSM_DEBUG_FIN caught a header whose n_pos / n_ang
  // were still the previous level's, with and without a per-block system-scope
  // release). So every writer ends a window with a seal: the launch's tag, who
  // wrote it and which lists it stored (tag_kind = tag | kind << 32), and a
  // checksum of the stored pieces and the tag (finish_seal_chk). The host
  // completes a window only from a copy whose checksum matches.
  uint64_t seal_tag_kind;
  uint64_t seal_chk;
};

// Seal kinds: the writer in bits 0-1, the lists stored in bits 2-3
// (bit 2 positional, bit 3 angular).
constexpr uint32_t kSealFast = 1, kSealExact = 2, kSealPending = 3;
constexpr int kFinishSealPiece = 34;  // 16-byte piece of the seal

// FinishOut's 16-byte pieces a writer stores for lists = (positional ? 1 : 0)
// | (angular ? 2 : 0): the header (0-3), then pos_idx (4-8) and pos_score
// (14-23) if positional, ang_idx (9-13) and ang_score (24-33) if angular.
__host__ __device__ inline int finish_n_pieces(int lists) {
  return 4 + ((lists & 1) ? 15 : 0) + ((lists & 2) ? 15 : 0);
}
__host__ __device__ inline int finish_piece(int t, int lists) {  // t < finish_n_pieces(lists)
  if (t < 4) return t;
  t -= 4;
  if (lists & 1) {
    if (t < 5) return 4 + t;          // pos_idx
    if (t < 15) return 14 + (t - 5);  // pos_score
    t -= 15;
  }
  return t < 5 ? 9 + t : 24 + (t - 5);  // ang_idx, ang_score
}
// One piece's share of the checksum (pieces add up in any order: the device
// sums its lanes' shares, the host its copy's).
__host__ __device__ inline uint64_t finish_piece_hash(int pc, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  const uint64_t a = ((uint64_t)w1 << 32) | w0, b = ((uint64_t)w3 << 32) | w2;
  uint64_t h = (a * 0x9E3779B97F4A7C15ull) ^ (b + 0xC2B2AE3D27D4EB4Full * (uint64_t)(pc + 1));
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  return h;
}
__host__ __device__ inline uint64_t finish_seal_share(uint64_t tag_kind) {
  return finish_piece_hash(kFinishSealPiece, (uint32_t)tag_kind, (uint32_t)(tag_kind >> 32), 0x5EA1u, 0u);
}

// The fused fast finish (r05, csm_tail.hpp): a scoring launch of the 3-level
// driver finishes its windows itself. Each (window, angle) wave stores its
// scores write-through and its angle's max, then counts in on its window; the
// last to arrive runs the fast finish's decisions for the window and writes
// its sealed FinishOut (or flags it for the exact pass, as before). The last
// window of the level-part sets the host flags. No separate fast-pass launch.
struct TailArgs {
  int32_t on;
  int32_t n_windows;   // windows of the level-part (every span of it)
  int32_t* win_ctr;    // per window: waves arrived (the window's finisher resets it to 0)
  int32_t* level_ctr;  // windows of the level-part finished (the last one resets it to 0)
  double* ang_max;     // per (window, angle): the angle's max score, NaN if any score is NaN
  FinishOut* out;      // FinishOut[n_windows] (pinned host memory with a host signal)
  FinishArgs A;        // the fast finish's arguments (need_exact, exact_list, host flags, tag)
};

// Launch-uniform description of one level.
struct LevelWork {
  int32_t n_angles;
  int32_t n_space;
  int64_t n_cand;          // n_angles * n_space^2 per window
  int32_t blocks_per_scan;
  int32_t n_scans;
  double step_cells;       // space_step_factor = res / map_resolution (:548)
  int32_t use_penalty;
  int32_t pad0;
  double dist_gain;        // kDistancePenaltyGain{Coarse,Fine} (:760-761)
  double size;             // search_space_size (max_distance_bound of :734)
  double mres;             // map_resolution (scale_factor of :733)
  const float* grid;       // packed fp32 grid(s), row-major
  int64_t grid_stride;     // floats between consecutive grids (submaps)
  int32_t size_x, size_y;
  float outside;
  int32_t int_mode;        // 1: accumulate the fixed-point copy gridi exactly
  const int32_t* gridi;    // value * 2^int_exp, exact (see csm_set_grid)
  double int_scale;        // 2^-int_exp
  int32_t outside_i;
  int32_t n_cols;          // n_angles * n_space (column kernel)
  int32_t ktiles;          // ceil(n_space / KT)
  int32_t col_blocks;      // ceil(n_cols / 64)
  int32_t pitch;           // gridi row pitch in cells (gridi_pitch(size_x))
  int64_t gridi_stride;    // int32 cells between consecutive gridi grids (pitch * (size_y +
                           // kGridiPadRows): each grid ends with zero rows)
  int32_t tile_n;          // box kernel over a large window: tiles per axis (0: untiled)
  int32_t tile_ns;         // ... and the window's own n_space (candidate indices are its)
  // The finish's flagged-window list header (FinishArgs::exact_list[0..1]) of
  // a host-signal launch: block 0 of the scoring kernel, which runs before the
  // finish on the stream, stores {count 0, clear_tag} there as one 8-byte word
  // (nullptr: nothing to clear). clear_tag is the launch's flag value: an
  // exact pass left over from the slot's previous launch (it had nothing to
  // do, or the host could not have gone on) finds another tag and exits.
  int32_t* clear_word;
  int32_t clear_tag;
  // The palette copy of gridi (score_box_pair_kernel's source): every cell's index
  // into pal_vals, the grid's distinct fixed-point values (pal_vals[0] = 0,
  // the outside value), one byte per cell in gridi's layout (row pitch
  // `pitch` bytes, pal_stride bytes per grid). pal_n = 0: no palette.
  int32_t pal_n;
  const uint8_t* pal_grid;
  const int32_t* pal_vals;
  int64_t pal_stride;
  // The strip copies of the palette grid (score_box_pair_kernel, pal_n <=
  // kPairMaxPal; csm_palette.hip strip_geom): bytes per strip, per copy and
  // per grid of the stack.
  const uint8_t* pal_strips;
  int32_t strip_bytes;
  int32_t strip_copy_bytes;
  int64_t strip_grid_bytes;
  // The strip copies of gridi (score_phase_kernel's strip form; csm_palette.hip
  // istrip_geom): bytes per strip, per copy and per grid of the stack.
  const int32_t* istrips;
  int32_t istrip_bytes;
  int32_t istrip_copy_bytes;
  int64_t istrip_grid_bytes;
  // the fused fast finish (tail.on = 0: scores only; csm_tail.hpp)
  TailArgs tail;
  // the largest n_used of the level's windows (0: unknown); the pair kernel
  // takes its run-free form at or below kPairNoRunBeams (csm_box.hip)
  int32_t max_n_used;
};

// Argmax partial: best score of a block and its flat candidate index.
struct BestPartial {
  double score;
  int64_t flat;
};

constexpr int kBlock = 256;      // 4 waves
constexpr int kChunk = 1024;     // beams staged in LDS per pass (16 KB)

constexpr int kFinishWaveScratch = 640;  // bytes of per-wave scratch
#ifndef CSM_FINISH_WAVES
#define CSM_FINISH_WAVES 4
#endif
constexpr int kFinishWaves = CSM_FINISH_WAVES;  // waves per window of the exact finish
// misc block of the finish carve (csm_finish.hip Shared): counts, limits,
// best (x, y), per-wave reductions
constexpr size_t kFinishMisc = (48 + 16 * (size_t)kFinishWaves + 4 + 15) & ~(size_t)15;

struct FinishLayout {
  size_t wave_scratch, defer, keys, vals, lpos, rpos, stack, fout, total;
};
constexpr int kFinishDefer = 64;  // segments the partial sort may set aside (12 B each)

// LDS carve of the finish kernel for n candidates (16-byte aligned pieces):
// misc | kFinishWaves wave scratches | deferred segments | keys f64[n] | vals u16[n] |
// lpos u16[n] | rpos u16[n] | shared segment stack | FinishOut.
constexpr FinishLayout finish_layout(int64_t n) {
  FinishLayout L{};
  size_t o = kFinishMisc;
  L.wave_scratch = o;
  o += (size_t)kFinishWaves * kFinishWaveScratch;
  L.defer = o;
  o += (size_t)kFinishDefer * 12;
  L.keys = o;
  o += (size_t)n * 8;
  L.vals = o;
  o += ((size_t)n * 2 + 15) & ~(size_t)15;
  L.lpos = o;
  o += ((size_t)n * 2 + 15) & ~(size_t)15;
  L.rpos = o;
  o += ((size_t)n * 2 + 15) & ~(size_t)15;
  L.stack = o;
  o += ((size_t)(n / 16 + 64) * 12 + 15) & ~(size_t)15;  // live segments
  L.fout = o;  // the window's FinishOut, assembled here and stored sealed
  o += (sizeof(FinishOut) + 15) & ~(size_t)15;
  L.total = o;
  return L;
}
constexpr size_t finish_lds_bytes(int64_t n) { return finish_layout(n).total; }

// A.host_flag (the few-window path): the caller's scoring launch zeroed
// exact_list[0] already; the exact pass then signals the host when done.
// exact_on_device = false: only the fast pass runs; the windows it flags
// (need_exact) are left for the host's std::sort (csm_api.cpp level_end).
// The fast pass (when A.need_exact) and the exact pass on `stream`; with
// exact_stream (and ev_fast, an event to record) the exact pass runs there,
// after the fast pass.
// fast_done: the scoring launches ran the fast pass's decisions themselves
// (the fused finish, csm_tail.hpp): only the exact pass is launched.
hipError_t launch_finish(const FinishArgs& A, const ScanWork* d_scans, const AngleEntry* d_angles,
                         const double* d_scores, FinishOut* d_out, int32_t n_windows,
                         hipStream_t stream, hipStream_t exact_stream = nullptr, hipEvent_t ev_fast = nullptr,
                         bool fast_done = false);

// Launchers (csm_kernels.hip). All enqueue on `stream` and return hipError_t.
// Column kernel (v2): lane = one (theta, x) column of a window, KT rows (y)
// per lane; L.blocks_per_scan = col_blocks * ktiles. kt = 4, 8 or 16.
hipError_t launch_score_cols(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials,
                             int kt, hipStream_t stream);
// Row-segment kernel (v3, INT mode only): lane = (theta, r); one angle group
// of ns lanes per angle, 64/ns groups per wave; L.blocks_per_scan =
// ceil(n_angles / (64/ns)). sq 16-byte loads per row segment (4*sq cells).
// rows_pick_sq returns the sq of an instantiation with 4*sq >= need_seg, or 0.
int rows_pick_sq(int ns, int need_seg);
// v4: row segments staged in LDS by LDS-DMA (score_rowsd_kernel).
hipError_t launch_score_rows(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials,
                             int ns, int sq, hipStream_t stream);
// FAST (branch-and-bound) tree scoring (csm_bnb.hip): every node of every
// level, per window and angle, laid out level max_depth first.
constexpr int kTreeMaxDepth = 12;
struct TreeWork {
  int32_t n_angles, n_low, depth, n_windows;
  int64_t nodes_per_angle;     // sum over levels of (n_low << (depth - l))^2
  double f_low;                // lowest-resolution step in cells (:347)
  double hw[kTreeMaxDepth + 1];  // hw[d]: half_width applied below depth d (:454-455)
  const float* grid;           // packed fp32 grid
  int32_t size_x, size_y;
  float outside;
  int32_t pad;
};
hipError_t launch_score_tree(const TreeWork& T, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, hipStream_t stream);

// Tiny-window kernel (v8, csm_tiny.hip): INT mode, 2 <= n_space <= 4 with
// (n_space - 1) * step < 1 cell; one wave per (window, angle), lanes are
// beams. blocks_per_scan = n_angles.
bool tiny_supported(int ns, double f);
hipError_t launch_score_tiny(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                             const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                             hipStream_t stream);
// Box kernel (v6, csm_box.hip): INT mode, window step exactly one cell,
// n_space <= 16; one wave per (window, angle), one 16-byte row piece per lane
// per beam. blocks_per_scan = n_angles.
bool box_supported(int ns);
// The grid's palette (the pair box kernel below): at most kPalMax distinct
// fixed-point values (L.pal_n > 0); boxes of n_space <= kPalMaxSpace.
constexpr int kPalMax = 256;
constexpr int kPalMaxSpace = 13;
// The palette of n int32 cells (gridi with its padding): distinct values
// (0 first, then ascending) into vals[0..kPalMax), their count into
// state[0] (kPalMax + 1: more than kPalMax, no palette) and each cell's index
// into idx. scratch: pal_scratch_ints(n) ints.
int64_t pal_scratch_ints(int64_t n);
// max over n points (x, y) of |x| + |y| (NaN if any is NaN) as the bits of a
// non-negative double, max-ed into *out (zeroed by the caller)
hipError_t launch_points_maxabs(const double* pts, int64_t n, unsigned long long* out, hipStream_t stream);
hipError_t launch_build_palette(const int32_t* gridi, int64_t n, int32_t* scratch, int32_t* vals, int32_t* state,
                                uint8_t* idx, hipStream_t stream);
// v11 pair box kernel: palettes of at most kPairMaxPal values, read from
// kStripCopies strip copies of the index grid (copy c holds cell x at byte
// x + 4c of its strip row; strips kStripW bytes wide, rows contiguous), so a
// box row piece is one aligned 16-byte strip row and a box's 13 rows are 208
// contiguous bytes (2.5 cache lines, not 13-14).
constexpr int kPairMaxPal = 16;
constexpr int kStripW = 16;
#ifndef CSM_STRIP_COPIES
#define CSM_STRIP_COPIES 16
#endif
// copies of the index grid, each kStripShift cells further along: 16 puts
// every box row at byte 0 of its strip row (64 MB for a 2000^2 grid); 4
// leaves a byte phase ix0 & 3 the kernel aligns (v_alignbyte, 16 MB). r04,
// isolated coarse launch of 4096 windows: 1.404 ms with 4, 1.358 with 16.
constexpr int kStripCopies = CSM_STRIP_COPIES;
constexpr int kStripShift = kStripW / kStripCopies;
static_assert(kStripCopies == 4 || kStripCopies == 16, "strip copies: 4 or 16");
constexpr int kStripPadRows = 16;  // zero rows below the grid (box rows and the zero run's rows)
// Columns and rows before the grid's first (pair strips): column -1 repeats
// column 0 and row -1 row 0, the rest hold index 0 (the outside value). The
// reference truncates toward zero, so a cell coordinate t in (-1, 0) reads
// cell 0 and t <= -1 reads outside (occu_grid_map.h GetCell's bounds): with
// this padding a box corner floor(t) >= -kStripPadLo reads what the reference
// reads, and a beam whose box straddles the grid's low edge stays on the fast
// path (r05: 10 % of the headline's waves had such beams, 0.8 % of beams,
// each summed cell by cell before).
constexpr int kStripPadLo = 16;
struct StripGeom {
  int32_t rows, n_strips;
  int64_t strip_bytes, copy_bytes, grid_bytes;
};
StripGeom strip_geom(int size_x, int size_y);
// idx: the palette index grid(s) (row pitch `pitch` bytes, idx_stride bytes
// per grid); out: n_grids * strip_geom().grid_bytes bytes.
hipError_t launch_build_strips(const uint8_t* idx, int pitch, int size_x, int size_y, int64_t idx_stride,
                               int n_grids, uint8_t* out, hipStream_t stream);
bool box_pair_supported(int ns);
// Strip copies of gridi for the phase kernel: copy c (of kIStripCopies) holds
// cell x of row y at cell x + 4c of its strip row, strips kIStripCells cells
// (32 bytes) wide with their rows contiguous, so a 5 x 5 phase box (corner
// phase <= 3 cells, two 16-byte pieces per row) is 160 contiguous bytes.
constexpr int kIStripCells = 8;
constexpr int kIStripCopies = 2;
constexpr int kIStripPadRows = 16;
// columns and rows before the grid's first in the phase strips, as
// kStripPadLo for the pair strips (column -1 repeats column 0, row -1 row 0,
// the rest outside): a box straddling the low edge stays on the fast path
// (r05: 6 % of the headline's fine-level waves summed such beams cell by cell)
constexpr int kIStripPadLo = 16;
StripGeom istrip_geom(int size_x, int size_y);
hipError_t launch_build_istrips(const int32_t* gridi, int pitch, int size_x, int size_y, int64_t gridi_stride,
                                int n_grids, int32_t* out, hipStream_t stream);
hipError_t launch_score_box_pair(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                                 const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                                 hipStream_t stream);
hipError_t launch_score_box(const LevelWork& L, const ScanWork* d_scans, const double* d_pts,
                            const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                            hipStream_t stream);
// Phase kernel (v7, csm_phase.hip): INT mode, sub-cell window step f < 1.
// A beam's cell offset for candidate j is floor(phase + j*f), constant over
// each phase bucket; the host builds the buckets (csm_api.cpp phase_table).
constexpr int kPhaseMaxBuckets = 8;
constexpr int kPhaseMaxSpace = 16;
struct PhaseTable {
  int32_t nq;                                  // buckets in use (<= the kernel's NQ)
  int32_t cells;                               // distinct offsets per axis: max ox + 1
  double lo[kPhaseMaxBuckets], hi[kPhaseMaxBuckets];  // bucket q: lo[q] <= phase <= hi[q]
  int8_t ox[kPhaseMaxBuckets][kPhaseMaxSpace]; // floor(phase + j*f) inside bucket q
  // Buckets of equal width 1 / nq (f a multiple of 1 / nq, e.g. 0.4 cells: 5):
  // bucket q = floor(phase * nq) when frac(phase * nq) is in [ulo, uhi]
  // (phase_table: inside every bucket's [lo, hi] with room for the product's
  // rounding), five comparisons a bucket fewer per beam and axis
  int32_t uniform;
  double ulo, uhi;
};
bool phase_supported(int ns, int cells, int nq);
hipError_t launch_score_phase(const LevelWork& L, const PhaseTable& T, const ScanWork* d_scans, const double* d_pts,
                              const AngleEntry* d_angles, double* d_out, BestPartial* d_partials, int ns,
                              hipStream_t stream);
// Split kernel (csm_split.hip): launches of few windows, INT mode, any window
// step. Lane = candidate, 256-candidate chunks, a window's beams split over
// `splits` blocks per chunk (<= kSplitMaxBeams each), int32 partial sums
// handed to the chunk's last block through a slab.
constexpr int kSplitThreads = 256;
constexpr int kSplitMaxBeams = 32;   // 32 * 2^26 <= 2^31: a split's int32 sum cannot overflow
constexpr int kSplitArgAngles = 64;  // angle rows a single window carries in the kernel arguments
struct SplitWork {
  int32_t splits;         // beam splits per chunk
  int32_t chunks;         // ceil(n_cand / kSplitThreads) per window
  int32_t inline_window;  // 1: one window, its ScanWork and angle rows in `sw` / `ang`
  int32_t clear_tag;      // with clear_word: LevelWork::clear_tag
  int32_t* slab;          // n_scans * chunks * splits * kSplitThreads int32 partial sums
  int32_t* arrive;        // n_scans * chunks arrival counters: zero before and after a launch
  int32_t* clear_word;    // set by block 0 (nullable): LevelWork::clear_word
  ScanWork* scans_out;    // inline window: block 0 stores it here for the finish ...
  AngleEntry* angles_out; // ... and its angle rows here
  ScanWork sw;
  AngleEntry ang[kSplitArgAngles];
};
hipError_t launch_score_split(const LevelWork& L, const SplitWork& W, const ScanWork* d_scans, const double* d_pts,
                              const AngleEntry* d_angles, double* d_out, hipStream_t stream);
// csm_trig.hip: rows[i].cosine / .sine = glibc sincos(rows[i].angle), bit-equal
// to the host's (libm_sincos.hpp; d_tab: libm's 440-double table); rows whose
// angle is outside the restated domain are left as they are.
hipError_t launch_angle_trig(AngleEntry* d_rows, int64_t n, const double* d_tab, hipStream_t stream);
// csm_trig.hip: the rows of windows d_sw[0..nw) whole (angle, cos, sin) from
// each window's ct: θ_a = (ct - offset) + a * ares, at rows[S.angle_off + a];
// every θ inside the restated domain (the caller checks).
hipError_t launch_angle_rows(const ScanWork* d_sw, int nw, int n_angles, double offset, double ares, AngleEntry* d_rows,
                             const double* d_tab, hipStream_t stream);
// gridi layout: row pitch = round4(size_x + kGridiPadCols) cells, size_y +
// kGridiPadRows rows; every cell outside [0,size_x) x [0,size_y) is zero, so a
// 16 x 16 box whose corner lies on the grid never leaves the buffer.
constexpr int kGridiPadCols = 15;
constexpr int kGridiPadRows = 16;
constexpr int32_t gridi_pitch(int32_t sx) { return (sx + kGridiPadCols + 3) & ~3; }
// Grid statistics for the exact integer path (csm_set_grid).
struct GridStats {
  int32_t min_gexp;       // every nonzero |v| is a multiple of 2^min_gexp
  uint32_t max_abs_bits;  // bits of max |v| (positive floats order as integers)
  int32_t nonfinite;
  int32_t pad;
};
// d_stats: 1 + kAnalyzeBlocks entries (result, then per-block partials).
constexpr int kAnalyzeBlocks = 1024;
hipError_t launch_analyze_grid(const float* g, int64_t n, GridStats* d_stats, hipStream_t stream);
// Row pitch of gridi is a multiple of 4 cells, so 16-byte row segments are
// aligned; size_y + kGridiPadRows rows are written, the pad zero.
// pad = false converts rows only (a row range of a resident grid, no pad rows).
hipError_t launch_fixed_point(const float* g, int32_t sx, int32_t sy, int32_t pitch, float outside,
                              int int_exp, int32_t* gi, hipStream_t stream, bool pad = true);
// One cell of an incremental grid refresh (csm_update_grid_cells).
struct CellUpdate {
  int32_t index;  // y * size_x + x
  float value;
};
// gi null: no fixed-point copy to keep in step.
hipError_t launch_update_cells(const CellUpdate* d_updates, int64_t n, float* g, int32_t sx, int32_t* gi,
                               int32_t pitch, float outside, int int_exp, hipStream_t stream);
// ---- Gauss-Newton scan matcher (csm_optimize.hip) --------------------------
// Per scan and iteration: the pose in map cells and the host glibc cos/sin of
// its angle (optimize_scan_matcher.h:94-97).
struct OptScan {
  double c, s, tx, ty;
  int32_t active;
  int32_t pad;
};
// Sums of UpdateCost (optimize_scan_matcher.h:154-221) in point order:
// v = {cost, H00, H10, H11, H20, H21, H22, b0, b1, b2}; valid = points in map.
struct OptSums {
  double v[10];
  int32_t valid;
  int32_t pad;
};
struct OptArgs {
  const float* grid;  // packed fp32 grid, row-major
  int32_t size_x, size_y;
  float outside;
  int32_t pad;
  const double* pts;        // map-cell (x, y) points of every scan
  const int64_t* offsets;   // n_scans + 1 prefix offsets into pts
  const OptScan* scans;
  OptSums* out;
};
hipError_t launch_optimize_cost(const OptArgs& A, int32_t n_scans, hipStream_t stream);

// Reduce per-window partials (blocks_per_scan each) to one BestPartial per window.
hipError_t launch_reduce_best(const BestPartial* d_partials, int32_t blocks_per_scan,
                              int32_t n_windows, BestPartial* d_out, hipStream_t stream);

}  // namespace csm
