/*
 * csm.h — C-ABI of the MI355X-native correlative scan matcher.
 *
 * This is the drop-in boundary for RoboRTS-Edu-SLAM's hot path, the
 * correlative (x, y, theta) search of src/scan_match/correlate_scan_matcher.h.
 * Plain C: POD structs, raw pointers, sizes and int status codes. No C++
 * exceptions, no torch or Eigen types cross this boundary.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository root):
 *
 *   csm_param                 CorrelationScanMatchParam  correlate_scan_matcher.h:41-86
 *   csm_match_type            CorrelationScanMatchType   correlate_scan_matcher.h:34-39
 *   csm_map_info              GridMapBase geometry       grid_map_base.h:47-71,307-309,371-378
 *   csm_set_grid              OccuGridMap cell storage read by GetGridProbValue
 *                                                        occu_grid_map.h:395-397, grid_map_base.h:352-354
 *   csm_update_grid_cells/rows  the cells UpdateMapByRange / ResetValueSpeedup rewrite
 *                                                        occu_grid_map.h:258-329, grid_map_base.h:114-120
 *   csm_scan_match            BasedCorrelationScanMatch::ScanMatch
 *                                                        correlate_scan_matcher.h:784-875
 *   csm_scan_matchers         ScanMatchers::ScanMatch (3-level coarse->fine->super)
 *                                                        scan_matchers.h:179-289
 *   csm_score_window          MultiResolutionCorrelateScanMatcher::ScanMatch enumeration +
 *                             GetResponse + PenalizeResponse, all candidate scores in
 *                             reference enumeration order (theta, x, y)
 *                                                        correlate_scan_matcher.h:516-603,637-662,718-745
 *   csm_best_window           same scoring, reduced on device to (max score, lowest flat index)
 *                             (large windows / loop-closure shards; no reference counterpart,
 *                             SURVEY.md 8e)
 *   csm_search_windows        the same argmax over many windows by an admissible
 *                             multi-resolution branch and bound (max-pooled levels);
 *                             the reference's FAST matcher is the non-admissible form
 *                                                        correlate_scan_matcher.h:271-502
 *   csm_optimize_scan_match   BasedOptimizeScanMatch::ScanMatch (Gauss-Newton)
 *                                                        optimize_scan_matcher.h:68-221
 *   csm_scan_match with       BranchAndBoundCorrelateScanMatcher::ScanMatch (FAST type,
 *   type == CSM_FAST          dispatched from BasedCorrelationScanMatch::ScanMatch :815-821)
 *                                                        correlate_scan_matcher.h:274-502
 *
 * Threading: every entry point locks the context; a context may be shared by
 * the front-end (ROS callback) thread and the back-end thread exactly like the
 * reference's shared ScanMatchers (scan_matchers.h:298, slam_processor.cpp:139,292).
 *
 * Error convention: 0 = success. The reference logs and returns 0.0 for an
 * uninitialised map or an empty scan (correlate_scan_matcher.h:792-795); this ABI
 * does the same (status CSM_OK, *response = 0.0, pose and covariance untouched).
 * Any other failure returns a non-zero status and csm_last_error() explains it;
 * the product never silently falls back to a CPU path.
 */
#ifndef ROBORTS_CSM_H
#define ROBORTS_CSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSM_ABI_VERSION 1

enum csm_status {
  CSM_OK = 0,
  CSM_ERR_INVALID_ARG = 1,
  CSM_ERR_HIP = 2,
  CSM_ERR_NO_GRID = 3,
  CSM_ERR_ALLOC = 4,
  CSM_ERR_UNSUPPORTED = 5
};

/* correlate_scan_matcher.h:34-39 */
enum csm_match_type {
  CSM_COARSE = 0,
  CSM_FINE = 1,
  CSM_SUPER = 2,
  CSM_FAST = 3
};

/* CorrelationScanMatchParam (correlate_scan_matcher.h:41-86). Units as in the
 * reference: sizes/resolutions in metres, angles in radians. */
typedef struct csm_param {
  double search_space_size;        /* full window width (m)                  */
  double search_space_resolution;  /* window step (m)                        */
  double search_angle_offset;      /* +/- angle half width (rad)             */
  double search_angle_resolution;  /* angle step (rad)                       */
  double response_threshold;       /* pose written back only above this      */
  int32_t use_point_size;          /* U: beam subsampling target             */
  int32_t max_depth;               /* BnB depth (FAST type only)             */
  int32_t use_center_penalty;      /* bool                                   */
  int32_t type;                    /* enum csm_match_type                    */
} csm_param;

/* Geometry of a ScanMatchMap (GridMapBase, grid_map_base.h:47-71).
 * world_to_map = Scaling(1/resolution) * Translation(offset). */
typedef struct csm_map_info {
  double resolution;    /* cell length used to build the map (m)             */
  double offset_x;      /* map_offset_ (m)                                   */
  double offset_y;
  int32_t size_x;       /* cells                                             */
  int32_t size_y;
  int32_t update_index; /* map_update_index_; < 0 means IsMapInit()==false    */
  int32_t reserved;
} csm_map_info;

/* Result of an argmax-only search (csm_best_window). flat_index is in the
 * reference enumeration order ((theta * n_space + x) * n_space + y); ties are
 * broken by the lowest flat index. */
typedef struct csm_best {
  double score;
  int64_t flat_index;
  double x, y, angle;   /* candidate pose in map cells / rad                 */
} csm_best;

/* Per-kernel accounting collected with HIP events on the context's stream
 * while profiling is on (csm_set_profiling). algorithmic_bytes counts one
 * fp32 grid read per summed beam per candidate (4*B bytes per scoring). */
typedef struct csm_kernel_stat {
  char name[48];
  int64_t launches;
  double total_ms;
  double algorithmic_bytes;
  double scorings;
} csm_kernel_stat;

typedef struct csm_ctx csm_ctx;

/* --- lifetime ---------------------------------------------------------- */
int csm_create(int device, csm_ctx** out);
int csm_destroy(csm_ctx* ctx);
const char* csm_last_error(const csm_ctx* ctx);
int csm_abi_version(void);
/* Digest of the library sources this build was compiled from
 * (tools/source_digest.py): tells a stale prebuilt .so from the tree's code. */
const char* csm_build_digest(void);
/* Value read for an endpoint outside the grid. The reference reads out of
 * bounds (UB, grid_map_base.h:352-354); this ABI defines it. Default 0.3f =
 * kMapUnknownCellProb (slam/slam_processor.h:264). */
int csm_set_outside_value(csm_ctx* ctx, float value);

/* --- grid residency ------------------------------------------------------ */
/* Upload a host grid. cells points at the first cell's probability (float);
 * cell_stride_bytes is 8 for the reference's AoS ProbabilityCell
 * {float prob_value_; int update_index_;} (grid_map_cell.h:301-328) and 4 for
 * a packed float grid. Row-major, index y*size_x + x (grid_map_base.h:352-354).
 * The device copy is keyed on (cells, stride, size, version): a call with an
 * unchanged key skips the upload. Pass version = -1 to force the upload. */
int csm_set_grid(csm_ctx* ctx, const void* cells, int64_t cell_stride_bytes,
                 const csm_map_info* info, int64_t version);
/* Incremental refresh of a grid made resident by csm_set_grid (the same
 * cells pointer, stride and geometry; otherwise the whole grid is uploaded).
 * Replaces re-uploading the map after OccuGridMap::UpdateMapByRange
 * (occu_grid_map.h:258-329): the reference rewrites only the cells it lists
 * in map_update_point_ (occu_grid_map.h:509,528,571) and resets only those in
 * ResetValueSpeedup (grid_map_base.h:114-120).
 *   csm_update_grid_cells: the listed cells (indices y*size_x + x, any order,
 *                          duplicates allowed) are re-read from cells.
 *   csm_update_grid_rows:  rows [row_begin, row_end) are re-read.
 * The grid's key takes the new version. Up to four host maps stay resident at
 * once, keyed on their cells pointer (least recently used evicted), so the
 * front end's and the back end's maps do not evict each other. */
int csm_update_grid_cells(csm_ctx* ctx, const void* cells, int64_t cell_stride_bytes,
                          const csm_map_info* info, int64_t version,
                          const int32_t* cell_indices, int64_t n_indices);
int csm_update_grid_rows(csm_ctx* ctx, const void* cells, int64_t cell_stride_bytes,
                         const csm_map_info* info, int64_t version,
                         int32_t row_begin, int32_t row_end);
/* Borrow a packed float grid that already lives in device memory of this
 * context's device (size_y * size_x floats). The caller keeps it alive. */
int csm_set_grid_device(csm_ctx* ctx, const float* device_prob,
                        const csm_map_info* info);

/* --- window geometry ----------------------------------------------------- */
/* n_angles = floor(2*offset/ares)+1 (correlate_scan_matcher.h:154),
 * n_space = Round(size/res)+1 (:538). */
int csm_window_dims(const csm_param* param, int32_t* n_angles, int32_t* n_space);

/* The angle rows' cos/sin as the 3-level driver computes them on the device
 * (AngleSearchLookUpTable::UpdateLookUpTable correlate_scan_matcher.h:171-172,
 * one glibc sincos per angle as GCC compiles it): glibc 2.35's sincos restated
 * for the GPU over the table of the libm this process has mapped, so each
 * result equals the host's sincos(x[i]) bit for bit. Arguments outside the
 * restated domain (|x| >= 105414350, not finite) are computed by the host.
 * CSM_ERR_UNSUPPORTED when the host's libm did not pass the table checks (the
 * driver then keeps the host sincos). Host buffers of n doubles. */
int csm_sincos_device(csm_ctx* ctx, const double* x, int64_t n, double* sin_out, double* cos_out);

/* --- drop-in entry points (host buffers) -------------------------------- */
/* BasedCorrelationScanMatch::ScanMatch. points_xy: n_points (x, y) pairs in
 * map-cell units, sensor frame (RangeDataContainer after CreateFrom with the
 * map's 1/resolution, sensor_data_manager.h:99-115). pose: world (x, y, theta)
 * in/out. cov: row-major 3x3 in/out (partially written per type, :835-858).
 * argmax_flat (nullable): enumeration index of the candidate std::sort put
 * first (-1 when the reference's early return applies). */
int csm_scan_match(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                   const csm_param* param, double pose[3], double cov[9],
                   double* response, int64_t* argmax_flat);

/* ScanMatchers::ScanMatch with use_optimize_scan_match = false (both reference
 * YAMLs) and the grid already sized by the caller's MapSizeCheck:
 * levels[0..2] = coarse, fine, super-fine params, all matched on the current
 * grid (scan_matchers.h:238,249,256). use_fine = false runs only the coarse
 * level. score = mean of the level responses (:281). */
int csm_scan_matchers(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                      const csm_param levels[3], int32_t use_fine,
                      double pose[3], double cov[9], double* score);

/* Batched forms: n_scans independent scans matched on the same grid in one
 * pass per level. point_offsets has n_scans+1 entries (prefix offsets in
 * points). poses n_scans*3, covs n_scans*9, responses n_scans. */
int csm_scan_match_batch(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                         const int64_t* point_offsets, const csm_param* param,
                         double* poses, double* covs, double* responses,
                         int64_t* argmax_flat);
int csm_scan_matchers_batch(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                            const int64_t* point_offsets, const csm_param levels[3],
                            int32_t use_fine, double* poses, double* covs,
                            double* scores);

/* Device-resident scan sets: csm_load_scans uploads a batch of scans once;
 * csm_scan_matchers_loaded runs the 3-level driver over it (poses/covs/scores
 * as in csm_scan_matchers_batch). Any other call that takes host points
 * replaces the loaded set. csm_load_scans, and the calls built on it
 * (csm_scan_matchers, csm_scan_matchers_batch, the *_grids forms), drop the
 * batches queued with csm_load_scans_async: the batch they load is the one
 * that is matched. */
int csm_load_scans(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                   const int64_t* point_offsets);
int csm_scan_matchers_loaded(csm_ctx* ctx, const csm_param levels[3], int32_t use_fine,
                             double* poses, double* covs, double* scores);

/* Streams of batches (the reference's points come from host memory,
 * sensor_data_manager.h:99-115): csm_load_scans_async queues a batch whose
 * upload runs on a copy stream of its own, concurrently with whatever the
 * context is matching; the next csm_scan_matchers_loaded takes the oldest
 * queued batch (waiting for its upload) before it matches. At most two
 * batches are queued. points_xy must stay unchanged until that call returns,
 * and should be pinned (csm_host_alloc): pageable memory makes the upload
 * synchronous. Typical loop: queue batch 0; for each i: queue batch i + 1,
 * then csm_scan_matchers_loaded (batch i, while batch i + 1 goes up). */
int csm_load_scans_async(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                         const int64_t* point_offsets);
/* Batches in flight back to back (no reference counterpart: a stream of
 * ScanMatchers::ScanMatch batches, scan_matchers.h:179-289, over the loaded
 * scans). csm_scan_matchers_submit does what csm_scan_matchers_loaded does
 * except that the batch's last level is left pending: the next submit's first
 * launch goes out before that level is completed, so the device does not wait
 * for the host between batches. poses / covs / scores of a submitted batch
 * are final once the next submit, csm_scan_matchers_wait, or any other call on
 * the context returns (every other entry point completes a pending batch
 * first); they must stay valid until then. Results equal
 * csm_scan_matchers_loaded's bit for bit. */
int csm_scan_matchers_submit(csm_ctx* ctx, const csm_param levels[3], int32_t use_fine, double* poses, double* covs,
                             double* scores);
int csm_scan_matchers_wait(csm_ctx* ctx);
/* Pinned (page-locked) host memory for csm_load_scans_async inputs. */
int csm_host_alloc(size_t bytes, void** out);
int csm_host_free(void* p);

/* --- host placement (one process per GPU) -------------------- */
/* A context's host worker pool (window planning and completion) runs on a
 * slice of the CPUs near its GPU: the process's affinity mask intersected with
 * the GPU's NUMA node, split into disjoint slices among the local ranks whose
 * GPUs share that node, and as many threads as the rank's share of the
 * cgroup's CPU quota allows (quota / local ranks, at most 16). csm_create takes
 * the local rank and count from LOCAL_RANK / LOCAL_WORLD_SIZE (torchrun,
 * bench.py), rank r driving device r; CSM_HOST_THREADS overrides the count.
 * No reference counterpart: the reference matches on one host thread. */
#define CSM_HOST_PLAN_MAX_CPUS 512
typedef struct csm_host_plan {
  int32_t threads;        /* pool size, the calling thread included */
  int32_t numa_node;      /* the GPU's NUMA node, -1 unknown */
  int32_t quota_cpus;     /* the cgroup's CPU quota in whole CPUs, -1 none */
  int32_t affinity_cpus;  /* CPUs in the process's affinity mask */
  int32_t n_cpus;         /* CPUs the pool's workers are pinned to (0: not pinned) */
  int32_t cpus[CSM_HOST_PLAN_MAX_CPUS];
} csm_host_plan;
/* The plan of local rank local_rank of local_world on this host, without a
 * GPU: numa_of_rank[r] is rank r's GPU NUMA node (-1 unknown; null: all
 * unknown), quota_cpus 0 reads the cgroup, -1 means none, > 0 is taken as is. */
int csm_host_plan_compute(int32_t local_rank, int32_t local_world, const int32_t* numa_of_rank,
                          int32_t quota_cpus, csm_host_plan* out);
/* The plan a context runs with. */
int csm_get_host_plan(csm_ctx* ctx, csm_host_plan* out);

/* --- Gauss-Newton scan matcher ---------------------- */
/* OptimizeScanMatchParam (optimize_scan_matcher.h:33-58), filled by
 * ScanMatchers::ScanMatchParamInit (scan_matchers.h:346-350). */
typedef struct csm_optimize_param {
  int32_t iterate_max_times;
  int32_t reserved;
  double cost_decrease_threshold;
  double cost_min_threshold;
  double max_update_distance;      /* m   */
  double max_update_angle;         /* rad */
} csm_optimize_param;

/* BasedOptimizeScanMatch::ScanMatch (optimize_scan_matcher.h:68-132) on the
 * current grid: Gauss-Newton on (x, y, theta) with the bilinear cell
 * interpolation of UpdateCost (:154-221). points_xy as in csm_scan_match
 * (cells of this grid, sensor frame); pose world in/out; *cost = the
 * reference's return value. As the reference: an uninitialised map, an empty
 * scan or a NaN step gives cost 1000 (kMaxCost) and leaves the pose untouched.
 * Sums over points are the reference's sequential fp64 sums; cos/sin and the
 * 3x3 LDLT solve (Eigen 3.3 restated) run on the host between iterations. */
int csm_optimize_scan_match(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                            const csm_optimize_param* param, double pose[3], double* cost);
/* n_scans independent scans on the same grid, one launch per iteration for
 * all of them. iterations (nullable): UpdateCost evaluations per scan. */
int csm_optimize_scan_match_batch(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                                  const int64_t* point_offsets, const csm_optimize_param* param,
                                  double* poses, double* costs, int32_t* iterations);

/* Test hook: one UpdateCost evaluation (optimize_scan_matcher.h:154-221) on
 * the device at a map-cell pose; cost normalised as the reference (:220), H
 * row-major (symmetric), b. */
int csm_optimize_update_cost(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                             const double est_map[3], double* cost, double H[9], double b[3]);

/* --- many scans, each on its own resident grid ------------------------------ */
/* As csm_load_scans / csm_scan_matchers_batch, with scan i matched on grid
 * grid_index[i] of the resident stack (csm_set_grid_stack or
 * csm_set_grid_stack_gridmaps); the grids share one geometry. Used by the
 * back-end's batched ScanMatchInterface (csm_backend.h). */
int csm_load_scans_grids(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                         const int64_t* point_offsets, const int32_t* grid_index);
int csm_scan_matchers_batch_grids(csm_ctx* ctx, int32_t n_scans, const double* points_xy,
                                  const int64_t* point_offsets, const int32_t* grid_index,
                                  const csm_param levels[3], int32_t use_fine, double* poses,
                                  double* covs, double* scores);

/* --- measurement ---------------------------------------------------------- */
/* HIP-event timing of scoring launches (resets the stats): 0 off, 1 every
 * launch and its finish, 2 the 3-level drivers' first-level scoring kernels
 * only (csm_scan_matchers_loaded / _submit: no events around their finish
 * passes or later levels). */
int csm_set_profiling(csm_ctx* ctx, int32_t on);
/* Copy up to capacity stats; *count = number of distinct kernels seen. */
int csm_kernel_stats(csm_ctx* ctx, csm_kernel_stat* out, int32_t capacity, int32_t* count);

/* Test hook: the permutation the device finish applies to n keys — its
 * emulation of libstdc++'s std::sort(greater) (correlate_scan_matcher.h:607).
 * n <= 10240. order receives n indices. */
int csm_sort_order(csm_ctx* ctx, const double* keys, int64_t n, int64_t* order);

/* Test hook (host only, no device): the phase buckets the v7 phase kernel
 * uses for a window step of step_cells (< 1) map cells over n_space
 * positions (csm_phase.hip; correlate_scan_matcher.h:569-572 enumeration).
 * Bucket q holds the phases lo[q] <= p <= hi[q] of t = (lx + x0) + 0.5, in
 * which candidate j reads column floor(t) + ox[q * 16 + j]. Arrays hold 8
 * buckets (ox: 8 x 16). Returns CSM_ERR_UNSUPPORTED when no table exists. */
int csm_phase_buckets(double step_cells, int32_t n_space, int32_t margin_log2, int32_t* n_buckets,
                      int32_t* cells, double* lo, double* hi, int8_t* ox);

/* --- raw scoring --------------------------------------------------------- */
/* Every candidate score of one window (after the centre penalty when
 * param->use_center_penalty), in reference enumeration order. center_map is
 * the window centre in map cells / rad (GetMapCoordsPose of the world pose).
 * n_out must equal n_angles * n_space^2. */
int csm_score_window(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                     const csm_param* param, const double center_map[3],
                     double* scores_out, int64_t n_out);

/* Argmax-only scoring of one window: max score, lowest flat index on ties.
 * Intended for windows far larger than the front end's (loop closure). */
int csm_best_window(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                    const csm_param* param, const double center_map[3],
                    csm_best* best);

/* --- loop-closure shards ----------------------------------- */
/* Make n_grids same-size packed fp32 grids resident back to back (submaps of
 * one shard: n_grids * size_y * size_x floats). info gives their common size
 * and resolution; every window names its grid and carries its own centre, so
 * per-submap offsets stay with the caller. Replaces the single grid of
 * csm_set_grid. */
int csm_set_grid_stack(csm_ctx* ctx, const float* cells, int32_t n_grids,
                       const csm_map_info* info, int64_t version);
/* Argmax-only scoring of one scan in n_windows windows, window i on grid
 * grid_index[i] (null: grid 0) centred at centers_map[3i..3i+2] (map cells /
 * rad). best[i] as csm_best_window. One launch for all windows. */
int csm_best_windows(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                     const csm_param* param, int32_t n_windows, const int32_t* grid_index,
                     const double* centers_map, csm_best* best);

/* --- admissible multi-resolution search (north_star: branch-and-bound
 *     across resolution levels; SURVEY.md 8e, BASELINE configs 3 and 4) ---- */
/* The best candidate of n_windows windows of one scan (window i on grid
 * grid_index[i], centred at centers_map[3i..3i+2], as csm_best_windows):
 * the maximum score, ties to the lowest (window, flat index) -- exactly what
 * reducing csm_best_windows' per-window results gives, and what the
 * reference's exhaustive MultiResolutionCorrelateScanMatcher::ScanMatch
 * (correlate_scan_matcher.h:516-603) ranks first, minus its sort.
 *
 * Unlike the reference's FAST matcher (BranchAndBoundCorrelateScanMatcher,
 * :271-502), whose lowest level reads the raw grid and so may prune the best
 * candidate, every level d >= 1 here reads a max-pooled copy of the grid
 * ((2^d + 1)^2 cells per anchor), so a node's score bounds every candidate
 * below it and the answer equals the exhaustive one. The pooled levels are
 * built once per resident grid (stack) and kept until it changes.
 *
 * Applies to windows with a step of exactly one map cell on a grid the exact
 * fixed-point path accepts; any other window is searched exhaustively on the
 * device (stats->exhaustive = 1), with the same result. */
typedef struct csm_search_options {
  int32_t max_depth;       /* top level: nodes of 2^max_depth x 2^max_depth candidates;
                              < 0: automatic (the smallest with ceil(n_space / 2^d) <= 32) */
  int32_t probe_min_nodes; /* below the top, a level of at least this many nodes first
                              scores its best node's leaves exactly (0: 4096; < 0: no
                              probe at any level, the top included: a test hook) */
  int64_t node_capacity;   /* nodes per level list (0: 2^25; a level never gets more than it has nodes); larger levels are split */
  int32_t top_kernel;      /* 0: the top level as beam boxes when eligible, 1: per-node gathers */
  int32_t reserved;
} csm_search_options;

typedef struct csm_search_stats {
  int32_t depth;           /* top level used                                          */
  int32_t exhaustive;      /* 1: the window did not qualify, searched exhaustively    */
  int64_t candidates;      /* n_windows * n_angles * n_space^2                        */
  int64_t nodes[11];       /* nodes scored at each level (nodes[0]: exact candidates)  */
  int64_t probe_leaves;    /* candidates scored exactly by incumbent probes           */
  int64_t beam_reads;      /* grid reads in all: (sum of nodes + probe_leaves) * B     */
  double build_ms;         /* pooled levels built by this call (0: cached)            */
  int64_t syncs;           /* node counts the host read back (level passes it waited on) */
  int32_t top_box;         /* 1: the top level ran as beam boxes                       */
  int32_t reserved;
} csm_search_stats;

int csm_search_windows(csm_ctx* ctx, const double* points_xy, int32_t n_points,
                       const csm_param* param, int32_t n_windows, const int32_t* grid_index,
                       const double* centers_map, const csm_search_options* options,
                       csm_best* best, int32_t* best_window, csm_search_stats* stats);

#ifdef __cplusplus
}
#endif

#endif /* ROBORTS_CSM_H */
