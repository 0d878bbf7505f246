"""ctypes view of include/csm.h (the C-ABI of libroborts_csm.so).

The shared library is the product; this module only binds it. It raises at
import time when the library is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", "libroborts_csm.so"))

CSM_OK = 0
CSM_ERR_INVALID_ARG = 1
CSM_ERR_HIP = 2
CSM_ERR_NO_GRID = 3
CSM_ERR_ALLOC = 4
CSM_ERR_UNSUPPORTED = 5

COARSE, FINE, SUPER, FAST = 0, 1, 2, 3

# Every function include/csm.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "csm_create", "csm_destroy", "csm_last_error", "csm_abi_version", "csm_build_digest",
    "csm_set_outside_value", "csm_set_grid", "csm_set_grid_device", "csm_update_grid_cells",
    "csm_update_grid_rows",
    "csm_window_dims", "csm_sincos_device", "csm_scan_match", "csm_scan_matchers",
    "csm_scan_match_batch", "csm_scan_matchers_batch", "csm_score_window",
    "csm_best_window", "csm_load_scans", "csm_scan_matchers_loaded", "csm_scan_matchers_submit", "csm_scan_matchers_wait", "csm_load_scans_async",
    "csm_host_alloc", "csm_host_free",
    "csm_set_profiling", "csm_kernel_stats", "csm_sort_order", "csm_phase_buckets",
    "csm_set_grid_stack", "csm_best_windows", "csm_optimize_scan_match", "csm_optimize_scan_match_batch",
    "csm_optimize_update_cost", "csm_load_scans_grids", "csm_scan_matchers_batch_grids",
    "csm_search_windows", "csm_host_plan_compute", "csm_get_host_plan",
    # include/csm_gridmap.h
    "csm_gridmap_create", "csm_gridmap_destroy", "csm_gridmap_last_error",
    "csm_gridmap_set_options", "csm_gridmap_set_cell_params", "csm_gridmap_set_map_offset",
    "csm_gridmap_reset", "csm_gridmap_update_bound", "csm_gridmap_update_by_range", "csm_gridmap_init_with_range_vec",
    "csm_gridmap_feedback_penalty", "csm_gridmap_get_state", "csm_gridmap_download",
    "csm_gridmap_device_prob", "csm_set_grid_gridmap", "csm_set_grid_stack_gridmaps",
    # include/csm_frontend.h
    "csm_frontend_create", "csm_frontend_destroy", "csm_frontend_last_error", "csm_frontend_process",
    "csm_frontend_map", "csm_frontend_correct_pose_and_map", "csm_frontend_kept_scans", "csm_frontend_matcher",
    "csm_frontend_last_phases",
    # include/csm_loop_closure.h
    "csm_loop_closure_create", "csm_loop_closure_destroy", "csm_loop_closure_last_error",
    "csm_loop_closure_set_submaps", "csm_loop_closure_match",
    # include/csm_backend.h
    "csm_backend_create", "csm_backend_destroy", "csm_backend_last_error", "csm_backend_add_scan",
    "csm_backend_set_scan_pose", "csm_backend_scan_match", "csm_backend_map",
)

PROBABILITY_CELL, COUNT_CELL = 0, 1


class CsmParam(C.Structure):
    """csm_param == CorrelationScanMatchParam (correlate_scan_matcher.h:41-86)."""

    _fields_ = [
        ("search_space_size", C.c_double),
        ("search_space_resolution", C.c_double),
        ("search_angle_offset", C.c_double),
        ("search_angle_resolution", C.c_double),
        ("response_threshold", C.c_double),
        ("use_point_size", C.c_int32),
        ("max_depth", C.c_int32),
        ("use_center_penalty", C.c_int32),
        ("type", C.c_int32),
    ]


class CsmMapInfo(C.Structure):
    _fields_ = [
        ("resolution", C.c_double),
        ("offset_x", C.c_double),
        ("offset_y", C.c_double),
        ("size_x", C.c_int32),
        ("size_y", C.c_int32),
        ("update_index", C.c_int32),
        ("reserved", C.c_int32),
    ]


class CsmBest(C.Structure):
    _fields_ = [
        ("score", C.c_double),
        ("flat_index", C.c_int64),
        ("x", C.c_double),
        ("y", C.c_double),
        ("angle", C.c_double),
    ]


class CsmSearchOptions(C.Structure):
    """csm_search_options (include/csm.h): the admissible multi-resolution search."""
    _fields_ = [
        ("max_depth", C.c_int32),
        ("probe_min_nodes", C.c_int32),
        ("node_capacity", C.c_int64),
        ("top_kernel", C.c_int32),
        ("reserved", C.c_int32),
    ]


class CsmSearchStats(C.Structure):
    _fields_ = [
        ("depth", C.c_int32),
        ("exhaustive", C.c_int32),
        ("candidates", C.c_int64),
        ("nodes", C.c_int64 * 11),
        ("probe_leaves", C.c_int64),
        ("beam_reads", C.c_int64),
        ("build_ms", C.c_double),
        ("syncs", C.c_int64),
        ("top_box", C.c_int32),
        ("reserved", C.c_int32),
    ]


CSM_HOST_PLAN_MAX_CPUS = 512


class CsmHostPlan(C.Structure):
    """csm_host_plan (include/csm.h): where a context's host worker pool runs."""
    _fields_ = [
        ("threads", C.c_int32),
        ("numa_node", C.c_int32),
        ("quota_cpus", C.c_int32),
        ("affinity_cpus", C.c_int32),
        ("n_cpus", C.c_int32),
        ("cpus", C.c_int32 * CSM_HOST_PLAN_MAX_CPUS),
    ]

    def as_dict(self) -> dict:
        return {"threads": self.threads, "numa_node": self.numa_node, "quota_cpus": self.quota_cpus,
                "affinity_cpus": self.affinity_cpus, "cpus": [int(c) for c in self.cpus[:self.n_cpus]]}


class CsmLoopClosureResult(C.Structure):
    """csm_loop_closure_result (include/csm_loop_closure.h)."""
    _fields_ = [
        ("score", C.c_double),
        ("global_index", C.c_int64),
        ("submap", C.c_int32),
        ("n_devices", C.c_int32),
        ("x", C.c_double),
        ("y", C.c_double),
        ("angle", C.c_double),
        ("pose_world", C.c_double * 3),
        ("search_ms", C.c_double),
        ("exchange_ms", C.c_double),
    ]


class CsmOptimizeParam(C.Structure):
    """csm_optimize_param == OptimizeScanMatchParam (optimize_scan_matcher.h:33-58)."""

    _fields_ = [
        ("iterate_max_times", C.c_int32),
        ("reserved", C.c_int32),
        ("cost_decrease_threshold", C.c_double),
        ("cost_min_threshold", C.c_double),
        ("max_update_distance", C.c_double),
        ("max_update_angle", C.c_double),
    ]


class CsmKernelStat(C.Structure):
    _fields_ = [
        ("name", C.c_char * 48),
        ("launches", C.c_int64),
        ("total_ms", C.c_double),
        ("algorithmic_bytes", C.c_double),
        ("scorings", C.c_double),
    ]


class CsmGridmapState(C.Structure):
    """csm_gridmap_state (include/csm_gridmap.h)."""

    _fields_ = [
        ("resolution", C.c_double),
        ("offset_x", C.c_double),
        ("offset_y", C.c_double),
        ("bound_min_x", C.c_double),
        ("bound_min_y", C.c_double),
        ("bound_max_x", C.c_double),
        ("bound_max_y", C.c_double),
        ("size_x", C.c_int32),
        ("size_y", C.c_int32),
        ("map_update_index", C.c_int32),
        ("cur_update_index", C.c_int32),
        ("half_kernel", C.c_int32),
        ("blur_states", C.c_int32),
        ("kind", C.c_int32),
        ("reserved", C.c_int32),
        ("scale_factor", C.c_double),
    ]


_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_ctx = C.c_void_p


def _bind(lib: C.CDLL) -> C.CDLL:
    sig = {
        "csm_create": (C.c_int, [C.c_int, C.POINTER(_ctx)]),
        "csm_destroy": (C.c_int, [_ctx]),
        "csm_last_error": (C.c_char_p, [_ctx]),
        "csm_abi_version": (C.c_int, []),
        "csm_build_digest": (C.c_char_p, []),
        "csm_set_outside_value": (C.c_int, [_ctx, C.c_float]),
        "csm_set_grid": (C.c_int, [_ctx, C.c_void_p, C.c_int64, C.POINTER(CsmMapInfo), C.c_int64]),
        "csm_set_grid_device": (C.c_int, [_ctx, C.c_void_p, C.POINTER(CsmMapInfo)]),
        "csm_update_grid_cells": (C.c_int, [_ctx, C.c_void_p, C.c_int64, C.POINTER(CsmMapInfo), C.c_int64, _i32p,
                                            C.c_int64]),
        "csm_update_grid_rows": (C.c_int, [_ctx, C.c_void_p, C.c_int64, C.POINTER(CsmMapInfo), C.c_int64,
                                           C.c_int32, C.c_int32]),
        "csm_window_dims": (C.c_int, [C.POINTER(CsmParam), _i32p, _i32p]),
        "csm_sincos_device": (C.c_int, [_ctx, _dp, C.c_int64, _dp, _dp]),
        "csm_scan_match": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), _dp, _dp, _dp, _i64p]),
        "csm_scan_matchers": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), C.c_int32, _dp, _dp, _dp]),
        "csm_scan_match_batch": (C.c_int, [_ctx, C.c_int32, _dp, _i64p, C.POINTER(CsmParam), _dp, _dp, _dp, _i64p]),
        "csm_scan_matchers_batch": (C.c_int, [_ctx, C.c_int32, _dp, _i64p, C.POINTER(CsmParam), C.c_int32, _dp, _dp, _dp]),
        "csm_score_window": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), _dp, _dp, C.c_int64]),
        "csm_best_window": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), _dp, C.POINTER(CsmBest)]),
        "csm_load_scans": (C.c_int, [_ctx, C.c_int32, _dp, _i64p]),
        "csm_load_scans_async": (C.c_int, [_ctx, C.c_int32, _dp, _i64p]),
        "csm_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
        "csm_host_free": (C.c_int, [C.c_void_p]),
        "csm_scan_matchers_loaded": (C.c_int, [_ctx, C.POINTER(CsmParam), C.c_int32, _dp, _dp, _dp]),
        "csm_scan_matchers_submit": (C.c_int, [_ctx, C.POINTER(CsmParam), C.c_int32, _dp, _dp, _dp]),
        "csm_scan_matchers_wait": (C.c_int, [C.c_void_p]),
        "csm_set_profiling": (C.c_int, [_ctx, C.c_int32]),
        "csm_kernel_stats": (C.c_int, [_ctx, C.POINTER(CsmKernelStat), C.c_int32, _i32p]),
        "csm_sort_order": (C.c_int, [_ctx, _dp, C.c_int64, _i64p]),
        "csm_phase_buckets": (C.c_int, [C.c_double, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), _dp, _dp, C.POINTER(C.c_int8)]),
        "csm_set_grid_stack": (C.c_int, [_ctx, C.c_void_p, C.c_int32, C.POINTER(CsmMapInfo), C.c_int64]),
        "csm_best_windows": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), C.c_int32, _i32p, _dp,
                                       C.POINTER(CsmBest)]),
        "csm_search_windows": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmParam), C.c_int32, _i32p, _dp,
                                         C.POINTER(CsmSearchOptions), C.POINTER(CsmBest), _i32p,
                                         C.POINTER(CsmSearchStats)]),
        "csm_host_plan_compute": (C.c_int, [C.c_int32, C.c_int32, _i32p, C.c_int32, C.POINTER(CsmHostPlan)]),
        "csm_get_host_plan": (C.c_int, [_ctx, C.POINTER(CsmHostPlan)]),
        "csm_optimize_scan_match": (C.c_int, [_ctx, _dp, C.c_int32, C.POINTER(CsmOptimizeParam), _dp, _dp]),
        "csm_optimize_scan_match_batch": (C.c_int, [_ctx, C.c_int32, _dp, _i64p, C.POINTER(CsmOptimizeParam), _dp,
                                                    _dp, _i32p]),
        "csm_optimize_update_cost": (C.c_int, [_ctx, _dp, C.c_int32, _dp, _dp, _dp, _dp]),
        "csm_gridmap_create": (C.c_int, [C.c_int, C.c_int32, C.c_double, C.c_int32, C.c_int32, C.c_double,
                                         C.c_double, C.c_double, C.c_float, C.POINTER(C.c_void_p)]),
        "csm_gridmap_destroy": (C.c_int, [C.c_void_p]),
        "csm_gridmap_last_error": (C.c_char_p, [C.c_void_p]),
        "csm_gridmap_set_options": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_double, C.c_double]),
        "csm_gridmap_set_cell_params": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_float]),
        "csm_gridmap_set_map_offset": (C.c_int, [C.c_void_p, C.c_double, C.c_double]),
        "csm_gridmap_reset": (C.c_int, [C.c_void_p]),
        "csm_gridmap_update_bound": (C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_double, C.c_double, _i32p]),
        "csm_gridmap_update_by_range": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, _dp, C.c_int32, _i32p]),
        "csm_gridmap_init_with_range_vec": (C.c_int, [C.c_void_p, C.c_int32, _dp, _i64p, _dp, _dp, C.c_int32,
                                                      C.c_int32]),
        "csm_gridmap_feedback_penalty": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, _dp, C.c_int32, C.c_double,
                                                   C.c_double, C.c_int32, _dp]),
        "csm_gridmap_get_state": (C.c_int, [C.c_void_p, C.POINTER(CsmGridmapState)]),
        "csm_gridmap_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
        "csm_gridmap_device_prob": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
        "csm_set_grid_gridmap": (C.c_int, [_ctx, C.c_void_p]),
        "csm_frontend_create": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
        "csm_frontend_destroy": (C.c_int, [C.c_void_p]),
        "csm_frontend_last_error": (C.c_char_p, [C.c_void_p]),
        "csm_frontend_process": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, C.c_void_p]),
        "csm_frontend_map": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
        "csm_frontend_matcher": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
        "csm_frontend_last_phases": (C.c_int, [C.c_void_p, _dp]),
        "csm_frontend_correct_pose_and_map": (C.c_int, [C.c_void_p, C.c_int32, _i32p, _dp]),
        "csm_frontend_kept_scans": (C.c_int, [C.c_void_p, _i32p, _dp]),
        "csm_load_scans_grids": (C.c_int, [_ctx, C.c_int32, _dp, _i64p, _i32p]),
        "csm_scan_matchers_batch_grids": (C.c_int, [_ctx, C.c_int32, _dp, _i64p, _i32p, C.POINTER(CsmParam), C.c_int32,
                                                    _dp, _dp, _dp]),
        "csm_set_grid_stack_gridmaps": (C.c_int, [_ctx, C.POINTER(C.c_void_p), C.c_int32]),
        "csm_loop_closure_create": (C.c_int, [C.c_int32, _i32p, C.POINTER(C.c_void_p)]),
        "csm_loop_closure_destroy": (C.c_int, [C.c_void_p]),
        "csm_loop_closure_last_error": (C.c_char_p, [C.c_void_p]),
        "csm_loop_closure_set_submaps": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(CsmMapInfo), _dp,
                                                   C.c_int64]),
        "csm_loop_closure_match": (C.c_int, [C.c_void_p, _dp, C.c_int32, C.POINTER(CsmParam), _dp, C.c_int32,
                                             C.POINTER(CsmLoopClosureResult)]),
        "csm_backend_create": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
        "csm_backend_destroy": (C.c_int, [C.c_void_p]),
        "csm_backend_last_error": (C.c_char_p, [C.c_void_p]),
        "csm_backend_add_scan": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, _i32p]),
        "csm_backend_set_scan_pose": (C.c_int, [C.c_void_p, C.c_int32, _dp]),
        "csm_backend_scan_match": (C.c_int, [C.c_void_p, C.c_void_p, _dp, C.c_void_p, C.c_int32]),
        "csm_backend_map": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load_library(path: str | None = None) -> C.CDLL:
    """Load libroborts_csm.so; raises OSError when it has not been built."""
    p = path or os.environ.get("CSM_LIB") or LIB_PATH  # CSM_LIB: A/B builds of the library
    if not os.path.exists(p):
        raise OSError(
            f"libroborts_csm.so not found at {p}; build it with "
            "`make -C roborts-edu-slam_amd` (or __graft_entry__.build())"
        )
    return _bind(C.CDLL(p))
