"""Parameter sets of the reference, as csm_param-compatible records.

Three default sets feed CorrelationScanMatchParam in the reference
(SURVEY.md Appendix C): the simulation/real-robot YAML
(config/simulatin_param.yaml:51-70), ParamConfig's nh.param defaults
(param_config.h:71-90) and ScanMatchParam's in-class defaults
(scan_matchers.h:136-157). The FAST (branch-and-bound) test parameters are
hard-coded at scan_matchers.h:337-343.
"""
from __future__ import annotations

from dataclasses import dataclass, replace

from ._abi import COARSE, FAST, FINE, SUPER, CsmOptimizeParam, CsmParam


@dataclass(frozen=True)
class CorrelationScanMatchParam:
    """Mirror of CorrelationScanMatchParam (correlate_scan_matcher.h:41-86)."""

    search_space_size: float
    search_space_resolution: float
    search_angle_offset: float
    search_angle_resolution: float
    response_threshold: float
    use_point_size: int
    max_depth: int = 0
    use_center_penalty: bool = True
    correlation_scan_match_type: int = COARSE

    def to_c(self) -> CsmParam:
        return CsmParam(
            self.search_space_size,
            self.search_space_resolution,
            self.search_angle_offset,
            self.search_angle_resolution,
            self.response_threshold,
            int(self.use_point_size),
            int(self.max_depth),
            1 if self.use_center_penalty else 0,
            int(self.correlation_scan_match_type),
        )

    def with_(self, **kw) -> "CorrelationScanMatchParam":
        return replace(self, **kw)


def _lv(size, res, off, ares, thr, use, typ, penalty=True):
    return CorrelationScanMatchParam(size, res, off, ares, thr, use, 0, penalty, typ)


# config/simulatin_param.yaml:51-70 (real_robot_param.yaml has the same levels)
SIM_YAML_LEVELS = (
    _lv(0.6, 0.05, 0.523, 0.0349, 0.6, 100, COARSE),
    _lv(0.2, 0.02, 0.175, 0.0349, 0.6, 100, FINE),
    _lv(0.02, 0.01, 0.0349, 0.00349, 0.6, 100, SUPER),
)

# ParamConfig nh.param defaults (param_config.h:71-90)
PARAM_CONFIG_LEVELS = (
    _lv(0.8, 0.1, 0.01745 * 100, 0.01745 * 2, 0.6, 100, COARSE),
    _lv(0.2, 0.02, 0.01745 * 20, 0.01745 * 2, 0.7, 100, FINE),
    _lv(0.02, 0.01, 0.01745 * 2, 0.01745 * 0.2, 0.7, 200, SUPER),
)

# ScanMatchParam in-class defaults (scan_matchers.h:136-157)
IN_CLASS_LEVELS = (
    _lv(0.8, 0.1, 0.01745 * 80, 0.01745 * 2, 0.6, 100, COARSE),
    _lv(0.2, 0.02, 0.01745 * 20, 0.01745 * 2, 0.7, 100, FINE),
    _lv(0.02, 0.01, 0.01745 * 2, 0.01745 * 0.2, 0.7, 200, SUPER),
)

# scan_matchers.h:337-343 (branch-and-bound test parameters)
FAST_PARAM = CorrelationScanMatchParam(0.8, 0.01, 0.523, 0.00349, 0.5, 100, 4, False, FAST)

# BASELINE config 1: +-0.5 m / +-15 deg window (1.0 m at 0.05 m, 0.2618 rad at 0.0349)
CONFIG1_PARAM = _lv(1.0, 0.05, 0.2617993877991494, 0.0349, 0.6, 100, COARSE)


@dataclass(frozen=True)
class OptimizeScanMatchParam:
    """Mirror of OptimizeScanMatchParam (optimize_scan_matcher.h:33-58)."""

    iterate_max_times: int
    cost_decrease_threshold: float
    cost_min_threshold: float
    max_update_distance: float
    max_update_angle: float

    def to_c(self) -> CsmOptimizeParam:
        return CsmOptimizeParam(int(self.iterate_max_times), 0, self.cost_decrease_threshold,
                                self.cost_min_threshold, self.max_update_distance, self.max_update_angle)


# config/simulatin_param.yaml:42-47 (use_optimize_scan_match: false there;
# optimize_failed_cost 2.0)
SIM_YAML_OPTIMIZE = OptimizeScanMatchParam(10, 0.1, 0.5, 0.5, 0.5)
SIM_YAML_OPTIMIZE_FAILED_COST = 2.0
# ParamConfig defaults (param_config.h:63-69; use_optimize_scan_match true,
# optimize_failed_cost 20)
PARAM_CONFIG_OPTIMIZE = OptimizeScanMatchParam(10, 1.0, 2.0, 0.5, 0.2)
PARAM_CONFIG_OPTIMIZE_FAILED_COST = 20.0


def headline_levels(use_point_size: int = 1081):
    """SIM_YAML levels with every beam summed (B = N = 1081): the BASELINE
    headline "1081-beam" configuration."""
    return tuple(l.with_(use_point_size=use_point_size) for l in SIM_YAML_LEVELS)


__all__ = [
    "CorrelationScanMatchParam", "SIM_YAML_LEVELS", "PARAM_CONFIG_LEVELS",
    "IN_CLASS_LEVELS", "FAST_PARAM", "CONFIG1_PARAM", "headline_levels",
    "COARSE", "FINE", "SUPER", "FAST", "OptimizeScanMatchParam", "SIM_YAML_OPTIMIZE",
    "SIM_YAML_OPTIMIZE_FAILED_COST", "PARAM_CONFIG_OPTIMIZE", "PARAM_CONFIG_OPTIMIZE_FAILED_COST",
]
