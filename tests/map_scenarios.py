"""Shared map-building scenarios (test infrastructure): the same operation
sequence is applied to the oracle (oracle/map_oracle.cpp), the independent
Python restatement (tests/map_pyref.py) and the device maps
(roborts_csm.gridmap), and their final states are compared bit for bit.

Scans are ray-cast in a seeded synthetic world (roborts_csm.worlds) and
expressed like RangeDataContainer after CreateFrom(raw, 1/resolution)
(slam/sensor_data_manager.h:99-115): map cells, sensor frame. Settings follow
the reference's maps (slam_processor.cpp:470-523, config/simulatin_param.yaml).
"""
from __future__ import annotations

import math

import numpy as np

from roborts_csm import worlds


def make_scans(n_scans, n_beams=241, seed=6, world_cells=240, world_res=0.05, res=0.05, range_max=5.0,
               step_m=0.15):
    """n_scans scans along a short straight path (metres), in cells of `res`."""
    w = worlds.make_world(world_cells, world_cells, world_res, seed=seed)
    laser = worlds.LaserSpec(n_beams=n_beams, range_max=range_max)
    rng = np.random.default_rng(seed)
    p0 = worlds.sample_free_poses(w, 1, rng, clearance_m=1.0)[0]
    poses = np.array([[p0[0] + step_m * k * math.cos(p0[2]), p0[1] + step_m * k * math.sin(p0[2]),
                       p0[2] + 0.05 * k] for k in range(n_scans)])
    rngs = worlds.raycast_ranges(w, poses, laser)
    scans = [worlds.scan_points(rngs[k], laser) * (1 / res) for k in range(n_scans)]
    return scans, poses


# (name, map kwargs, options, cell params, ops) — ops: ("update", k, use_blur),
# ("init", [k...], use_blur, speedup), ("offset", (ox, oy)), ("reset",),
# ("penalty", k, check_point_num, bound_tolerance, gain, use_blur)
def scenarios():
    return {
        # front-end ScanMatchMap: just_update_occu + blur, auto-resize from a small map
        "prob_blur_grow": dict(kind=0, res=0.05, size=(40, 40), off=None, dev=0.15, default=0.3,
                               opts=(True, True, 0.88, 0.2), cell=None,
                               ops=[("update", k, True) for k in range(4)]),
        # just_update_occu without blur: once-per-scan occupied increments
        "prob_occupied": dict(kind=0, res=0.05, size=(160, 160), off="centre", dev=0.15, default=0.3,
                              opts=(False, True, 0.88, 0.2), cell=None,
                              ops=[("update", k, False) for k in range(4)]),
        # PubMap: CountCell, full Bresenham, first-frame then running factors
        "count_lines": dict(kind=1, res=0.05, size=(160, 160), off="centre", dev=0.0, default=0.5,
                            opts=(True, False, 0.72, 0.2), cell=(4.0, 8.0, 0.5, 1.0),
                            ops=[("update", 0, False), ("cell", (0.3, 0.7, 0.2, 3.0)),
                                 ("update", 1, False), ("update", 2, False), ("update", 3, False),
                                 ("penalty", 2, 50, 2.5, 0.015, False), ("penalty", 3, 100, 1.0, 0.05, False)]),
        # ProbabilityCell with full lines (free decrements), growing
        "prob_lines_grow": dict(kind=0, res=0.05, size=(50, 50), off=None, dev=0.15, default=0.3,
                                opts=(True, False, 0.88, 0.3), cell=None,
                                ops=[("update", k, False) for k in range(3)]),
        # back-end ScanMatchMap (CreateScanMatchMapWithRangeVec + ResetScanMatchMapWithRangeVec):
        # init with growth, then offset change and speedup re-inits without resize
        "prob_reset_speedup": dict(kind=0, res=0.05, size=(60, 60), off=None, dev=0.15, default=0.3,
                                   opts=(True, True, 0.88, 1.0), cell=None,
                                   ops=[("init", [0, 1], True, False), ("opts", (False, True, 0.88, 1.0)),
                                        ("offset", "shift"), ("init", [2, 3], True, True),
                                        ("init", [1], True, True), ("penalty", 1, 30, 2.0, 0.05, True)]),
    }


def map_offset(sc, size, res, pose):
    """Map offset putting `pose` at the map centre (CreateScanMatchMapWithRangeVec,
    slam_processor.cpp:433-437) or at cell (5, 5) for growth tests."""
    if sc["off"] == "centre":
        return (-(pose[0] - 0.5 * size[0] * res), -(pose[1] - 0.5 * size[1] * res))
    return (-(pose[0] - 5 * res), -(pose[1] - 5 * res))


def run(engine_factory, sc, scans, poses):
    """Apply a scenario; returns (map, list of penalty results)."""
    off = map_offset(sc, sc["size"], sc["res"], poses[0])
    m = engine_factory(sc["kind"], sc["res"], sc["size"], off, sc["dev"], sc["default"])
    m.set_options(*sc["opts"])
    if sc["cell"]:
        m.set_cell_params(*sc["cell"])
    pens = []
    for op in sc["ops"]:
        if op[0] == "update":
            m.update(scans[op[1]], poses[op[1]], op[2])
        elif op[0] == "init":
            m.init([scans[k] for k in op[1]], [poses[k] for k in op[1]], op[2], op[3])
        elif op[0] == "opts":
            m.set_options(*op[1])
        elif op[0] == "cell":
            m.set_cell_params(*op[1])
        elif op[0] == "offset":
            st = m.state()
            m.set_offset((st["offset"][0] + 0.35, st["offset"][1] - 0.2))
        elif op[0] == "penalty":
            pens.append(m.penalty(scans[op[1]], poses[op[1]], op[2], op[3], op[4], op[5]))
    return m, pens
