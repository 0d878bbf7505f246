"""Phase timing of the v11 pair box kernel from a CSM_BOX_TRACE build
(s_memtime stamps of every 61st wave, csm_box.hip): where a wave's life goes
(prologue, run-list build, counting sort, accumulation, the sums' transpose,
the cell-by-cell pass, epilogue), as mean cycles per wave, plus the runs and
pairs per wave and how many waves were alive at once.

  make -C roborts-edu-slam_amd VARIANT=btrace EXTRA=-DCSM_BOX_TRACE
  CSM_LIB=roborts-edu-slam_amd/lib/libroborts_csm-btrace.so python tools/box_trace.py [--scans 4096]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd")]
os.environ.setdefault("CSM_PIPELINE", "0")
os.environ.setdefault("CSM_FIRST_WINDOWS", "0")

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=4096)
    ap.add_argument("--use-point-size", type=int, default=0, help="the level's U (0: every beam; 100: B = 109)")
    ap.add_argument("--xcd", action="store_true",
                    help="a CSM_BOX_TRACE_XCD build: per-XCD (blockIdx % 8) summed wave life and last exit")
    a = ap.parse_args()
    import roborts_csm
    from roborts_csm import _lib, worlds
    from roborts_csm.params import headline_levels
    fn = _lib.csm_debug_box_trace
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, a.scans, seed=7)
    lv = headline_levels()[0]
    if a.use_point_size:
        lv = lv.with_(use_point_size=a.use_point_size)
    c = roborts_csm.Context(0)
    c.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    eye = np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1))
    buf = (C.c_ulonglong * (4096 * 12))()
    for it in range(3):
        fn(buf, 4096)  # reset
        poses = np.ascontiguousarray(b.init_poses.copy())
        c.scan_match_batch(b.points_cells, b.offsets, lv, poses, eye.copy())
    n = fn(buf, 4096)
    t = np.frombuffer(buf, dtype=np.uint64, count=n * 12).reshape(n, 12).astype(np.float64)
    life = t[:, 7] - t[:, 0]
    pro = t[:, 1] - t[:, 0]
    tail = t[:, 7] - t[:, 6]
    body = t[:, 5] - t[:, 1] - t[:, 2] - t[:, 3] - t[:, 4]
    phases = {"prologue": pro, "build": t[:, 2], "sort": t[:, 3], "accumulate": t[:, 4],
              "transpose+other": body, "cell_by_cell": t[:, 6] - t[:, 5], "epilogue": tail}
    span = t[:, 7].max() - t[:, 0].min()
    out = {"waves_sampled": int(n), "mean_life_cycles": float(life.mean()),
           "phase_mean_cycles": {k: float(v.mean()) for k, v in phases.items()},
           "phase_share": {k: float(v.mean() / life.mean()) for k, v in phases.items()},
           "runs_per_wave": float(t[:, 8].mean()), "pair_slots_per_wave": float(t[:, 9].mean()),
           "beams": float(t[:, 10].mean()), "kernel_span_cycles": float(span),
           "sampled_waves_alive_mean": float(life.sum() / span) if span > 0 else None,
           "life_p10_p50_p90": [float(np.percentile(life, q)) for q in (10, 50, 90)]}
    if a.xcd:  # the samples are the last launch's (each iteration resets them)
        x = t[:, 11].astype(np.int64) % 8
        ex = t[:, 10]
        last = np.ones(n, bool)
        per = {}
        for k in range(8):
            m = (x == k) & last
            per[k] = {"waves": int(m.sum()), "life_sum": float(life[m].sum()),
                      "last_exit_us": float((ex[m].max() - ex[last].min()) / 100.0) if m.any() else None}
        ls = [v["life_sum"] for v in per.values()]
        out["per_xcd"] = per
        out["xcd_life_max_over_mean"] = float(max(ls) / (sum(ls) / 8)) if sum(ls) else None
    print(json.dumps(out), flush=True)
    c.close()


if __name__ == "__main__":
    main()
