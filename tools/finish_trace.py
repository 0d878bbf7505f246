"""Phase timing of the exact device finish (finish_kernel) on the config-2
workload, from a CSM_FINISH_TRACE build of the library:
  make -C roborts-edu-slam_amd OUT=libtrace OBJ=buildtrace EXTRA=-DCSM_FINISH_TRACE
  CSM_LIB=roborts-edu-slam_amd/libtrace/libroborts_csm.so python tools/finish_trace.py
Prints, per traced window, n_cand, the partial-sort limit and the microseconds
spent in: load+max, counts, sort levels, FindBest, stage 2, lists."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roborts-edu-slam_amd"))
import roborts_csm  # noqa: E402
from roborts_csm import _abi, worlds  # noqa: E402
from roborts_csm.params import headline_levels  # noqa: E402

lib = C.CDLL(os.environ["CSM_LIB"])
lib.csm_debug_finish_trace.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
n_scans = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
# optional: which headline levels to run as the three levels (e.g. "2,2,2":
# the super-fine window three times)
level_sel = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else None
world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
batch = worlds.make_scan_batch(world, n_scans, seed=1000)
ctx = roborts_csm.Context(0)
ctx.set_grid(roborts_csm.ScanMatchMap(world.grid, world.resolution, world.offset, 0, 1))
ctx.load_scans(batch.points_cells, batch.offsets)
buf = (C.c_ulonglong * (256 * 10))()
for it in range(2):
    lib.csm_debug_finish_trace(buf, 256)  # reset
    poses = np.ascontiguousarray(batch.init_poses.copy())
    covs = np.ascontiguousarray(np.tile(np.eye(3).reshape(1, 9), (n_scans, 1)))
    lv = headline_levels()
    ctx.scan_matchers_loaded([lv[i] for i in level_sel] if level_sel else lv, poses, covs)
lv = (C.c_ulonglong * (256 * 32))()
lib.csm_debug_finish_levels.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
nl = lib.csm_debug_finish_levels(lv, 256)  # before the reset below (same window count)
n = lib.csm_debug_finish_trace(buf, 256)
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 10)[:n].astype(np.int64)
print("windows traced:", n)
print("   n  plim   load  count  sort  find  stage2 lists  total  (us)")
rows = []
for r in a:
    d = np.diff(r[:7]) / 100.0  # wall_clock64: 100 MHz
    rows.append(list(d) + [(r[6] - r[0]) / 100.0])
    print("%5d %5d " % (r[9], r[8]) + " ".join("%6.1f" % x for x in d) + "  %6.1f" % ((r[6] - r[0]) / 100.0))
if rows:
    print("mean        " + " ".join("%6.1f" % x for x in np.mean(np.array(rows), axis=0)))

# stage-1 levels of the first windows: (segments, first segment's length, us)
L = np.frombuffer(lv, dtype=np.uint64).reshape(256, 32)[:max(nl, 0)].astype(np.int64)
for r in L[:6]:
    out = []
    for l in range(15):
        t0, t1 = r[2 * l], r[2 * l + 2]
        if t0 == 0 or t1 == 0 or t1 < t0:
            break
        out.append("%d:%d %.1f" % (r[2 * l + 1] >> 32, r[2 * l + 1] & 0xFFFFFFFF, (t1 - t0) / 100.0))
    print("levels:", " | ".join(out))
