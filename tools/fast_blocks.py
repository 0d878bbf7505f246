"""Per-block timing of the fast finish on the config-2 workload (CSM_TRACE_FASTBLK
build: `make VARIANT=fastblk EXTRA=-DCSM_TRACE_FASTBLK`, loaded with CSM_LIB).
After each 3-level call the stamps hold the call's last fast-finish launch (the
super-fine level of the second part): its span, the block durations and how the
block starts spread over the span (dispatch rounds)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "roborts-edu-slam_amd"))
import roborts_csm  # noqa: E402
from roborts_csm import worlds  # noqa: E402
from roborts_csm.params import headline_levels  # noqa: E402


def main():
    n_scans = int(os.environ.get("N_SCANS", "4096"))
    lib = roborts_csm._lib
    f = lib.csm_debug_fast_blocks
    f.restype = C.c_int
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    batch = worlds.make_scan_batch(world, n_scans, seed=1000)
    levels = headline_levels()
    buf = (C.c_ulonglong * (4096 * 16))()
    with roborts_csm.Context(0) as ctx:
        ctx.set_grid(roborts_csm.ScanMatchMap(world.grid, world.resolution, world.offset, 0, 1))
        ctx.load_scans(batch.points_cells, batch.offsets)
        poses0 = np.ascontiguousarray(batch.init_poses)
        covs0 = np.ascontiguousarray(np.tile(np.eye(3).reshape(1, 9), (n_scans, 1)))
        # NCAND: record only launches of this many candidates (5070 / 1331 / 189 at config 2)
        lib.csm_debug_fast_select(C.c_int(int(os.environ.get("NCAND", "0"))))
        for it in range(int(os.environ.get("CALLS", "6"))):
            p, c = poses0.copy(), covs0.copy()
            if "LEVEL" in os.environ:  # one level alone (csm_scan_match_batch), nothing else on the device
                ctx.scan_match_batch(batch.points_cells, batch.offsets, levels[int(os.environ["LEVEL"])], p, c)
            else:
                ctx.scan_matchers_loaded(levels, p, c)
            n = f(buf, 4096)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16)[:n]
            nb = int(np.count_nonzero(a[:, 1]))
            a = a[:nb].astype(np.int64)
            t0 = a[:, 0].min()
            st = (a[:, 0] - t0) / 100.0  # wall clock: 100 MHz -> us
            en = (a[:, 1] - t0) / 100.0
            du = en - st
            q = np.percentile
            print(f"call {it}: {nb} blocks, span {en.max():.1f} us; block duration p10/50/90/max "
                  f"{q(du, 10):.1f}/{q(du, 50):.1f}/{q(du, 90):.1f}/{du.max():.1f} us; start p10/50/90/max "
                  f"{q(st, 10):.1f}/{q(st, 50):.1f}/{q(st, 90):.1f}/{st.max():.1f} us; cus {len(np.unique(a[:, 2]))}")
            names = {3: "start", 4: "loads", 5: "max", 6: "counts", 7: "ranked", 8: "prefix", 9: "near",
                     10: "nrank", 11: "body", 12: "signal"}
            prev = a[:, 3]
            row = []
            for k in range(4, 13):
                ok = a[:, k] > 0
                if not ok.any():
                    continue
                d = (a[ok, k] - prev[ok]) / 100.0
                row.append(f"{names[k]} {np.median(d):.2f}/{np.percentile(d, 90):.2f}")
                prev = np.where(ok, a[:, k], prev)
            print("   phase median/p90 us (last window of each block):", ", ".join(row))
            hist, edges = np.histogram(st, bins=10)
            print("   starts per 10 % of the span:", hist.tolist())
            buf[:] = [0] * (4096 * 16)


if __name__ == "__main__":
    main()
