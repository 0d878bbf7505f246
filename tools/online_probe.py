"""What one slow scan of the config-5 stream does (GPU box): the stream of
bench.py --workload online (same world, same seed) up to scan K, then scans
K..K+2 with the fine matcher's profiling on, each call's phases and the
matcher's per-kernel / host-phase stats printed as JSON lines.

  python tools/online_probe.py [K ...]      (default: 42)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd")]

from roborts_csm import worlds  # noqa: E402
from roborts_csm.frontend import FrontEndParam, SlamFrontEnd  # noqa: E402


def main():
    ks = sorted(int(a) for a in sys.argv[1:]) or [42]
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    stream = worlds.make_scan_stream(world, ks[-1] + 3, seed=77)
    fe = SlamFrontEnd(FrontEndParam(), device=0)
    m = fe.matcher()
    k = 0
    for target in ks:
        while k < target:
            fe.process(stream.points_m[k], stream.odom_poses[k])
            k += 1
        for j in range(3):
            m.set_profiling(True)
            t = time.perf_counter()
            fe.process(stream.points_m[k], stream.odom_poses[k])
            ms = (time.perf_counter() - t) * 1e3
            st = [s for s in m.kernel_stats() if s["launches"]]
            m.set_profiling(False)
            top = sorted(st, key=lambda s: -s["total_ms"])[:14]
            print(json.dumps({"scan": k, "ms": round(ms, 4), "phases": fe.last_phases(),
                              "n_points": int(len(stream.points_m[k])),
                              "stats": [(s["name"], s["launches"], round(s["total_ms"], 4)) for s in top]}),
                  flush=True)
            k += 1
    m.close()


if __name__ == "__main__":
    main()
