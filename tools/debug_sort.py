"""Small GPU check of the device std::sort emulation (csm_sort_order)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
import roborts_csm  # noqa: E402

ctx = roborts_csm.Context(0)
rng = np.random.default_rng(0)
for n in [1, 2, 5, 16, 17, 20, 40, 64, 65, 70, 100, 200, 1000, 5070]:
    for kind in ["rand", "ties", "zeros"]:
        k = rng.random(n) if kind == "rand" else (rng.integers(0, 4, n).astype(float) if kind == "ties" else np.zeros(n))
        t = time.time()
        try:
            got = ctx.sort_order(k)
            ok = np.array_equal(got, O.std_sort_order(k))
        except Exception as e:  # noqa: BLE001
            ok = f"ERR {e}"
        print(n, kind, ok, f"{(time.time()-t)*1e3:.2f} ms", flush=True)
