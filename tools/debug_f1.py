"""F1 scan match under each finish mode (GPU debug helper)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "tests")]
import roborts_csm
from roborts_csm.params import CorrelationScanMatchParam
f1 = np.load(os.path.join(ROOT, "tests", "golden", "f1_config1.npz"))
a = f1["param"]
p = CorrelationScanMatchParam(float(a[0]), float(a[1]), float(a[2]), float(a[3]), float(a[4]), int(a[5]), int(a[6]), bool(a[7]), int(a[8]))
for mode in ("host", "exact", None):
    if mode:
        os.environ["CSM_FINISH"] = mode
    c = roborts_csm.Context(0)
    os.environ.pop("CSM_FINISH", None)
    c.set_grid(roborts_csm.ScanMatchMap(f1["grid"], float(f1["resolution"]), tuple(f1["offset"]), 0, 0))
    c.set_profiling(True)
    pose = np.array(f1["init_pose"], dtype=np.float64)
    cov = np.eye(3).reshape(9).copy()
    r, am = c.scan_match(f1["points"], p, pose, cov, return_argmax=True)
    st = {k["name"]: k["scorings"] for k in c.kernel_stats()}
    print(mode, r == f1["response"], am == f1["argmax"], np.array_equal(pose, f1["pose"]), np.array_equal(cov, f1["cov"]),
          "exact windows:", st.get("finish:exact_windows"))
    print("   cov", cov, "\n   ref", f1["cov"])
    c.close()
