"""Per-step kernel/host table of a bench.py JSON line (the `kernels` list)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or d["config"].get("kernels") or []
steps = d["steps"]
print(f"value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.3f}  steps {steps}")
for r in k:
    if r["launches"]:
        print(f"  {r['name']:40s} launches/step {r['launches'] / steps:6.2f}  avg_ms {r['total_ms'] / r['launches']:.4f}"
              f"  ms/step {r['total_ms'] / steps:.4f}")
