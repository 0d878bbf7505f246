"""Shared pieces of bench.py and bench_host.py: the host's CPU share, the
build digest, and the roofline placement of a kernel from its live average
launch time and its PMC counters (profiles/<round>/counters*.json)."""
from __future__ import annotations

import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))

# MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s (spec), 256 CUs x 4 SIMD-32,
# 2400 MHz max clock; a 64-lane VALU instruction issues over 2 cycles (4 for
# fp64 arithmetic: FP64 vector peak = half the FP32 rate).
HBM_PEAK_GBS = 8000.0
N_CU, N_SIMD, CLK_GHZ = 256, 1024, 2.4
COUNTERS_JSON = os.path.join(ROOT, "profiles", "r06", "counters.json")
# the reference-default beam rule's leg (B = 109: the same kernels, other counters)
COUNTERS_B109_JSON = os.path.join(ROOT, "profiles", "r06", "counters_b109.json")
# the loop-closure / willow legs' counters (tools/pmc_topbox.sh: the search's top-level kernel)
COUNTERS_LC_JSON = os.path.join(ROOT, "profiles", "r06", "counters_lc.json")


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cgroup_cpus():
    """CPUs the cgroup's quota allows (cpu.max "quota period"), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) // int(per)))
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def host_cpu_share() -> dict:
    """What this process may run on: the affinity mask, the cgroup's CPU quota,
    and nproc (os.cpu_count(): the whole machine on the GPU box)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"affinity": aff, "cgroup_quota_cpus": _cgroup_cpus(), "nproc": os.cpu_count(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def _host_threads() -> int:
    """The all-cores CPU baseline's thread count: every CPU of the affinity
    mask, capped by the cgroup's CPU quota when one is set (threads beyond the
    quota only time-slice)."""
    share = host_cpu_share()
    n = share["affinity"]
    if share["cgroup_quota_cpus"]:
        n = min(n, share["cgroup_quota_cpus"])
    return max(1, n)



def source_digest() -> str:
    """SHA-1 over the library's sources and public headers (tools/source_digest.py):
    ties counters.json (and a bench line) to the build it was measured on."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import source_digest as _sd
    return _sd.digest(ROOT)


def load_counters(path: str):
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def roofline(kernel: str, avg_ms: float, algorithmic_bytes: float, counters, counters_path: str):
    """The kernel against each ceiling its PMC counters price (per launch, from
    tools/pmc_roofline.sh) over the live average launch time. frac > 1 is
    refused: the ceiling or the counter reading would be wrong."""
    t = avg_ms * 1e-3
    out = {"kernel": kernel, "avg_launch_ms": avg_ms,
           "algorithmic_bytes_per_launch": algorithmic_bytes,
           "algorithmic_GBs": algorithmic_bytes / t / 1e9,
           "algorithmic_note": "4 B per summed beam per candidate (SURVEY 8d); served from L2/MALL and "
                               "deduplicated on chip, so not an HBM rate"}
    ks = (counters or {}).get("kernels", {}).get(kernel)
    if ks is None and kernel.endswith(",tiles>"):  # the tiled box argmax: rocprof's name has no tile flag
        ks = (counters or {}).get("kernels", {}).get(kernel[:-len(",tiles>")] + ">")
    if ks is None:
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                    "traffic": None, "note": f"no PMC counters for {kernel} in {counters_path}"})
        return out
    ceilings = {}
    hbm = ks.get("hbm_bytes_per_launch")
    if hbm is not None:
        ceilings["hbm"] = (hbm / t / 1e9, HBM_PEAK_GBS, "GB/s")
    if ks.get("TA_BUSY_avr") is not None:  # busy cycles of one TA (one per CU)
        ceilings["ta"] = (ks["TA_BUSY_avr"] / t / 1e9, CLK_GHZ, "TA-busy Gcycles/s per CU")
    if ks.get("SQ_INSTS_VALU") is not None:
        f64 = ks.get("valu_f64_insts")
        cyc = 2.0 * ks["SQ_INSTS_VALU"] + (2.0 * f64 if f64 else 0.0)
        ceilings["valu"] = (cyc / N_SIMD / t / 1e9, CLK_GHZ, "VALU issue Gcycles/s per SIMD")
    if ks.get("SQ_INSTS_LDS") is not None and ks.get("SQ_LDS_BANK_CONFLICT") is not None:
        # ds instructions at >= 1 cycle each plus the measured conflict cycles, per CU
        cyc = ks["SQ_INSTS_LDS"] + ks["SQ_LDS_BANK_CONFLICT"]
        ceilings["lds"] = (cyc / N_CU / t / 1e9, CLK_GHZ, "LDS Gcycles/s per CU (lower bound)")
    fr = {k: a / p for k, (a, p, _) in ceilings.items()}
    bad = {k: v for k, v in fr.items() if v > 1.0}
    out["ceilings"] = {k: {"achieved": a, "peak": p, "unit": u, "frac": (a / p if k not in bad else None)}
                       for k, (a, p, u) in ceilings.items()}
    good = {k: v for k, v in fr.items() if k not in bad}
    if bad:
        out["refused"] = {k: f"frac {v:.2f} > 1 refused" for k, v in bad.items()}
    b = max(good, key=good.get) if good else None
    if b is not None:
        a, p, u = ceilings[b]
        out.update({"bound": b, "achieved": a, "peak": p, "unit": u, "frac": a / p})
    else:
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None})
    out["traffic"] = hbm
    out["hbm_frac"] = fr.get("hbm")
    if ks.get("SQ_WAVE_CYCLES") and ks.get("GRBM_GUI_ACTIVE"):
        cyc = ks["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        out["waves_per_simd"] = ks["SQ_WAVE_CYCLES"] * 4.0 / N_SIMD / cyc
        out["effective_clock_GHz"] = cyc / t / 1e9
        if ks.get("SQ_WAIT_ANY"):
            out["wait_frac"] = ks["SQ_WAIT_ANY"] / ks["SQ_WAVE_CYCLES"]
    if b is not None and fr[b] < 0.6:
        out["limiter"] = (f"latency: best ceiling {b} at {fr[b]:.2f}; "
                          f"{out.get('waves_per_simd', float('nan')):.1f} waves/SIMD, "
                          f"{out.get('wait_frac', float('nan')):.0%} of wave time parked on waitcnt")
    out["counters_source"] = os.path.relpath(counters_path, ROOT)
    out["counters_build"] = (counters or {}).get("source_digest")
    out["counters_stale"] = (counters or {}).get("source_digest") != source_digest()
    return out


COUNTERS_SMALL_JSON = os.path.join(ROOT, "profiles", "r06", "counters_small.json")

# The driver reads the LAST stdout line of a bounded tail: r05's 24 KB line
# (per-kernel tables inlined) was not parsed. The final line keeps the headline
# keys, the roofline, cpu_baseline, parity and a B=109 summary; everything
# else goes to a side file (DETAIL_JSON) and is named in the line's "detail".
LINE_BUDGET_BYTES = 6000
DETAIL_JSON = os.path.join("gpurun_out", "bench_detail.json")
_HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
             "scaling", "vs_baseline", "dtype", "data")
_RL_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "hbm_frac", "avg_launch_ms",
            "algorithmic_bytes_per_launch", "algorithmic_GBs", "waves_per_simd", "wait_frac", "counters_source",
            "counters_stale", "note")


def _pick(d, keys):
    return {k: d[k] for k in keys if d is not None and k in d}


def compact_roofline(rl):
    """The roofline object of the final line: the binding ceiling plus every
    ceiling's fraction (the achieved/peak/unit of each stays in the detail)."""
    if rl is None:
        return None
    out = _pick(rl, _RL_KEYS)
    if rl.get("ceilings"):
        out["ceiling_fracs"] = {k: v.get("frac") for k, v in rl["ceilings"].items()}
    return out


def _cpu(c):
    return _pick(c, ("value", "unit", "cores", "kind", "sample"))


def compact_line(out: dict, detail_path: str | None = None) -> dict:
    """The driver-facing line of a config-2 result `out` (bench.py main)."""
    line = _pick(out, _HEADLINE)
    cfg = out.get("config") or {}
    line["config"] = _pick(cfg, ("workload", "levels", "scans_per_gpu", "scorings_per_scan", "parallelism"))
    if isinstance(cfg.get("beams_summed"), dict):
        line["config"]["beams_summed"] = _pick(cfg["beams_summed"], ("mean", "use_point_size"))
    line["roofline"] = compact_roofline(out.get("roofline"))
    line["cpu_baseline"] = _cpu(out.get("cpu_baseline"))
    if out.get("cpu_baseline_all_cores"):
        line["cpu_baseline_all_cores"] = _pick(out["cpu_baseline_all_cores"], ("value", "unit", "cores", "kind"))
    line["parity"] = _pick(out.get("parity"), ("scans_checked", "mismatches", "ranks"))
    for k in ("kernel_stream_ms_per_step", "kernel_share_of_step", "single_scan_latency_ms", "median_pose_error_m"):
        if k in out:
            line[k] = out[k]
    if out.get("value_host_inputs"):
        line["value_host_inputs"] = _pick(out["value_host_inputs"], ("value", "ms_per_step", "same_result_as_resident"))
    b = out.get("b109")
    if b:
        line["b109"] = dict(_pick(b, ("value", "unit", "ms_per_step", "kernel_stream_ms_per_step")),
                            beams_summed=(b.get("beams_summed") or {}).get("mean"),
                            roofline=compact_roofline(b.get("roofline")),
                            parity=_pick(b.get("parity"), ("scans_checked", "mismatches", "ranks")),
                            cpu_baseline=_cpu(b.get("cpu_baseline")))
    lc = out.get("loop_closure_rccl")
    if lc:
        line["loop_closure_rccl"] = _pick(lc, ("status", "metric", "value", "unit", "ms_per_query", "n_devices",
                                               "n_devices_requested", "command", "error"))
        if isinstance(lc.get("verify"), dict):
            line["loop_closure_rccl"]["same_as_one_device"] = lc["verify"].get("same_as_one_device")
        if isinstance(line["loop_closure_rccl"].get("error"), str):
            line["loop_closure_rccl"]["error"] = line["loop_closure_rccl"]["error"][-600:]
    for k in ("world", "build", "rank_units"):
        if k in out:
            line[k] = out[k]
    if detail_path:
        line["detail"] = detail_path
    return line


def emit(out: dict, detail_path: str | None = DETAIL_JSON, compact=compact_line) -> dict:
    """Write the whole result to `detail_path` (best effort) and print the
    compact line as the process's last stdout line."""
    wrote = None
    if detail_path:
        try:
            d = os.path.dirname(detail_path)
            if d:
                os.makedirs(d, exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(out, f)
            wrote = detail_path
        except OSError:
            wrote = None
    line = compact(out, wrote)
    s = json.dumps(line)
    if len(s) > LINE_BUDGET_BYTES:  # never let the line outgrow the driver's tail again
        for k in ("loop_closure_rccl", "value_host_inputs", "cpu_baseline_all_cores", "median_pose_error_m"):
            line.pop(k, None)
        s = json.dumps(line)
    print(s)
    sys.stdout.flush()
    return line


def split_roofline(stats, counters_path: str | None = None):
    """Roofline of the few-window path's dominant kernel from HIP-event stats
    (csm_kernel_stats): the split kernel's launches of every level pooled (one
    kernel, rocprof cannot tell the levels apart), PMC counters per launch
    from counters_path (tools/pmc_roofline.sh --workload online)."""
    if counters_path is None:  # CSM_COUNTERS_SMALL: counters measured for this build elsewhere
        counters_path = os.environ.get("CSM_COUNTERS_SMALL", COUNTERS_SMALL_JSON)
    agg = {}
    for s in stats:  # the scoring kernels (the hot path); the finish is bookkeeping
        if not s["name"].startswith("score_") or not s["launches"]:
            continue
        base = s["name"].split("<")[0]
        a = agg.setdefault(base, {"launches": 0, "total_ms": 0.0, "bytes": 0.0})
        a["launches"] += s["launches"]
        a["total_ms"] += s["total_ms"]
        a["bytes"] += s["algorithmic_bytes"]
    if not agg:
        return None
    name, a = max(agg.items(), key=lambda kv: kv[1]["total_ms"])
    rl = roofline(name, a["total_ms"] / a["launches"], a["bytes"] / a["launches"], load_counters(counters_path),
                  counters_path)
    rl["launches_pooled"] = a["launches"]
    if rl.get("bound") is None and rl["algorithmic_bytes_per_launch"]:
        # without counters: the algorithmic rate against HBM (an upper bound on the
        # bytes the kernel could have fetched)
        ach = rl["algorithmic_GBs"]
        rl.update({"bound": "hbm (algorithmic)", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": ach / HBM_PEAK_GBS})
    return rl


def _device() -> int:
    """This rank's GPU: LOCAL_RANK, or LOCAL_RANK modulo the visible devices
    when CSM_BENCH_SHARE_GPU=1 (rehearsing N ranks on fewer GPUs, gloo)."""
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CSM_BENCH_SHARE_GPU") == "1":
        import torch
        return lr % max(1, torch.cuda.device_count())
    return lr


def worlds_mod():
    from roborts_csm import worlds
    return worlds
