"""Benchmark: candidate-pose scorings/s of the correlative scan matcher.

Workload (BASELINE.json configs[1]): 1081-beam scans against a 2000x2000
@5 cm probability grid, full 3-level coarse -> fine -> super-fine search
(sim-YAML windows: 5,070 + 1,331 + 189 = 6,590 candidate poses per scan), every
beam summed (use_point_size = 1081 -> B = 1081, the "1081-beam" headline of
SURVEY.md 8d). One step = the whole 3-level match of a batch of scans that is
already resident in HBM (grid and points uploaded before the timed region);
the step includes every device launch, the device->host score copies and the
host finish (std::sort / FindBestCandidate / covariance) of all windows.

Multi-GPU: one process per GPU; each rank matches its own batch (weak scaling,
no data-path collective — independent scans). Timing: barrier +
synchronize on both sides of exactly --steps steps, max over ranks.

Roofline: the dominant kernel is placed against every ceiling its counters
can be priced on (HBM bytes, TA address-unit busy cycles, VALU issue cycles),
each from rocprofv3 --pmc passes of the same build (tools/pmc_roofline.sh ->
profiles/<round>/counters.json) divided by the kernel's average launch time
measured live with HIP events on the stream it runs on. `bound` is the ceiling
with the highest fraction; a fraction above 1 is refused (printed as null).
The algorithmic rate (4 B per summed beam per candidate) is kept
beside it as `algorithmic_GBs`: those reads are served from L2 / Infinity
Cache and deduplicated by the kernels, so it is not an HBM rate.
cpu_baseline: the oracle (single-threaded restatement of the reference) on a
bounded sample of the same workload, rank 0 at N=1 only, plus its all-cores
variant (OpenMP over theta) and the reference-default B=109 levels.

Multi-GPU: `python bench.py --gpus N` with no torch.distributed environment
spawns N child processes itself (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set before
any GPU call) and prints rank 0's line; under torchrun it joins the given group.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# the CPU baseline's OpenMP threads sleep between windows instead of spinning
# (read by libgomp when the oracle library loads)
os.environ.setdefault("OMP_WAIT_POLICY", "passive")
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

from bench_common import (COUNTERS_B109_JSON, COUNTERS_JSON, COUNTERS_LC_JSON, DETAIL_JSON,  # noqa: E402,F401
                          _cpu_model, _device, _host_threads, emit, host_cpu_share, load_counters, roofline,
                          source_digest, split_roofline, worlds_mod)
from bench_host import adapter_bench, backend_bench, online_bench  # noqa: E402

METRIC = "candidate-pose scorings/sec (1081-beam scan, 2000×2000 grid) at 1/2/4/8 GPUs"
# The admissible search resolves every candidate of a window without scoring
# most of them: its lines carry this metric, never METRIC
RESOLVED_METRIC = "candidate poses resolved/sec by the admissible search (answer = the exhaustive argmax)"


def _metric(search):
    """(metric, unit) of a loop-closure / willow line for its search kind."""
    return (RESOLVED_METRIC, "candidates/s") if search == "pyramid" else (METRIC, "scorings/s")


def kernel_accounting(stats, elapsed_s: float, steps: int) -> dict:
    """Device time of the timed steps from the HIP-event stats, without double
    counting: the scoring launches and the fast finish passes run back to back
    on the kernel stream (their sum / elapsed = kernel_share_of_step <= 1); the
    exact finish passes run on x_stream beside the other part's scoring and are
    reported apart. "finish_kernel<n>" is the fast + exact interval, "finish:*"
    and "span2:*" are sub-intervals, "host:*" and "pool:*" host phases: none of
    them is added again."""
    by = {s["name"]: s for s in stats}
    main_ms = exact_ms = finish_ms = 0.0
    scorings = 0.0
    for s in stats:
        n = s["name"]
        if n.startswith("score_"):
            main_ms += s["total_ms"]
            scorings += s["scorings"]
        elif n.startswith("finish_kernel"):
            lt = n[len("finish_kernel"):]
            fast, exact = by.get("finish:fast" + lt), by.get("finish:exact" + lt)
            finish_ms += s["total_ms"]
            if fast is not None and exact is not None:
                main_ms += fast["total_ms"]
                exact_ms += exact["total_ms"]
            else:
                main_ms += s["total_ms"]
    return {"kernel_stream_ms_per_step": main_ms / steps,
            "exact_finish_side_stream_ms_per_step": exact_ms / steps,
            "finish_ms_per_step": finish_ms / steps,
            "kernel_share_of_step": main_ms * 1e-3 / elapsed_s,
            "kernel_scorings_per_s": scorings / (main_ms * 1e-3) if main_ms else None}


def breakdown_note(elapsed_s: float, steps: int) -> dict:
    """Where kernel_accounting's figures come from."""
    return {"ms_per_step": elapsed_s / steps * 1e3, "steps": steps,
            "how": "a second region of the same steps right after the timed one, HIP events around every "
                   "launch (the timed region has them around the first level's scoring kernels only)"}


def dominant_kernel(stats, timed_stats=None):
    """The scoring or finish kernel with the most device time in `stats` (the
    every-launch breakdown), and its average launch time from `timed_stats`
    (the value's own region, when it timed that kernel) as rocprof sees it over
    whole-part dispatches
    (`CSM_FIRST_WINDOWS=0`). The first part's coarse level goes out in spans
    ("span2:<name>", each with its own ramp and tail) and the parts differ in
    size (`CSM_PART0_PERMILLE`), so the time is the one-dispatch launches' bytes
    per ms at the mean launch's algorithmic bytes."""
    ks = [s for s in stats if s["name"].startswith(("score_", "finish_kernel"))]
    dom = max(ks, key=lambda s: s["total_ms"])
    if timed_stats:
        own = next((s for s in timed_stats if s["name"] == dom["name"]), None)
        if own is not None:
            stats, dom = timed_stats, own
    two = next((s for s in stats if s["name"] == "span2:" + dom["name"]), None)
    n1 = dom["launches"] - (two["launches"] if two else 0)
    info = {"launches": dom["launches"], "two_span_launches": two["launches"] if two else 0}
    mean_bytes = dom["algorithmic_bytes"] / dom["launches"]
    if two and n1 > 0:
        t1 = dom["total_ms"] - two["total_ms"]
        b1 = dom["algorithmic_bytes"] - two["algorithmic_bytes"]
        avg = mean_bytes * t1 / b1 if b1 > 0 and mean_bytes > 0 else t1 / n1
        info["avg_ms_one_dispatch_launches"] = t1 / n1
        info["avg_ms_all_launches"] = dom["total_ms"] / dom["launches"]
        info["avg_ms_two_span_launches"] = two["total_ms"] / two["launches"]
        info["how"] = "one-dispatch launches' bytes per ms, at the mean launch's bytes"
    else:
        avg = dom["total_ms"] / dom["launches"]
    return dom, avg, info


def cpu_baseline(world, batch, levels, seconds: float, threads: int = 1, label: str = "", collect=None):
    """Oracle (test infrastructure, CPU restatement) on a bounded sample.
    threads > 1: the all-cores variant (OpenMP over theta inside each window;
    identical results). collect: a list that receives (n, (scores, poses,
    covs)) of the sample (scans 0 .. n-1), the parity check's expected values."""
    import pyoracle as O
    O.set_threads(threads)
    m = O.Map(world.grid, world.resolution, world.offset)
    eye = np.tile(np.eye(3).reshape(1, 9), (1, 1))

    def run(k0, k1):
        off = batch.offsets[k0:k1 + 1] - batch.offsets[k0]
        pts = batch.points_cells[batch.offsets[k0]:batch.offsets[k1]]
        t = time.perf_counter()
        res = O.scan_matchers_batch(m, pts, off, levels, batch.init_poses[k0:k1],
                                    np.tile(eye, (k1 - k0, 1)))
        return time.perf_counter() - t, res

    probe = run(0, 2)[0] / 2
    n = int(max(2, min(batch.offsets.size - 1, seconds / max(probe, 1e-6))))
    dt, res = run(0, n)
    O.set_threads(1)
    if collect is not None:
        collect.append((n, res))
    per_scan = sum(_window_cands(l) for l in levels)
    how = "single-threaded" if threads == 1 else f"{threads} threads (OpenMP over theta)"
    out = {"value": n * per_scan / dt, "unit": "scorings/s", "cores": threads, "kind": "port",
           "sample": f"{label}{n} scans x 3 levels ({n * per_scan} scorings, {dt:.1f} s) {how} "
                     f"oracle/csm_oracle.cpp on {_cpu_model()}"}
    if threads > 1:
        out["host_cpu_share"] = host_cpu_share()
    return out


def parity_check(gpu, runs, what: str) -> dict:
    """The timed configuration's own outputs against the oracle's: gpu =
    (scores, poses, covs) of the last timed step, runs = cpu_baseline's
    collected samples (scans 0 .. n-1 of the same batch from the same initial
    poses). Bit for bit; a mismatching scan is one whose score, pose or
    covariance differs in any bit."""
    n, (s2, p2, c2) = max(runs, key=lambda r: r[0])
    s, p, c = (np.asarray(a)[:n] for a in gpu)
    bad = (s != s2) | np.any(p.reshape(n, 3) != p2.reshape(n, 3), axis=1) | \
        np.any(c.reshape(n, 9) != c2.reshape(n, 9), axis=1)
    out = {"scans_checked": int(n), "mismatches": int(np.sum(bad)),
           "what": f"{what}: scores, poses and covariances of the last timed step, bit for bit, against "
                   "oracle/csm_oracle.cpp on the cpu_baseline samples (scans 0 .. scans_checked-1)"}
    if out["mismatches"]:
        out["first_mismatch"] = int(np.argmax(bad))
    return out


def oracle_sample(world, batch, levels, n: int, threads: int):
    """The oracle's outputs for scans 0 .. n-1 (parity only, not timed)."""
    import pyoracle as O
    n = int(max(1, min(n, batch.offsets.size - 1)))
    O.set_threads(threads)
    try:
        m = O.Map(world.grid, world.resolution, world.offset)
        res = O.scan_matchers_batch(m, batch.points_cells[:batch.offsets[n]], batch.offsets[:n + 1], levels,
                                    batch.init_poses[:n], np.tile(np.eye(3).reshape(1, 9), (n, 1)))
    finally:
        O.set_threads(1)
    return n, res


def _beams_summed(offsets, use_point_size: int) -> dict:
    """Beams GetResponse sums per candidate (correlate_scan_matcher.h:561-566):
    N < 2U -> every point, else every (N / (U - 1))-th. The scans keep only
    in-range beams (roborts_slam_node.cpp:300), so N varies per scan."""
    n = np.diff(np.asarray(offsets, dtype=np.int64))
    u = int(use_point_size)
    step = np.where(n < 2 * u, 1, n // max(1, u - 1))
    b = -(-n // np.maximum(step, 1))
    return {"mean": float(np.mean(b)), "max": int(np.max(b)), "use_point_size": u,
            "laser_beams": 1081}


def _window_cands(p) -> int:
    import roborts_csm
    na, ns = roborts_csm.window_dims(p)
    return na * ns * ns


def loop_closure_bench(args, rank, world_size, dist, torch):
    """Config 3: one 1081-beam query (U=100 -> B=109) against
    512 submaps of 800x800 @5 cm, +-8 m / +-pi window (181 x 321^2 =
    18,650,421 candidates per submap). Submaps are sharded [r*512/G,
    (r+1)*512/G) over ranks (strong scaling), each rank's share resident as
    one stack; one step = the whole query incl. the MAX/MIN exchange."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.loop_closure import ShardedLoopClosure, shard_range
    from roborts_csm.params import CorrelationScanMatchParam
    n_sub, side, res = args.submaps, 800, 0.05
    lo, hi = shard_range(n_sub, rank, world_size)
    bases = [worlds.make_world(side, side, res, seed=20261015 + k) for k in range(8)]
    stack = np.empty((hi - lo, side, side), dtype=np.float32)
    for i, s in enumerate(range(lo, hi)):  # distinct submaps: shifted copies of 8 bases
        stack[i] = np.roll(bases[s % 8].grid, ((s // 8) * 7, (s // 8) * 11), axis=(0, 1))
    batch = worlds.make_scan_batch(bases[0], 1, seed=7)
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    pose = batch.init_poses[0]
    offsets = np.tile(np.array(bases[0].offset), (hi - lo, 1))
    param = CorrelationScanMatchParam(16.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    na, ns = roborts_csm.window_dims(param)
    ctx = roborts_csm.Context(_device())
    ctx.set_grid_stack(stack, res, version=1)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    lc = ShardedLoopClosure(ctx, n_sub, res, offsets, rank=rank, world=world_size, device=dev,
                            search=args.search)
    if args.search == "pyramid" and args.depth >= 0:
        sw = ctx.search_windows
        ctx.search_windows = lambda *a, **k: sw(*a, max_depth=args.depth, **k)
    for _ in range(args.warmup):
        lc.match(pts, param, pose)
    ctx.set_profiling(True)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = lc.match(pts, param, pose)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.kernel_stats()
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    total = float(n_sub) * na * ns * ns * args.steps
    # the dominant kernel; the search's own aggregate ("pyramid_search") is
    # not a kernel: its top-level kernel is priced instead
    kst = [s for s in stats if not s["name"].startswith("host:") and s["name"] != "pyramid_search"]
    kst = kst or [s for s in stats if not s["name"].startswith("host:")]
    dom = max(kst, key=lambda s: s["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    cj = COUNTERS_LC_JSON if args.counters_json == COUNTERS_JSON else args.counters_json
    rl = roofline(dom["name"], avg_ms, dom["algorithmic_bytes"] / dom["launches"], load_counters(cj), cj)
    search = None
    if args.search == "pyramid":
        st = lc.last_stats or {}
        search = {"kind": "admissible multi-resolution branch and bound (csm_search_windows)",
                  "depth": st.get("depth"), "top_level_as_beam_boxes": st.get("top_box"),
                  "nodes_per_level": st.get("nodes"),
                  "probe_leaves": st.get("probe_leaves"),
                  "nodes_scored_per_query_rank0": (sum(st.get("nodes", [])) + st.get("probe_leaves", 0)),
                  "beam_reads_per_query_rank0": st.get("beam_reads"),
                  "candidates_per_query_rank0": st.get("candidates"),
                  "value_note": "value counts every candidate of every window as resolved (the answer equals "
                                "the exhaustive argmax, tests/test_gpu_search.py); the nodes actually scored "
                                "are nodes_scored_per_query_rank0"}
        if world_size == 1:  # the exhaustive search of the same query, same run
            ex = ShardedLoopClosure(ctx, n_sub, res, offsets, search="exhaustive")
            ex.match(pts, param, pose)
            te = time.perf_counter()
            r2 = ex.match(pts, param, pose)
            search["exhaustive_ms_per_query"] = (time.perf_counter() - te) * 1e3
            search["same_answer_as_exhaustive"] = bool(r2.global_index == r.global_index and r2.score == r.score)
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu:
        cpu = lc_cpu_baseline(bases, pts, param, pose, args.cpu_seconds, na * ns * ns)
    met, unit = _metric(args.search)
    if search is not None:  # what the device actually scored, per second
        search["nodes_scored_per_s_rank0"] = search["nodes_scored_per_query_rank0"] * args.steps / elapsed
    return {
        "metric": met, "value": total / elapsed, "unit": unit, "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (8 seeded 800x800 wall maps, shifted into 512 submaps; one ray-cast query)",
        "config": {"workload": f"config3: loop closure, 1 query x {n_sub} submaps 800x800 @5cm, "
                               f"+-8 m / +-pi window ({na}x{ns}^2 candidates per submap), B=109",
                   "search": args.search,
                   "parallelism": f"submaps sharded x{world_size}, MAX/MIN all-reduce"},
        "roofline": rl,
        "result": {"score": r.score, "submap": r.submap, "global_index": r.global_index},
        "search": search,
        "kernels": stats, "cpu_baseline": cpu,
    }


def _lc_config3(n_sub: int):
    """Config 3's inputs (the torch-sharded leg's too): 512 submaps of 800x800 @5 cm,
    shifted copies of 8 seeded wall maps, one ray-cast query scan (B = 109)."""
    from roborts_csm import worlds
    from roborts_csm.params import CorrelationScanMatchParam
    side, res = 800, 0.05
    bases = [worlds.make_world(side, side, res, seed=20261015 + k) for k in range(8)]
    stack = np.empty((n_sub, side, side), dtype=np.float32)
    for s in range(n_sub):
        stack[s] = np.roll(bases[s % 8].grid, ((s // 8) * 7, (s // 8) * 11), axis=(0, 1))
    batch = worlds.make_scan_batch(bases[0], 1, seed=7)
    pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    offsets = np.tile(np.array(bases[0].offset), (n_sub, 1))
    param = CorrelationScanMatchParam(16.0, 0.05, math.pi, 0.0349, 0.5, 100, 0, False, 0)
    return bases, stack, pts, batch.init_poses[0], offsets, param, res


def loop_closure_capi_bench(args):
    """Config 3 through the C-ABI TryCloseLoop would call from C++
    (include/csm_loop_closure.h; range_scan_pose_graph.cpp:299-355): ONE
    process drives args.gpus devices, csm_loop_closure_create makes a matcher
    context and an RCCL communicator per device (ncclCommInitAll), the 512
    submaps are sharded over them, and each query ends in the MAX / MIN / SUM
    all-reduces. n_devices is what the library reports in the result.
    --lc-verify: the same query on ONE device holding every submap (a plain
    matcher context, no communicator), compared field by field."""
    import roborts_csm
    from roborts_csm.loop_closure import DeviceLoopClosure, ShardedLoopClosure, shard_range
    n_sub = args.submaps
    t_setup = time.perf_counter()
    lc = DeviceLoopClosure(list(range(args.gpus)))  # first: no device or no RCCL fails before the inputs are made
    bases, stack, pts, pose, offsets, param, res = _lc_config3(n_sub)
    na, ns = roborts_csm.window_dims(param)
    search_ms, exchange_ms, query_ms = [], [], []
    try:
        lc.set_submaps(stack, res, offsets, version=1)
        for _ in range(args.warmup):
            r = lc.match(pts, param, pose, search=args.search)
        setup_s = time.perf_counter() - t_setup
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tq = time.perf_counter()
            r = lc.match(pts, param, pose, search=args.search)
            query_ms.append((time.perf_counter() - tq) * 1e3)
            search_ms.append(lc.last_search_ms)
            exchange_ms.append(lc.last_exchange_ms)
        elapsed = time.perf_counter() - t0
        n_dev = lc.last_n_devices
        pose_world = lc.last_pose_world.tolist()
    finally:
        lc.close()
    total = float(n_sub) * na * ns * ns * args.steps
    met, unit = _metric(args.search)
    verify = None
    if args.lc_verify:  # the one-device answer, same process, no communicator
        ctx = roborts_csm.Context(0)
        try:
            ctx.set_grid_stack(stack, res, version=1)
            one = ShardedLoopClosure(ctx, n_sub, res, offsets, search=args.search).match(pts, param, pose)
        finally:
            ctx.close()
        verify = {"one_device": {"score": one.score, "submap": one.submap, "global_index": one.global_index,
                                 "x": one.x, "y": one.y, "angle": one.angle},
                  "same_as_one_device": bool(one.score == r.score and one.global_index == r.global_index and
                                             one.submap == r.submap and one.x == r.x and one.y == r.y and
                                             one.angle == r.angle)}
    return {
        "metric": met, "value": total / elapsed, "unit": unit, "n_gpus": args.gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (8 seeded 800x800 wall maps, shifted into 512 submaps; one ray-cast query)",
        "config": {"workload": f"config3 via the C-ABI (csm_loop_closure_*): 1 query x {n_sub} submaps 800x800 "
                               f"@5cm, +-8 m / +-pi window ({na}x{ns}^2 candidates per submap), B=109",
                   "search": args.search, "lc": "capi",
                   "parallelism": f"one process, submaps sharded over {n_dev} devices, in-process RCCL "
                                  f"communicator (ncclCommInitAll), MAX/MIN/SUM all-reduce",
                   "n_devices": n_dev,
                   "submaps_per_device": [hi - lo for lo, hi in (shard_range(n_sub, d, n_dev)
                                                                 for d in range(n_dev))]},
        "query_ms": {"median": float(np.median(query_ms)), "min": float(np.min(query_ms)),
                     "max": float(np.max(query_ms))},
        "search_ms_median": float(np.median(search_ms)),
        "exchange_us": {"median": float(np.median(exchange_ms)) * 1e3, "min": float(np.min(exchange_ms)) * 1e3,
                        "max": float(np.max(exchange_ms)) * 1e3},
        "setup_s": setup_s,
        "roofline": None,
        "result": {"score": r.score, "submap": r.submap, "global_index": r.global_index, "x": r.x, "y": r.y,
                   "angle": r.angle, "pose_world": pose_world},
        "verify": verify,
        "cpu_baseline": None,
    }


def lc_leg(args) -> dict:
    """The config-3 leg of the default line: the north
    star's RCCL best-score exchange at args.gpus devices, in a child process
    started before this process makes any GPU call (`--workload loop_closure
    --lc capi --lc-verify`), under a time limit of its own so that a hung
    communicator can cost the line this key but never the line. Called on
    rank 0 only; the other ranks are still in the process-group rendezvous."""
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "loop_closure", "--lc", "capi", "--lc-verify",
           "--gpus", str(args.gpus), "--steps", str(args.lc_steps), "--warmup", "2",
           "--submaps", str(args.submaps)]
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
            "MASTER_PORT")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC")}
    t = time.perf_counter()
    out = {"command": " ".join(os.path.basename(c) if i == 1 else c for i, c in enumerate(cmd[1:], 1)),
           "n_devices_requested": args.gpus}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.lc_timeout, env=env)
    except subprocess.TimeoutExpired:
        out.update(status="timeout", limit_s=args.lc_timeout, wall_s=time.perf_counter() - t)
        return out
    out["wall_s"] = time.perf_counter() - t
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        err = [l for l in r.stderr.splitlines() if l.strip()]
        out.update(status="failed", returncode=r.returncode, error=err[-1] if err else None,
                   stderr_tail=r.stderr[-600:])
        return out
    d = json.loads(lines[-1])
    out.update(status="ok", metric=d["metric"], value=d["value"], unit=d["unit"], steps=d["steps"],
               ms_per_query=d["ms_per_step"], query_ms=d["query_ms"], search_ms_median=d["search_ms_median"],
               exchange_us=d["exchange_us"], setup_s=d["setup_s"], n_devices=d["config"]["n_devices"],
               submaps_per_device=d["config"]["submaps_per_device"], workload=d["config"]["workload"],
               parallelism=d["config"]["parallelism"], result=d["result"], verify=d["verify"],
               scaling="strong (512 submaps in total, whatever the device count)")
    return out


def lc_cpu_baseline(bases, pts, param, pose, seconds, per_submap):
    """Config-3 CPU leg: the oracle's argmax over whole submap windows (the
    reference's GetResponse loop over 181 x 321^2 candidates), all host
    threads (OpenMP over theta); one submap takes seconds, so the sample is
    the submaps that fit in `seconds`."""
    import pyoracle as O
    from roborts_csm.loop_closure import world_to_map
    th = _host_threads()
    O.set_threads(th)
    b = bases[0]
    m = O.Map(b.grid, b.resolution, b.offset)
    c = world_to_map(pose, b.resolution, b.offset)
    t = time.perf_counter()
    n = 0
    while n < 1 or time.perf_counter() - t < seconds:
        O.best_window(m, pts, param, c)
        n += 1
    dt = time.perf_counter() - t
    O.set_threads(1)
    return {"value": n * per_submap / dt, "unit": "scorings/s", "cores": th, "kind": "port",
            "sample": f"{n} submap window(s) of {per_submap} candidates, B=109, {dt:.1f} s, oracle "
                      f"best_window with {th} threads (OpenMP over theta) on {_cpu_model()}",
            "host_cpu_share": host_cpu_share()}


def willow_map(grid_cells: int, seed: int):
    """Config 4's map: the reference's willow map (1165x945, padded by 200
    cells to 1565x1345), or with grid_cells > 0 a grid_cells^2 @5cm grid tiled
    from config 2's 2000^2 synthetic world (the HBM-stress variant of SURVEY
    8d: 16384^2 = 1 GiB of fp32). Returns (world, scan batch, tile side)."""
    from roborts_csm import worlds
    if grid_cells <= 0:
        w = worlds.willow_world()
        return w, None, 0
    base = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    reps = -(-grid_cells // 2000)
    grid = np.ascontiguousarray(np.tile(base.grid, (reps, reps))[:grid_cells, :grid_cells])
    return worlds.World(grid, None, base.resolution, base.offset), base, 2000


def willow_bench(args, rank, world_size, dist, torch):
    """Config 4: the reference's willow map (1165x945, padded
    by 200 cells to 1565x1345), argmax-only windows, +-pi at 0.0349 (181
    angles), every beam summed (U = 1081). The window is --window-m metres
    around each query scan's initial pose, or with --whole-map the whole
    padded map (1566^2 cells around the map's centre: 181 x 1566^2 = 444 M
    candidates per query, the survey's definition). --grid-cells N: an N x N
    grid tiled from config 2's world instead, one scan per step searched in
    --windows windows spread over every tile (the 1 GiB HBM-stress grid at
    16384). Queries are independent: weak scaling, one replica per GPU."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import CorrelationScanMatchParam
    w, base, tile = willow_map(args.grid_cells, 20261015)
    batch = worlds.make_scan_batch(base if base is not None else w, max(1, args.steps + args.warmup), seed=31 + rank)
    sy, sx = w.grid.shape
    window_m = max(sx, sy) * w.resolution if args.whole_map else args.window_m
    param = CorrelationScanMatchParam(window_m, 0.05, math.pi, 0.0349, 0.5, 1081, 0, False, 0)
    na, ns = roborts_csm.window_dims(param)
    ctx = roborts_csm.Context(_device())
    ctx.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    from roborts_csm.loop_closure import world_to_map
    n_win = args.windows if tile else 1
    rng = np.random.default_rng(7 + rank)
    reps = -(-sx // tile) if tile else 1

    def centers(k):
        """Query k's window centres (map cells): the scan's initial pose, in
        n_win tiles drawn over the whole grid (the same map around it in every
        tile); the map's centre with --whole-map."""
        c = world_to_map(batch.init_poses[k], w.resolution, w.offset)
        if args.whole_map:
            c = np.array([sx / 2.0, sy / 2.0, c[2]])
        if not tile:
            return c.reshape(1, 3)
        t = rng.integers(0, reps, size=(n_win, 2))
        out = np.tile(c, (n_win, 1))
        out[:, 0] += t[:, 0] * tile
        out[:, 1] += t[:, 1] * tile
        return out
    qc = [centers(k) for k in range(args.steps + args.warmup)]
    last = {}

    def query(k, search=args.search):
        pts = batch.points_cells[batch.offsets[k]:batch.offsets[k + 1]]
        c = qc[k]
        if search == "exhaustive":
            if c.shape[0] == 1:
                return ctx.best_window(pts, param, c[0])
            sc, fl, x, y, a = ctx.best_windows(pts, param, np.zeros(c.shape[0], np.int32), c)
            i = int(np.lexsort((np.arange(sc.size), -sc))[0])  # max score, then the lowest window
            return roborts_csm.CsmBest(sc[i], fl[i], x[i], y[i], a[i])
        b, _, st = ctx.search_windows(pts, param, [0] * c.shape[0], c, max_depth=args.depth)
        last.update(st)
        return b

    for k in range(args.warmup):
        query(args.steps + k)
    ctx.set_profiling(True)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    beams = 0
    for k in range(args.steps):
        query(k)
        beams += int(batch.offsets[k + 1] - batch.offsets[k])
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.kernel_stats()
    search = None
    if args.search == "pyramid":
        search = {"kind": "admissible multi-resolution branch and bound (csm_search_windows)",
                  "depth": last.get("depth"), "top_level_as_beam_boxes": last.get("top_box"),
                  "nodes_per_level_last_query": last.get("nodes"),
                  "beam_reads_last_query": last.get("beam_reads"),
                  "value_note": "value counts every candidate of the window as resolved (the answer equals "
                                "the exhaustive argmax, tests/test_gpu_search.py)"}
        if world_size == 1:
            same = True
            te = time.perf_counter()
            for k in range(args.steps):
                b1 = query(k, "exhaustive")
            search["exhaustive_ms_per_query"] = (time.perf_counter() - te) / args.steps * 1e3
            for k in range(min(args.steps, 3)):
                b1, b2 = query(k, "exhaustive"), query(k)
                same = same and b1.score == b2.score and b1.flat_index == b2.flat_index
            search["same_answer_as_exhaustive"] = bool(same)
    local = float(na * ns * ns * n_win * args.steps)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    if dist is not None:
        t = torch.tensor([elapsed, local], dtype=torch.float64, device=dev)
        e, s = t[:1].clone(), t[1:].clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, total = float(e.item()), float(s.item())
    else:
        total = local
    # the dominant kernel; the search's own aggregate ("pyramid_search") is
    # not a kernel: its top-level kernel is priced instead
    kst = [s for s in stats if not s["name"].startswith("host:") and s["name"] != "pyramid_search"]
    kst = kst or [s for s in stats if not s["name"].startswith("host:")]
    dom = max(kst, key=lambda s: s["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    cj = COUNTERS_LC_JSON if args.counters_json == COUNTERS_JSON else args.counters_json
    rl = roofline(dom["name"], avg_ms, dom["algorithmic_bytes"] / dom["launches"], load_counters(cj), cj)
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu:
        import pyoracle as O
        th = _host_threads()
        O.set_threads(th)
        om = O.Map(w.grid, w.resolution, w.offset)
        # a bounded sample: windows of more than 30 M candidates (the whole
        # map: ~2 min of all cores per query) are sampled by a 20 m window
        # around the same centre (the oracle's rate per candidate, all beams)
        cp, cna, cns = param, na, ns
        if na * ns * ns > 30e6:
            cp = CorrelationScanMatchParam(20.0, 0.05, math.pi, 0.0349, 0.5, 1081, 0, False, 0)
            cna, cns = roborts_csm.window_dims(cp)
        tc = time.perf_counter()
        m = 0
        while m < 1 or time.perf_counter() - tc < args.cpu_seconds:
            q = m % args.steps  # the timed queries, cycled
            pts = batch.points_cells[batch.offsets[q]:batch.offsets[q + 1]]
            O.best_window(om, pts, cp, qc[q][0])
            m += 1
        dtc = time.perf_counter() - tc
        O.set_threads(1)
        cpu = {"value": m * cna * cns * cns / dtc, "unit": "scorings/s", "cores": th, "kind": "port",
               "sample": f"{m} of the same queries ({cna}x{cns}^2 candidates"
                         f"{' (a 20 m window around the same centre)' if cp is not param else ''}, all beams), "
                         f"{dtc:.1f} s, oracle best_window with {th} threads (OpenMP over theta) on {_cpu_model()}"}
    met, unit = _metric(args.search)
    return {
        "metric": met, "value": total / elapsed, "unit": unit, "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": ("willow-full-0.05 occupancy (tests/golden/willow_walls.npz) with the blur splat; "
                 "ray-cast scans at free poses") if not tile else
                (f"{sx}x{sy} @5cm grid tiled from config 2's 2000x2000 synthetic world ({sx * sy * 4 / 2**30:.2f} GiB "
                 f"fp32); ray-cast scans of that world, each searched in {n_win} windows over random tiles"),
        "config": {"workload": (f"config4: {'willow 1565x1345' if not tile else f'{sx}x{sy} tiled'} @5cm, "
                                f"{'whole-map ' if args.whole_map else ''}{window_m:.2f} m / +-pi window "
                                f"({na}x{ns}^2 candidates) x {n_win} windows, all beams"),
                   "search": args.search, "windows_per_query": n_win,
                   "mean_beams": beams / args.steps, "parallelism": f"replicas x{world_size}"},
        "roofline": rl, "search": search,
        "kernels": stats, "cpu_baseline": cpu,
    }


def plumbing_bench(args, rank, world_size, dist, torch):
    """The launcher and timing protocol without the matcher (CPU tests of
    `--gpus N`): barrier, --steps timed sleeps of 1 ms, max over ranks, sum of
    per-rank units."""
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(1e-3)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    units = float(args.steps)
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64)
        u = torch.tensor([units], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        elapsed, units = float(e.item()), float(u.item())
    # per-kernel tables of config 2's size, so the tests see the compact line
    # hold its budget with the side file carrying the rest
    kernels = [{"name": f"kernel<{i}>", "launches": 40, "total_ms": 1.0, "algorithmic_bytes": 0.0, "scorings": 0.0}
               for i in range(64)]
    return {"metric": "plumbing", "value": units / elapsed, "unit": "steps/s", "n_gpus": world_size,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "rank_units": units, "kernels": kernels, "kernels_timed_region": kernels[:20],
            "b109": {"value": units / elapsed, "unit": "steps/s", "ms_per_step": elapsed / args.steps * 1e3,
                     "kernels": kernels}}


def build_info() -> dict:
    """Which library ran: the source digest compiled into it (csm_build_digest)
    against the tree's sources (a stale prebuilt .so shows match: false)."""
    import roborts_csm
    lib = roborts_csm.build_digest()
    return {"library_digest": lib, "source_digest": source_digest(), "match": lib == source_digest()}


def host_plans(plan: dict, dist, torch) -> list:
    """Every rank's host worker pool (csm_get_host_plan): threads, NUMA node
    and the CPU slice it is pinned to, gathered to rank 0."""
    cpus = plan["cpus"]
    row = [plan["threads"], plan["numa_node"], len(cpus), min(cpus) if cpus else -1, max(cpus) if cpus else -1,
           plan["quota_cpus"]]
    rows = [row]
    if dist is not None:
        t = torch.tensor(row, dtype=torch.int64, device="cuda" if torch.cuda.is_available() else "cpu")
        out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        rows = [[int(v) for v in o.tolist()] for o in out]
    return [{"rank": r, "threads": a, "numa_node": b, "n_cpus": c, "cpu_min": d, "cpu_max": e, "quota_cpus": f}
            for r, (a, b, c, d, e, f) in enumerate(rows)]


def world_info(dist) -> dict:
    """What actually ran: world size and backend of the process group."""
    if dist is None:
        return {"world_size": 1, "backend": None}
    return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend())}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh child processes, one
    per GPU, with the torch.distributed environment set. The parent never
    touches the GPU and never re-execs; it relays rank 0's stdout and returns
    the first non-zero exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0]
    codes = [p.wait() for p in procs]
    # only the result line goes to stdout (communication libraries print
    # their own status lines to the process's stdout)
    for line in out.decode().splitlines():
        (sys.stdout if line.startswith("{") else sys.stderr).write(line + "\n")
    sys.stdout.flush()
    return next((c for c in codes if c != 0), 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # config 2 defaults to 30 timed steps after 5 warmups (~0.2 s): with 5 steps
    # one host stall of a few ms on a shared box moved ms_per_step by up to 60 %
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 30 for config2, else 5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 40 for config2, else 2)")
    ap.add_argument("--scans", type=int, default=4096, help="scans per GPU per step")
    ap.add_argument("--levels", choices=["headline", "sim"], default="headline",
                    help="headline: every beam summed (B=1081); sim: reference YAML U=100 (B=109)")
    ap.add_argument("--workload", choices=["config2", "loop_closure", "willow", "online", "backend", "adapter",
                                           "plumbing"],
                    default="config2",
                    help="config2: the headline front-end batch; loop_closure: config 3; willow: config 4; "
                         "online: config 5 (steps = scans); backend: f2 pose-graph jobs")
    ap.add_argument("--jobs", type=int, default=16, help="backend: ScanMatchInterface jobs per step")
    ap.add_argument("--rate-hz", type=float, default=0.0,
                    help="online: pace the scan stream (40 = the Hokuyo's rate; 0 = as fast as possible)")
    ap.add_argument("--attach-backend", action="store_true",
                    help="online: run the back end's per-vertex jobs in a thread beside the front end (config 5)")
    ap.add_argument("--window-m", type=float, default=20.0, help="willow: window edge (m)")
    ap.add_argument("--whole-map", action="store_true",
                    help="willow: the window is the whole map around its centre (SURVEY 8d config 4)")
    ap.add_argument("--grid-cells", type=int, default=0,
                    help="willow: an N x N grid tiled from config 2's world instead (16384: the 1 GiB HBM stress)")
    ap.add_argument("--windows", type=int, default=64, help="willow --grid-cells: windows per query scan")
    ap.add_argument("--submaps", type=int, default=512, help="loop_closure: submaps in total")
    ap.add_argument("--search", choices=["pyramid", "exhaustive"], default="pyramid",
                    help="loop_closure / willow: the admissible multi-resolution search (csm_search_windows) "
                         "or every candidate scored (csm_best_windows); both give the same answer")
    ap.add_argument("--depth", type=int, default=-1, help="pyramid search: top level (-1: automatic)")
    ap.add_argument("--lc", choices=["torch", "capi"], default="torch",
                    help="loop_closure: torch = one rank per GPU, the exchange over torch.distributed (RCCL); "
                         "capi = ONE process over --gpus devices through csm_loop_closure_* (in-process "
                         "RCCL communicator), what TryCloseLoop calls from C++")
    ap.add_argument("--sync-steps", action="store_true",
                    help="config2: one csm_scan_matchers_loaded call per step (no batches in flight back to back)")
    ap.add_argument("--no-host-inputs", action="store_true",
                    help="config2: skip the value_host_inputs leg (batches uploaded from pinned host memory)")
    ap.add_argument("--lc-verify", action="store_true",
                    help="loop_closure --lc capi: also answer the query on one device holding every submap")
    ap.add_argument("--no-lc-leg", action="store_true",
                    help="config2: leave out the config-3 RCCL leg (loop_closure_rccl key)")
    ap.add_argument("--lc-leg", action="store_true", help="plumbing: run the config-3 leg too (launch tests)")
    ap.add_argument("--lc-steps", type=int, default=20, help="config-3 leg: timed queries")
    ap.add_argument("--lc-timeout", type=float, default=240.0, help="config-3 leg: the child's time limit (s)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--parity-scans", type=int, default=256,
                    help="config2: scans each rank checks against the oracle when no cpu_baseline runs "
                         "(N > 1 or --no-cpu)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-scan latency probe (profiling runs: keeps rocprof "
                         "per-kernel averages equal to the timed steps' launches)")
    ap.add_argument("--counters-json", default=COUNTERS_JSON,
                    help="per-kernel PMC counters per launch (tools/pmc_roofline.sh -> tools/pmc_roofline.py)")
    ap.add_argument("--counters-b109-json", default=COUNTERS_B109_JSON,
                    help="the B=109 leg's PMC counters (tools/pmc_roofline.sh with --levels sim)")
    ap.add_argument("--no-b109", action="store_true",
                    help="config2: skip the reference-default B=109 (U=100) line beside the headline")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="torch.distributed backend (auto: nccl = RCCL on a GPU box, gloo on CPU)")
    ap.add_argument("--detail-json", default=DETAIL_JSON,
                    help="config2 / plumbing: the whole result (per-kernel tables, breakdowns) goes here; "
                         "the last stdout line is the compact headline ('' = no side file)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 30 if args.workload == "config2" else 5
    if args.warmup is None:
        # config 2: ~0.15 s of untimed steps, so the host cores and the GPU clocks
        # have ramped up before the timed region (a fresh box's first run measured
        # up to 10 % slower after 5)
        args.warmup = 40 if args.workload == "config2" else 2

    if args.workload == "loop_closure" and args.lc == "capi":  # one process, every device
        out = loop_closure_capi_bench(args)
        out["world"] = {"world_size": 1, "backend": "rccl (in-process communicator)"}
        print(json.dumps(out))
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_size}")
    # the config-3 RCCL leg, before this process makes any GPU call (the child
    # drives every device; the other ranks wait in the rendezvous below)
    leg = None
    if rank == 0 and ((args.workload == "config2" and not args.no_lc_leg) or
                      (args.workload == "plumbing" and args.lc_leg)):
        leg = lc_leg(args)
    local_rank = _device()
    dist = None
    import torch
    if world_size > 1:
        import torch.distributed as dist
        backend = args.backend if args.backend != "auto" else (
            "nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)

    if args.workload in ("loop_closure", "willow", "online", "backend", "adapter", "plumbing"):
        fn = {"loop_closure": loop_closure_bench, "willow": willow_bench, "online": online_bench,
              "backend": backend_bench, "adapter": adapter_bench, "plumbing": plumbing_bench}[args.workload]
        out = fn(args, rank, world_size, dist, torch)
        if rank == 0:
            if leg is not None:
                out["loop_closure_rccl"] = leg
            out["world"] = world_info(dist)
            out["build"] = build_info()
            if args.workload == "plumbing":  # the config-2 line's emit path, side file included
                emit(out, args.detail_json or None)
            else:
                print(json.dumps(out))
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import SIM_YAML_LEVELS, headline_levels

    levels = headline_levels() if args.levels == "headline" else SIM_YAML_LEVELS
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    batch = worlds.make_scan_batch(world, args.scans, seed=1000 + rank)

    ctx = roborts_csm.Context(local_rank)
    ctx.set_grid(roborts_csm.ScanMatchMap(world.grid, world.resolution, world.offset, 0, 1))
    ctx.load_scans(batch.points_cells, batch.offsets)
    poses0 = np.ascontiguousarray(batch.init_poses)
    covs0 = np.ascontiguousarray(np.tile(np.eye(3).reshape(1, 9), (args.scans, 1)))
    host = host_plans(ctx.host_plan(), dist, torch)

    poses_w, covs_w = np.empty_like(poses0), np.empty_like(covs0)  # reset in place each step
    # submitted batches (csm_scan_matchers_submit): each step is one whole
    # batch, but step k + 1's first launch goes out before step k's last level
    # is completed; two sets of outputs alternate (a batch's are final once
    # the next submit returns), the timed region ends with the last one's wait
    sets = [(np.empty_like(poses0), np.empty_like(covs0), np.zeros(args.scans)) for _ in range(2)]
    k_step = [0]

    def step(lv=levels):
        """One whole batch; returns its (scores, poses, covs), final after settle()."""
        if args.sync_steps:
            np.copyto(poses_w, poses0)
            np.copyto(covs_w, covs0)
            sc = ctx.scan_matchers_loaded(lv, poses_w, covs_w)
            return sc, poses_w, covs_w
        p, c, sc = sets[k_step[0] % 2]
        k_step[0] += 1
        np.copyto(p, poses0)
        np.copyto(c, covs0)
        ctx.scan_matchers_submit(lv, p, c, sc)
        return sc, p, c

    def settle():  # the last submitted step completes
        if not args.sync_steps:
            ctx.scan_matchers_wait()

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def timed(lv, warmup, steps, events=2):
        """warmup untimed steps, then exactly `steps` timed ones between
        barriers; returns (elapsed s, kernel stats, last step's outputs).
        events: csm_set_profiling's mode (2: HIP events around the first
        level's scoring kernels only, the dominant kernel; 1: every launch and
        finish, for the per-kernel breakdown)."""
        for _ in range(warmup):
            step(lv)
        settle()
        # HIP events around every launch feed the live roofline below
        ctx.set_profiling(events)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = step(lv)
        settle()
        barrier()
        el = time.perf_counter() - t0
        st = ctx.kernel_stats()
        ctx.set_profiling(False)
        return el, st, tuple(np.array(a, copy=True) for a in res)

    # the A/B knob CSM_BENCH_NO_EVENTS=1 leaves the HIP events out to price their overhead
    # (CSM_BENCH_EVENTS=1 times every launch inside the value's region, as r05's first builds did)
    ev_mode = 0 if os.environ.get("CSM_BENCH_NO_EVENTS") == "1" else int(os.environ.get("CSM_BENCH_EVENTS", "2"))
    elapsed, stats_value, final = timed(levels, args.warmup, args.steps, ev_mode)
    # the per-kernel breakdown: the same steps once more, every launch timed
    # (its events add ~50 us of kernel-stream gaps a step, so not in `value`)
    el_all, stats, _ = timed(levels, 5, args.steps, 1)
    poses = final[1]
    poses_resident = poses.copy()

    per_scan = sum(_window_cands(l) for l in levels)
    local_scorings = float(args.scans * per_scan * args.steps)
    if dist is not None:
        t = torch.tensor([elapsed, local_scorings], dtype=torch.float64,
                         device="cuda" if torch.cuda.is_available() else "cpu")
        e = t[:1].clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        s = t[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, total_scorings = float(e.item()), float(s.item())
    else:
        total_scorings = local_scorings

    # single-scan latency (front-end, config 5 shape): one 3-level match
    lat = []
    one_pts = batch.points_cells[batch.offsets[0]:batch.offsets[1]]
    for _ in range(0 if args.no_latency else 20):
        pose = poses0[0].copy()
        cov = np.eye(3).reshape(9).copy()
        t = time.perf_counter()
        ctx.scan_matchers(one_pts, levels, pose, cov)
        lat.append(time.perf_counter() - t)
    # the PCIe-inclusive cost of the host-buffer entry points: one H2D copy of
    # the batch's points (never part of `value`)
    t = time.perf_counter()
    ctx.load_scans(batch.points_cells, batch.offsets)
    h2d_ms = (time.perf_counter() - t) * 1e3

    # value_host_inputs: every step's scans come from (pinned) host memory,
    # uploaded on the copy stream while the previous batch is matched
    # (csm_load_scans_async, double-buffered); the first upload is not hidden
    host_inputs = None
    if not args.no_host_inputs:
        pins = [roborts_csm.PinnedArray(batch.points_cells.shape) for _ in range(2)]
        for p in pins:
            np.copyto(p.array, batch.points_cells)
        t = time.perf_counter()
        ctx.load_scans(pins[0].array, batch.offsets)
        h2d_pinned_ms = (time.perf_counter() - t) * 1e3

        def run_host(k):
            ctx.load_scans_async(pins[0].array, batch.offsets)
            res = None
            for i in range(k):
                if i + 1 < k:
                    ctx.load_scans_async(pins[(i + 1) % 2].array, batch.offsets)
                res = step()
            settle()
            return res[1]

        run_host(max(2, min(args.warmup, 10)))
        barrier()
        t = time.perf_counter()
        ph = run_host(args.steps)
        barrier()
        eh = time.perf_counter() - t
        if dist is not None:
            e = torch.tensor([eh], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            eh = float(e.item())
        host_inputs = {"value": world_size * args.scans * sum(_window_cands(l) for l in levels) * args.steps / eh,
                       "unit": "scorings/s", "ms_per_step": eh / args.steps * 1e3, "steps": args.steps,
                       "bytes_per_step": int(batch.points_cells.nbytes),
                       "h2d_pinned_ms_one_batch": h2d_pinned_ms,
                       "same_result_as_resident": bool(np.array_equal(ph, poses_resident)),
                       "how": "each step's 4096 scans (1081 beams, fp64) uploaded from pinned host memory "
                              "(csm_host_alloc) on a copy stream of its own while the previous batch is matched "
                              "(csm_load_scans_async, two device buffers); the first step's upload is not hidden"}
        ctx.load_scans(batch.points_cells, batch.offsets)
        for p in pins:
            p.close()

    # the reference-default beam rule next to the headline: sim-YAML U=100 ->
    # B=109, driven exactly as the headline (submitted batches, HIP events)
    b109 = None
    if args.levels == "headline" and not args.no_b109:
        e109, stats109_value, final109 = timed(SIM_YAML_LEVELS, args.warmup, args.steps, ev_mode)
        e109_all, stats109, _ = timed(SIM_YAML_LEVELS, 5, args.steps, 1)
        if dist is not None:
            e = torch.tensor([e109], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            e109 = float(e.item())
        ps = sum(_window_cands(l) for l in SIM_YAML_LEVELS)
        b109 = {"value": world_size * args.scans * ps * args.steps / e109, "unit": "scorings/s",
                "ms_per_step": e109 / args.steps * 1e3, "beams_summed": _beams_summed(batch.offsets, 100),
                "levels": "sim YAML (U=100 at every level: B=109)",
                "batches": "submitted back to back, as the headline",
                "breakdown": breakdown_note(e109_all, args.steps),
                **kernel_accounting(stats109, e109_all, args.steps)}
        dom109, avg109, info109 = dominant_kernel(stats109, stats109_value)
        b109["dominant_kernel"] = {"name": dom109["name"], "avg_ms": avg109,
                                   "share_of_step": dom109["total_ms"] * 1e-3 / e109, **info109}
        b109["roofline"] = roofline(dom109["name"], avg109, dom109["algorithmic_bytes"] / dom109["launches"],
                                    load_counters(args.counters_b109_json), args.counters_b109_json)
        b109["kernels"] = stats109

    # parity of the timed configuration itself: every rank checks its own
    # batch's last timed step against the oracle (rank 0 at N = 1 on the
    # cpu_baseline samples, which run anyway; otherwise a bounded sample)
    runs, runs109 = [], []
    cpu = cpu_all = cpu109 = None
    if rank == 0 and world_size == 1 and not args.no_cpu:
        cpu = cpu_baseline(world, batch, levels, args.cpu_seconds, collect=runs)
        cpu_all = cpu_baseline(world, batch, levels, args.cpu_seconds / 2, threads=_host_threads(), collect=runs)
        if b109 is not None:
            cpu109 = cpu_baseline(world, batch, SIM_YAML_LEVELS, args.cpu_seconds / 2,
                                  label="B=109 (sim YAML, U=100): ", collect=runs109)
    else:
        th = max(1, _host_threads() // int(os.environ.get("LOCAL_WORLD_SIZE", world_size)))
        runs.append(oracle_sample(world, batch, levels, args.parity_scans, th))
        if b109 is not None:
            runs109.append(oracle_sample(world, batch, SIM_YAML_LEVELS, args.parity_scans, th))
    parity = parity_check(final, runs, "headline (B=1081)")
    parity109 = parity_check(final109, runs109, "B=109") if b109 is not None else None
    if dist is not None:  # summed over ranks: each checked its own scans
        for d in (parity, parity109):
            if d is None:
                continue
            t = torch.tensor([d["scans_checked"], d["mismatches"]], dtype=torch.float64,
                             device="cuda" if torch.cuda.is_available() else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            d["scans_checked"], d["mismatches"] = int(t[0].item()), int(t[1].item())
            d["ranks"] = world_size
    failed = parity["mismatches"] > 0 or (parity109 is not None and parity109["mismatches"] > 0)

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        if failed:
            sys.exit(1)
        return

    if os.environ.get("CSM_BENCH_NO_EVENTS") == "1":  # A/B of the event overhead only: no roofline
        print(json.dumps({"ms_per_step": elapsed / args.steps * 1e3, "events": False}))
        return
    # device kernels only (kernel_accounting: no sub-interval or host phase twice)
    dom, avg_ms, dom_info = dominant_kernel(stats, stats_value)
    # a B = 109 run prices its launches with the B = 109 counters (the kernels
    # share names with the B = 1081 ones; the pair kernel even changes form)
    cj = (args.counters_b109_json if args.levels == "sim" and args.counters_json == COUNTERS_JSON
          else args.counters_json)
    rl = roofline(dom["name"], avg_ms, dom["algorithmic_bytes"] / dom["launches"], load_counters(cj), cj)
    rl["launch_time"] = dict(dom_info, source="HIP events on the kernel stream around each one-dispatch "
                                              "launch of the dominant kernel in the timed steps")
    acct = {"breakdown": breakdown_note(el_all, args.steps), **kernel_accounting(stats, el_all, args.steps)}

    err = np.hypot(*(poses[:, :2] - batch.true_poses[:, :2]).T)
    out = {
        "metric": METRIC,
        "value": total_scorings / elapsed,
        "unit": "scorings/s",
        "n_gpus": world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded 2000x2000 @5cm wall map with the reference's blur splat; "
                "ray-cast 1081-beam Hokuyo scans at distinct poses)",
        "config": {
            "workload": "config2: 1081-beam scans vs 2000x2000 @5cm fp32 grid, full 3-level "
                        "coarse->fine->super-fine (sim-YAML windows 5070+1331+189 candidates/scan)",
            "levels": args.levels,
            "beams_summed": _beams_summed(batch.offsets, levels[0].use_point_size),
            "scans_per_gpu": args.scans,
            "scorings_per_scan": per_scan,
            "parallelism": f"replicas x{world_size} (scan-sharded, no collective)",
            "batches": ("one csm_scan_matchers_loaded call per step" if args.sync_steps else
                        "submitted back to back (csm_scan_matchers_submit): step k + 1's first launch goes out "
                        "before step k's last level is completed; every step is one whole batch, the timed "
                        "region ends when the last one is complete"),
            "inputs": "grid and scans resident in HBM before the timed region (csm_load_scans); the "
                      f"host-buffer entry points add one H2D copy of the points: "
                      f"{batch.points_cells.nbytes / 1e6:.1f} MB per step here, timed below as h2d_ms",
        },
        "roofline": rl,
        **acct,
        "single_scan_latency_ms": float(np.median(lat) * 1e3) if lat else None,
        "median_pose_error_m": float(np.median(err)),
        "kernels": stats,
        "kernels_timed_region": stats_value,
    }
    out["h2d_ms"] = h2d_ms
    if host_inputs is not None:
        out["value_host_inputs"] = host_inputs
    out["parity"] = parity
    if b109 is not None:
        b109["parity"] = parity109
        if cpu109 is not None:
            b109["cpu_baseline"] = cpu109
        out["b109"] = b109
    out["cpu_baseline"] = cpu
    if cpu_all is not None:
        out["cpu_baseline_all_cores"] = cpu_all
    if leg is not None:
        out["loop_closure_rccl"] = leg
    out["host_threads"] = host
    out["world"] = world_info(dist)
    out["build"] = build_info()
    # the per-kernel tables and breakdowns go to the side file; the last
    # stdout line stays under LINE_BUDGET_BYTES (a 24 KB line
    # was not parsed by the driver)
    emit(out, args.detail_json or None)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if failed:
        sys.exit("bench.py: the timed configuration's outputs differ from the oracle's (parity.mismatches)")


if __name__ == "__main__":
    main()
