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

Roofline: the dominant kernel's algorithmic bytes (4 B per summed beam per
candidate) over its HIP-event time, measured live on the stream it runs on.
cpu_baseline: the oracle (single-threaded restatement of the reference) on a
bounded sample of the same workload, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

METRIC = "candidate-pose scorings/sec (1081-beam scan, 2000×2000 grid) at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(world, batch, levels, seconds: float):
    """Oracle (test infrastructure, CPU restatement) on a bounded sample."""
    import pyoracle as O
    m = O.Map(world.grid, world.resolution, world.offset)
    eye = np.tile(np.eye(3).reshape(1, 9), (1, 1))

    def run(k0, k1):
        off = batch.offsets[k0:k1 + 1] - batch.offsets[k0]
        pts = batch.points_cells[batch.offsets[k0]:batch.offsets[k1]]
        t = time.perf_counter()
        O.scan_matchers_batch(m, pts, off, levels, batch.init_poses[k0:k1],
                              np.tile(eye, (k1 - k0, 1)))
        return time.perf_counter() - t

    probe = run(0, 2) / 2
    n = int(max(2, min(batch.offsets.size - 1, seconds / max(probe, 1e-6))))
    dt = run(0, n)
    per_scan = sum(_window_cands(l) for l in levels)
    return {"value": n * per_scan / dt, "unit": "scorings/s", "cores": 1, "kind": "port",
            "sample": f"{n} scans x 3 levels ({n * per_scan} scorings, {dt:.1f} s) single-threaded "
                      f"oracle/csm_oracle.cpp on {_cpu_model()}"}


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
    ctx = roborts_csm.Context(int(os.environ.get("LOCAL_RANK", "0")))
    ctx.set_grid_stack(stack, res, version=1)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    lc = ShardedLoopClosure(ctx, n_sub, res, offsets, rank=rank, world=world_size, device=dev)
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
    kst = [s for s in stats if not s["name"].startswith("host:")]
    dom = max(kst, key=lambda s: s["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    achieved = dom["algorithmic_bytes"] / dom["launches"] / (avg_ms * 1e-3) / 1e9
    return {
        "metric": METRIC, "value": total / elapsed, "unit": "scorings/s", "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (8 seeded 800x800 wall maps, shifted into 512 submaps; one ray-cast query)",
        "config": {"workload": f"config3: loop closure, 1 query x {n_sub} submaps 800x800 @5cm, "
                               f"+-8 m / +-pi window ({na}x{ns}^2 candidates per submap), B=109",
                   "parallelism": f"submaps sharded x{world_size}, MAX/MIN all-reduce"},
        "roofline": {"bound": "hbm", "kernel": dom["name"], "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "avg_launch_ms": avg_ms},
        "result": {"score": r.score, "submap": r.submap, "global_index": r.global_index},
        "kernels": stats, "cpu_baseline": None,
    }


def willow_bench(args, rank, world_size, dist, torch):
    """Config 4: the reference's willow map (1165x945, padded
    by 200 cells to 1565x1345), one argmax-only window per query scan,
    +-pi at 0.0349 (181 angles), every beam summed (U = 1081). The window
    edge is --window-m (the whole-map window of the survey is ~78 m: 181 x
    1566^2 candidates, minutes per query; scale it here). Queries are
    independent: weak scaling, one replica per GPU."""
    import roborts_csm
    from roborts_csm import worlds
    from roborts_csm.params import CorrelationScanMatchParam
    w = worlds.willow_world()
    batch = worlds.make_scan_batch(w, max(1, args.steps + args.warmup), seed=31 + rank)
    param = CorrelationScanMatchParam(args.window_m, 0.05, math.pi, 0.0349, 0.5, 1081, 0, False, 0)
    na, ns = roborts_csm.window_dims(param)
    ctx = roborts_csm.Context(int(os.environ.get("LOCAL_RANK", "0")))
    ctx.set_grid(roborts_csm.ScanMatchMap(w.grid, w.resolution, w.offset, 0, 1))
    from roborts_csm.loop_closure import world_to_map

    def query(k):
        pts = batch.points_cells[batch.offsets[k]:batch.offsets[k + 1]]
        return ctx.best_window(pts, param, world_to_map(batch.init_poses[k], w.resolution, w.offset))

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
    local = float(na * ns * ns * args.steps)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    if dist is not None:
        t = torch.tensor([elapsed, local], dtype=torch.float64, device=dev)
        e, s = t[:1].clone(), t[1:].clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, total = float(e.item()), float(s.item())
    else:
        total = local
    kst = [s for s in stats if not s["name"].startswith("host:")]
    dom = max(kst, key=lambda s: s["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    achieved = dom["algorithmic_bytes"] / dom["launches"] / (avg_ms * 1e-3) / 1e9
    return {
        "metric": METRIC, "value": total / elapsed, "unit": "scorings/s", "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "willow-full-0.05 occupancy (tests/golden/willow_walls.npz) with the blur splat; "
                "ray-cast scans at free poses",
        "config": {"workload": f"config4: willow 1565x1345 @5cm, {args.window_m} m / +-pi window "
                               f"({na}x{ns}^2 candidates), all beams",
                   "mean_beams": beams / args.steps, "parallelism": f"replicas x{world_size}"},
        "roofline": {"bound": "hbm", "kernel": dom["name"], "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "avg_launch_ms": avg_ms},
        "kernels": stats, "cpu_baseline": None,
    }


def online_bench(args, rank, world_size, dist, torch):
    """Config 5: a 40 Hz-style 1081-beam scan stream through the
    device-resident front-end (include/csm_frontend.h: SlamProcessor::process
    with the 3-level match on the 1 cm fine map, the PubMap check and the
    three map updates; config/simulatin_param.yaml settings). One step = one
    scan; the maps grow as the drive leaves the initial 30 m square. Replicas
    only (one independent robot per rank)."""
    from roborts_csm import worlds
    from roborts_csm.frontend import CsmFrontendResult, FrontEndParam, SlamFrontEnd
    n = args.warmup + args.steps
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    stream = worlds.make_scan_stream(world, n, seed=77 + rank)
    fe = SlamFrontEnd(FrontEndParam(), device=int(os.environ.get("LOCAL_RANK", "0")))
    for k in range(args.warmup):
        fe.process(stream.points_m[k], stream.odom_poses[k])
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    lat = []
    err = []
    t0 = time.perf_counter()
    for k in range(args.warmup, n):
        t = time.perf_counter()
        r = fe.process(stream.points_m[k], stream.odom_poses[k])
        lat.append(time.perf_counter() - t)
        err.append(r.pose)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    lat_ms = np.array(lat) * 1e3
    # pose error against the drive (the SLAM frame is the first scan's pose)
    t0p = stream.true_poses[0]
    c, s = math.cos(-t0p[2]), math.sin(-t0p[2])
    d = stream.true_poses[args.warmup:n] - t0p
    rel = np.stack([c * d[:, 0] - s * d[:, 1], s * d[:, 0] + c * d[:, 1]], 1)
    perr = np.linalg.norm(np.array(err)[:, :2] - rel, axis=1)
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu:
        import pyoracle as O
        ofe = O.FrontEnd(FrontEndParam().to_c())
        tc = time.perf_counter()
        m = 0
        while m < n and (m < args.warmup + 2 or time.perf_counter() - tc < args.cpu_seconds):
            if m == args.warmup:
                tc2 = time.perf_counter()
            ofe.process(stream.points_m[m], stream.odom_poses[m], CsmFrontendResult())
            m += 1
        dtc = time.perf_counter() - tc2
        cpu = {"value": (m - args.warmup) / dtc, "unit": "scans/s", "cores": 1, "kind": "port",
               "sample": f"scans {args.warmup}..{m - 1} of the same stream through the oracle's restatement "
                         f"of the front-end (oracle/map_oracle.cpp), single-threaded, {dtc:.1f} s on {_cpu_model()}"}
    return {
        "metric": "front-end scans/sec (config 5 online: 1081-beam stream, 3-level match + map check + 3 map "
                  "updates)",
        "value": world_size * args.steps / elapsed, "unit": "scans/s", "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic drive (roborts_csm.worlds.make_scan_stream) in the seeded 2000x2000 @5cm world; "
                "ray-cast 1081-beam Hokuyo scans, noisy odometry",
        "config": {"workload": "config5: online front-end, simulatin_param.yaml (fine map 1 cm, coarse 8 cm, "
                               "PubMap 5 cm, U=100)", "parallelism": f"replicas x{world_size}",
                   "latency_ms": {"mean": float(lat_ms.mean()), "p50": float(np.median(lat_ms)),
                                  "p99": float(np.percentile(lat_ms, 99)), "max": float(lat_ms.max())},
                   "rate_40hz_headroom": float(world_size * args.steps / elapsed / 40.0),
                   "median_pose_error_m": float(np.median(perr)), "max_pose_error_m": float(perr.max())},
        "roofline": None, "cpu_baseline": cpu,
    }


def backend_bench(args, rank, world_size, dist, torch):
    """the back-end's ScanMatchInterface
    (slam_processor.cpp:250-326) for a batch of pose-graph jobs per step —
    --jobs near-chain links of a 1081-beam drive, each rebuilding its coarse
    (8 cm) and fine (1 cm) back-end maps from a 10-scan chain, the 3-level
    match on the fine map and the logistic PubMap check (simulatin_param.yaml
    settings). One step = one batch. Replicas only (one back-end per rank)."""
    from roborts_csm.backend import BackEndParam, ScanMatchService, job_results, make_jobs
    from roborts_csm.gridmap import OccuGridMap
    n_scans = 160
    w = worlds_mod().make_world(1000, 1000, 0.05, seed=20261015)
    st = worlds_mod().make_scan_stream(w, n_scans, seed=55 + rank)
    prm = BackEndParam()
    svc = ScanMatchService(prm, device=int(os.environ.get("LOCAL_RANK", "0")))
    for k in range(n_scans):
        svc.AddRangeData(st.points_m[k], st.true_poses[k])
    pub = OccuGridMap(w.resolution, (w.size_x, w.size_y), w.offset, 0.0, 0.5, kind=1)
    pub.set_options(True, False, 0.72, 0.2)
    for k in range(n_scans):
        pub.UpdateMapByRange(st.points_m[k] / w.resolution, st.true_poses[k])
    rng = np.random.default_rng(3)
    J = args.jobs
    qs = list(range(n_scans - J, n_scans))
    chains = [list(range(q - 20, q - 1, 2)) for q in qs]  # sparse 10-scan chains (LinkNearChains :131-146)
    init = [st.true_poses[q] + rng.normal(size=3) * [0.05, 0.05, 0.02] for q in qs]
    cur = st.true_poses[-1]
    queries = [st.points_m[q] for q in qs]

    def step():
        return svc.scan_match_jobs(queries, chains, init, cur, pub)

    for _ in range(args.warmup):
        step()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the same jobs one call at a time (the reference's calling pattern)
    t1 = time.perf_counter()
    for j in range(J):
        svc.scan_match_jobs([queries[j]], [chains[j]], [init[j]], cur, pub)
    seq = time.perf_counter() - t1
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    err = [float(np.hypot(*(r.pose[:2] - st.true_poses[q][:2]))) for r, q in zip(res, qs)]
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu:
        import pyoracle as O
        opub = O.GridMap(1, w.resolution, (w.size_x, w.size_y), w.offset, 0.0, 0.5)
        opub.set_options(True, False, 0.72, 0.2)
        for k in range(n_scans):
            opub.update_by_range(st.points_m[k] / w.resolution, st.true_poses[k])
        obe = O.BackEnd(prm.to_c())
        for k in range(n_scans):
            obe.add_scan(st.points_m[k], st.true_poses[k])
        tc = time.perf_counter()
        m = 0
        while m < J and (m < 2 or time.perf_counter() - tc < args.cpu_seconds):
            arr = make_jobs([queries[m]], [chains[m]], [init[m]])
            obe.scan_match(arr, 1, cur, opub)
            m += 1
        dtc = time.perf_counter() - tc
        cpu = {"value": m / dtc, "unit": "jobs/s", "cores": 1, "kind": "port",
               "sample": f"{m} of the same jobs through the oracle's restatement of ScanMatchInterface "
                         f"(oracle/map_oracle.cpp), single-threaded, {dtc:.1f} s on {_cpu_model()}"}
    return {
        "metric": "back-end ScanMatchInterface jobs/sec (f2: map pair rebuild from a 10-scan chain + 3-level "
                  "match + logistic map check)",
        "value": world_size * J * args.steps / elapsed, "unit": "jobs/s", "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic drive in the seeded 1000x1000 @5cm world; ray-cast 1081-beam scans at true poses",
        "config": {"workload": f"backend: {J} near-chain jobs per step, simulatin_param.yaml (fine 1 cm, coarse "
                               f"8 cm, U=100)", "parallelism": f"replicas x{world_size}",
                   "sequential_jobs_per_s": J / seq, "median_pose_error_m": float(np.median(err))},
        "roofline": None, "cpu_baseline": cpu,
    }


def worlds_mod():
    from roborts_csm import worlds
    return worlds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scans", type=int, default=4096, help="scans per GPU per step")
    ap.add_argument("--levels", choices=["headline", "sim"], default="headline",
                    help="headline: every beam summed (B=1081); sim: reference YAML U=100 (B=109)")
    ap.add_argument("--workload", choices=["config2", "loop_closure", "willow", "online", "backend"],
                    default="config2",
                    help="config2: the headline front-end batch; loop_closure: config 3; willow: config 4; "
                         "online: config 5 (steps = scans); backend: f2 pose-graph jobs")
    ap.add_argument("--jobs", type=int, default=16, help="backend: ScanMatchInterface jobs per step")
    ap.add_argument("--window-m", type=float, default=20.0, help="willow: window edge (m)")
    ap.add_argument("--submaps", type=int, default=512, help="loop_closure: submaps in total")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-scan latency probe (profiling runs: keeps rocprof "
                         "per-kernel averages equal to the timed steps' launches)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01", "traffic.json"),
                    help="PMC-derived HBM bytes per launch per kernel (tools/pmc_run.sh -> "
                         "tools/pmc_traffic.py; FETCH_SIZE and WRITE_SIZE passes of the same command)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch
    if world_size > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)

    if args.workload in ("loop_closure", "willow", "online", "backend"):
        fn = {"loop_closure": loop_closure_bench, "willow": willow_bench, "online": online_bench,
              "backend": backend_bench}[args.workload]
        out = fn(args, rank, world_size, dist, torch)
        if rank == 0:
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

    def step():
        poses, covs = poses0.copy(), covs0.copy()
        ctx.scan_matchers_loaded(levels, poses, covs)
        return poses

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    # HIP events around every launch feed the live roofline below; the A/B knob
    # CSM_BENCH_NO_EVENTS=1 leaves them out to price their overhead
    ctx.set_profiling(os.environ.get("CSM_BENCH_NO_EVENTS") != "1")
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        poses = step()
    barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)

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
    ctx.load_scans(batch.points_cells, batch.offsets)

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    if os.environ.get("CSM_BENCH_NO_EVENTS") == "1":  # A/B of the event overhead only: no roofline
        print(json.dumps({"ms_per_step": elapsed / args.steps * 1e3, "events": False}))
        return
    # device kernels only; "host:*" entries are wall-clock phases of the driver
    kstats = [s for s in stats if not s["name"].startswith("host:")]
    dom = max(kstats, key=lambda s: s["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    bytes_per_launch = dom["algorithmic_bytes"] / dom["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)  # tools/pmc_traffic.py output, keyed by kernel
        traffic = tj.get(dom["name"], {}).get("hbm_bytes_per_launch")
    kernel_total_ms = sum(s["total_ms"] for s in kstats)
    kernel_scorings = sum(s["scorings"] for s in kstats)

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
            "beams_summed": 1081 if args.levels == "headline" else 109,
            "scans_per_gpu": args.scans,
            "scorings_per_scan": per_scan,
            "parallelism": f"replicas x{world_size} (scan-sharded, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom["name"],
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": (os.path.relpath(args.traffic_json, ROOT) if traffic is not None else None),
            "avg_launch_ms": avg_ms,
            "algorithmic_bytes_per_launch": bytes_per_launch,
        },
        "kernel_scorings_per_s": kernel_scorings / (kernel_total_ms * 1e-3) if kernel_total_ms else None,
        "kernel_share_of_step": kernel_total_ms * 1e-3 / elapsed,
        "single_scan_latency_ms": float(np.median(lat) * 1e3) if lat else None,
        "median_pose_error_m": float(np.median(err)),
        "kernels": stats,
    }
    if not args.no_cpu and world_size == 1:
        out["cpu_baseline"] = cpu_baseline(world, batch, levels, args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
