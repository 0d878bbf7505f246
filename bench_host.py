"""The host-side workloads of bench.py around the matcher: config 5 (the
online front end, optionally with the back end attached), f2 (the back end's
ScanMatchInterface jobs) and the reference-side adapter. Same JSON line
contract as bench.py's config 2; called from bench.py's main."""
from __future__ import annotations

import json
import math
import os
import subprocess
import time

import numpy as np

from bench_common import ROOT, _cpu_model, _device, split_roofline, worlds_mod



class _AttachedBackEnd:
    """The back end beside the front end (SlamProcessor::BackEndProcessThread,
    slam_processor.cpp:384-426): a host thread fed the kept scans. Per new
    vertex it adds the scan (AddRangeData) and runs the vertex's
    ScanMatchInterface jobs (slam_processor.cpp:250-326) in one batch: the
    near-chain link against the previous 10 kept scans (LinkNearChains,
    range_scan_pose_graph.cpp:120-167) and, once enough scans are kept, a
    loop-closure candidate against a chain 40-50 vertices back (TryCloseLoop,
    :299-355). Its own device context and stream on the same GPU; ctypes
    releases the GIL, so the front end keeps running. The pose-graph solve
    itself is out of scope."""

    def __init__(self, device: int, pub_map=None):
        import queue
        import threading
        from roborts_csm.backend import BackEndParam, ScanMatchService
        self.svc = ScanMatchService(BackEndParam(), device=device)
        # the front end's PubMap (MapCheckPenalize with logistic in every job,
        # slam_processor.cpp:312-317): its checks and the front end's updates
        # run in order on the map's own stream, under the map's lock
        self.pub_map = pub_map
        self.q = queue.Queue()
        self.kept = []
        self.jobs = 0
        self.lags = []
        self.busy = 0.0
        self.err = None
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def submit(self, points_m, pose):
        self.q.put((np.array(points_m, copy=True), np.array(pose, dtype=np.float64), time.perf_counter()))

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            try:
                pts, pose, t_enq = item
                t = time.perf_counter()
                rid = self.svc.AddRangeData(pts, pose)
                self.kept.append(rid)
                queries, chains, inits = [], [], []
                if len(self.kept) >= 11:
                    queries.append(pts), chains.append(self.kept[-11:-1]), inits.append(pose)
                if len(self.kept) >= 51:
                    queries.append(pts), chains.append(self.kept[-51:-41]), inits.append(pose)
                if queries:
                    self.svc.scan_match_jobs(queries, chains, inits, pose, self.pub_map)
                    self.jobs += len(queries)
                now = time.perf_counter()
                self.busy += now - t
                self.lags.append(now - t_enq)
            except Exception as e:  # reported, not raised in the thread
                self.err = repr(e)
            self.q.task_done()

    def drain(self):
        self.q.join()

    def reset_stats(self):
        self.drain()
        self.jobs, self.lags, self.busy = 0, [], 0.0

    def finish(self, fe_elapsed: float) -> dict:
        self.drain()
        self.q.put(None)
        self.th.join()
        lag = np.array(self.lags) * 1e3 if self.lags else np.zeros(1)
        out = {"vertices": len(self.lags), "jobs": self.jobs, "kept_total": len(self.kept),
               "busy_fraction_of_stream": self.busy / fe_elapsed if fe_elapsed > 0 else None,
               "vertex_lag_ms": {"p50": float(np.median(lag)), "max": float(lag.max())},
               "what": "per kept scan: AddRangeData + near-chain job (+ a loop-closure job 40-50 vertices back) "
                       "on a second device context, concurrently with the front end; every job ends with the "
                       "logistic MapCheckPenalize on the front end's PubMap; no pose-graph solve"}
        if self.err:
            out["error"] = self.err
        self.svc.close()
        return out


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
    n_prof = 60  # profiled scans after the timed ones (HIP events perturb latency)
    world = worlds.make_world(2000, 2000, 0.05, seed=20261015)
    stream = worlds.make_scan_stream(world, n + n_prof, seed=77 + rank)
    fe = SlamFrontEnd(FrontEndParam(), device=_device())
    be = None
    if args.attach_backend:
        fe.process(stream.points_m[0], stream.odom_poses[0])  # the first scan creates the maps (CreateAllMap)
        be = _AttachedBackEnd(_device(), pub_map=fe.map(0))  # CSM_PUB_MAP
        be.submit(stream.points_m[0], fe.kept_poses()[0])
    for k in range(1 if be is not None else 0, args.warmup):
        r = fe.process(stream.points_m[k], stream.odom_poses[k])
        if be is not None and r.map_updated:
            be.submit(stream.points_m[k], r.pose)
    if be is not None:
        be.drain()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    lat = []
    err = []
    try:  # the 1 cm fine map: its growth (ExtendSize) per scan, for the latency tail
        fine = fe.map(2)
    except RuntimeError:  # no scan processed yet (--warmup 0)
        fine = None
    fine_size = (lambda: (fine.GetSizeX(), fine.GetSizeY())) if fine is not None else (lambda: None)
    sizes = [fine_size()]
    kept_flags = []
    phases = []  # per scan: the front end's host phases (csm_frontend_last_phases)
    t0 = time.perf_counter()
    if be is not None:
        be.reset_stats()
    period = 1.0 / args.rate_hz if args.rate_hz > 0 else 0.0
    for k in range(args.warmup, n):
        if period:  # paced stream: scan k arrives at t0 + (k - warmup) * period
            wait = t0 + (k - args.warmup) * period - time.perf_counter()
            if wait > 0:
                time.sleep(wait)
        t = time.perf_counter()
        r = fe.process(stream.points_m[k], stream.odom_poses[k])
        if be is not None and r.map_updated:  # a kept scan: a new vertex for the back end
            be.submit(stream.points_m[k], r.pose)
        lat.append(time.perf_counter() - t)
        phases.append(fe.last_phases())
        err.append(r.pose)
        kept_flags.append(bool(r.map_updated))
        sizes.append(fine_size())
    fe_elapsed = time.perf_counter() - t0
    backend = be.finish(fe_elapsed) if be is not None else None
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
    # the latency tail: the slowest scans and what they did (kept / drawn into
    # the maps, the fine map grew), and the percentiles without growth scans
    grew = np.array([sizes[i + 1] != sizes[i] for i in range(len(lat))])
    kept_a = np.array(kept_flags)
    order = np.argsort(lat_ms)[::-1][:8]
    steady = lat_ms[~grew] if (~grew).any() else lat_ms
    ph_names = ("prepare", "match", "map_check", "update_map", "update_pub", "update_coarse", "update_fine")
    ph = np.array([[p[n] for n in ph_names] for p in phases]) if phases else np.zeros((1, len(ph_names)))
    tail = {"slowest": [{"scan": int(args.warmup + i), "ms": float(lat_ms[i]), "kept": bool(kept_a[i]),
                         "fine_map_grew": bool(grew[i]),
                         "phases_ms": {n: round(float(ph[i, c]), 4) for c, n in enumerate(ph_names)},
                         "outside_call_ms": round(float(lat_ms[i] - ph[i, :4].sum()), 4)} for i in order],
            "phase_ms": {n: {"p50": float(np.median(ph[:, c])), "p99": float(np.percentile(ph[:, c], 99)),
                             "max": float(ph[:, c].max())} for c, n in enumerate(ph_names)},
            "p99_not_kept_ms": float(np.percentile(lat_ms[~kept_a], 99)) if (~kept_a).any() else None,
            "p99_kept_ms": float(np.percentile(lat_ms[kept_a], 99)) if kept_a.any() else None,
            "growth_scans": int(grew.sum()), "kept_scans": int(kept_a.sum()),
            "p50_kept_ms": float(np.median(lat_ms[kept_a])) if kept_a.any() else None,
            "p50_not_kept_ms": float(np.median(lat_ms[~kept_a])) if (~kept_a).any() else None,
            "p99_without_growth_ms": float(np.percentile(steady, 99))}
    mctx = fe.matcher()
    mctx.set_profiling(True)
    for k in range(n, n + n_prof):
        fe.process(stream.points_m[k], stream.odom_poses[k])
    rl = split_roofline(mctx.kernel_stats())
    mctx.set_profiling(False)
    mctx.close()
    # SlamProcessor::CorrectPoseAndMap (slam_processor.cpp:329-370) after the
    # drive: every kept scan's pose nudged as a pose-graph solve would, all
    # three maps rebuilt on the device from every kept scan
    kept = fe.kept_poses()
    rng = np.random.default_rng(5)
    ids = np.arange(kept.shape[0], dtype=np.int32)
    corr = kept + rng.uniform(-1, 1, size=kept.shape) * np.array([0.02, 0.02, 0.005])
    tcp = time.perf_counter()
    fe.correct_pose_and_map(ids, corr)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    correct_ms = (time.perf_counter() - tcp) * 1e3
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
        obe, okept = None, []
        if be is not None:  # the back end's jobs too, on the same thread after each kept scan
            from roborts_csm.backend import BackEndParam, make_jobs
            obe = O.BackEnd(BackEndParam().to_c())
        tc = time.perf_counter()
        m = 0
        olat = []  # per-scan oracle time (front end + that scan's back-end jobs), timed scans only
        while m < n and (m < args.warmup + 2 or time.perf_counter() - tc < args.cpu_seconds):
            if m == args.warmup:
                tc2 = time.perf_counter()
            ts = time.perf_counter()
            res = CsmFrontendResult()
            ofe.process(stream.points_m[m], stream.odom_poses[m], res)
            if obe is not None and res.map_updated:
                okept.append(obe.add_scan(stream.points_m[m], np.array(res.pose[:])))
                qs, cs, ps = [], [], []
                if len(okept) >= 11:
                    qs.append(stream.points_m[m]), cs.append(okept[-11:-1]), ps.append(np.array(res.pose[:]))
                if len(okept) >= 51:
                    qs.append(stream.points_m[m]), cs.append(okept[-51:-41]), ps.append(np.array(res.pose[:]))
                if qs:
                    obe.scan_match(make_jobs(qs, cs, ps), len(qs), np.array(res.pose[:]), ofe.map(0))
            if m >= args.warmup:
                olat.append((time.perf_counter() - ts) * 1e3)
            m += 1
        dtc = time.perf_counter() - tc2
        what = "front end" + (" + the back end's per-vertex jobs (near-chain link, loop-closure candidate, "
                              "logistic PubMap check)" if obe is not None else "")
        olat = np.array(olat)
        cpu = {"value": (m - args.warmup) / dtc, "unit": "scans/s", "cores": 1, "kind": "port",
               "latency_ms": {"p50": float(np.median(olat)), "p99": float(np.percentile(olat, 99)),
                              "max": float(olat.max())},
               "sample": f"scans {args.warmup}..{m - 1} of the same stream through the oracle's restatement "
                         f"of the {what} (oracle/map_oracle.cpp), single-threaded, unpaced, {dtc:.1f} s on "
                         f"{_cpu_model()}"}
        if args.rate_hz > 0:  # the paced line's value is a latency: the oracle's per-scan time beside it
            cpu.update(value=float(np.median(olat)), unit="ms per scan (p50)",
                       scans_per_s_unpaced=(m - args.warmup) / dtc)
        if m == n:  # the oracle kept the same scans: time its CorrectPoseAndMap too
            tco = time.perf_counter()
            try:
                ofe.correct_pose_and_map(ids, corr)
                cpu["correct_pose_and_map_ms"] = (time.perf_counter() - tco) * 1e3
            except ValueError:
                pass
    if args.rate_hz > 0:  # paced: the stream's rate is the input, the latency per scan is the result
        head = {"metric": f"front-end per-scan latency p50 (config 5 online at {args.rate_hz:g} Hz: 1081-beam "
                          f"stream, 3-level match + map check + 3 map updates"
                          + (", back end attached)" if be is not None else ")"),
                "value": float(np.median(lat_ms)), "unit": "ms", "higher_is_better": False,
                "p99_ms": float(np.percentile(lat_ms, 99)), "scans_per_s_paced": world_size * args.steps / elapsed}
    else:
        head = {"metric": "front-end scans/sec (config 5 online: 1081-beam stream, 3-level match + map check + 3 "
                          "map updates)" + (", back end attached" if be is not None else ""),
                "value": world_size * args.steps / elapsed, "unit": "scans/s", "higher_is_better": True}
    return {
        **head, "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic drive (roborts_csm.worlds.make_scan_stream) in the seeded 2000x2000 @5cm world; "
                "ray-cast 1081-beam Hokuyo scans, noisy odometry",
        "config": {"workload": "config5: online front-end, simulatin_param.yaml (fine map 1 cm, coarse 8 cm, "
                               "PubMap 5 cm, U=100)", "parallelism": f"replicas x{world_size}",
                   "latency_ms": {"mean": float(lat_ms.mean()), "p50": float(np.median(lat_ms)),
                                  "p99": float(np.percentile(lat_ms, 99)), "max": float(lat_ms.max())},
                   "latency_tail": tail,
                   "rate_40hz_headroom": float(world_size * args.steps / elapsed / 40.0),
                   "paced_hz": args.rate_hz or None,
                   "median_pose_error_m": float(np.median(perr)), "max_pose_error_m": float(perr.max()),
                   "backend_attached": backend,
                   "correct_pose_and_map": {"kept_scans": int(kept.shape[0]), "ms": correct_ms,
                                            "what": "CorrectPoseAndMap: all kept poses corrected, PubMap + coarse + "
                                                    "fine rebuilt from every kept scan on the device"}},
        "roofline": rl, "cpu_baseline": cpu,
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
    svc = ScanMatchService(prm, device=_device())
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


def adapter_bench(args, rank, world_size, dist, torch):
    """The reference-side drop-in (include/csm_reference_adapter.hpp) as the
    reference calls it: ScanMatchers::ScanMatch's three levels per scan
    (scan_matchers.h:238,249,256) on the front end's 1 cm fine map (3000 x
    3000 AoS ProbabilityCell, slam_processor.cpp:469,499-500) with ~1e5 cells
    rewritten between scans (UpdateMapByRange). Timed in C++ by
    tests/cpp/adapter_run: per-scan latency including the grid refresh, with
    the incremental refresh (csm_update_grid_cells) and with whole-grid
    uploads, next to the oracle's CPU matcher on the same scans. Replicas
    only; rank 0 reports."""
    exe = os.path.join(ROOT, "tests", "cpp", "build", "adapter_run")
    if not os.path.exists(exe):
        raise SystemExit("tests/cpp/build/adapter_run missing: run __graft_entry__.build()")
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("LOCAL_RANK", "0")) if world_size > 1 else dict(os.environ)
    # latency run first; then a run with per-kernel HIP-event stats (CSM_STATS_DUMP) for the roofline
    r = subprocess.run([exe, "bench", str(max(args.steps, 3) + 1), "3000"], capture_output=True, text=True,
                       timeout=600, env=env)
    rs = subprocess.run([exe, "bench", "21", "3000"], capture_output=True, text=True, timeout=600,
                        env=dict(env, CSM_STATS_DUMP="1"))
    stats = []
    for line in rs.stderr.splitlines():
        if line.startswith("csm stats:"):
            f = line[len("csm stats:"):].split()
            stats.append({"name": f[0], "launches": int(f[2]), "total_ms": float(f[6]),
                          "algorithmic_bytes": float(f[8]), "scorings": 0.0})
    if r.returncode != 0:
        raise SystemExit(f"adapter_run failed ({r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}")
    a = json.loads(r.stdout.strip().splitlines()[-1])
    lat = a["adapter_incremental_ms_p50"]
    return {
        "metric": "drop-in adapter 3-level ScanMatch latency per scan (config 5 shape, incl. grid refresh)",
        "value": 1e3 / lat, "unit": "scans/s", "n_gpus": world_size, "steps": a["scans"] - 1,
        "warmup": 1, "ms_per_step": lat, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic 3000x3000 @1cm AoS map with walls; 1081-beam ray-marched scans; "
                                "1e5 random cells rewritten between scans",
        "config": {"workload": "adapter: BasedCorrelationScanMatchGpu x 3 levels per scan (sim YAML, U=100)",
                   "incremental_ms_p50": lat, "whole_upload_ms_p50": a["adapter_whole_upload_ms_p50"],
                   "host_map_mutation_ms_p50": a["host_map_mutation_ms_p50"],
                   "first_level_incl_refresh_ms_p50": a.get("adapter_first_level_ms_p50"),
                   "parallelism": f"replicas x{world_size}"},
        "roofline": split_roofline(stats),
        "cpu_baseline": {"value": 1e3 / a["oracle_cpu_ms_p50"], "unit": "scans/s", "cores": 1, "kind": "port",
                         "sample": f"the same {a['scans'] - 1} scans x 3 levels through oracle_scan_match "
                                   f"(single-threaded restatement of the reference) on {_cpu_model()}"},
    }
