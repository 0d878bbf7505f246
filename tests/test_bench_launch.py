"""bench.py's multi-GPU launch protocol on the CPU (gloo): `--gpus N` with no
torch.distributed environment spawns N ranks itself, times with barriers, takes
the max over ranks and sums the units; rank 0 prints exactly one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launch_gloo(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--workload",
                        "plumbing", "--backend", "gloo", "--steps", "4"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["world"] == {"world_size": n, "backend": "gloo"}
    assert out["n_gpus"] == n
    assert out["rank_units"] == 4.0 * n  # every rank's units summed


def test_bench_lc_leg_spawned_once_by_rank0():
    """The config-3 RCCL leg at world size 2 on the CPU:
    rank 0 alone starts the child (`--workload loop_closure --lc capi` over
    --gpus devices) before any GPU call; with no GPU here the child fails, and
    the line still prints with the leg's status and the child's error, never
    the line lost."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload",
                        "plumbing", "--backend", "gloo", "--steps", "3", "--lc-leg"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    leg = out["loop_closure_rccl"]
    assert leg["n_devices_requested"] == 2
    assert "--lc capi" in leg["command"] and "--gpus 2" in leg["command"] and "--lc-verify" in leg["command"]
    assert leg["status"] == "failed" and "csm_create" in leg["error"], leg
    assert out["world"] == {"world_size": 2, "backend": "gloo"} and out["rank_units"] == 6.0


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload",
                        "plumbing"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_search_lines_use_their_own_metric():
    """The admissible search's lines (config 3 / willow, --search pyramid) count
    candidates resolved, not scorings: they never carry the headline metric."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench._metric("pyramid") == (bench.RESOLVED_METRIC, "candidates/s")
    assert bench._metric("exhaustive") == (bench.METRIC, "scorings/s")
    assert bench.RESOLVED_METRIC != bench.METRIC


def test_roofline_launch_time_and_kernel_accounting():
    """The roofline's launch time: the one-dispatch launches' bytes per ms at
    the mean launch's bytes (parts of different sizes, a first part in spans);
    kernel_share counts scoring launches and the fast finish passes once."""
    sys.path.insert(0, ROOT)
    import bench

    # part 0: 1.2 GB in spans over 1.0 ms (span2 entry), part 1: 0.8 GB in 0.4 ms, per step, 2 steps
    stats = [
        {"name": "score_box_pair_kernel<13,all>", "launches": 4, "total_ms": 2 * (1.0 + 0.4),
         "algorithmic_bytes": 2 * (1.2e9 + 0.8e9), "scorings": 4.0},
        {"name": "span2:score_box_pair_kernel<13,all>", "launches": 2, "total_ms": 2.0,
         "algorithmic_bytes": 2.4e9, "scorings": 0.0},
        {"name": "finish_kernel<5070>", "launches": 4, "total_ms": 1.0, "algorithmic_bytes": 0.0, "scorings": 0.0},
        {"name": "finish:fast<5070>", "launches": 4, "total_ms": 0.2, "algorithmic_bytes": 0.0, "scorings": 0.0},
        {"name": "finish:exact<5070>", "launches": 4, "total_ms": 0.8, "algorithmic_bytes": 0.0, "scorings": 0.0},
        {"name": "host:wait", "launches": 9, "total_ms": 5.0, "algorithmic_bytes": 0.0, "scorings": 0.0},
    ]
    dom, avg, info = bench.dominant_kernel(stats)
    assert dom["name"] == "score_box_pair_kernel<13,all>"
    # one-dispatch rate 0.8 GB / 0.4 ms = 2 GB/ms; the mean launch is 1.0 GB -> 0.5 ms
    assert abs(avg - 0.5) < 1e-12 and info["two_span_launches"] == 2
    # the value's own region timed only the first level: its launches give the time
    first = [dict(stats[0], total_ms=2 * (1.1 + 0.44)), dict(stats[1], total_ms=2.2)]
    dom2, avg2, _ = bench.dominant_kernel(stats, first)
    assert dom2["name"] == dom["name"] and abs(avg2 - 0.55) < 1e-12
    # a timed region without that kernel falls back to the breakdown's
    assert bench.dominant_kernel(stats, [stats[2]])[1] == avg
    acct = bench.kernel_accounting(stats, elapsed_s=4e-3, steps=2)
    assert abs(acct["kernel_stream_ms_per_step"] - (2.8 + 0.2) / 2) < 1e-12
    assert abs(acct["exact_finish_side_stream_ms_per_step"] - 0.4) < 1e-12
    assert acct["kernel_share_of_step"] <= 1.0


def test_compact_line_of_the_r05_result():
    """the driver could not parse r05's 24 KB line. The
    whole r05 config-2 result (tests/golden/bench_line_r05.json, the line the
    r05 build printed) compacts to a last line under the budget that still
    carries the headline keys, the roofline, cpu_baseline, parity and B=109."""
    sys.path.insert(0, ROOT)
    import bench_common as bc

    with open(os.path.join(ROOT, "tests", "golden", "bench_line_r05.json")) as f:
        full = json.load(f)
    assert len(json.dumps(full)) > 20000
    line = bc.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bc.LINE_BUDGET_BYTES, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "parity", "b109", "build"):
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert line["roofline"][k] == full["roofline"][k]
    assert line["cpu_baseline"] == {k: full["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind", "sample")}
    assert line["parity"]["mismatches"] == 0 and line["parity"]["scans_checked"] > 0
    b = line["b109"]
    assert b["value"] == full["b109"]["value"] and b["roofline"]["frac"] == full["b109"]["roofline"]["frac"]
    assert b["cpu_baseline"]["value"] == full["b109"]["cpu_baseline"]["value"] and b["parity"]["mismatches"] == 0
    assert "kernels" not in line and "kernels_timed_region" not in line and "kernels" not in b


def test_bench_plumbing_last_line_size_and_side_file(tmp_path):
    """The plumbing mode runs the config-2 emit path: the last stdout line is
    the compact one (under the budget, headline keys), the per-kernel tables
    land in the side file."""
    sys.path.insert(0, ROOT)
    import bench_common as bc

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    detail = str(tmp_path / "detail.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "plumbing", "--steps", "3",
                        "--detail-json", detail], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    last = [l for l in r.stdout.splitlines() if l.strip()][-1]
    assert len(last) <= bc.LINE_BUDGET_BYTES
    out = json.loads(last)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "b109", "world"):
        assert k in out, k
    assert "kernels" not in out and out["detail"] == detail
    with open(detail) as f:
        full = json.load(f)
    assert len(full["kernels"]) == 64 and len(full["b109"]["kernels"]) == 64
