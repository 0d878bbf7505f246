"""Host placement of the per-context worker pool (include/csm.h
csm_host_plan, csm_placement.cpp) for one process per GPU, on
the CPU: every local rank of a gloo group computes its plan; the slices are
disjoint, lie in the affinity mask, and the thread counts are the rank's share
of the CPU quota (at most 16)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir, numa, quota):
    import torch.distributed as dist
    import roborts_csm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = roborts_csm.host_plan(rank, world, numa, quota)
    plans = [None] * world
    dist.all_gather_object(plans, p)
    if rank == 0:
        np.save(os.path.join(out_dir, "plans.npy"), np.array(plans, dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def _node0():
    try:
        with open("/sys/devices/system/node/node0/cpulist") as f:
            import re
            out = set()
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                out.update(range(int(a), int(b or a) + 1))
            return out
    except OSError:
        return None


@pytest.mark.parametrize("numa,quota", [((0, 0), 8), ((0, 0), 2), (None, -1), ((0, 0), -1)])
def test_gloo_ranks_get_disjoint_quota_sized_pools(tmp_path, numa, quota):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), numa, quota), nprocs=world, join=True)
    plans = list(np.load(tmp_path / "plans.npy", allow_pickle=True))
    aff = set(os.sched_getaffinity(0))
    node = _node0() if numa is not None else None
    seen = set()
    for r, p in enumerate(plans):
        cpus = set(p["cpus"])
        assert cpus and cpus <= aff, (r, p)
        if node is not None and node & aff:
            assert cpus <= node, (r, p)
        assert not (cpus & seen), ("pools overlap", plans)
        seen |= cpus
        want = min(16, len(cpus), quota // world if quota > 0 else 10 ** 9)
        assert p["threads"] == max(1, want), (r, p, quota)
        assert p["affinity_cpus"] == len(aff)


def test_plan_more_ranks_than_cpus_and_other_nodes():
    import roborts_csm
    aff = sorted(os.sched_getaffinity(0))
    # more local ranks than CPUs: one (shared) CPU each, one thread
    n = len(aff) + 3
    for r in (0, n - 1):
        p = roborts_csm.host_plan(r, n, None, -1)
        assert len(p["cpus"]) == 1 and p["threads"] == 1
    # a rank whose GPU sits on a node with no allowed CPU falls back to the
    # whole mask, split among every local rank
    p = roborts_csm.host_plan(1, 2, (0, 999), -1)
    assert set(p["cpus"]) <= set(aff) and p["numa_node"] == 999
    with pytest.raises(roborts_csm.CsmError):
        roborts_csm.host_plan(2, 2)
