"""Loop-closure sharding on the CPU: world_size 1 and 2 over
gloo, the oracle standing in for the device scorer (csm_best_windows), so the
exchange step itself -- MAX score, MIN global index among equal scores, the
winner's pose from its owner -- is what is tested here. The GPU scorer is
checked against the same oracle in test_gpu_parity.py."""
import os
import socket

import numpy as np
import pytest

import pyoracle as O
from roborts_csm.loop_closure import ShardedLoopClosure, shard_range, world_to_map
from roborts_csm.params import CorrelationScanMatchParam

RES = 0.05
PARAM = CorrelationScanMatchParam(0.6, 0.05, 0.175, 0.0349, 0.5, 100, 0, False, 0)


class OracleScorer:
    """best_windows over a stack of grids, by the CPU oracle (test double)."""

    def __init__(self, grids):
        self.grids = grids

    def best_windows(self, points, param, grid_index, centers):
        import roborts_csm
        na, ns = roborts_csm.window_dims(param)
        mres = 1 / (1 / RES)
        f = param.search_space_resolution / mres
        out = [[], [], [], [], []]
        for g, c in zip(grid_index, centers):
            m = O.Map(self.grids[g], RES, (0.0, 0.0))
            s, flat = O.best_window(m, points, param, c)
            x0 = c[0] - (param.search_space_size / mres) * 0.5
            y0 = c[1] - (param.search_space_size / mres) * 0.5
            out[0].append(s)
            out[1].append(flat)
            out[2].append(x0 + int((flat // ns) % ns) * f)
            out[3].append(y0 + int(flat % ns) * f)
            out[4].append((c[2] - (param.search_angle_offset * 2) / 2) + (flat // (ns * ns)) * param.search_angle_resolution)
        return tuple(np.array(v) for v in out)

    def search_windows(self, points, param, grid_index, centers):
        """csm_search_windows' contract: the best over all windows, ties to
        the lowest (window, flat)."""
        import roborts_csm
        from roborts_csm._abi import CsmBest
        na, ns = roborts_csm.window_dims(param)
        sc, flat, x, y, a = self.best_windows(points, param, grid_index, centers)
        gidx = np.arange(sc.size) * (na * ns * ns) + flat
        k = int(np.argmin(np.where(sc == sc.max(), gidx, np.iinfo(np.int64).max)))
        return CsmBest(sc[k], int(flat[k]), x[k], y[k], a[k]), k, {}


def _world():
    rng = np.random.default_rng(77)
    base = rng.choice(np.array([0.3, 0.45, 0.7, 1.0], dtype=np.float32), size=(4, 90, 90))
    # submaps 4 and 5 duplicate 1: equal best scores in several submaps (ties
    # across shards are broken by the lowest global index)
    grids = np.concatenate([base, base[1:2], base[1:2]])
    offsets = np.zeros((grids.shape[0], 2))
    pts = rng.uniform(-25, 25, size=(150, 2))
    pose = np.array([2.2, 2.3, 0.1])
    return grids, offsets, pts, pose


def test_shard_range_covers():
    for n in (1, 5, 8, 512, 13):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def _single(grids, offsets, pts, pose, search="exhaustive"):
    lc = ShardedLoopClosure(OracleScorer(grids), grids.shape[0], RES, offsets, search=search)
    return lc.match(pts, PARAM, pose)


@pytest.mark.parametrize("search", ["exhaustive", "pyramid"])
def test_world1_matches_bruteforce(search):
    grids, offsets, pts, pose = _world()
    r = _single(grids, offsets, pts, pose, search)
    import roborts_csm
    na, ns = roborts_csm.window_dims(PARAM)
    best = (-np.inf, None)
    for g in range(grids.shape[0]):
        m = O.Map(grids[g], RES, (0.0, 0.0))
        s, flat = O.best_window(m, pts, PARAM, world_to_map(pose, RES, offsets[g]))
        gi = g * na * ns * ns + flat
        if s > best[0] or (s == best[0] and gi < best[1]):
            best = (s, gi)
    assert (r.score, r.global_index) == best


def _rank_main(rank, world, port, out_dir, search):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grids, offsets, pts, pose = _world()
    lo, hi = shard_range(grids.shape[0], rank, world)
    lc = ShardedLoopClosure(OracleScorer(grids[lo:hi]), grids.shape[0], RES, offsets[lo:hi],
                            rank=rank, world=world, search=search)
    r = lc.match(pts, PARAM, pose)
    np.save(os.path.join(out_dir, f"r{rank}.npy"),
            np.array([r.score, r.global_index, r.submap, r.x, r.y, r.angle], dtype=np.float64))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,search", [(2, "exhaustive"), (3, "exhaustive"), (2, "pyramid"), (3, "pyramid")])
def test_gloo_shards_agree_with_single_process(tmp_path, world, search):
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), search), nprocs=world, join=True)
    grids, offsets, pts, pose = _world()
    ref = _single(grids, offsets, pts, pose)
    want = np.array([ref.score, ref.global_index, ref.submap, ref.x, ref.y, ref.angle])
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        assert np.array_equal(got, want), (r, got, want)
