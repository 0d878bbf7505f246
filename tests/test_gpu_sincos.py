"""The angle rows' cos/sin on the device (csm_trig.hip, csrc/libm_sincos.hpp):
glibc 2.35's sincos restated for the GPU must equal the host libm's sincos
(AngleSearchLookUpTable correlate_scan_matcher.h:171-172 as GCC compiles it)
bit for bit, checked here against the oracle's batch call of the host's
::sincos (oracle_sincos_batch), and the 3-level driver must return the same
poses with the rows computed on the host (CSM_DEVICE_TRIG=0) and on the
device. Tolerance 0 throughout.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import pyoracle as O  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    import roborts_csm
    c = roborts_csm.Context(0)
    yield c
    c.close()


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def _arguments(n, seed):
    """Arguments over every branch of the restated sincos: tiny (< 2^-27), the
    table range (< 0.855), the pi/2 - x range (< 2.426), the reduced range (up
    to 1e8), the window grids the driver plans (centre +- offset in steps of
    the angle resolution), and the branch thresholds' neighbours."""
    rng = np.random.default_rng(seed)
    parts = [
        np.ldexp(rng.random(n), rng.integers(-40, 12, n)),
        (rng.random(n) - 0.5) * 16.0,
        (rng.random(n) - 0.5) * 2.0e8,
    ]
    centre = (rng.random(n // 64) - 0.5) * 8.0
    for res, off in ((np.deg2rad(1.0), np.deg2rad(15.0)), (np.deg2rad(0.25), np.deg2rad(2.0)), (0.0005, 0.004)):
        k = np.arange(int(2 * off / res) + 1)
        parts.append(((centre - off)[:, None] + k[None, :] * res).ravel())
    edges = np.array([0x3E400000, 0x3FEB6000, 0x400368FD, 0x41991000], dtype=np.uint64) << np.uint64(32)
    d = np.arange(-256, 257, dtype=np.int64)
    e = (edges[:, None].astype(np.int64) + d[None, :]).ravel().astype(np.uint64).view(np.float64)
    parts += [e, -e]
    x = np.concatenate(parts)
    return np.where(rng.random(x.size) < 0.5, x, -x)


@pytest.mark.parametrize("seed", [1, 2])
def test_device_sincos_equals_host_libm(ctx, seed):
    x = _arguments(1 << 20, seed)
    s, c = ctx.sincos_device(x)
    s0, c0 = O.sincos_batch(x)
    bad = ~((s.view(np.uint64) == s0.view(np.uint64)) & (c.view(np.uint64) == c0.view(np.uint64)))
    assert not bad.any(), f"{int(bad.sum())} of {x.size} differ, first at x={x[np.argmax(bad)]!r}"


def test_device_sincos_outside_domain(ctx):
    """Beyond 105414350 (glibc's __branred range, not restated), zeros,
    subnormals, inf and NaN: the host computes what the device does not."""
    x = np.array([0.0, -0.0, 5e-324, -2.2e-308, 105414350.0, 105414349.9, -1.0e9, 1.0e300,
                  np.inf, -np.inf, np.nan, 2.0 ** -27, 0.855469, 2.426265, np.pi, -np.pi / 2])
    s, c = ctx.sincos_device(x)
    s0, c0 = O.sincos_batch(x)
    fin = np.isfinite(x)
    assert _bits_equal(s[fin], s0[fin]) and _bits_equal(c[fin], c0[fin])
    assert np.isnan(s[~fin]).all() and np.isnan(c[~fin]).all()


def _ctx_env(**env):
    import roborts_csm
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return roborts_csm.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def world2000():
    from roborts_csm import worlds
    w = worlds.make_world(2000, 2000, 0.05)
    b = worlds.make_scan_batch(w, 96, seed=7)
    return w, b


@pytest.mark.parametrize("parts", ["2", "3"])
def test_driver_rows_device_equal_host(world2000, parts):
    """The 3-level driver with its angle rows' cos/sin from the device and from
    the host's ::sincos: the same poses, covariances and responses, and the
    oracle's; the device path really ran (host:trig_rows counts its levels)."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    out = {}
    for trig in ("1", "0"):
        c = _ctx_env(CSM_PIPELINE="16", CSM_PIPELINE_PARTS=parts, CSM_DEVICE_TRIG=trig, CSM_SMALL="0")
        try:
            c.set_grid(roborts_csm.ScanMatchMap(w.grid, float(w.resolution), tuple(w.offset), 0, 1))
            poses = np.ascontiguousarray(b.init_poses.copy())
            covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
            c.set_profiling(True)
            s = c.scan_matchers_batch(b.points_cells, b.offsets, headline_levels(), poses, covs)
            st = {k["name"]: k["launches"] for k in c.kernel_stats()}
            c.set_profiling(False)
            out[trig] = (s, poses, covs, st.get("host:trig_rows", 0) + st.get("host:trig_rows:gen", 0))
        finally:
            c.close()
    assert out["1"][3] >= 2 * int(parts) and out["0"][3] == 0
    for a, b_ in zip(out["1"][:3], out["0"][:3]):
        assert _bits_equal(a, b_)
    m = O.Map(w.grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), b.init_poses,
                                       np.tile(np.eye(3).reshape(1, 9), (b.init_poses.shape[0], 1)))
    assert np.array_equal(out["1"][0], s2) and np.array_equal(out["1"][1], p2) and np.array_equal(out["1"][2], c2)


def test_driver_rows_outside_domain(world2000):
    """Scans whose pose angle lies beyond the restated sincos's domain (|theta|
    >= 105414350 rad, glibc's __branred range): their launches copy the host's
    rows and the kernel fills the rest in place; the results are the oracle's."""
    import roborts_csm
    from roborts_csm.params import headline_levels
    w, b = world2000
    init = b.init_poses.copy()
    init[::5, 2] += 1.2e8  # every fifth scan far outside (the same direction modulo 2 pi, roughly)
    c = _ctx_env(CSM_PIPELINE="16", CSM_PIPELINE_PARTS="2", CSM_SMALL="0")
    try:
        c.set_grid(roborts_csm.ScanMatchMap(w.grid, float(w.resolution), tuple(w.offset), 0, 1))
        poses = np.ascontiguousarray(init.copy())
        covs = np.tile(np.eye(3).reshape(1, 9), (poses.shape[0], 1))
        c.set_profiling(True)
        s = c.scan_matchers_batch(b.points_cells, b.offsets, headline_levels(), poses, covs)
        st = {k["name"]: k["launches"] for k in c.kernel_stats()}
        c.set_profiling(False)
    finally:
        c.close()
    assert st.get("host:trig_rows", 0) > 0
    m = O.Map(w.grid, w.resolution, w.offset)
    s2, p2, c2 = O.scan_matchers_batch(m, b.points_cells, b.offsets, headline_levels(), init,
                                       np.tile(np.eye(3).reshape(1, 9), (init.shape[0], 1)))
    assert _bits_equal(s, s2) and _bits_equal(poses, p2) and _bits_equal(covs, c2)
