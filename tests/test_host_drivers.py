"""Host force phase of an ensemble with one driver per trajectory: the sameq cache
per trajectory (md.py:437-474, 767-779) and concurrent driver calls.  Host logic only: md objects
touch the device only when stepped."""
import threading
import time

import numpy as np
import pytest

from sclmd_amd import md as MD
from sclmd_amd import synthetic
from sclmd_amd.drivers import HarmonicDriver


class SlowDriver(HarmonicDriver):
    """HarmonicDriver whose force call takes a while and records how many calls overlap."""

    active = 0
    peak = 0
    lock = threading.Lock()

    def force(self, q):
        with SlowDriver.lock:
            SlowDriver.active += 1
            SlowDriver.peak = max(SlowDriver.peak, SlowDriver.active)
        time.sleep(0.05)
        try:
            return super().force(q)
        finally:
            with SlowDriver.lock:
                SlowDriver.active -= 1


def _md(ntraj):
    natom = 6
    dyn = synthetic.chain_dyn(natom)
    axyz = synthetic.axyz_chain(natom)
    return MD.md(synthetic.DT, 16, 300.0, axyz=axyz, ntraj=ntraj, verbose=False), dyn, axyz


def test_per_trajectory_drivers_concurrent_and_cached(monkeypatch):
    monkeypatch.setenv("SCLMD_FORCE_WORKERS", "8")
    B = 8
    m, dyn, axyz = _md(B)
    drivers = [SlowDriver(dyn, axyz) for _ in range(B)]
    m.AddPotential(drivers)
    rng = np.random.default_rng(3)
    qs = rng.normal(size=(B, m.nph)) * 1e-2
    cache = [([], None)] * B
    SlowDriver.peak = 0
    t0 = time.perf_counter()
    f = m._host_forces(qs, cache)
    wall = time.perf_counter() - t0
    np.testing.assert_allclose(f, -(qs @ dyn.T), rtol=1e-14, atol=1e-18)
    assert SlowDriver.peak > 1 and wall < 0.05 * B * 0.75   # calls overlapped
    assert all(d.ncalls == 2 for d in drivers)              # initforce + one force each
    # the same configurations hit every trajectory's cache: no driver call
    f2 = m._host_forces(qs.copy(), cache)
    assert np.array_equal(f, f2) and all(d.ncalls == 2 for d in drivers)
    # one trajectory moves: only its driver is called
    qs[5] += 1e-6
    m._host_forces(qs, cache)
    assert [d.ncalls for d in drivers] == [2] * 5 + [3] + [2] * 2
    m.close()


def test_single_driver_serial_matches_list():
    B = 4
    m1, dyn, axyz = _md(B)
    d1 = HarmonicDriver(dyn, axyz)
    m1.AddPotential(d1)
    m2, _, _ = _md(B)
    m2.AddPotential([HarmonicDriver(dyn, axyz) for _ in range(B)])
    qs = np.random.default_rng(5).normal(size=(B, m1.nph))
    f1 = m1._host_forces(qs, [([], None)] * B)
    f2 = m2._host_forces(qs, [([], None)] * B)
    assert np.array_equal(f1, f2) and d1.ncalls == 1 + B
    with pytest.raises(ValueError):
        m1.AddPotential([d1, d1])
    m1.close()
    m2.close()
