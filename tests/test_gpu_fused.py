"""GPU tests of the fused velocity-iteration stage (dof_BC: md.py:401-408 in one launch via the
precomputed K0^2, K0 P dyn, K0 Kq products) against the two-launch B + C path, which the golden
trajectory tests pin to the reference: ordinary dynamics, a biased electron bath next to a
memory-kernel phonon bath (the q channel), constraints, and a near-static start where md.potforce's
cache hits at q~ (the K0 Fc branch).  Tolerance 1e-10 relative (K0 p1 is re-associated)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _system(biased):
    from sclmd_amd import synthetic

    natom, ml, nmd = 12, 24, 96
    dyn, axyz, baths, meta = synthetic.junction("C3", seed=3, natom=natom, ml=ml, nmd=nmd, nw=80)
    if biased:
        rng = np.random.default_rng(8)
        baths = [baths[0], synthetic.make_biased_ebath(300.0, list(range(3 * 9, 3 * 12)), nmd, rng)]
    return dyn, baths, meta


def _run(fused, biased, scale_p, scale_q, scale_n, constr, nsteps=60, ntraj=4):
    from sclmd_amd import _native as N

    dyn, baths, meta = _system(biased)
    old = os.environ.get("GLE_FUSE_BC")
    os.environ["GLE_FUSE_BC"] = "1" if fused else "0"
    try:
        st = N.Stepper(meta["nph"], ntraj, meta["nmd"], meta["dt"], 0)
        for b in baths:
            if b.kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        if constr:
            st.set_constraint(list(range(3, 6)))
        rng = np.random.default_rng(21)
        st.set_state(rng.normal(size=(ntraj, meta["nph"])) * scale_p,
                     rng.normal(size=(ntraj, meta["nph"])) * scale_q, 0)
        for i, b in enumerate(baths):
            st.set_history(i, None)
            st.set_noise(i, rng.normal(size=(ntraj, meta["nmd"], b.nc)) * scale_n)
        st.run(nsteps)
        p, q, _ = st.get_state()
        cur = st.get_current()[:, :, :nsteps]
        st.close()
        return p, q, cur
    finally:
        if old is None:
            del os.environ["GLE_FUSE_BC"]
        else:
            os.environ["GLE_FUSE_BC"] = old


@pytest.mark.parametrize("biased,constr", [(False, False), (False, True), (True, True)])
def test_fused_matches_two_launch_path(biased, constr):
    a = _run(True, biased, 1e-2, 1e-2, 1e-3, constr)
    b = _run(False, biased, 1e-2, 1e-2, 1e-3, constr)
    for x, y in zip(a, b):
        assert rel(x, y) < 1e-10


def test_fused_potforce_cache_hits():
    """At rest with no noise and displacements far below md.potforce's 1e-9 cache radius, the id1
    force comes from the cache (K0 Fc branch of the fused stage)."""
    a = _run(True, False, 0.0, 1e-13, 0.0, False, nsteps=20)
    b = _run(False, False, 0.0, 1e-13, 0.0, False, nsteps=20)
    assert np.max(np.abs(a[1])) > 0
    for x, y in zip(a[:2], b[:2]):
        assert rel(x, y) < 1e-10
