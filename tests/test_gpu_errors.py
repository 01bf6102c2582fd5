"""The C-ABI's error behaviour: misuse returns an error code with a message (the reference prints and
calls sys.exit for its shape errors, md.py / baths.py; the drop-in raises) and leaves the handle
usable -- after every rejected call below, a valid run still matches the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _expect(fn, code):
    from sclmd_amd import _native as N

    with pytest.raises(N.GLEError) as e:
        fn()
    assert code in str(e.value), str(e.value)


def test_gle_create_rejects_bad_config():
    from sclmd_amd import _native as N

    _expect(lambda: N.Stepper(12, 2, 63, 0.5, 0), "GLE_ERR_ARG")   # odd nmd (functions.py:47-50)
    _expect(lambda: N.Stepper(0, 2, 64, 0.5, 0), "GLE_ERR_ARG")
    _expect(lambda: N.Stepper(12, 0, 64, 0.5, 0), "GLE_ERR_ARG")
    _expect(lambda: N.Stepper(12, 2, 64, -0.5, 0), "GLE_ERR_ARG")


def test_misuse_is_rejected_and_the_handle_stays_usable():
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C3", natom=20, ml=24, nmd=128, nw=60, seed=4)
    nph, nmd, dt, B = meta["nph"], meta["nmd"], meta["dt"], 5
    st = N.Stepper(nph, B, nmd, dt, 0)
    try:
        bad = np.asarray(baths[0].cids).copy()
        bad[-1] = nph  # a DOF past the system
        _expect(lambda: st.add_bath(N.GLE_BATH_PHONON, bad, baths[0].kernel), "GLE_ERR_ARG")
        for b in baths:
            st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        _expect(lambda: st.set_constraint([0, nph]), "GLE_ERR_ARG")
        _expect(lambda: st.run(3), "GLE_ERR_STATE")                       # no state yet
        rng = np.random.default_rng(1)
        p = rng.normal(size=(B, nph)) * 1e-2
        q = rng.normal(size=(B, nph)) * 1e-2
        st.set_state(p, q, 0)
        _expect(lambda: st.set_plan_class("large"), "GLE_ERR_STATE")     # the plan is built
        _expect(lambda: st.run(3), "GLE_ERR_STATE")                       # no noise yet
        assert st.lib.gle_set_noise(st.h, len(baths), None) == -1            # bad bath id: GLE_ERR_ARG
        noise = [rng.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
        for i in range(len(baths)):
            st.set_noise(i, noise[i])
        _expect(lambda: st.power_spectrum([[0, 1]]), "GLE_ERR_STATE")    # nothing recorded
        _expect(lambda: st.power_spectrum([[0, nph]]), "GLE_ERR")
        # a step begun with a host force must end with one
        qt = st.step_begin(-(q @ dyn.T))
        _expect(lambda: st.step_end(None), "GLE_ERR_STATE")
        st.step_end(-(qt @ dyn.T))
        ob = [O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)]
        sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=B)
        sim.p, sim.q = p.T.copy(), q.T.copy()
        sim.step()
        st.run(40)
        for _ in range(40):
            sim.step()
        pg, qg, t = st.get_state()
        assert t == 41
        assert rel(qg, sim.q.T) < 1e-10 and rel(pg, sim.p.T) < 1e-10
    finally:
        st.close()

