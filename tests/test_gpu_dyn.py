"""The device copy of the dynamical matrix (gle_set_dyn, include/hipgle.h) drops the roundoff that
md.setDyn's U diag(w^2) U^T reconstruction (reference md.py:264-292) leaves in the entries the
matrix does not couple: the pair d_ij, d_ji goes when max(|d_ij|, |d_ji|) <= 16 * 2^-52 *
max(max_k |d_ik|, max_k |d_jk|) (symmetric: both entries or neither).  Checked here: the rule keeps exactly
the physical pattern of the benched junctions (CPU), a run fed the setDyn-processed (dense) matrix
is bit-identical to one fed the matrix with those entries zeroed, and both match the oracle's
dense product to the parity tolerance (GPU)."""
import numpy as np
import pytest

from conftest import load_golden, oracle_from_golden

DROP = 16.0 * 2.0 ** -52
RTOL_TRAJ = 1e-10   # as tests/test_gpu_parity.py


def clean(dyn):
    d = np.array(dyn, dtype=float)
    rmax = np.max(np.abs(d), axis=1)
    thr = DROP * np.maximum.outer(rmax, rmax)
    d[np.maximum(np.abs(d), np.abs(d.T)) <= thr] = 0.0
    return d


@pytest.mark.parametrize("cfg", ["C3", "C5"])
def test_drop_rule_keeps_the_physical_pattern(cfg):
    """md.setDyn's reconstruction of the benched junctions: the dropped entries are exactly the
    ones the raw matrix does not couple, and they are all roundoff (<= 16 eps of the row max)."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    dyn, axyz, _, meta = synthetic.junction(cfg, seed=1234, gmem_device=True)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=1, seed=1, verbose=False)
    dense = np.asarray(m.dyn)
    assert np.count_nonzero(dense) > 10 * np.count_nonzero(dyn)  # the reconstruction is dense
    kept = clean(dense) != 0.0
    np.testing.assert_array_equal(kept, np.asarray(dyn) != 0.0)


def _run(g, dyn, nsteps):
    from conftest import constr_from
    from sclmd_amd import _native as N

    nph = 3 * int(g["natom"])
    st = N.Stepper(nph, 1, int(g["nmd"]), float(g["dt"]), 0, 0, "auto")
    try:
        for i in range(int(g["nbath"])):
            kind = str(g["b%d_kind" % i])
            if kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, g["b%d_cids" % i], g["b%d_kernel" % i],
                            float(g["b%d_bias" % i]), g["b%d_exim" % i], g["b%d_zeta1" % i],
                            g["b%d_zeta2" % i])
            else:
                st.add_bath(N.GLE_BATH_PHONON, g["b%d_cids" % i], g["b%d_kernel" % i])
        st.set_dyn(dyn)
        c = constr_from(g)
        if c:
            st.set_constraint([d for r in c for d in r])
        st.set_state(g["p0"][None], g["q0"][None], 0)
        dropped = st.plan_detail()["dyn_dropped"]
        assert dropped == np.count_nonzero(dyn) - np.count_nonzero(clean(dyn)), dropped
        for i in range(int(g["nbath"])):
            st.set_history(i, None)
            st.set_noise(i, g["b%d_noise" % i][None])
        qs = []
        for _ in range(nsteps):
            st.step_begin(None, want_qt=False)
            st.step_end(None)
            qs.append(st.get_state()[1][0].copy())
        return np.array(qs)
    finally:
        st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["vv_mixed", "vv_biased"])
def test_roundoff_entries_do_not_change_the_device_run(case):
    g = load_golden(case)
    nsteps = int(g["nsteps"])
    # the golden setDyn-processed matrices are physically dense: nothing is dropped from them
    np.testing.assert_array_equal(clean(g["dyn_md"]), g["dyn_md"])
    # a banded physical matrix (a chain's coupling pattern) from the golden one, and the same
    # matrix carrying reconstruction-sized roundoff (<= 8 eps of the row max, random signs) in
    # every entry it does not couple
    n = g["dyn_md"].shape[0]
    band = np.abs(np.subtract.outer(np.arange(n), np.arange(n))) <= 3
    phys = np.where(band, g["dyn_md"], 0.0)
    rng = np.random.default_rng(7)
    rowmax = np.max(np.abs(phys), axis=1, keepdims=True)
    noisy = np.where(band, phys, rng.uniform(-8.0, 8.0, size=phys.shape) * 2.0 ** -52 * rowmax)
    assert np.count_nonzero(noisy) == n * n and np.array_equal(clean(noisy), phys)
    q_phys = _run(g, phys, nsteps)
    q_noisy = _run(g, noisy, nsteps)
    np.testing.assert_array_equal(q_noisy, q_phys)
    # the oracle multiplies by the dense noisy matrix (the reference's own arithmetic)
    sim = oracle_from_golden(g)
    sim.dyn = noisy
    worst = 0.0
    for k in range(nsteps):
        sim.step()
        worst = max(worst, float(np.max(np.abs(q_noisy[k] - sim.q)) / max(np.max(np.abs(sim.q)), 1e-300)))
    assert worst < RTOL_TRAJ, worst
