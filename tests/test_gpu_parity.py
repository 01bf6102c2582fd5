"""GPU parity: the HIP stepper (through the C-ABI) against the reference-pinned golden
trajectories and the CPU oracle.  fp64 throughout; tolerances are stated per assertion."""
import numpy as np
import pytest

from conftest import constr_from, load_golden, oracle_from_golden, vv_cases

pytestmark = pytest.mark.gpu

RTOL_TRAJ = 1e-10   # q, p after every step, relative to the trajectory's max magnitude
RTOL_CUR = 1e-9     # heat current per step (north star: 1e-6 on the time-averaged current)


def relerr(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def stepper_from_golden(g, ntraj=1, block_len=0, far_mode="auto"):
    from sclmd_amd import _native as N

    nph = 3 * int(g["natom"])
    st = N.Stepper(nph, ntraj, int(g["nmd"]), float(g["dt"]), 0, block_len, far_mode)
    for i in range(int(g["nbath"])):
        kind = str(g["b%d_kind" % i])
        if kind == "ebath":
            st.add_bath(N.GLE_BATH_ELECTRON, g["b%d_cids" % i], g["b%d_kernel" % i],
                        float(g["b%d_bias" % i]), g["b%d_exim" % i], g["b%d_zeta1" % i],
                        g["b%d_zeta2" % i])
        else:
            st.add_bath(N.GLE_BATH_PHONON, g["b%d_cids" % i], g["b%d_kernel" % i])
    st.set_dyn(g["dyn_md"])
    c = constr_from(g)
    if c:
        st.set_constraint([d for r in c for d in r])
    st.set_state(np.tile(g["p0"], (ntraj, 1)), np.tile(g["q0"], (ntraj, 1)), 0)
    for i in range(int(g["nbath"])):
        st.set_history(i, None)
        st.set_noise(i, np.tile(g["b%d_noise" % i][None], (ntraj, 1, 1)))
    return st


FAR_VARIANTS = [("auto", 0), ("direct", 1), ("direct", 3), ("direct", 16), ("spectral", 2), ("spectral", 5), ("spectral", 16)]


@pytest.mark.parametrize("case", vv_cases())
@pytest.mark.parametrize("far_mode,block_len", FAR_VARIANTS)
def test_vv_golden(case, far_mode, block_len):
    g = load_golden(case)
    st = stepper_from_golden(g, 1, block_len, far_mode)
    pow2 = block_len > 1 and (block_len & (block_len - 1)) == 0
    if far_mode == "spectral" and pow2 and max(int(g["b%d_ml" % i]) for i in range(int(g["nbath"]))) > 2 * block_len:
        assert st.plan_info()["far_mode"] == "spectral"
    nmd = int(g["nmd"])
    qs, ps = [], []
    for _ in range(int(g["nsteps"])):
        st.step_begin(None, want_qt=False)
        st.step_end(None)
        p, q, _ = st.get_state()
        ps.append(p[0])
        qs.append(q[0])
    assert relerr(qs, g["q"]) < RTOL_TRAJ, case
    assert relerr(ps, g["p"]) < RTOL_TRAJ, case
    cur = st.get_current()[:, 0, :]
    et = st.get_energy()[0]
    n = int(g["nsteps"])
    tn = [t % nmd for t in range(max(0, n - nmd), n)]
    gold_cur = g["cur"][max(0, n - nmd):n].T
    assert relerr(cur[:, tn], gold_cur) < RTOL_CUR, case
    assert relerr(et[tn], g["etot"][max(0, n - nmd):n]) < RTOL_TRAJ, case
    st.close()


@pytest.mark.parametrize("case", ["vv_mixed", "vv_biased", "vv_twoph"])
@pytest.mark.parametrize("far_mode", ["direct", "spectral"])
def test_vv_batched_trajectories(case, far_mode):
    """B trajectories with different initial states and noise vs the oracle, one by one."""
    g = load_golden(case)
    B = 5
    rng = np.random.default_rng(7)
    st = stepper_from_golden(g, B, 4 if far_mode == "spectral" else 0, far_mode)
    p0 = g["p0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    q0 = g["q0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    st.set_state(p0, q0, 0)
    noises = []
    for i in range(int(g["nbath"])):
        st.set_history(i, None)
        nz = g["b%d_noise" % i][None] * (1 + rng.normal(size=(B, 1, 1)))
        noises.append(nz)
        st.set_noise(i, nz)
    nsteps = int(g["nsteps"])
    st.run(nsteps)
    p, q, t = st.get_state()
    assert t == nsteps
    for b in range(B):
        sim = oracle_from_golden(g)
        sim.p, sim.q = p0[b].copy(), q0[b].copy()
        for i, bath in enumerate(sim.baths):
            bath.noise = noises[i][b]
        for _ in range(nsteps):
            sim.step()
        assert relerr(q[b], sim.q) < RTOL_TRAJ
        assert relerr(p[b], sim.p) < RTOL_TRAJ
    st.close()


@pytest.mark.parametrize("case", ["vv_biased", "vv_mixed"])
def test_vv_wide_batch_across_noise_periods(case):
    """64 trajectories (several chain column tiles) run across two ends of the noise ring -- the
    last time slot is where an operand read past the ring once faulted -- checked against the
    oracle on a few trajectories."""
    g = load_golden(case)
    B, nmd = 64, int(g["nmd"])
    rng = np.random.default_rng(11)
    st = stepper_from_golden(g, B)
    p0 = g["p0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    q0 = g["q0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    st.set_state(p0, q0, 0)
    noises = []
    for i in range(int(g["nbath"])):
        st.set_history(i, None)
        nz = g["b%d_noise" % i][None] * (1 + rng.normal(size=(B, 1, 1)))
        noises.append(nz)
        st.set_noise(i, nz)
    nsteps = 2 * nmd + 3
    st.run(nsteps)
    p, q, t = st.get_state()
    assert t == nsteps
    for b in (0, 17, 63):
        sim = oracle_from_golden(g)
        sim.p, sim.q = p0[b].copy(), q0[b].copy()
        for i, bath in enumerate(sim.baths):
            bath.noise = noises[i][b]
        for _ in range(nsteps):
            sim.step()
        assert relerr(q[b], sim.q) < RTOL_TRAJ
        assert relerr(p[b], sim.p) < RTOL_TRAJ
    st.close()


def test_no_bath_nve_vs_oracle():
    """md without baths (md.py: the bath loops of force() are empty): velocity Verlet on the harmonic
    potential alone, with constraints, against the oracle; energy stays constant to the integrator's
    order."""
    from sclmd_amd import _native as N
    from oracle import sclmd_oracle as O

    g = load_golden("vv_mixed")
    nph, nmd, dt = 3 * int(g["natom"]), int(g["nmd"]), float(g["dt"])
    B = 3
    st = N.Stepper(nph, B, nmd, dt, 0)
    st.set_dyn(g["dyn_md"])
    st.set_constraint([0, 1])
    rng = np.random.default_rng(2)
    p0 = rng.normal(size=(B, nph)) * 1e-2
    q0 = rng.normal(size=(B, nph)) * 1e-1
    p0[:, :2] = q0[:, :2] = 0.0
    st.set_state(p0, q0, 0)
    nsteps = 2 * nmd + 5
    st.run(nsteps)
    p, q, t = st.get_state()
    assert t == nsteps
    for b in range(B):
        sim = O.GLE(nph, dt, nmd, [], dyn=g["dyn_md"], constr=[range(0, 2)])
        sim.p, sim.q = p0[b].copy(), q0[b].copy()
        for _ in range(nsteps):
            sim.step()
        assert relerr(q[b], sim.q) < RTOL_TRAJ and relerr(p[b], sim.p) < RTOL_TRAJ
    st.close()


@pytest.mark.parametrize("case", vv_cases())
@pytest.mark.parametrize("far_mode,block_len", [("auto", 0), ("spectral", 4)])
def test_vv_golden_through_run(case, far_mode, block_len):
    """The golden trajectories through gle_run (st.run), the path bench and md.Run take: the composed
    one-launch step where the plan allows it (GLE_PLAN_COMPOSED_STEP; the biased ebath and the
    overlapping phonon baths keep the two-launch path), one step per call with the state read after
    each, then the whole run in one call -- against the reference's own fixtures."""
    g = load_golden(case)
    st = stepper_from_golden(g, 1, block_len, far_mode)
    composed = st.plan_detail()["composed_step"]
    if case == "vv_mixed":  # unbiased ebath + memory-kernel phonon bath + constraints
        assert composed
    if case in ("vv_biased", "vv_twoph"):
        assert not composed
    n = int(g["nsteps"])
    qs, ps = [], []
    for _ in range(n):
        st.run(1)
        p, q, _ = st.get_state()
        ps.append(p[0])
        qs.append(q[0])
    assert relerr(qs, g["q"]) < RTOL_TRAJ, case
    assert relerr(ps, g["p"]) < RTOL_TRAJ, case
    st.close()
    st = stepper_from_golden(g, 1, block_len, far_mode)
    st.run(n)
    p, q, t = st.get_state()
    assert t == n
    assert relerr(q[0], g["q"][-1]) < RTOL_TRAJ and relerr(p[0], g["p"][-1]) < RTOL_TRAJ, case
    nmd = int(g["nmd"])
    tn = [t % nmd for t in range(max(0, n - nmd), n)]
    assert relerr(st.get_current()[:, 0, tn], g["cur"][max(0, n - nmd):n].T) < RTOL_CUR, case
    assert st.cache_audit() == (0, 0)
    st.close()
