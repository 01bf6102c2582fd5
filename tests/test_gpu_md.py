"""GPU tests of the drop-in md API and of the noise generator, plus full-size (C3) properties.

Tolerances: trajectories 1e-10 relative to the trajectory scale, heat currents 1e-9 relative
(north star: 1e-6 on the time-averaged current), noise 1e-12; statistical tests state theirs."""
import numpy as np
import pytest

from conftest import constr_from, load_golden, oracle_from_golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_seeded_run_matches_reference(tmp_path, monkeypatch):
    """md.Run with the numpy-compatible noise: initialise + per-run gnoi + nmd vv steps + kappa files,
    against the real reference run with the same numpy seed (golden run_seeded)."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath

    g = load_golden("run_seeded")
    monkeypatch.chdir(tmp_path)
    dt, nmd, T = float(g["dt"]), int(g["nmd"]), float(g["T"])
    m = MD.md(dt, nmd, T, axyz=synthetic.axyz_chain(int(g["natom"])), dyn=g["dyn"], nstart=0,
              nstop=int(g["nrun"]), verbose=False)
    b1 = phbath(float(g["T1"]), g["c1"], debye=float(g["debye1"]), nw=int(g["nw1"]), dt=dt, nmd=nmd,
                ml=int(g["ml1"]), gamma=g["gam1"], gwl=g["gwl1"])
    b1.gmem()
    b2 = ebath(g["c2"], float(g["T2"]), dt, nmd, wmax=1.0, nw=50, bias=0.0, efric=g["efric2"])
    m.AddBath(b1)
    m.AddBath(b2)
    m.AddConstr([range(6, 8)])
    np.random.seed(int(g["seed"]))
    m.Run()
    assert m.t == int(g["t_end"])
    assert rel(m.p, g["p_end"]) < 1e-9 and rel(m.q, g["q_end"]) < 1e-9
    assert rel(np.array(m.kappa_runs), g["kappa"]) < 1e-9
    for j in range(int(g["nrun"])):
        for i in range(2):
            row = open("kappa.%s.bath%d.run%d.dat" % (str(T), i, j)).read().split()
            assert int(row[0]) == j and abs(float(row[2]) - g["kappa"][j, i]) < 2e-6
    assert rel(b1.cur, g["cur"][-1, 0]) < 1e-9
    m.close()


def _md_from_golden(g, driver=False):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath
    from sclmd_amd.drivers import HarmonicDriver

    dt, nmd = float(g["dt"]), int(g["nmd"])
    axyz = synthetic.axyz_chain(int(g["natom"]))
    m = MD.md(dt, nmd, float(g["T"]), axyz=axyz, dyn=None if driver else g["dyn_md"], verbose=False)
    for i in range(int(g["nbath"])):
        cids = g["b%d_cids" % i]
        if str(g["b%d_kind" % i]) == "ebath":
            b = ebath(cids, 300.0, dt, nmd, bias=float(g["b%d_bias" % i]), efric=g["b%d_efric" % i],
                      exim=g["b%d_exim" % i], zeta1=g["b%d_zeta1" % i], zeta2=g["b%d_zeta2" % i])
        else:
            b = phbath(300.0, cids, 0.2, 10, dt, nmd, ml=int(g["b%d_ml" % i]))
            b.kernel = g["b%d_kernel" % i]
            b.ml = int(g["b%d_ml" % i])
        b.noise = g["b%d_noise" % i]
        m.AddBath(b)
    c = constr_from(g)
    if c:
        m.AddConstr(c)
    drv = None
    if driver:
        drv = HarmonicDriver(g["dyn_md"], axyz)
        m.AddPotential(drv)
    m.p, m.q, m.t = g["p0"], g["q0"], 0
    m.ResetHis()
    return m, drv


@pytest.mark.parametrize("case", ["vv_mixed", "vv_biased", "vv_twoph"])
def test_host_driver_path(case):
    """Forces from a host plugin (.force(q), the lammpsdriver surface) at q_t and q~ each step."""
    g = load_golden(case)
    m, drv = _md_from_golden(g, driver=True)
    qs = []
    for _ in range(int(g["nsteps"])):
        m.vv(0)
        qs.append(np.array(m.q))
    assert rel(qs, g["q"]) < 1e-10
    assert rel(m.p, g["p"][-1]) < 1e-10
    # md.potforce cache: one driver call per step without constraints, two with (md.py:449)
    n = int(g["nsteps"])
    if constr_from(g):
        assert n + 1 <= drv.ncalls - 1 <= 2 * n + 1
    else:
        assert drv.ncalls - 1 == n + 1
    m.close()


def test_md_vv_device_harmonic():
    g = load_golden("vv_mixed")
    m, _ = _md_from_golden(g)
    for _ in range(int(g["nsteps"])):
        m.vv(0)
    assert rel(m.q, g["q"][-1]) < 1e-10
    et = np.asarray(m.etot)
    n, nmd = int(g["nsteps"]), int(g["nmd"])
    assert rel(et[(n - 1) % nmd], g["etot"][n - 1]) < 1e-10
    m.close()


@pytest.mark.parametrize("tag", ["ph_q", "ph_nozp"])
def test_phnoise_device_matches_reference(tag):
    from sclmd_amd import noise as N

    g = load_golden("noise")
    T, phcut, cl, zp = g["params_" + tag]
    np.random.seed(11)
    nz = N.phnoise(g["gam"], g["gwl"], T, phcut, float(g["dt"]), int(g["nmd"]), bool(cl), bool(zp))
    assert rel(nz, np.real(g["noise_" + tag])) < 1e-12


@pytest.mark.parametrize("tag", ["e_eq", "e_bias"])
def test_enoise_device_matches_reference(tag):
    from sclmd_amd import noise as N
    from sclmd_amd.functions import antisymmetrize, symmetrize

    g = load_golden("noise")
    bias, T, ecut, cl, zp = g["params_" + tag]
    np.random.seed(12)
    nz = N.enoise(symmetrize(g["efric"]), antisymmetrize(g["exim"]), symmetrize(g["exip"]), bias, T,
                  ecut, float(g["dt"]), int(g["nmd"]), bool(cl), bool(zp))
    assert rel(nz, np.real(g["noise_" + tag])) < 1e-12


@pytest.mark.parametrize("kind", ["ph", "e"])
def test_device_noise_covariance(kind):
    """Philox ensemble noise: the time-averaged covariance over 1024 trajectories matches
    scale^2 (A+_0 + A+_h + 2 sum_{0<w<h} A+_w) (the PSD part of the reference's spectrum).
    Statistical tolerance: 6% of the largest diagonal entry."""
    from sclmd_amd import noise as N
    from sclmd_amd.functions import antisymmetrize, symmetrize

    g = load_golden("noise")
    dt, nmd = float(g["dt"]), int(g["nmd"])
    if kind == "ph":
        spec = N.phonon_spectrum(g["gam"], g["gwl"], 300.0, 0.4, dt, nmd)
    else:
        spec = N.electron_spectrum(symmetrize(g["efric"]), antisymmetrize(g["exim"]),
                                   symmetrize(g["exip"]), 0.3, 300.0, 1.0, dt, nmd)
    f = N.NoiseFactor(spec)
    nz = N.generate(f, dt, nmd, ntraj=1024, seed=12345)
    emp = np.einsum("btk,btl->kl", nz, nz) / (nz.shape[0] * nz.shape[1])
    m = f.scaled()
    ap = np.real(np.einsum("wik,wjk->wij", m, np.conj(m)))
    h = nmd // 2
    scale = 1.0 / (dt * nmd)
    theory = scale ** 2 * (ap[0] + ap[h] + 2.0 * ap[1:h].sum(axis=0))
    assert np.max(np.abs(emp - theory)) < 0.06 * np.max(np.diag(theory))
    # different seeds give different realisations, same seed the same one
    nz2 = N.generate(f, dt, nmd, ntraj=4, seed=12345)
    nz3 = N.generate(f, dt, nmd, ntraj=4, seed=777)
    assert np.array_equal(nz2, nz[:4]) and not np.allclose(nz3, nz2)


def _c3_stepper(ntraj, ml=1024, nmd=4096, block_len=0, far_mode="auto"):
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", ml=ml, nmd=nmd)
    st = N.Stepper(meta["nph"], ntraj, meta["nmd"], meta["dt"], 0, block_len, far_mode)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    return st, baths, meta


@pytest.mark.parametrize("far_mode", ["direct", "spectral"])
def test_c3_linearity_full_size(far_mode):
    """At the full C3 shape (nph 900, 2 x nc 300, ml 1024): the step is linear in (state, noise), so
    trajectory(s1+s2, n1+n2) == trajectory(s1, n1) + trajectory(s2, n2) within fp64 rounding."""
    st, baths, meta = _c3_stepper(3, far_mode=far_mode)
    nph, nmd = meta["nph"], meta["nmd"]
    rng = np.random.default_rng(5)
    p = rng.normal(size=(3, nph)) * 1e-3
    q = rng.normal(size=(3, nph)) * 1e-3
    p[2], q[2] = p[0] + p[1], q[0] + q[1]
    st.set_state(p, q, 0)
    for i, b in enumerate(baths):
        st.set_history(i, None)
        n = rng.normal(size=(3, nmd, b.nc)) * 1e-3
        n[2] = n[0] + n[1]
        st.set_noise(i, n)
    st.run(70)
    p, q, t = st.get_state()
    assert t == 70
    assert rel(q[2], q[0] + q[1]) < 1e-11 and rel(p[2], p[0] + p[1]) < 1e-11
    st.close()


@pytest.mark.parametrize("far_mode", ["direct", "spectral"])
def test_c3_trajectory_vs_oracle_short(far_mode):
    """Full C3 shape, 1 trajectory, a few steps against the oracle (reference-shaped numpy)."""
    from oracle import sclmd_oracle as O

    st, baths, meta = _c3_stepper(1, far_mode=far_mode)
    nph, nmd, dt = meta["nph"], meta["nmd"], meta["dt"]
    rng = np.random.default_rng(9)
    p = rng.normal(size=nph) * 1e-3
    q = rng.normal(size=nph) * 1e-3
    noise = [rng.normal(size=(nmd, b.nc)) * 1e-3 for b in baths]
    st.set_state(p[None], q[None], 0)
    for i in range(len(baths)):
        st.set_history(i, None)
        st.set_noise(i, noise[i][None])
    bs = [O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)]
    from sclmd_amd import synthetic

    sim = O.GLE(nph, dt, nmd, bs, dyn=synthetic.chain_dyn(meta["natom"]))
    sim.p, sim.q = p.copy(), q.copy()
    nst = 40  # crosses the first spectral block boundary (P = 32)
    for _ in range(nst):
        sim.step()
    st.run(nst)
    pg, qg, _ = st.get_state()
    assert rel(qg[0], sim.q) < 1e-10 and rel(pg[0], sim.p) < 1e-10
    cur = st.get_current()[:, 0, :nst]
    assert rel(cur, np.array([b.cur[:nst] for b in bs])) < 1e-9
    st.close()


@pytest.mark.parametrize("far_mode,block_len", [("auto", 0), ("direct", 5), ("spectral", 4), ("spectral", 7)])
def test_ring_wraparound_vs_oracle(far_mode, block_len):
    """Run well past the history ring length (R = ml + 3L + 2 slots) and across the noise period."""
    from sclmd_amd import _native as N
    from oracle import sclmd_oracle as O

    g = load_golden("vv_twoph")
    nph, nmd, dt = 3 * int(g["natom"]), int(g["nmd"]), float(g["dt"])
    st = N.Stepper(nph, 2, nmd, dt, 0, block_len, far_mode)
    for i in range(int(g["nbath"])):
        st.add_bath(N.GLE_BATH_PHONON, g["b%d_cids" % i], g["b%d_kernel" % i])
    st.set_dyn(g["dyn_md"])
    st.set_constraint([0])
    st.set_state(np.tile(g["p0"], (2, 1)), np.tile(g["q0"], (2, 1)), 0)
    for i in range(int(g["nbath"])):
        st.set_history(i, None)
        st.set_noise(i, np.tile(g["b%d_noise" % i][None], (2, 1, 1)))
    nsteps = 260
    st.run(nsteps)
    sim = oracle_from_golden(g)
    for _ in range(nsteps):
        sim.step()
    p, q, t = st.get_state()
    assert t == nsteps
    assert rel(q[0], sim.q) < 1e-9 and rel(q[1], sim.q) < 1e-9
    hist = st.get_history(0)  # newest first, p at t-1, t-2, ... on the bath's DOFs
    assert rel(hist[0, 0], sim.phis[0][g["b0_cids"]]) < 1e-9
    st.close()


def test_deterministic():
    st1, baths, meta = _c3_stepper(2, ml=256, nmd=512)
    st2, _, _ = _c3_stepper(2, ml=256, nmd=512)
    rng = np.random.default_rng(3)
    p = rng.normal(size=(2, meta["nph"])) * 1e-3
    outs = []
    for st in (st1, st2):
        st.set_state(p, p, 0)
        for i, b in enumerate(baths):
            st.set_history(i, None)
            st.noise_factors(i, b.noise_factor().scaled())
            st.noise_generate(i, None, seed=99)
        st.run(30)
        outs.append(st.get_state()[0])
        st.close()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("far_mode,block_len,max_block",
                         [("auto", 0, 0), ("direct", 0, 0), ("spectral", 0, 64), ("spectral", 2, 0), ("direct", 3, 16)])
def test_ladder_long_kernel_vs_oracle(far_mode, block_len, max_block):
    """Every rung of the memory-sum ladder against the oracle: a 1024-slice kernel on a small
    junction, started at an unaligned t with a nonzero history, run past several blocks of the
    largest level (block 256 at the defaults) and across the noise period."""
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic
    from oracle import sclmd_oracle as O

    ml, nmd, t0, nst, B = 1024, 512, 37, 700, 8
    dyn, _, baths, meta = synthetic.junction("C3", ml=ml, nmd=nmd, natom=12, nw=200)
    nph, dt = meta["nph"], meta["dt"]
    st = N.Stepper(nph, B, nmd, dt, 0, block_len, far_mode, max_block)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    rng = np.random.default_rng(21)
    # two distinct trajectories, tiled over the batch
    p = rng.normal(size=(2, nph)) * 1e-3
    q = rng.normal(size=(2, nph)) * 1e-3
    hist = [rng.normal(size=(2, ml, b.nc)) * 1e-3 for b in baths]
    noise = [rng.normal(size=(2, nmd, b.nc)) * 1e-3 for b in baths]
    tile = np.arange(B) % 2
    st.set_state(p[tile], q[tile], t0)
    for i in range(len(baths)):
        st.set_history(i, hist[i][tile])
        st.set_noise(i, noise[i][tile])
    info = st.plan_info()
    if far_mode == "spectral":
        assert info["far_mode"] == "spectral"
    st.run(nst)
    pg, qg, t = st.get_state()
    assert t == t0 + nst
    for j in range(2):
        bs = [O.Bath("ph", b.cids, b.kernel, noise[i][j], dt, nmd) for i, b in enumerate(baths)]
        sim = O.GLE(nph, dt, nmd, bs, dyn=dyn)
        sim.p, sim.q, sim.t = p[j].copy(), q[j].copy(), t0
        for i, b in enumerate(baths):
            sim.phis[:, b.cids] = hist[i][j]
        for _ in range(nst):
            sim.step()
        for b_ in (j, j + 2, B - 2 + j):
            assert rel(qg[b_], sim.q) < 1e-9 and rel(pg[b_], sim.p) < 1e-9, (b_, rel(qg[b_], sim.q))
    st.close()


@pytest.mark.parametrize("case", ["vv_mixed", "vv_biased"])
def test_host_driver_ensemble_per_trajectory_drivers(case):
    """An ensemble whose host forces come from one driver per trajectory (called concurrently):
    every trajectory follows the device-harmonic trajectory of the same initial state and noise."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath
    from sclmd_amd.drivers import HarmonicDriver

    g = load_golden(case)
    B = 3
    dt, nmd = float(g["dt"]), int(g["nmd"])
    axyz = synthetic.axyz_chain(int(g["natom"]))
    rng = np.random.default_rng(9)
    p0 = g["p0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    q0 = g["q0"][None] * (1 + 0.1 * rng.normal(size=(B, 1)))
    out = []
    for use_driver in (True, False):
        m = MD.md(dt, nmd, float(g["T"]), axyz=axyz, dyn=None if use_driver else g["dyn_md"], ntraj=B,
                  verbose=False)
        for i in range(int(g["nbath"])):
            cids = g["b%d_cids" % i]
            if str(g["b%d_kind" % i]) == "ebath":
                b = ebath(cids, 300.0, dt, nmd, bias=float(g["b%d_bias" % i]), efric=g["b%d_efric" % i],
                          exim=g["b%d_exim" % i], zeta1=g["b%d_zeta1" % i], zeta2=g["b%d_zeta2" % i])
            else:
                b = phbath(300.0, cids, 0.2, 10, dt, nmd, ml=int(g["b%d_ml" % i]))
                b.kernel = g["b%d_kernel" % i]
                b.ml = int(g["b%d_ml" % i])
            b.noise = g["b%d_noise" % i]
            m.AddBath(b)
        c = constr_from(g)
        if c:
            m.AddConstr(c)
        if use_driver:
            m.AddPotential([HarmonicDriver(g["dyn_md"], axyz) for _ in range(B)])
        m.p, m.q, m.t = p0.copy(), q0.copy(), 0
        m.ResetHis()
        for _ in range(int(g["nsteps"])):
            m.vv(0)
        out.append((np.array(m.p), np.array(m.q)))
        m.close()
    assert rel(out[0][1], out[1][1]) < 1e-10 and rel(out[0][0], out[1][0]) < 1e-10


@pytest.mark.parametrize("ntraj,cut", [(16, 8), (40, 33)])
def test_ensemble_sharding_invariance(tmp_path, monkeypatch, ntraj, cut):
    """The multi-GPU ensemble by construction: trajectory g's initial state and device noise are keyed
    by its global index (seed + traj_offset + b), so one md of ntraj trajectories equals two shards with
    traj_offset 0 and cut -- what ranks 0 and 1 hold -- up to the summation order of the batched
    kernels (1e-9 relative on p, q and the heat currents).  Also per trajectory: the recorded p / q / bath
    force series (savep, saveq, saveall), the bath history rings, the full-DOF histories MD{j}.nc
    stores, and the per-trajectory power spectra.  (40 = 33 + 7: partial column tiles everywhere.)"""
    from sclmd_amd import _native as NV
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    monkeypatch.chdir(tmp_path)

    def run(n, offset):
        dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=12, ml=64, nmd=256, nw=80)
        m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=n, seed=77,
                  traj_offset=offset, noise_mode="device", verbose=False)
        for b in baths:
            m.AddBath(b)
        m.Savep()
        m.Saveq()
        m.SaveAll()
        m.initialise()
        m.ResetHis()
        for i in range(len(baths)):
            m.gen_noise(i, 0)
        m._in_run = True  # record the full-DOF p / q rings as md.Run does (REC_HIST)
        m.steps(300)
        st = m._st
        p, q, _ = st.get_state()
        out = {"p": p, "q": q, "cur": st.get_current().transpose(1, 0, 2),
               "ps": st.get_record(NV.REC_P), "qs": st.get_record(NV.REC_Q),
               "f0": st.get_record(NV.REC_F, 0), "f1": st.get_record(NV.REC_F, 1),
               "h0": st.get_history(0), "h1": st.get_history(1),
               "fullp": st.get_full_history(64)[0],
               "pow": st.power_spectrum([list(range(0, 6)), list(range(20, 36))]).transpose(1, 0, 2)}
        m._in_run = False
        m.close()
        return out

    whole, a, b = run(ntraj, 0), run(cut, 0), run(ntraj - cut, cut)
    for k in whole:
        assert rel(np.concatenate([a[k], b[k]]), whole[k]) < 1e-9, k
