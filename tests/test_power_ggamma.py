"""Power spectra (functions.powerspecp, md.GetPower) and the self-energy bath (phbath.ggamma) against
fixtures made by the real reference (tests/golden/make_golden.py power / ggamma).

CPU: the host restatements against the fixtures.  GPU: md with CalPowerSpec + AddPowerSection +
CalAveStruct + SaveAll stepped on the device; the device-recorded ps / qs / fhis, the device power
spectra (gle_power_spectrum), the average structure and the checkpoint histories against the
reference's run (1e-10 relative); the ggamma-built bath stepped on the device against the oracle."""
import os

import numpy as np
import pytest

from conftest import constr_from, load_golden, oracle_from_golden


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_powerspecp_matches_reference_getpower():
    from sclmd_amd.functions import powerspecp

    g = load_golden("power")
    dt, nmd = float(g["dt"]), int(g["nmd"])
    assert rel(powerspecp(g["ps"], dt, nmd), g["power"]) < 1e-12
    for layer, dofs in enumerate(g["atomlist"]):
        assert rel(powerspecp(g["ps"][:, dofs], dt, nmd), g["poweratomlist"][layer]) < 1e-12


def test_oracle_reproduces_power_run_fhis_and_ps():
    g = load_golden("power")
    sim = oracle_from_golden(g)
    nmd = int(g["nmd"])
    ps = np.zeros((nmd, sim.nph))
    for _ in range(int(g["nsteps"])):
        ps[sim.t % nmd] = sim.p
        sim.step()
    assert rel(ps, g["ps"]) < 1e-12
    assert rel(sim.fhis[0], g["fhis0"]) < 1e-11 and rel(sim.fhis[1], g["fhis1"]) < 1e-11


def test_ggamma_and_gmem_match_reference():
    from sclmd_amd.baths import phbath

    g = load_golden("ggamma")
    b = phbath(300.0, g["cids"], debye=float(g["debye"]), nw=int(g["nw"]), dt=float(g["dt"]), nmd=int(g["nmd"]),
               ml=int(g["ml"]), sig=g["sig"], gwl=g["gwl"])
    assert rel(b.gamma, g["gamma"]) < 1e-14
    b.gmem()
    assert rel(b.kernel, g["kernel"]) < 1e-12


def _power_md(g, ntraj=1):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath

    dt, nmd = float(g["dt"]), int(g["nmd"])
    m = MD.md(dt, nmd, float(g["T"]), axyz=synthetic.axyz_chain(int(g["natom"])), dyn=g["dyn_md"], ntraj=ntraj,
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
    m.AddConstr(constr_from(g))
    m.CalPowerSpec()
    m.AddPowerSection([list(a) for a in g["atomlist"]])
    m.CalAveStruct()
    m.SaveAll()
    p0, q0 = g["p0"], g["q0"]
    if ntraj > 1:
        p0, q0 = np.tile(p0, (ntraj, 1)), np.tile(q0, (ntraj, 1))
    m.p, m.q, m.t = p0, q0, 0
    m.ResetHis()
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("ntraj", [1, 3])
def test_device_recordings_and_power_match_reference(ntraj, tmp_path, monkeypatch):
    from sclmd_amd import _native as N

    monkeypatch.chdir(tmp_path)
    g = load_golden("power")
    m = _power_md(g, ntraj)
    m.steps(int(g["nsteps"]))
    one = (lambda a: a) if ntraj == 1 else (lambda a: a[ntraj - 1])
    assert rel(one(m.q), g["q_end"]) < 1e-10
    assert rel(one(m.ps), g["ps"]) < 1e-10 and rel(one(m.qs), g["qs"]) < 1e-10
    assert rel(one(m.fhis_of(0)), g["fhis0"]) < 1e-10 and rel(one(m.fhis_of(1)), g["fhis1"]) < 1e-10
    power, al = m.power_spectra()  # ensemble mean of identical trajectories == the reference's
    assert rel(power, g["power"]) < 1e-10
    assert rel(np.array(al), g["poweratomlist"]) < 1e-10
    # the device spectra are functions.powerspecp of the device-recorded series, per trajectory
    spec = m._st.power_spectrum([np.arange(m.nph)])
    ps = m._st.get_record(N.REC_P)
    for b in range(ntraj):
        f = np.abs(np.fft.fft(ps[b], axis=0)) ** 2
        assert rel(spec[0, b], f.sum(axis=1)) < 1e-12
    m._avestructure(0)
    rows = [l.split() for l in open("avestructure.%s.run0.dat" % str(m.T)).read().splitlines()[2:]]
    ave = np.array([[float(x) for x in r[1:4]] for r in rows]).ravel()
    assert rel(ave, g["avestructure"]) < 1e-10
    m.close()


@pytest.mark.gpu
def test_run_power_files_and_checkpoint_histories(tmp_path, monkeypatch):
    """md.Run with savep + AddPowerSection + SaveAll: power.*.dat and poweratomlist.*.dat files of
    the reference's format, MD{j}.nc with fhis{i}, ps, qs, power, poweratomlist and full-DOF
    phis / qhis that equal the oracle's histories (the reference's md.phis / md.qhis)."""
    from sclmd_amd.checkpoint import ReadNetCDFVar

    monkeypatch.chdir(tmp_path)
    g = load_golden("power")
    m = _power_md(g)
    m.nstart, m.nstop = 0, 1
    m.initialise = lambda: None  # keep the fixture's initial state (Run would re-draw it)
    m.gen_noise = lambda i, run=0: None  # and its injected noise (Run would draw new noise)
    m.Run()
    sim = oracle_from_golden(g)
    for _ in range(int(g["nmd"])):
        sim.step()
    assert rel(ReadNetCDFVar("MD0.nc", "q"), sim.q) < 1e-10
    assert rel(ReadNetCDFVar("MD0.nc", "phis"), sim.phis) < 1e-10
    assert rel(ReadNetCDFVar("MD0.nc", "qhis"), sim.qhis) < 1e-10
    assert rel(ReadNetCDFVar("MD0.nc", "fhis1"), g["fhis1"]) < 1e-10
    assert rel(np.transpose(ReadNetCDFVar("MD0.nc", "poweratomlist"), (1, 0, 2)), g["poweratomlist"]) < 1e-10
    # the file stops at 1.5 max(hw) (md.py:631-636): here after the first row; the whole spectrum is m.power
    pw = np.loadtxt("power.%s.run0.dat" % str(m.T), ndmin=2)
    n = len(pw)
    assert 0 < n <= int(g["nmd"]) and np.allclose(pw, np.round(g["power"][:n], 6), atol=2e-6)
    assert rel(m.power, g["power"]) < 1e-10
    for layer in range(len(g["atomlist"])):
        assert os.path.isfile("poweratomlist.%d.%s.run0.dat" % (layer, str(m.T)))
    m.close()


@pytest.mark.gpu
def test_ggamma_bath_device_kernel_and_step():
    """phbath(sig=...) -> ggamma -> gmem(on_device=True) -> device steps, against the reference's
    kernel (golden ggamma) and the oracle stepped with it."""
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd.baths import phbath
    from sclmd_amd import synthetic

    g = load_golden("ggamma")
    dt, nmd, ml = float(g["dt"]), int(g["nmd"]), int(g["ml"])
    b = phbath(300.0, g["cids"], debye=float(g["debye"]), nw=int(g["nw"]), dt=dt, nmd=nmd, ml=ml, sig=g["sig"],
               gwl=g["gwl"])
    b.gmem(on_device=True)
    natom = 3
    nph = 3 * natom
    st = N.Stepper(nph, 2, nmd, dt, 0)
    W, gm = b.gmem_recipe
    st.add_bath_gmem(b.cids, W, gm)
    assert rel(st.get_kernel(0), g["kernel"]) < 1e-12
    dyn = synthetic.chain_dyn(natom)
    st.set_dyn(dyn)
    rng = np.random.default_rng(3)
    p = rng.normal(size=(2, nph)) * 1e-3
    q = rng.normal(size=(2, nph)) * 1e-3
    noise = rng.normal(size=(2, nmd, len(g["cids"]))) * 1e-3
    st.set_state(p, q, 0)
    st.set_history(0, None)
    st.set_noise(0, noise)
    st.run(50)
    pg, qg, _ = st.get_state()
    st.close()
    for j in range(2):
        sim = O.GLE(nph, dt, nmd, [O.Bath("ph", g["cids"], g["kernel"], noise[j], dt, nmd)], dyn=dyn)
        sim.p, sim.q = p[j].copy(), q[j].copy()
        for _ in range(50):
            sim.step()
        assert rel(qg[j], sim.q) < 1e-10 and rel(pg[j], sim.p) < 1e-10
