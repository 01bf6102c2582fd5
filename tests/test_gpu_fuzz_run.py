"""Seeded random md.Run configurations against the oracle's restatement of the reference's run
(md.py:493-682 as in tests/test_oracle_golden.py::test_oracle_matches_reference_run): the drop-in
md API with the numpy-compatible noise (np.random.seed, the reference's RandomState draws in the
reference's order: initialise, then per run each bath's gnoi) against oracle.initial_state +
oracle.phnoise / enoise + the reference-shaped oracle.GLE stepping and the per-run kappa.  Each case
draws a chain junction, 1-3 baths (phonon baths with gamma spectra, ml in [1, 40], electron baths
with random exim / exip, biased or not; T = 0 sometimes, classical or without zero-point motion), constraints, nrun in [1, 3], npie and an even nmd that is
sometimes not a power of two (the device noise then takes the mixed-radix / Bluestein transforms).
1e-9 relative on the final p, q, on every run's kappa and on the power spectra (CalPowerSpec, with
random AddPowerSection groups: the running mean over the runs of functions.powerspecp of the
recorded velocities)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NCASE = int(os.environ.get("SCLMD_FUZZ_RUNS", "16"))  # a wider sweep: SCLMD_FUZZ_RUNS=120


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _case(seed):
    r = np.random.default_rng(5000 + seed)
    natom = int(r.integers(4, 20))
    nph = 3 * natom
    nmd = int(r.choice([64, 100, 128, 2 * 97, 256]))
    npie = int(r.choice([1, 2, 4]))
    while nmd % npie:
        npie //= 2
    nrun = int(r.integers(1, 4))
    baths = []
    for k in range(int(r.integers(1, 4))):
        nc = int(r.integers(2, min(nph, 24) + 1))
        a0 = int(r.integers(0, nph - nc + 1))
        cids = list(range(a0, a0 + nc)) if r.random() < 0.6 else sorted(int(x) for x in r.choice(nph, nc, replace=False))
        if r.random() < 0.4:
            n = nc
            s = 1e-3
            baths.append(dict(kind="e", cids=cids, T=float(r.choice([0.0, 300.0 * (1 + 0.05 * k)], p=[0.2, 0.8])),
                              classical=bool(r.random() < 0.2), zpmotion=bool(r.random() < 0.8),
                              efric=np.eye(n) * 1e-2 + s * (lambda m: m @ m.T / n)(r.normal(size=(n, n))),
                              exim=s * r.normal(size=(n, n)), exip=s * r.normal(size=(n, n)),
                              zeta1=s * r.normal(size=(n, n)), zeta2=s * r.normal(size=(n, n)),
                              bias=float(r.choice([0.0, 0.5])), wmax=1.0, nw=50))
        else:
            ngw = 41
            gwl = np.linspace(0.0, 0.5, ngw)
            A = r.normal(size=(nc, nc))
            A = A @ A.T / nc + np.eye(nc)
            gam = (0.658 / 100.0) * np.exp(-(gwl / 0.1) ** 2)[:, None, None] * A[None]
            baths.append(dict(kind="ph", cids=cids, T=float(r.choice([0.0, 300.0 * (1 + 0.05 * k)], p=[0.2, 0.8])),
                              classical=bool(r.random() < 0.2), zpmotion=bool(r.random() < 0.8), gam=gam, gwl=gwl, debye=0.2,
                              nw=int(r.integers(20, 80)), ml=int(r.choice([1, 2, 5, 16, 40]))))
    constr = None
    if r.random() < 0.5:
        c0 = int(r.integers(0, nph - 3))
        constr = [range(c0, c0 + int(r.integers(1, 4)))]
    groups = None
    if r.random() < 0.5:  # AddPowerSection: DOF groups of the power spectra (md.py:604-653)
        groups = [sorted(int(x) for x in r.choice(nph, int(r.integers(1, nph + 1)), replace=False))
                  for _ in range(int(r.integers(1, 4)))]
    return dict(natom=natom, nph=nph, nmd=nmd, npie=npie, nrun=nrun, baths=baths, constr=constr, seed=seed,
                np_seed=int(r.integers(0, 2 ** 31)), groups=groups)


def _describe(c):
    return "seed %d natom %d nmd %d npie %d nrun %d constr %s baths %s" % (
        c["seed"], c["natom"], c["nmd"], c["npie"], c["nrun"], c["constr"],
        [(b["kind"], len(b["cids"]), b.get("ml", 1), b.get("bias")) for b in c["baths"]])


def _oracle_run(c, dyn, dt, T):
    from oracle import sclmd_oracle as O

    np.random.seed(c["np_seed"])
    p0, q0, dyn_used = O.initial_state(dyn, T, c["constr"])
    obs = []
    for b in c["baths"]:
        if b["kind"] == "ph":
            wl = [2.0 * b["debye"] * i / b["nw"] for i in range(b["nw"])]
            k, _ = O.gmem(b["ml"], dt, wl, b["gwl"], b["gam"])
            obs.append(O.Bath("ph", b["cids"], k, None, dt, c["nmd"]))
        else:
            obs.append(O.Bath("e", b["cids"], np.array([O.symm(b["efric"])]), None, dt, c["nmd"], bias=b["bias"],
                              exim=O.antisymm(b["exim"]), zeta1=O.symm(b["zeta1"]), zeta2=O.antisymm(b["zeta2"])))
    from sclmd_amd.functions import powerspecp  # the host restatement, pinned by tests/golden/power.npz

    sim = O.GLE(c["nph"], dt, c["nmd"], obs, dyn=dyn_used, constr=c["constr"])
    sim.p, sim.q = p0, q0
    kappa, powers = [], []
    for _ in range(c["nrun"]):
        for b, ob in zip(c["baths"], obs):
            if b["kind"] == "ph":
                ob.noise = np.real(O.phnoise(b["gam"], b["gwl"], b["T"], 2.0 * b["debye"], dt, c["nmd"],
                                             b["classical"], b["zpmotion"]))
            else:
                ob.noise = np.real(O.enoise(O.symm(b["efric"]), O.antisymm(b["exim"]), O.symm(b["exip"]), b["bias"],
                                            b["T"], b["wmax"], dt, c["nmd"], b["classical"], b["zpmotion"]))
        ps = np.zeros((c["nmd"], c["nph"]))
        for _ in range(c["nmd"]):
            ps[int(sim.t) % c["nmd"]] = sim.p  # savep: md.ps[t % nmd] = p_t (md.py:374-375)
            sim.step()
        kappa.append([np.mean(ob.cur) * O.CURCOF for ob in obs])
        powers.append([powerspecp(ps, dt, c["nmd"])] + [powerspecp(ps[:, g], dt, c["nmd"]) for g in c["groups"] or []])
    # md.Run keeps the running mean over its runs (md.py:604-653)
    power = np.mean(np.array(powers), axis=0)
    return sim.p, sim.q, np.array(kappa), power


@pytest.mark.parametrize("seed", range(NCASE))
def test_random_run_vs_oracle(seed, tmp_path, monkeypatch):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath

    c = _case(seed)
    desc = _describe(c)
    monkeypatch.chdir(tmp_path)
    dt, T = synthetic.DT, 300.0
    dyn = synthetic.chain_dyn(c["natom"])
    m = MD.md(dt, c["nmd"], T, axyz=synthetic.axyz_chain(c["natom"]), dyn=dyn, nstart=0, nstop=c["nrun"],
              npie=c["npie"], verbose=False)
    for b in c["baths"]:
        if b["kind"] == "ph":
            pb = phbath(b["T"], b["cids"], debye=b["debye"], nw=b["nw"], dt=dt, nmd=c["nmd"], ml=b["ml"],
                        gamma=b["gam"], gwl=b["gwl"], classical=b["classical"], zpmotion=b["zpmotion"])
            pb.gmem()
            m.AddBath(pb)
        else:
            m.AddBath(ebath(b["cids"], b["T"], dt, c["nmd"], wmax=b["wmax"], nw=b["nw"], bias=b["bias"], efric=b["efric"],
                            exim=b["exim"], exip=b["exip"], zeta1=b["zeta1"], zeta2=b["zeta2"],
                            classical=b["classical"], zpmotion=b["zpmotion"]))
    if c["constr"] is not None:
        m.AddConstr(c["constr"])
    m.CalPowerSpec()
    if c["groups"] is not None:
        m.AddPowerSection(c["groups"])
    np.random.seed(c["np_seed"])
    m.Run()
    p, q, kap, t = np.array(m.p), np.array(m.q), np.array(m.kappa_runs), m.t
    power = np.array(m.power)
    al = None if c["groups"] is None else np.array(m.poweratomlist)
    m.close()
    wp, wq, wk, wpow = _oracle_run(c, dyn, dt, T)
    assert t == c["nrun"] * c["nmd"], desc
    assert rel(q, wq) < 1e-9 and rel(p, wp) < 1e-9, (desc, rel(q, wq), rel(p, wp))
    assert rel(kap, wk) < 1e-9, (desc, kap, wk)
    assert rel(power, wpow[0]) < 1e-9, (desc, "power")
    if al is not None:
        assert rel(al, wpow[1:]) < 1e-9, (desc, "poweratomlist")


@pytest.mark.parametrize("seed", range(4))
def test_numpy_noise_ensemble_equals_single_trajectories(seed, tmp_path, monkeypatch):
    """The numpy-compatible noise with md(seed=s): trajectory b draws from RandomState(s + b) (its
    initial state and every run's vargau draws), so a 3-trajectory md.Run equals three one-trajectory
    runs with traj_offset = b -- the reference's per-trajectory sequence, batched."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic
    from sclmd_amd.baths import ebath, phbath

    c = _case(seed)
    dt, T = synthetic.DT, 300.0
    dyn = synthetic.chain_dyn(c["natom"])

    def run(ntraj, offset):
        d = tmp_path / ("n%d_o%d" % (ntraj, offset))
        d.mkdir()
        monkeypatch.chdir(d)
        m = MD.md(dt, c["nmd"], T, axyz=synthetic.axyz_chain(c["natom"]), dyn=dyn, nstart=0, nstop=c["nrun"],
                  npie=c["npie"], ntraj=ntraj, seed=77, traj_offset=offset, noise_mode="numpy", verbose=False)
        for b in c["baths"]:
            if b["kind"] == "ph":
                pb = phbath(b["T"], b["cids"], debye=b["debye"], nw=b["nw"], dt=dt, nmd=c["nmd"], ml=b["ml"],
                            gamma=b["gam"], gwl=b["gwl"], classical=b["classical"], zpmotion=b["zpmotion"])
                pb.gmem()
                m.AddBath(pb)
            else:
                m.AddBath(ebath(b["cids"], b["T"], dt, c["nmd"], wmax=b["wmax"], nw=b["nw"], bias=b["bias"],
                                efric=b["efric"], exim=b["exim"], exip=b["exip"], zeta1=b["zeta1"], zeta2=b["zeta2"],
                                classical=b["classical"], zpmotion=b["zpmotion"]))
        if c["constr"] is not None:
            m.AddConstr(c["constr"])
        m.Run()
        p, q = np.array(m.p).reshape(ntraj, -1), np.array(m.q).reshape(ntraj, -1)
        m.close()
        return p, q

    p, q = run(3, 0)
    for b in range(3):
        pb, qb = run(1, b)
        assert rel(qb[0], q[b]) < 1e-9 and rel(pb[0], p[b]) < 1e-9, (_describe(c), b)
