#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REAL reference (sclmd).

This script is the only thing in the repository that imports /root/reference.  It runs ONCE in
the build container (where the reference is mounted read-only) and writes small .npz fixtures;
nothing at test time, in smoke() or in bench.py reads /root/reference.  The reference has no test
suite of its own, so these fixtures are what pins the oracle.

    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/make_golden.py

The reference's md.py imports netCDF4 (absent here) only for dump/ReadNetCDFVar (md.py:684-764),
which this script never reaches, so a stub module is injected.

Fixtures (each < 1 MB):
  scalars.npz     bose / equ / flinterp tables over their edge cases   (functions.py:80-143, noise.py:249-270)
  gamt.npz        memory kernels, eta_ad = 0 and != 0                   (baths.py:19-52, 412-445)
  noise.npz       phnoise / enoise realisations + per-omega vargau draws (noise.py:50-100, 149-206, 273-305)
  vv_*.npz        md.vv trajectories with injected noise/kernels        (md.py:367-474, baths.py:224-255, 448-458)
  run_seeded.npz  initialise + per-run gnoi + vv + kappa, seeded numpy RNG (md.py:294-338, 493-664)
  tools.npz       calHF / calTC outputs on synthetic kappa files        (tools.py:132-215)
  power.npz       savep / saveq vv run: ps, qs, fhis, GetPower's power and per-section spectra,
                  average structure                                     (md.py:351-360, 374-398, 604-675,
                                                                         functions.py:221-236)
  ggamma.npz      phbath built from a self-energy sig: gamma = -Im sig / w, gmem kernel
                                                                        (baths.py:294-340, 375-395, 412-445)
  helpers.npz     public helpers: coth / xcoth / fermi / dagger / mm / powerspecq, phnoisew /
                  nonequm / nonequp / vargau, exlist, ebath.GetSig    (functions.py:59-218, noise.py:28-305,
                                                                         baths.py:12-14, 194-208)

    python3 tests/golden/make_golden.py [name ...]     (default: all)
"""
import contextlib
import io
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.modules["netCDF4"] = types.SimpleNamespace(Dataset=None)

import sclmd.baths as RB  # noqa: E402
import sclmd.functions as RF  # noqa: E402
import sclmd.md as RMD  # noqa: E402
import sclmd.noise as RN  # noqa: E402
import sclmd.tools as RT  # noqa: E402
import sclmd.units as RU  # noqa: E402


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


def chain_dyn(natom, k=0.01, onsite=1e-3, seed=None):
    """1-D chain: nearest-neighbour spring k on each Cartesian axis plus an on-site term."""
    n = 3 * natom
    d = np.zeros((n, n))
    for a in range(natom):
        for x in range(3):
            i = 3 * a + x
            d[i, i] += onsite
            if a + 1 < natom:
                j = 3 * (a + 1) + x
                d[i, i] += k
                d[j, j] += k
                d[i, j] -= k
                d[j, i] -= k
    if seed is not None:  # small symmetric perturbation so the matrix is not block-trivial
        r = np.random.default_rng(seed).normal(size=(n, n)) * 1e-4
        d += r + r.T
    return d


def axyz_for(natom):
    return [["C", 1.42 * a, 0.0, 0.0] for a in range(natom)]


def spd(n, rng, scale):
    r = rng.normal(size=(n, n))
    return scale * (r @ r.T / n + np.eye(n))


def anti(n, rng, scale):
    r = rng.normal(size=(n, n)) * scale
    return r - r.T


def sym(n, rng, scale):
    r = rng.normal(size=(n, n)) * scale
    return r + r.T


def gamma_table(nc, rng, ngw=21, wmax=0.5, g0=0.658 / 100, wc=0.1):
    gwl = np.linspace(0.0, wmax, ngw)
    A = spd(nc, rng, 1.0)
    gam = np.array([g0 * A * np.exp(-(w / wc) ** 2) for w in gwl])
    return gwl, gam


# ----------------------------------------------------------------------------- F1 scalars
def make_scalars():
    kb = RU.kb
    ws = np.array([0.0, 1e-4, 0.01, 0.05, 0.1, 0.3, 0.99, 1.0, 1.5, -0.02, -1e-3])
    Ts = np.array([0.0, 4.2, 300.0, 1000.0])
    bose = np.array([[RF.bose(w, T) for w in ws] for T in Ts])
    equ = []
    for classical in (False, True):
        for zp in (True, False):
            for cut in (0.2, 1.0):
                equ.append([[RN.equ(w, cut, T, classical, zp) for w in ws] for T in Ts])
    equ = np.array(equ)
    rng = np.random.default_rng(1)
    xs = np.linspace(0.0, 0.5, 11)
    ys = rng.normal(size=(11, 3, 3))
    xq = np.array([-0.1, 0.0, 0.01, 0.024, 0.025, 0.026, 0.13, 0.25, 0.31, 0.476, 0.49, 0.5, 0.7])
    fl = np.array([RF.flinterp(x, xs, ys) for x in xq])
    np.savez_compressed(os.path.join(HERE, "scalars.npz"), ws=ws, Ts=Ts, bose=bose, equ=equ,
                        equ_order=np.array(["classical,zp,cut"]), xs=xs, ys=ys, xq=xq, flinterp=fl,
                        kb=kb)


# ----------------------------------------------------------------------------- F2 gamt
def make_gamt():
    rng = np.random.default_rng(2)
    nc, ml, nw = 4, 16, 40
    dt = 0.25 / 0.658
    gwl, gam = gamma_table(nc, rng)
    out = {"gwl": gwl, "gam": gam, "dt": dt, "ml": ml, "nw": nw}
    for tag, eta in (("eta0", 0.0), ("eta1", 0.02)):
        with quiet():
            b = RB.phbath(300.0, list(range(nc)), debye=0.2, nw=nw, dt=dt, nmd=64, ml=ml,
                          mcof=2.0, gamma=gam.copy(), gwl=gwl, eta_ad=eta)
            b.gmem()
        out["kernel_" + tag] = b.kernel
        out["gamma_after_" + tag] = b.gamma
    # a direct gamt call on an uneven time list
    tl = [0.0, 0.3, 1.7, 5.0]
    wl = [0.4 * i / 25 for i in range(25)]
    with quiet():
        out["gamt_direct"] = RB.gamt(tl, wl, gwl, gam)
    out["gamt_tl"] = np.array(tl)
    out["gamt_wl"] = np.array(wl)
    # Debye/local bath (baths.py:336-340, 419-422)
    with quiet():
        b = RB.phbath(300.0, list(range(nc)), debye=0.15, nw=nw, dt=dt, nmd=64, ml=8)
        b.gmem()
    out["kernel_debye"] = b.kernel
    out["ml_debye"] = b.ml
    np.savez_compressed(os.path.join(HERE, "gamt.npz"), **out)


# ----------------------------------------------------------------------------- F3 noise
class Recorder:
    def __init__(self):
        self.calls = []
        self.orig = RN.vargau

    def __call__(self, ev, evec, cof=1.0):
        st = np.random.get_state()
        r = self.orig(ev, evec, cof)
        self.calls.append((np.array(ev), np.array(r)))
        return r


def make_noise():
    rng = np.random.default_rng(3)
    nc, nmd = 5, 64
    dt = 0.25 / 0.658
    gwl, gam = gamma_table(nc, rng)
    out = {"nc": nc, "nmd": nmd, "dt": dt, "gwl": gwl, "gam": gam}
    rec = Recorder()
    RN.vargau = rec
    try:
        for tag, T, phcut, classical, zp in (("ph_q", 300.0, 0.4, False, True),
                                             ("ph_c", 300.0, 0.4, True, True),
                                             ("ph_nozp", 100.0, 0.3, False, False)):
            np.random.seed(11)
            rec.calls = []
            with quiet():
                nz = RN.phnoise(gam, gwl, T, phcut, dt, nmd, classical, zp)
            out["noise_" + tag] = nz
            out["amp_" + tag] = np.array([c[1] for c in rec.calls])
            out["eval_" + tag] = np.array([c[0] for c in rec.calls])
            out["params_" + tag] = np.array([T, phcut, float(classical), float(zp)])
        efric = spd(nc, rng, 0.658 / 100)
        exim = anti(nc, rng, 1e-3)
        exip = sym(nc, rng, 1e-3) + 0.5 * efric
        out["efric"], out["exim"], out["exip"] = efric, exim, exip
        for tag, bias, T, ecut, classical, zp in (("e_eq", 0.0, 300.0, 1.0, False, True),
                                                  ("e_bias", 0.3, 300.0, 1.0, False, True),
                                                  ("e_cold", 0.2, 0.0, 0.5, False, True)):
            np.random.seed(12)
            rec.calls = []
            with quiet():
                nz = RN.enoise(symf(efric), antif(exim), symf(exip), bias, T, ecut, dt, nmd,
                               classical, zp)
            out["noise_" + tag] = nz
            out["amp_" + tag] = np.array([c[1] for c in rec.calls])
            out["eval_" + tag] = np.array([c[0] for c in rec.calls])
            out["params_" + tag] = np.array([bias, T, ecut, float(classical), float(zp)])
    finally:
        RN.vargau = rec.orig
    np.savez_compressed(os.path.join(HERE, "noise.npz"), **out)


def symf(a):
    return RF.symmetrize(a)


def antif(a):
    return RF.antisymmetrize(a)


# ----------------------------------------------------------------------------- F4 vv trajectories
def build_md(natom, dt, nmd, T, dyn, baths, constr, seed_init, noranvel=False):
    with quiet():
        m = RMD.md(dt, nmd, T, axyz=axyz_for(natom), dyn=dyn)
        for b in baths:
            m.AddBath(b)
        if constr is not None:
            m.AddConstr(constr)
        if noranvel:
            m.noranvel()
        np.random.seed(seed_init)
        m.initialise()
        m.ResetHis()
    return m


def run_vv(m, nsteps):
    qs, ps, curs, etots = [], [], [], []
    for _ in range(nsteps):
        t = int(m.t)
        m.vv(0)
        qs.append(np.array(m.q))
        ps.append(np.array(m.p))
        curs.append([b.cur[t % m.nmd] for b in m.baths])
        etots.append(m.etot[t % m.nmd])
    return np.array(qs), np.array(ps), np.array(curs), np.array(etots)


def bath_record(prefix, b, out):
    out[prefix + "_cids"] = np.array(b.cids)
    out[prefix + "_noise"] = np.array(b.noise)
    out[prefix + "_kernel"] = np.array(b.kernel)
    out[prefix + "_ml"] = b.ml


def make_vv_cases():
    dt = 0.25 / 0.658
    T = 300.0
    cases = {}
    # ---- mixed: ebath (eq) + phbath(ml=16) + constraints, harmonic chain
    rng = np.random.default_rng(4)
    natom, nmd = 5, 32
    nph = 3 * natom
    dyn = chain_dyn(natom, seed=5)
    ecids = [0, 1, 2, 3]
    pcids = [10, 11, 12, 13, 14]
    with quiet():
        eb = RB.ebath(ecids, T * 1.05, dt, nmd, wmax=1.0, nw=100, bias=0.0,
                      efric=spd(len(ecids), rng, 0.658 / 100))
        gwl, gam = gamma_table(len(pcids), rng)
        pb = RB.phbath(T * 0.95, pcids, debye=0.2, nw=60, dt=dt, nmd=nmd, ml=16, gamma=gam, gwl=gwl)
        pb.gmem()
    eb.noise = rng.normal(size=(nmd, len(ecids))) * 1e-3
    pb.noise = rng.normal(size=(nmd, len(pcids))) * 1e-3
    cases["vv_mixed"] = (natom, nmd, dyn, [eb, pb], [range(5, 7), range(8, 9)], 70, False)

    # ---- biased ebath with exim, zeta1, zeta2 all nonzero + local phbath (ml=1, no dt factor)
    rng = np.random.default_rng(6)
    natom, nmd = 4, 24
    dyn = chain_dyn(natom, seed=7)
    ecids = [3, 4, 5, 6, 7, 8]
    pcids = [0, 1, 2]
    ne = len(ecids)
    with quiet():
        eb = RB.ebath(ecids, T, dt, nmd, wmax=1.0, nw=100, bias=0.5,
                      efric=spd(ne, rng, 0.658 / 100), exim=anti(ne, rng, 2e-3),
                      exip=sym(ne, rng, 1e-3), zeta1=sym(ne, rng, 2e-3), zeta2=anti(ne, rng, 2e-3))
        pb = RB.phbath(T * 1.1, pcids, debye=0.1, nw=60, dt=dt, nmd=nmd, ml=4)
        pb.gmem()
    eb.noise = rng.normal(size=(nmd, ne)) * 1e-3
    pb.noise = rng.normal(size=(nmd, len(pcids))) * 1e-3
    cases["vv_biased"] = (natom, nmd, dyn, [eb, pb], [range(11, 12)], 60, False)

    # ---- biased ebath with zeta = None: bias only enters the noise (baths.py:233 quirk)
    rng = np.random.default_rng(8)
    natom, nmd = 3, 16
    dyn = chain_dyn(natom, seed=9)
    ecids = [0, 1, 2, 3, 4, 5, 6, 7, 8]
    with quiet():
        eb = RB.ebath(ecids, T, dt, nmd, wmax=1.0, nw=100, bias=0.7,
                      efric=spd(9, rng, 0.658 / 100), exim=anti(9, rng, 2e-3), exip=sym(9, rng, 1e-3))
    eb.noise = rng.normal(size=(nmd, 9)) * 1e-3
    cases["vv_zeta0"] = (natom, nmd, dyn, [eb], None, 40, False)

    # ---- two phonon baths with long memory (ml=24 > nmd-steps crossing), overlapping cids,
    #      noranvel start (p=q=0: exercises sameq cache hits at t=0)
    rng = np.random.default_rng(10)
    natom, nmd = 4, 20
    dyn = chain_dyn(natom, seed=11)
    c1 = [0, 1, 2, 3, 4, 5]
    c2 = [4, 5, 6, 7, 8, 9, 10, 11]
    with quiet():
        g1, gm1 = gamma_table(len(c1), rng)
        b1 = RB.phbath(T * 1.05, c1, debye=0.2, nw=50, dt=dt, nmd=nmd, ml=24, gamma=gm1, gwl=g1)
        b1.gmem()
        g2, gm2 = gamma_table(len(c2), rng)
        b2 = RB.phbath(T * 0.95, c2, debye=0.2, nw=50, dt=dt, nmd=nmd, ml=9, gamma=gm2, gwl=g2)
        b2.gmem()
    b1.noise = rng.normal(size=(nmd, len(c1))) * 1e-3
    b2.noise = rng.normal(size=(nmd, len(c2))) * 1e-3
    cases["vv_twoph"] = (natom, nmd, dyn, [b1, b2], [range(0, 1)], 50, True)

    for name, (natom, nmd, dyn, baths, constr, nsteps, norv) in cases.items():
        m = build_md(natom, dt, nmd, T, dyn, baths, constr, seed_init=21, noranvel=norv)
        out = {"natom": natom, "nmd": nmd, "dt": dt, "T": T, "dyn": dyn, "nsteps": nsteps,
               "noranvel": norv, "p0": np.array(m.p), "q0": np.array(m.q), "nbath": len(baths),
               "dyn_md": np.array(m.dyn)}
        out["constr"] = (np.concatenate([np.array(list(r)) for r in constr]) if constr is not None
                         else np.zeros(0, dtype=int))
        out["constr_ranges"] = (np.array([[r.start, r.stop] for r in constr]) if constr is not None
                                else np.zeros((0, 2), dtype=int))
        for i, b in enumerate(baths):
            bath_record("b%d" % i, b, out)
            out["b%d_kind" % i] = "ebath" if isinstance(b, RB.ebath) else "phbath"
            if isinstance(b, RB.ebath):
                out["b%d_bias" % i] = b.bias
                for nm in ("efric", "exim", "exip", "zeta1", "zeta2"):
                    out["b%d_%s" % (i, nm)] = np.array(getattr(b, nm))
        q, p, cur, et = run_vv(m, nsteps)
        out.update(q=q, p=p, cur=cur, etot=et)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


# ----------------------------------------------------------------------------- F5 seeded run
def make_run_seeded():
    """md.Run without the NetCDF files: initialise, then per run j gnoi() (in AddBath order) and
    nmd vv steps, then kappa_j = mean(cur)*curcof (md.py:500-506, 569-570, 582-585, 657-664)."""
    dt = 0.25 / 0.658
    T = 300.0
    delta = 0.1
    natom, nmd, nrun = 4, 16, 3
    dyn = chain_dyn(natom, seed=13)
    rng = np.random.default_rng(14)
    c1 = [0, 1, 2]
    c2 = [9, 10, 11]
    with quiet():
        g1, gm1 = gamma_table(3, rng)
        b1 = RB.phbath(T * (1 + delta / 2), c1, debye=0.2, nw=50, dt=dt, nmd=nmd, ml=6,
                       gamma=gm1, gwl=g1)
        b1.gmem()
        b2 = RB.ebath(c2, T * (1 - delta / 2), dt, nmd, wmax=1.0, nw=50, bias=0.0,
                      efric=spd(3, rng, 0.658 / 100))
        m = RMD.md(dt, nmd, T, axyz=axyz_for(natom), dyn=dyn, nstart=0, nstop=nrun)
        m.AddBath(b1)
        m.AddBath(b2)
        m.AddConstr([range(6, 8)])
        np.random.seed(2024)
        m.initialise()
        m.ResetHis()
        p0, q0 = np.array(m.p), np.array(m.q)
        kappa = np.zeros((nrun, 2))
        curs = np.zeros((nrun, 2, nmd))
        noises = []
        for j in range(nrun):
            for b in m.baths:
                b.gnoi()
            noises.append([np.array(b.noise) for b in m.baths])
            for _ in range(nmd):
                m.vv(j)
            for i, b in enumerate(m.baths):
                kappa[j, i] = np.mean(b.cur) * RU.curcof
                curs[j, i] = b.cur
    out = dict(natom=natom, nmd=nmd, nrun=nrun, dt=dt, T=T, delta=delta, dyn=dyn, seed=2024,
               c1=np.array(c1), c2=np.array(c2), gwl1=g1, gam1=gm1, debye1=0.2, nw1=50, ml1=6,
               T1=T * (1 + delta / 2), T2=T * (1 - delta / 2), efric2=np.array(b2.efric),
               kernel1=np.array(b1.kernel), constr=np.array([6, 7]), p0=p0, q0=q0,
               dyn_md=np.array(m.dyn), kappa=kappa, cur=curs, p_end=np.array(m.p), q_end=np.array(m.q), t_end=m.t,
               noise1=np.array([n[0] for n in noises]), noise2=np.array([n[1] for n in noises]))
    np.savez_compressed(os.path.join(HERE, "run_seeded.npz"), **out)


# ----------------------------------------------------------------------------- tools
def make_tools():
    rng = np.random.default_rng(15)
    T = 300
    nrun = 6
    kb = rng.normal(size=(3, nrun)) * 10.0
    out = {"kb": kb, "T": T, "nrun": nrun}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            for i in range(3):
                for j in range(nrun):
                    with open("kappa.%s.bath%d.run%d.dat" % (str(float(T)), i, j), "w") as f:
                        f.write("%i %f    %f \n" % (j, float(T), kb[i, j]))
            # md.py writes str(self.T) into the name; calHF/calTC read str(int(T)) -> use T int.
            for i in range(3):
                for j in range(nrun):
                    os.rename("kappa.%s.bath%d.run%d.dat" % (str(float(T)), i, j),
                              "kappa.%d.bath%d.run%d.dat" % (T, i, j))
            with quiet():
                RT.calHF(dlist=2, bathnum=2)
                RT.calTC(delta=0.1, dlist=2, bathnum=2, L=10.0, A=4.0)
            out["heatflux_2"] = np.loadtxt("heatflux.%d.dat" % T)
            out["tc_2"] = np.loadtxt("thermalconductance.%d.dat" % T)
            out["tcy_2"] = np.loadtxt("thermalconductivity.%d.dat" % T)
            out["hfb_2"] = np.loadtxt("heatflux-between-baths.%d.dat" % T)
            with quiet():
                RT.calHF(dlist=1, bathnum=3)
                RT.calTC(delta=0.1, dlist=1, bathnum=3)
            out["heatflux_3"] = np.loadtxt("heatflux.%d.dat" % T)
            out["tc_3"] = np.loadtxt("thermalconductance.%d.dat" % T)
            out["hfb_3"] = np.loadtxt("heatflux-between-baths.%d.dat" % T)
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "tools.npz"), **out)


# ----------------------------------------------------------------------------- power spectra
def make_power():
    """A vv run with CalPowerSpec + AddPowerSection + CalAveStruct (md.py:185-197): the recorded ps /
    qs / fhis, GetPower's power and poweratomlist (md.py:351-360), the average structure
    (md.py:665-675).  Same system shape as vv_mixed; nsteps = nmd so every ps row is written."""
    dt = 0.25 / 0.658
    T = 300.0
    rng = np.random.default_rng(41)
    natom, nmd = 5, 32
    dyn = chain_dyn(natom, seed=42)
    ecids = [0, 1, 2, 3]
    pcids = [10, 11, 12, 13, 14]
    with quiet():
        eb = RB.ebath(ecids, T * 1.05, dt, nmd, wmax=1.0, nw=100, bias=0.0,
                      efric=spd(len(ecids), rng, 0.658 / 100))
        gwl, gam = gamma_table(len(pcids), rng)
        pb = RB.phbath(T * 0.95, pcids, debye=0.2, nw=60, dt=dt, nmd=nmd, ml=16, gamma=gam, gwl=gwl)
        pb.gmem()
    eb.noise = rng.normal(size=(nmd, len(ecids))) * 1e-3
    pb.noise = rng.normal(size=(nmd, len(pcids))) * 1e-3
    atomlist = [[0, 1, 2, 3, 4, 5], [9, 10, 11, 12, 13, 14]]
    m = build_md(natom, dt, nmd, T, dyn, [eb, pb], [range(5, 7)], seed_init=43)
    with quiet():
        m.CalPowerSpec()
        m.AddPowerSection(atomlist)
        m.CalAveStruct()
        m.ResetSavepq()
        p0, q0 = np.array(m.p), np.array(m.q)
        run_vv(m, nmd)
        m.GetPower()
    ave = m.conv * (m.qs.mean(axis=0)) + m.xyz
    out = {"natom": natom, "nmd": nmd, "dt": dt, "T": T, "dyn": dyn, "nsteps": nmd, "noranvel": False,
           "p0": p0, "q0": q0, "nbath": 2, "dyn_md": np.array(m.dyn),
           "constr": np.array([5, 6]), "constr_ranges": np.array([[5, 7]]),
           "atomlist": np.array(atomlist), "ps": np.array(m.ps), "qs": np.array(m.qs),
           "power": np.array(m.power), "poweratomlist": np.array(m.poweratomlist),
           "fhis0": np.array(m.fhis[0]), "fhis1": np.array(m.fhis[1]), "avestructure": ave,
           "hw": np.array(m.hw), "p_end": np.array(m.p), "q_end": np.array(m.q)}
    for i, b in enumerate([eb, pb]):
        bath_record("b%d" % i, b, out)
        out["b%d_kind" % i] = "ebath" if isinstance(b, RB.ebath) else "phbath"
        if isinstance(b, RB.ebath):
            out["b%d_bias" % i] = b.bias
            for nm in ("efric", "exim", "exip", "zeta1", "zeta2"):
                out["b%d_%s" % (i, nm)] = np.array(getattr(b, nm))
    np.savez_compressed(os.path.join(HERE, "power.npz"), **out)


# ----------------------------------------------------------------------------- ggamma
def make_ggamma():
    """phbath from a self-energy: gamma(w) = -Im sig(w) / w, the w = 0 row from the next point
    (baths.py:375-395), then gmem (baths.py:412-445)."""
    dt = 0.25 / 0.658
    rng = np.random.default_rng(51)
    nc, ngw, ml, nmd = 4, 21, 24, 32
    gwl = np.linspace(0.0, 0.4, ngw)
    base = spd(nc, rng, 0.658 / 100)
    sig = np.array([(rng.normal(size=(nc, nc)) * 1e-4 + 0.0j) - 1j * w * (base * np.exp(-(w / 0.15) ** 2))
                    for w in gwl])
    with quiet():
        b = RB.phbath(300.0, [3, 4, 5, 6], debye=0.2, nw=50, dt=dt, nmd=nmd, ml=ml, sig=sig, gwl=gwl)
        gamma = np.array(b.gamma)
        b.gmem()
    np.savez_compressed(os.path.join(HERE, "ggamma.npz"), sig=sig, gwl=gwl, nc=nc, ml=ml, nmd=nmd, dt=dt,
                        debye=0.2, nw=50, cids=np.array([3, 4, 5, 6]), gamma=gamma, kernel=np.array(b.kernel))


def make_helpers():
    """The reference's small public helpers a user script may import: functions.coth / xcoth /
    fermi / dagger / mm / powerspecq, noise.phnoisew / nonequm / nonequp / vargau, baths.exlist,
    ebath.GetSig.  (np.complex, removed in numpy 2, is aliased for GetSig.)"""
    rng = np.random.default_rng(21)
    had = hasattr(np, "complex")
    if not had:
        np.complex = complex
    try:
        out = {}
        xs = np.array([-3.0, -0.5, 1e-6, 0.25, 2.0, 30.0])
        out["coth_x"] = xs
        out["coth"] = np.array([RF.coth(x) for x in xs])
        xs0 = np.concatenate([[0.0], xs])
        out["xcoth_x"] = xs0
        out["xcoth"] = np.array([RF.xcoth(x) for x in xs0])
        fe = [(e, mu, T) for e in (-0.2, 0.0, 0.1) for mu in (0.0, 0.1) for T in (0.0, 300.0)]
        out["fermi_args"] = np.array(fe)
        out["fermi"] = np.array([RF.fermi(e, mu, T) for e, mu, T in fe])
        a = rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4))
        out["dagger_in"], out["dagger"] = a, RF.dagger(a)
        m1, m2, m3 = rng.normal(size=(3, 4)), rng.normal(size=(4, 5)), rng.normal(size=(5, 2))
        out["mm_1"], out["mm_2"], out["mm_3"], out["mm"] = m1, m2, m3, RF.mm(m1, m2, m3)
        nmd, dt = 64, 0.25 / 0.658
        qs = rng.normal(size=(nmd, 6))
        out["qs"], out["powerspecq"], out["pq_dt"] = qs, RF.powerspecq(qs, dt, nmd), dt
        nc = 4
        gwl, gam = gamma_table(nc, rng)
        wl = np.linspace(0.0, 0.6, 13)
        gamw = np.array([RF.flinterp(w, gwl, gam) for w in wl])
        out["phw_wl"], out["phw_gam"] = wl, gamw
        for tag, T, cut, cl, zp in (("q", 300.0, 0.4, False, True), ("c", 300.0, 0.4, True, True),
                                    ("nozp", 50.0, 0.3, False, False)):
            out["phnoisew_" + tag] = RN.phnoisew(gamw, wl, T, cut, cl, zp)
            out["phw_params_" + tag] = np.array([T, cut, float(cl), float(zp)])
        efric = spd(nc, rng, 0.658 / 100)
        exim, exip = anti(nc, rng, 1e-3), sym(nc, rng, 1e-3)
        out["ew_efric"], out["ew_exim"], out["ew_exip"] = efric, exim, exip
        # (the reference's enoisew raises: its local `np = chkShape(exip)` shadows numpy before
        # np.zeros, noise.py:122-128; enoise's own spectral matrix pins the formula instead)
        neq = [(w, b, T, cl) for w in (0.0, 0.05, 0.3) for b in (0.0, 0.1, -0.2) for T in (0.0, 300.0)
               for cl in (False, True) if not (cl and T == 0.0)]
        out["neq_args"] = np.array(neq, dtype=float)
        with quiet():
            out["nonequm"] = np.array([RN.nonequm(w, b, T, cl) for w, b, T, cl in neq])
            out["nonequp"] = np.array([RN.nonequp(w, b, T, cl) for w, b, T, cl in neq])
        ev = np.array([-1e-3, 0.0, 2.0, 0.5])
        evec = np.linalg.qr(rng.normal(size=(4, 4)))[0]
        np.random.seed(5)
        out["vargau_ev"], out["vargau_evec"] = ev, evec
        out["vargau"] = np.array([RN.vargau(ev, evec, 1.5) for _ in range(3)])
        arr = rng.normal(size=(10, 3))
        idx = np.array([7, 2, 2, 9])
        out["exlist_in"], out["exlist_idx"], out["exlist"] = arr, idx, RB.exlist(arr, idx)
        cats = [3, 4, 5]
        with quiet():
            eb = RB.ebath(cats, 300.0, 0.5, 64, wmax=1.0, nw=7, bias=0.4, efric=spd(3, rng, 0.01),
                          exim=anti(3, rng, 1e-3), exip=sym(3, rng, 1e-3), zeta1=sym(3, rng, 1e-3),
                          zeta2=anti(3, rng, 1e-3))
            eb.GetSig()
        out["sig_efric"], out["sig_exim"], out["sig_zeta1"], out["sig_zeta2"] = eb.efric, eb.exim, eb.zeta1, eb.zeta2
        out["sig_wl"], out["sig"] = np.array(eb.wl), eb.sig
    finally:
        if not had:
            del np.complex
    np.savez_compressed(os.path.join(HERE, "helpers.npz"), **out)


if __name__ == "__main__":
    makers = {"scalars": make_scalars, "gamt": make_gamt, "noise": make_noise, "vv": make_vv_cases,
              "run_seeded": make_run_seeded, "tools": make_tools, "power": make_power, "ggamma": make_ggamma,
              "helpers": make_helpers}
    for name in (sys.argv[1:] or list(makers)):
        makers[name]()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
