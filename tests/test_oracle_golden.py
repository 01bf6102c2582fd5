"""Pin the CPU oracle against fixtures produced by the real reference (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from conftest import constr_from, load_golden, oracle_from_golden, vv_cases
from oracle import sclmd_oracle as O

RTOL = 1e-12


def close(a, b, rtol=RTOL):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(np.max(np.abs(b)), 1e-300)
    return np.max(np.abs(a - b)) <= rtol * scale


def test_scalars():
    g = load_golden("scalars")
    bose = np.array([[O.bose(w, T) for w in g["ws"]] for T in g["Ts"]])
    np.testing.assert_array_equal(bose, g["bose"])
    k = 0
    for classical in (False, True):
        for zp in (True, False):
            for cut in (0.2, 1.0):
                e = np.array([[O.equ(w, cut, T, classical, zp) for w in g["ws"]] for T in g["Ts"]])
                np.testing.assert_array_equal(e, g["equ"][k])
                k += 1
    fl = np.array([O.flinterp(x, g["xs"], g["ys"]) for x in g["xq"]])
    np.testing.assert_allclose(fl, g["flinterp"], rtol=0, atol=1e-15)
    assert float(g["kb"]) == O.KB


def test_gamt():
    g = load_golden("gamt")
    ml, nw, dt = int(g["ml"]), int(g["nw"]), float(g["dt"])
    wmax = 2.0 * 0.2
    wl = [wmax * i / nw for i in range(nw)]  # baths.py:305-308
    for tag, eta in (("eta0", 0.0), ("eta1", 0.02)):
        k, gam = O.gmem(ml, dt, wl, g["gwl"], g["gam"], eta)
        assert close(k, g["kernel_" + tag]), tag
        assert close(gam, g["gamma_after_" + tag]), tag
    direct = O.gamt(g["gamt_tl"], g["gamt_wl"], g["gwl"], g["gam"])
    assert close(direct, g["gamt_direct"])
    # Debye/local bath: kernel = [diag(debye*pi/6)], ml forced to 1 (baths.py:336-340)
    assert int(g["ml_debye"]) == 1
    np.testing.assert_allclose(g["kernel_debye"][0], np.diag(np.full(4, 0.15 * np.pi / 6)), rtol=0,
                               atol=0)


@pytest.mark.parametrize("tag", ["ph_q", "ph_c", "ph_nozp"])
def test_phnoise(tag):
    g = load_golden("noise")
    T, phcut, classical, zp = g["params_" + tag]
    np.random.seed(11)
    rec = []
    nz = O.phnoise(g["gam"], g["gwl"], T, phcut, float(g["dt"]), int(g["nmd"]), bool(classical),
                   bool(zp), record=rec)
    assert close(rec[0], g["amp_" + tag])
    assert close(nz, g["noise_" + tag])


@pytest.mark.parametrize("tag", ["e_eq", "e_bias", "e_cold"])
def test_enoise(tag):
    g = load_golden("noise")
    bias, T, ecut, classical, zp = g["params_" + tag]
    np.random.seed(12)
    rec = []
    nz = O.enoise(O.symm(g["efric"]), O.antisymm(g["exim"]), O.symm(g["exip"]), bias, T, ecut,
                  float(g["dt"]), int(g["nmd"]), bool(classical), bool(zp), record=rec)
    assert close(rec[0], g["amp_" + tag])
    assert close(nz, g["noise_" + tag])


def test_spectrum_to_series_matches_amplitudes():
    """Stage check used by the GPU generator parity test: mirror+FFT of the recorded amplitudes."""
    g = load_golden("noise")
    for tag in ("ph_q", "e_bias"):
        s = O.spectrum_to_series(g["amp_" + tag], float(g["dt"]), int(g["nmd"]))
        assert close(s, g["noise_" + tag], 1e-14)


@pytest.mark.parametrize("case", vv_cases())
def test_vv_trajectory(case):
    g = load_golden(case)
    sim = oracle_from_golden(g)
    q, p, cur, et = [], [], [], []
    nmd = int(g["nmd"])
    for _ in range(int(g["nsteps"])):
        t = sim.t
        sim.step()
        q.append(sim.q.copy())
        p.append(sim.p.copy())
        cur.append([b.cur[t % nmd] for b in sim.baths])
        et.append(sim.etot[t % nmd])
    assert close(q, g["q"]), case
    assert close(p, g["p"]), case
    assert close(cur, g["cur"], 1e-11), case
    assert close(et, g["etot"]), case


def test_initialise_and_seeded_runs():
    g = load_golden("run_seeded")
    np.random.seed(int(g["seed"]))
    constr = [range(6, 8)]
    p0, q0, dyn_used = O.initial_state(g["dyn"], float(g["T"]), constr)
    assert close(p0, g["p0"]) and close(q0, g["q0"])
    assert close(dyn_used, g["dyn_md"])
    nmd, dt = int(g["nmd"]), float(g["dt"])
    wl1 = [2.0 * float(g["debye1"]) * i / int(g["nw1"]) for i in range(int(g["nw1"]))]
    k1, _ = O.gmem(int(g["ml1"]), dt, wl1, g["gwl1"], g["gam1"])
    assert close(k1, g["kernel1"])
    b1 = O.Bath("ph", g["c1"], k1, None, dt, nmd)
    b2 = O.Bath("e", g["c2"], np.array([g["efric2"]]), None, dt, nmd)
    sim = O.GLE(len(p0), dt, nmd, [b1, b2], dyn=dyn_used, constr=constr)
    sim.p, sim.q = p0, q0
    kappa = []
    z = np.zeros_like(g["efric2"])
    for j in range(int(g["nrun"])):
        b1.noise = np.real(O.phnoise(g["gam1"], g["gwl1"], float(g["T1"]), 2.0 * float(g["debye1"]),
                                     dt, nmd))
        b2.noise = np.real(O.enoise(g["efric2"], z, z, 0.0, float(g["T2"]), 1.0, dt, nmd))
        assert close(b1.noise, g["noise1"][j]) and close(b2.noise, g["noise2"][j])
        for _ in range(nmd):
            sim.step()
        kappa.append([np.mean(b.cur) * O.CURCOF for b in sim.baths])
    assert close(kappa, g["kappa"], 1e-10)
    assert close(sim.p, g["p_end"]) and close(sim.q, g["q_end"])
    assert sim.t == int(g["t_end"])


def test_tools_tables():
    g = load_golden("tools")
    kb = g["kb"]
    np.testing.assert_allclose(O.heat_flux_table(kb[:2], 2), g["heatflux_2"], rtol=1e-6)
    m, s = O.conductance(kb, 0.1, float(g["T"]), 2, 2)
    np.testing.assert_allclose([m, s], g["tc_2"], rtol=1e-6)
    m, s = O.conductance(kb, 0.1, float(g["T"]), 1, 3)
    np.testing.assert_allclose([m, s], g["tc_3"], rtol=1e-6)


@pytest.mark.parametrize("case", vv_cases())
def test_batch_oracle_matches_reference_trajectory(case):
    """GLEBatch (one memory-tail product per step, trajectories in columns) reproduces the
    reference-generated vv trajectories (ntr = 1) like GLE does."""
    from oracle import sclmd_oracle as O

    g = load_golden(case)
    sim = oracle_from_golden(g)
    bt = O.GLEBatch(sim.nph, sim.dt, sim.nmd, sim.baths, g["dyn_md"], ntr=1, constr=sim.constr)
    bt.p, bt.q = g["p0"].copy()[:, None], g["q0"].copy()[:, None]
    nmd, cur = int(g["nmd"]), []
    for _ in range(int(g["nsteps"])):
        t = bt.t
        bt.step()
        cur.append([c[0, t % nmd] for c in bt.cur])
    assert close(bt.q[:, 0], g["q"][-1], 1e-12) and close(bt.p[:, 0], g["p"][-1], 1e-12)
    assert close(cur, g["cur"], 1e-11)


def test_batch_oracle_matches_reference_shaped_oracle_long_memory():
    """GLEBatch vs GLE with a 64-slice kernel, a nonzero history, an unaligned start, a biased
    electron bath and constraints: three distinct trajectories, 150 steps (1e-12)."""
    from oracle import sclmd_oracle as O
    from sclmd_amd import synthetic

    rng = np.random.default_rng(3)
    dyn, _, baths, meta = synthetic.junction("C5", natom=12, ml=64, nmd=128, nw=60, seed=4)
    nph, dt, nmd = meta["nph"], meta["dt"], meta["nmd"]
    ntr, t0, nst = 3, 11, 150
    p = rng.normal(size=(nph, ntr)) * 1e-3
    q = rng.normal(size=(nph, ntr)) * 1e-3
    hist = [rng.normal(size=(ntr, b.ml, b.nc)) * 1e-3 for b in baths]
    noise = [rng.normal(size=(ntr, nmd, b.nc)) * 1e-3 for b in baths]
    constr = [range(0, 3)]

    def obath(b, nz):
        if b.kind == "ebath":
            return O.Bath("e", b.cids, b.kernel, nz, dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1,
                          zeta2=b.zeta2)
        return O.Bath("ph", b.cids, b.kernel, nz, dt, nmd)

    bt = O.GLEBatch(nph, dt, nmd, [obath(b, noise[i]) for i, b in enumerate(baths)], dyn, ntr=ntr, constr=constr)
    bt.p, bt.q, bt.t = p.copy(), q.copy(), t0
    for i in range(len(baths)):
        bt.set_history(i, hist[i])
    for _ in range(nst):
        bt.step()
    assert any(ob.biased() for ob in bt.baths)
    for j in range(ntr):
        sim = O.GLE(nph, dt, nmd, [obath(b, noise[i][j]) for i, b in enumerate(baths)], dyn=dyn, constr=constr)
        sim.p, sim.q, sim.t = p[:, j].copy(), q[:, j].copy(), t0
        for i, b in enumerate(baths):
            sim.phis[: b.ml, b.cids] = hist[i][j]
        for _ in range(nst):
            sim.step()
        assert close(bt.q[:, j], sim.q, 1e-12) and close(bt.p[:, j], sim.p, 1e-12)
        for i, ob in enumerate(sim.baths):
            assert close(bt.cur[i][j], ob.cur, 1e-11)
