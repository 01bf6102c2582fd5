"""Landauer limit of the GLE ensemble: a harmonic chain between two ohmic electron
baths (ml = 1, efric = I / damp) at T(1 +- delta/2) carries, in steady state, the NEGF current
  J = int_0^inf dw/2pi  hbar w  T(w) [n(w, T_hot) - n(w, T_cold)]
(sclmd negf.py:242-267 computes it; sclmd_amd.negf.bpt is its restatement, pinned to the reference
in tests/test_negf.py).  The semiclassical Langevin equation with quantum (zero-point + Bose) noise
reproduces it exactly in the harmonic limit, so the device ensemble's time-averaged current must
match it within its statistical error: an end-to-end physics check of the noise spectrum, the
friction, the integrator and the heat-current estimator together.

Tolerance: |J_gle - J_negf| < 4 standard errors of the ensemble mean + 3 % of J (Verlet
discretisation at w dt < 0.08 and the finite noise grid) for the antisymmetric estimator
(J_hot - J_cold)/2, + 5 % for each bath's current on its own (slow relaxation of the chain's
interior modes after the first run)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NATOM = 8
FIXED = [list(range(0, 3)), list(range(21, 24))]
BATHS = [list(range(3, 9)), list(range(15, 21))]


def landauer_case(ntraj=2048, nmd=8192, neq=1024, T=300.0, delta=1.0, damp=100.0, seed=11, zpmotion=False,
                  nrun=2):
    """Ensemble heat currents of the last of nrun md.Run runs (the earlier ones relax the initial
    state, which carries zero-point energy) and the NEGF current, in nW: a dict with the hot and
    cold bath currents, their antisymmetric combination (J_hot - J_cold) / 2 (the system's energy
    drift cancels in it), the standard errors of the ensemble means, and J_negf.

    zpmotion=False drops the zero-point part of both baths' noise: the current depends on the
    difference of the two baths' spectra only, so its mean is unchanged, while the zero-point
    fluctuations (temperature-independent, and the bulk of the variance) are gone."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic, units as U
    from sclmd_amd.baths import ebath
    from sclmd_amd.negf import bpt

    dt = synthetic.DT
    dyn = synthetic.chain_dyn(NATOM)
    m = MD.md(dt, nmd, T, axyz=synthetic.axyz_chain(NATOM), dyn=dyn, nstart=0, nstop=nrun, ntraj=ntraj,
              seed=seed, noise_mode="device", verbose=False)
    temps = [T * (1 + delta / 2), T * (1 - delta / 2)]
    for dofs, Tb in zip(BATHS, temps):
        m.AddBath(ebath(dofs, Tb, dt, nmd, wmax=2.0, nw=100, bias=0.0, efric=np.eye(len(dofs)) / damp,
                            zpmotion=zpmotion))
    m.AddConstr([range(a[0], a[-1] + 1) for a in FIXED])
    m.Run()
    allc = m._st.get_current()                                        # (nbath, ntraj, nmd)
    cur = [allc[i][:, neq:] * U.curcof for i in range(len(m.baths))]  # (ntraj, steps) nW
    per = [c.mean(axis=1) for c in cur]
    per.append((per[0] - per[1]) / 2)
    m.close()
    neg = bpt.from_md(dyn, damp, BATHS, FIXED, maxomega=0.4, num=4000)
    out = {"J_negf": float(neg.thermalcurrent(T, delta))}
    for name, v in zip(("hot", "cold", "anti"), per):
        out["J_" + name] = float(v.mean())
        out["sem_" + name] = float(v.std(ddof=1) / np.sqrt(ntraj))
    return out


def test_ensemble_current_matches_landauer(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    r = landauer_case()
    jn = r["J_negf"]
    assert jn > 0
    assert abs(r["J_anti"] - jn) < 4 * r["sem_anti"] + 0.03 * jn, r
    # after the relaxation run: each bath on its own, energy balance J_hot + J_cold ~ 0
    assert abs(r["J_hot"] - jn) < 4 * r["sem_hot"] + 0.05 * jn, r
    assert abs(-r["J_cold"] - jn) < 4 * r["sem_cold"] + 0.05 * jn, r
