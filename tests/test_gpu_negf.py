"""Landauer limit of the GLE ensemble: a harmonic chain between two ohmic electron
baths (ml = 1, efric = I / damp) at T(1 +- delta/2) carries, in steady state, the NEGF current
  J = int_0^inf dw/2pi  hbar w  T(w) [n(w, T_hot) - n(w, T_cold)]
(sclmd negf.py:242-267 computes it; sclmd_amd.negf.bpt is its restatement, pinned to the reference
in tests/test_negf.py).  The semiclassical Langevin equation with quantum (zero-point + Bose) noise
reproduces it exactly in the harmonic limit, so the device ensemble's time-averaged current must
match it within its statistical error: an end-to-end physics check of the noise spectrum, the
friction, the integrator and the heat-current estimator together.

Tolerance: |J_gle - J_negf| < 4 standard errors of the ensemble mean + 3 % of J (Verlet
discretisation at w dt < 0.08 and the finite noise grid).  Energy balance: hot and cold bath
currents agree in magnitude within the same bound."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NATOM = 8
FIXED = [list(range(0, 3)), list(range(21, 24))]
BATHS = [list(range(3, 9)), list(range(15, 21))]


def landauer_case(ntraj=512, nmd=8192, neq=1024, T=300.0, delta=1.0, damp=100.0, seed=11):
    """(J_hot, J_cold, sem_hot, sem_cold, J_negf) in nW for the chain junction above."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic, units as U
    from sclmd_amd.baths import ebath
    from sclmd_amd.negf import bpt

    dt = synthetic.DT
    dyn = synthetic.chain_dyn(NATOM)
    m = MD.md(dt, nmd, T, axyz=synthetic.axyz_chain(NATOM), dyn=dyn, nstart=0, nstop=1, ntraj=ntraj,
              seed=seed, noise_mode="device", verbose=False)
    temps = [T * (1 + delta / 2), T * (1 - delta / 2)]
    for dofs, Tb in zip(BATHS, temps):
        m.AddBath(ebath(dofs, Tb, dt, nmd, wmax=2.0, nw=100, bias=0.0, efric=np.eye(len(dofs)) / damp))
    m.AddConstr([range(a[0], a[-1] + 1) for a in FIXED])
    m.Run()
    cur = [np.asarray(b.cur)[:, neq:] * U.curcof for b in m.baths]    # (ntraj, steps) nW
    per = [c.mean(axis=1) for c in cur]
    m.close()
    neg = bpt.from_md(dyn, damp, BATHS, FIXED, maxomega=0.4, num=4000)
    jn = neg.thermalcurrent(T, delta)
    return (float(per[0].mean()), float(per[1].mean()), float(per[0].std(ddof=1) / np.sqrt(ntraj)),
            float(per[1].std(ddof=1) / np.sqrt(ntraj)), float(jn))


@pytest.mark.skip(reason="local-bath-only ensemble run under investigation (device fault)")
def test_ensemble_current_matches_landauer(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    jh, jc, sh, sc, jn = landauer_case()
    assert jn > 0
    assert abs(jh - jn) < 4 * sh + 0.03 * jn, (jh, sh, jn)
    assert abs(-jc - jn) < 4 * sc + 0.03 * jn, (jc, sc, jn)
