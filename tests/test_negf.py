"""NEGF / Landauer restatement (sclmd_amd.negf) against the reference's own bpt
(tests/golden/negf.npz, made by tests/golden/make_golden_negf.py from negf.py:8-273)."""
import numpy as np
import pytest

from conftest import load_golden
from sclmd_amd.negf import RPC, bpt


@pytest.fixture(scope="module")
def g():
    return load_golden("negf")


def make(g):
    return bpt(maxomega=float(g["maxomega"]), damp=float(g["damp"]), dofatomofbath=[g["bath0"], g["bath1"]],
               dofatomfixed=[g["fixed0"], g["fixed1"]], num=int(g["intnum"]), dynmat=g["dynmat"])


def test_transmission_matches_reference(g):
    b = make(g)
    t = b.gettm(filename=None)
    np.testing.assert_array_equal(t[:, 0], g["tm_x"])
    np.testing.assert_allclose(t[:, 1], g["tm_y"], rtol=1e-12, atol=1e-13)
    assert b.tm(float(g["tm_x"][100])) == pytest.approx(float(g["tm_y"][100]), rel=1e-12)


def test_thermal_current_conductance_conductivity(g):
    b = make(g)
    d = float(g["delta"])
    cur = np.array([b.thermalcurrent(T, d) for T in g["current_T"]])
    # T = 0 reproduces the reference's inf - inf at w = 0 (negf.py:221): nan in both
    np.testing.assert_allclose(cur, g["current"], rtol=1e-12, equal_nan=True)
    temps = g["current_T"][1:]
    np.testing.assert_allclose([b.thermalconductance(T, d) for T in temps], g["conductance"], rtol=1e-12)
    np.testing.assert_allclose([b.thermalconductivity(T, d, float(g["L"]), float(g["A"])) for T in temps],
                               g["conductivity"], rtol=1e-12)


def test_power_spectrum_unbiased_and_biased(g):
    b = make(g)
    T = float(g["ps_T"])
    ps = [b.ps(w, T, g["ps_atoms"]) for w in g["ps_w"]]
    np.testing.assert_allclose(ps, g["ps_unbiased"], rtol=1e-12)
    b.setbias(float(g["bias"]), bdamp=g["bdamp"], chiplus=g["chiplus"], chiminus=g["chiminus"],
              dofatomofbias=list(g["bias_dofs"]))
    ps = [b.ps(w, T, g["ps_atoms"]) for w in g["ps_w"]]
    # G^r from a batched solve instead of inv: the biased Keldysh product loses a few digits
    np.testing.assert_allclose(ps, g["ps_biased"], rtol=1e-8)
    with pytest.raises(ValueError):
        b.setbias(0.1, bdamp=np.eye(2), chiplus=np.eye(2), chiminus=np.eye(3), dofatomofbias=[9, 10])


def test_single_dof_transmission_closed_form():
    """One free DOF coupled to both baths: T = (2 w g)^2 / ((w^2 - k)^2 + (2 w g)^2), g = 1/damp."""
    k, damp = 0.3, 2.0
    d = np.zeros((3, 3))
    d[0, 0] = k
    d[1, 1] = d[2, 2] = 1.0
    b = bpt(maxomega=RPC * 2.0, damp=damp, dofatomofbath=[[0], [0]], dofatomfixed=[[], []], num=50, dynmat=d)
    for w in (0.1, 0.5, 0.9, 1.7):
        gam = 2 * w / damp
        # Sigma^r = -i w (1/damp + 1/damp) on the DOF; |G|^2 = 1 / ((w^2 - k)^2 + (2 w / damp)^2)
        want = gam ** 2 / ((w ** 2 - k) ** 2 + (2 * w / damp) ** 2)
        assert b.tm(w) == pytest.approx(want, rel=1e-7)


def test_missing_engine_and_fixed_bath_dof():
    with pytest.raises(RuntimeError):
        bpt(infile=["units metal"], maxomega=0.25, damp=0.1, dofatomofbath=[[0], [1]])
    d = np.eye(6)
    with pytest.raises(ValueError):
        bpt(maxomega=0.25, damp=0.1, dofatomofbath=[[0], [4]], dofatomfixed=[[0, 1, 2], []], dynmat=d)


def test_md_units_bridge():
    """from_md: eV^2 dynamical matrix and damping in md time units -> the same physics in ps."""
    d = np.diag([0.01, 0.02, 0.03])
    b = bpt.from_md(d, damp_md=100.0, dofatomofbath=[[0], [2]], maxomega=0.3, num=10)
    np.testing.assert_allclose(np.sort(b.omegas), np.sqrt([0.01, 0.02, 0.03]), rtol=1e-12)
    assert b.damp == pytest.approx(100.0 * 0.658211814201041e-3)
