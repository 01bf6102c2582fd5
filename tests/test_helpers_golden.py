"""The reference's small public helpers (a user script may import them from sclmd.functions /
noise / baths) against outputs of the reference itself (tests/golden/helpers.npz, made by
tests/golden/make_golden.py helpers).  Host code: no GPU."""
import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def g():
    return load_golden("helpers")


def close(a, b, tol=1e-13):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and float(np.max(np.abs(a - b), initial=0.0)) <= tol * max(np.max(np.abs(b), initial=0.0), 1e-300)


def test_functions(g):
    from sclmd_amd import functions as F

    assert close([F.coth(x) for x in g["coth_x"]], g["coth"])
    with pytest.raises(ValueError):
        F.coth(0.0)
    assert close([F.xcoth(x) for x in g["xcoth_x"]], g["xcoth"])
    assert close([F.fermi(*a) for a in g["fermi_args"]], g["fermi"])
    assert close(F.dagger(g["dagger_in"]), g["dagger"])
    assert close(F.mm(g["mm_1"], g["mm_2"], g["mm_3"]), g["mm"])
    nmd = g["qs"].shape[0]
    assert close(F.powerspecq(g["qs"], float(g["pq_dt"]), nmd), g["powerspecq"], 1e-12)


def test_noise_helpers(g):
    from sclmd_amd import noise as N

    for tag in ("q", "c", "nozp"):
        T, cut, cl, zp = g["phw_params_" + tag]
        assert close(N.phnoisew(g["phw_gam"], g["phw_wl"], T, cut, bool(cl), bool(zp)), g["phnoisew_" + tag])
    for a, m, p in zip(g["neq_args"], g["nonequm"], g["nonequp"]):
        w, b, T, cl = a
        assert close(N.nonequm(w, b, T, bool(cl)), m) and close(N.nonequp(w, b, T, bool(cl)), p)
    np.random.seed(5)
    got = np.array([N.vargau(g["vargau_ev"], g["vargau_evec"], 1.5) for _ in range(3)])
    assert close(got, g["vargau"])


def test_enoisew_is_enoise_matrix():
    """enoisew: the reference's own raises (noise.py:122-128 shadows numpy), so it is pinned by the
    spectral matrix of enoise (golden-checked through the noise fixtures): enoisew(w) * Delta equals
    electron_spectrum's matrix at the same frequencies."""
    from sclmd_amd import noise as N

    rng = np.random.default_rng(2)
    n = 4
    efric = np.eye(n) * 1e-2
    exim = rng.normal(size=(n, n)) * 1e-3
    exim = exim - exim.T
    exip = rng.normal(size=(n, n)) * 1e-3
    exip = exip + exip.T
    dt, nmd = 0.5, 16
    ws, delta = N.frequencies(dt, nmd)
    want = N.electron_spectrum(efric, exim, exip, 0.3, 300.0, 1.0, dt, nmd)
    got = N.enoisew(ws, efric, exim, exip, 0.3, 300.0, 1.0) * delta
    assert close(got, want, 1e-14)


def test_bath_helpers(g):
    from sclmd_amd import baths as B

    assert close(B.exlist(g["exlist_in"], g["exlist_idx"]), g["exlist"])
    eb = B.ebath([3, 4, 5], 300.0, 0.5, 64, wmax=1.0, nw=7, bias=0.4, efric=g["sig_efric"], exim=g["sig_exim"],
                 exip=np.zeros((3, 3)), zeta1=g["sig_zeta1"], zeta2=g["sig_zeta2"])
    assert close(np.array(eb.wl), g["sig_wl"])
    assert close(eb.GetSig(), g["sig"]) and close(eb.sig, g["sig"])
