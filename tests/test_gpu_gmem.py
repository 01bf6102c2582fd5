"""GPU tests of the device memory-kernel construction (phbath.gmem / gamt, baths.py:19-52,
412-445) through the C-ABI: gle_gamt against the reference's golden kernels, gle_add_bath_gmem
against the host-built kernel (small and full C3 size) and trajectories stepped with either.

Tolerance: 1e-12 relative to max|K| (the device contracts over the ngw spectrum nodes instead of the
reference's nw frequencies -- a re-association, fp64 rounding only); trajectories 1e-10."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("tag,eta", [("eta0", 0.0), ("eta1", 0.02)])
def test_gamt_device_matches_reference(tag, eta):
    from sclmd_amd import _native as N
    from sclmd_amd import baths as B

    g = load_golden("gamt")
    ml, nw, dt = int(g["ml"]), int(g["nw"]), float(g["dt"])
    wl = [0.4 * i / nw for i in range(nw)]   # phbath: wmax = mcof * debye = 2.0 * 0.2
    W = B.gmem_coefficients([dt * i for i in range(ml)], wl, g["gwl"], eta)
    K = N.gamt_device(W, g["gam"])
    assert K.shape == g["kernel_" + tag].shape
    assert rel(K, g["kernel_" + tag]) < 1e-12
    Wd = B.gmem_coefficients(g["gamt_tl"], g["gamt_wl"], g["gwl"])
    assert rel(N.gamt_device(Wd, g["gam"]), g["gamt_direct"]) < 1e-12


@pytest.mark.parametrize("ml,ngw,nel", [(1, 1, 1), (17, 5, 65), (100, 130, 200), (33, 300, 64)])
def test_gamt_device_ragged_shapes(ml, ngw, nel):
    """Ragged tails: ml not a multiple of 16, nel not a multiple of 64, ngw beyond one LDS chunk."""
    from sclmd_amd import _native as N

    rng = np.random.default_rng(ml * 1000 + ngw)
    W = rng.normal(size=(ml, ngw))
    G = rng.normal(size=(ngw, nel))
    out = N.gamt_device(W, G)
    assert rel(out, W @ G) < 1e-13


def _device_vs_host_baths(natom, ml, nmd, ntraj, nsteps, far_mode="auto"):
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    out = []
    for dev in (False, True):
        dyn, axyz, baths, meta = synthetic.junction("C3", seed=7, natom=natom, ml=ml, nmd=nmd, nw=120,
                                                    gmem_device=dev)
        st = N.Stepper(meta["nph"], ntraj, nmd, meta["dt"], 0, 0, far_mode)
        for b in baths:
            if dev:
                W, G = b.gmem_recipe
                st.add_bath_gmem(b.cids, W, G)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        rng = np.random.default_rng(3)
        p0 = rng.normal(size=(ntraj, meta["nph"])) * 1e-2
        q0 = rng.normal(size=(ntraj, meta["nph"])) * 1e-2
        st.set_state(p0, q0, 0)
        for i, b in enumerate(baths):
            st.set_history(i, None)
            st.set_noise(i, np.random.default_rng(11 + i).normal(size=(ntraj, nmd, b.nc)) * 1e-3)
        kern = [st.get_kernel(i) for i in range(len(baths))]
        st.run(nsteps)
        p, q, _ = st.get_state()
        out.append((kern, p, q, [b.kernel for b in baths]))
        st.close()
    return out


def test_gmem_bath_trajectory_matches_host_kernel():
    (kh, ph, qh, _), (kd, pd, qd, khost_lazy) = _device_vs_host_baths(natom=30, ml=96, nmd=128, ntraj=4,
                                                                     nsteps=150)
    for a, b, c in zip(kd, kh, khost_lazy):
        assert rel(a, b) < 1e-12 and rel(c, b) < 1e-12
    assert rel(qd, qh) < 1e-10 and rel(pd, ph) < 1e-10


def test_gmem_full_c3_kernel():
    """Full C3 shape (nc = 300, ml = 1024): device kernel vs numpy gamt on sampled slices."""
    import time

    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", seed=1234, gmem_device=True)
    st = N.Stepper(meta["nph"], 64, meta["nmd"], meta["dt"], 0)
    t0 = time.perf_counter()
    for b in baths:
        W, G = b.gmem_recipe
        st.add_bath_gmem(b.cids, W, G)
    build_s = time.perf_counter() - t0
    for i, b in enumerate(baths):
        W, G = b.gmem_recipe
        for s0 in (0, 511, 1023 - 7):
            dev = st.get_kernel(i, s0, 8)
            host = np.einsum("ig,gab->iab", W[s0:s0 + 8], G)
            assert rel(dev, host) < 1e-12
    print("C3 device gmem: %.3f s for %d baths" % (build_s, len(baths)))
    st.close()
