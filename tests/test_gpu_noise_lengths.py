"""Noise and power spectra at run lengths that are not a power of two <= 8192.  The reference takes
any even nmd (myfft.iFourier1D checks only the length, functions.py:36-53): its profile runs
nmd = 1000 and examples/current-induced/rundp.py nmd = 2 10^5.  Lengths of 2, 3, 5 and 7 factors go
through mixed-radix transforms in global memory, other primes through Bluestein's chirp-z
(gle_kernels.hip, gfft_*); powers of two above the LDS limit through the same passes.

* phnoise / enoise on the device with the reference's RandomState draws against the oracle's
  restatement of noise.py (eigh, vargau, mirror, numpy FFT) at 1e-12 relative;
* the streamed generator (C5's path) equals the resident one at such lengths;
* the device power spectrum of recorded velocities against numpy's |FFT|^2;
* md.Run at nmd = 1000 with device noise: finite, and one md of 6 trajectories equals two shards."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LENGTHS = [6, 10, 1000, 2 * 97, 2 * 1009, 12288, 16384, 2 * 3 * 5 * 7 * 11]


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("nmd", LENGTHS)
def test_phnoise_any_length_vs_oracle(nmd):
    from oracle import sclmd_oracle as O
    from sclmd_amd import noise as N
    from sclmd_amd import synthetic

    rng = np.random.default_rng(nmd)
    gwl, gam = synthetic.gamma_spectrum(5, rng)
    dt = synthetic.DT
    np.random.seed(17)
    got = N.phnoise(gam, gwl, 300.0, 0.4, dt, nmd)
    np.random.seed(17)
    want = np.real(O.phnoise(gam, gwl, 300.0, 0.4, dt, nmd))
    assert got.shape == (nmd, 5)
    assert rel(got, want) < 1e-12, rel(got, want)


@pytest.mark.parametrize("nmd", [10, 1000, 2 * 1009, 12288])
def test_enoise_any_length_vs_oracle(nmd):
    from oracle import sclmd_oracle as O
    from sclmd_amd import noise as N
    from sclmd_amd.functions import antisymmetrize, symmetrize

    rng = np.random.default_rng(nmd + 1)
    n = 4
    efric = symmetrize(np.eye(n) * 1e-2 + 1e-3 * rng.normal(size=(n, n)))
    exim = antisymmetrize(1e-3 * rng.normal(size=(n, n)))
    exip = symmetrize(1e-3 * rng.normal(size=(n, n)))
    dt = 0.5 / 0.658
    np.random.seed(23)
    got = N.enoise(efric, exim, exip, 1.0, 300.0, 2.0, dt, nmd)
    np.random.seed(23)
    want = np.real(O.enoise(efric, exim, exip, 1.0, 300.0, 2.0, dt, nmd))
    assert rel(got, want) < 1e-12, rel(got, want)


@pytest.mark.parametrize("nmd", [1000, 2 * 97, 12288])
def test_stream_equals_resident_any_length(nmd):
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    rng = np.random.default_rng(5)
    B = 7
    b = synthetic.make_phbath(300.0, list(range(9)), 8, nmd, rng, nw=40)
    fac = b.noise_factor().scaled()
    out = []
    for streamed in (False, True):
        st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((1, b.nc, b.nc)))
        if streamed:
            st.noise_stream(0, ((w0, fac[w0:w0 + 50]) for w0 in range(0, fac.shape[0], 50)), False, seed=5,
                            max_chunk=50)
        else:
            st.noise_factors(0, fac)
            st.noise_generate(0, None, seed=5)
        out.append(st.get_noise(0))
        st.close()
    assert rel(out[1], out[0]) < 1e-12


@pytest.mark.parametrize("nmd", [10, 1000, 2 * 97, 12288])
def test_power_spectrum_any_length_vs_numpy(nmd):
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C3", natom=6, ml=4, nmd=nmd, nw=40, seed=2)
    B, nph = 3, meta["nph"]
    st = N.Stepper(nph, B, nmd, meta["dt"], 0)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    rng = np.random.default_rng(1)
    st.set_state(rng.normal(size=(B, nph)) * 1e-2, rng.normal(size=(B, nph)) * 1e-2, 0)
    for i, b in enumerate(baths):
        st.set_noise(i, rng.normal(size=(B, nmd, b.nc)) * 1e-3)
    st.record(N.REC_P)
    st.run(nmd)
    ps = st.get_record(N.REC_P)  # (B, nmd, nph)
    groups = [[0, 1, 2], [5], list(range(3, nph))]
    got = st.power_spectrum(groups)
    st.close()
    X = np.fft.fft(ps, axis=1)
    want = np.stack([np.sum(np.abs(X[:, :, g]) ** 2, axis=2) for g in groups])
    assert rel(got, want) < 1e-12, rel(got, want)


def test_md_run_nmd_1000_device_noise(tmp_path, monkeypatch):
    """md.Run with nmd = 1000 (the reference profile's length), device noise, power spectra: finite
    results, and 6 trajectories equal shards of 4 + 2 (trajectory-keyed noise and state)."""
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    def run(ntraj, offset):
        d = tmp_path / ("n%d_o%d" % (ntraj, offset))  # md.Run resumes from MD{j}.nc in the working directory
        d.mkdir()
        monkeypatch.chdir(d)
        dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=12, ml=32, nmd=1000, nw=80)
        m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=ntraj, seed=9, nstart=0, nstop=1,
                  traj_offset=offset, noise_mode="device", verbose=False)
        for b in baths:
            m.AddBath(b)
        m.CalPowerSpec()
        m.Run()
        p, q = np.array(m.p).reshape(ntraj, -1), np.array(m.q).reshape(ntraj, -1)
        power = np.array(m.power)
        m.close()
        return p, q, power

    p, q, power = run(6, 0)
    assert np.all(np.isfinite(p)) and np.all(np.isfinite(q)) and np.all(np.isfinite(power))
    assert np.abs(q).max() > 0
    p0, q0, _ = run(4, 0)
    p1, q1, _ = run(2, 4)
    assert rel(np.concatenate([q0, q1]), q) < 1e-9 and rel(np.concatenate([p0, p1]), p) < 1e-9


def test_generic_transforms_chunked_equal_unchunked():
    """Above ~1 GiB of work buffers the generic transforms run in chunks of series: a 64-trajectory
    ensemble at nmd = 24576 (2 noise chunks) and its power spectrum at nmd = 12288 (2 chunks) equal
    the same trajectories transformed one at a time (one chunk each)."""
    from sclmd_amd import _native as N
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    rng = np.random.default_rng(8)
    nmd, B, nc = 24576, 64, 60
    gwl, gam = synthetic.gamma_spectrum(nc, rng)
    fac = Nz.NoiseFactor(Nz.phonon_spectrum(gam, gwl, 300.0, 0.4, synthetic.DT, nmd))
    x = np.stack([fac.draws(np.random.RandomState(100 + b)) for b in range(B)])

    def gen(xs):
        st = N.Stepper(nc, len(xs), nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(nc), np.zeros((1, nc, nc)))
        st.noise_factors(0, fac.evecs)
        st.noise_generate(0, xs)
        out = st.get_noise(0)
        st.close()
        return out

    whole = gen(x)
    for b in (0, 31, 63):
        assert rel(gen(x[b:b + 1])[0], whole[b]) < 1e-13, b

    nmd = 12288
    dyn, _, baths, meta = synthetic.junction("C3", natom=20, ml=4, nmd=nmd, nw=40, seed=2)
    nph = meta["nph"]
    r = np.random.default_rng(3)
    st = N.Stepper(nph, B, nmd, meta["dt"], 0)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    st.set_state(r.normal(size=(B, nph)) * 1e-2, r.normal(size=(B, nph)) * 1e-2, 0)
    for i, b in enumerate(baths):
        st.set_noise(i, r.normal(size=(B, nmd, b.nc)) * 1e-3)
    st.record(N.REC_P)
    st.run(nmd)
    groups = [list(range(0, nph, 2)), list(range(1, nph, 2))]
    got = st.power_spectrum(groups)  # 64 x 60 series of 12288: two chunks
    ps = st.get_record(N.REC_P)
    st.close()
    for b in (0, 40):
        X = np.fft.fft(ps[b], axis=0)
        want = np.stack([np.sum(np.abs(X[:, g]) ** 2, axis=1) for g in groups])
        assert rel(got[:, b], want) < 1e-12, b
