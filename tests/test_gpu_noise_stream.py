"""Streamed device noise (gle_noise_stream_*, the C5 path) on the GPU.

1. Same factors and seed: the streamed generator equals gle_noise_factors + gle_noise_generate
   (the same Philox keys, the same mirror + FFT; 1e-12 relative, summation order only).
2. md.gen_noise through the stream (noise_stream_bytes = 0) for a reduced C5 bath set -- two phonon
   baths and a biased electron bath -- gives an ensemble whose time-averaged covariance matches the
   reference spectrum's positive part, scale^2 (A+_0 + A+_h + 2 sum_{0<w<h} A+_w) (statistical, 6 %
   of the largest diagonal entry; 2048 trajectories of 1024 steps: the phonon spectra have few
   effective frequencies under their cutoff, so fewer samples leave ~5 % scatter)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("B,nc", [(5, 20), (40, 70), (33, 130)])
@pytest.mark.parametrize("kind", ["ph", "e"])
def test_stream_equals_resident_generator(kind, B, nc):
    """(partial 64-row factor tiles and 32-trajectory tiles of noise_gemm at B = 33 / 40, nc = 70 / 130)"""
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    rng = np.random.default_rng(2)
    nmd = 256
    if kind == "ph":
        b = synthetic.make_phbath(300.0, list(range(nc)), 8, nmd, rng, nw=40)
    else:
        b = synthetic.make_biased_ebath(300.0, list(range(nc - 2)), nmd, rng)
    fac = b.noise_factor().scaled()
    cplx = np.iscomplexobj(fac)
    out = []
    for streamed in (False, True):
        st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((1, b.nc, b.nc)))
        if streamed:
            chunks = ((w0, fac[w0:w0 + 7]) for w0 in range(0, fac.shape[0], 7))
            st.noise_stream(0, chunks, cplx, seed=77, traj_offset=3, max_chunk=7)
        else:
            st.noise_factors(0, fac)
            st.noise_generate(0, None, seed=77, traj_offset=3)
        out.append(st.get_noise(0))
        st.close()
    assert rel(out[1], out[0]) < 1e-12


def test_md_streamed_noise_covariance_reduced_c5():
    from sclmd_amd import md as MD
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C5", natom=12, ml=8, nmd=1024, nw=60, seed=8)
    B = 2048
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=B, seed=5, noise_mode="device",
              verbose=False)
    m.noise_stream_bytes = 0  # force the streamed path
    for b in baths:
        m.AddBath(b)
    m.initialise()
    m.ResetHis()
    assert any(b.kind == "ebath" and b.biased() for b in baths)
    dt, nmd = meta["dt"], meta["nmd"]
    h = nmd // 2
    scale = 1.0 / (dt * nmd)
    for i, b in enumerate(baths):
        m.gen_noise(i, 0)
        nz = m._st.get_noise(i)                       # (B, nmd, nc)
        emp = np.einsum("btk,btl->kl", nz, nz) / (B * nmd)
        f = b.noise_factor().scaled()
        ap = np.real(np.einsum("wik,wjk->wij", f, np.conj(f)))
        theory = scale ** 2 * (ap[0] + ap[h] + 2.0 * ap[1:h].sum(axis=0))
        assert np.max(np.abs(emp - theory)) < 0.06 * np.max(np.diag(theory)), (i, b.kind)
    m.close()


def test_stream_failure_releases_scratch_and_recovers():
    """A factor generator that raises between gle_noise_stream_begin and _end: the
    exception reaches the caller, gle_noise_stream_abort releases the spectrum scratch (device
    memory returns to its level before begin), and a later complete stream gives the same noise as
    a fresh handle."""
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    rng = np.random.default_rng(4)
    nmd, B = 4096, 64  # spectrum scratch 2049 x 64 x 64 doubles = 67 MB: a leak shows in mem_get_info
    b = synthetic.make_phbath(300.0, list(range(64)), 8, nmd, rng, nw=40)
    fac = b.noise_factor().scaled()

    def chunks(fail_at=None):
        for w0 in range(0, fac.shape[0], 64):
            if fail_at is not None and w0 >= fail_at:
                raise np.linalg.LinAlgError("factorisation failed (test)")
            yield w0, fac[w0:w0 + 64]

    def fresh():
        st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((1, b.nc, b.nc)))
        return st

    st = fresh()
    st.sync()
    free0 = N.device_mem_info(0)[0]
    with pytest.raises(np.linalg.LinAlgError):
        st.noise_stream(0, chunks(fail_at=640), False, seed=11, max_chunk=64)
    st.sync()
    assert N.device_mem_info(0)[0] >= free0 - (8 << 20)  # 67 MB scratch released (slack 8 MB)
    st.noise_stream(0, chunks(), False, seed=11, max_chunk=64)
    got = st.get_noise(0)
    st.close()
    ref = fresh()
    ref.noise_stream(0, chunks(), False, seed=11, max_chunk=64)
    want = ref.get_noise(0)
    ref.close()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kind", ["ph", "e"])
def test_stream_plan_equals_chunks_and_reuses_cache(kind, monkeypatch):
    """The work-segment stream (noise.stream_factor_plan: zero frequencies skipped, shared-matrix
    frequencies as one factor times per-frequency scales, dense factors per frequency) gives the
    noise of the full per-frequency chunk stream for the same seed (1e-12); a second run with the
    factor cache factorises nothing and, for the same seed, repeats the first run's noise exactly."""
    from sclmd_amd import _native as N
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    rng = np.random.default_rng(6)
    nmd, B = 1024, 6
    if kind == "ph":
        b = synthetic.make_phbath(300.0, list(range(36)), 8, nmd, rng, nw=40)
    else:
        b = synthetic.make_biased_ebath(300.0, list(range(30)), nmd, rng)
    cplx = kind == "e"

    def stepper():
        st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((1, b.nc, b.nc)))
        return st

    st = stepper()
    st.noise_stream(0, Nz.stream_factor_chunks(b, chunk=16), cplx, seed=21, traj_offset=2, max_chunk=16)
    want = st.get_noise(0)
    cache = {}
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16, cache=cache), cplx, seed=21, traj_offset=2,
                         max_chunk=16)
    got = st.get_noise(0)
    kinds = {s[0] for s in cache["segments"]}
    assert kinds == {"shared", "dense"}, kinds
    assert rel(got, want) < 1e-12
    calls = []
    monkeypatch.setattr(Nz, "dense_factor", lambda a: calls.append(1) or Nz.positive_factor(a))
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16, cache=cache), cplx, seed=21, traj_offset=2,
                         max_chunk=16)
    again = st.get_noise(0)
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16, cache=cache), cplx, seed=22, traj_offset=2,
                         max_chunk=16)
    other = st.get_noise(0)
    st.close()
    assert not calls
    assert np.array_equal(again, got)
    assert rel(other, got) > 0.1


@pytest.mark.parametrize("kind", ["ph", "e"])
def test_retained_plan_replay_equals_stream(kind, monkeypatch):
    """Device-retained factors (gle_noise_stream_retain / _replay): replaying the retained plan with a
    seed gives exactly the noise of streaming the plan again with that seed; md.gen_noise's later runs
    replay (no factorisation, no host factor cache kept) and give the noise a fresh stream gives."""
    from sclmd_amd import _native as N
    from sclmd_amd import md as MD
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    rng = np.random.default_rng(9)
    nmd, B = 1024, 6
    if kind == "ph":
        b = synthetic.make_phbath(300.0, list(range(36)), 8, nmd, rng, nw=40)
    else:
        b = synthetic.make_biased_ebath(300.0, list(range(30)), nmd, rng)
    cplx = kind == "e"

    def stepper():
        st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
        st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((1, b.nc, b.nc)))
        return st

    ref = stepper()
    want = {}
    for sd in (31, 32):
        ref.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16), cplx, seed=sd, traj_offset=4, max_chunk=16)
        want[sd] = ref.get_noise(0)
    ref.close()
    st = stepper()
    assert st.noise_stream_retained(0) == 0
    with pytest.raises(N.GLEError):
        st.noise_stream_replay(0, 31, 4)
    st.noise_stream_retain(0, True)
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16), cplx, seed=31, traj_offset=4, max_chunk=16)
    assert np.array_equal(st.get_noise(0), want[31])
    assert st.noise_stream_retained(0) > 0
    st.noise_stream_replay(0, 32, 4)
    assert np.array_equal(st.get_noise(0), want[32])
    st.noise_stream_replay(0, 31, 4)
    assert np.array_equal(st.get_noise(0), want[31])
    st.noise_stream_retain(0, False)
    assert st.noise_stream_retained(0) == 0
    st.close()

    # md: the second run's noise comes from the retained plan
    dyn, axyz, baths, meta = synthetic.junction("C5", natom=12, ml=8, nmd=nmd, nw=60, seed=8)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=B, seed=3, noise_mode="device",
              verbose=False)
    m.noise_stream_bytes = 0  # force the streamed path
    for bb in baths:
        m.AddBath(bb)
    m.initialise()
    i = [k for k, bb in enumerate(baths) if (bb.kind == "ebath") == cplx][0]
    bi = baths[i]
    m.gen_noise(i, 0)
    assert m._st.noise_stream_retained(i) > 0 and getattr(bi, "_stream_cache", None) is None
    calls = []
    monkeypatch.setattr(Nz, "dense_factor", lambda a: calls.append(1) or Nz.positive_factor(a))
    m.gen_noise(i, 1)
    got = m._st.get_noise(i)
    seed1 = m._noise_seed(i, 1)
    m.close()
    assert not calls
    monkeypatch.undo()
    fresh = N.Stepper(bi.nc, B, nmd, meta["dt"], 0)
    fresh.add_bath(N.GLE_BATH_PHONON, np.arange(bi.nc), np.zeros((1, bi.nc, bi.nc)))
    fresh.noise_stream_plan(0, Nz.stream_factor_plan(bi), cplx, seed=seed1, traj_offset=0)
    assert np.array_equal(got, fresh.get_noise(0))
    fresh.close()


def test_retention_cap_streams_without_keeping():
    """Retention that would exceed the handle's cap (gle_noise_stream_retain_cap; the same path as
    running short of free device memory beside the plan) keeps nothing and streams as without it:
    the noise is bit-identical, the bath's run and the history getters (md.dump's snapshot buffer)
    still work, and md.gen_noise falls back to the host factor cache."""
    from sclmd_amd import _native as N
    from sclmd_amd import md as MD
    from sclmd_amd import noise as Nz
    from sclmd_amd import synthetic

    rng = np.random.default_rng(4)
    nmd, B = 512, 4
    b = synthetic.make_phbath(300.0, list(range(24)), 8, nmd, rng, nw=40)
    st = N.Stepper(b.nc, B, nmd, synthetic.DT, 0)
    st.add_bath(N.GLE_BATH_PHONON, np.arange(b.nc), np.zeros((2, b.nc, b.nc)))
    st.set_dyn(np.eye(b.nc) * 0.01)
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16), False, seed=5, traj_offset=0, max_chunk=16)
    want = st.get_noise(0)
    st.noise_stream_retain(0, True)
    st.noise_stream_retain_cap(4096)  # far below one chunk of factors
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16), False, seed=5, traj_offset=0, max_chunk=16)
    assert st.noise_stream_retained(0) == 0
    assert np.array_equal(st.get_noise(0), want)
    with pytest.raises(N.GLEError):
        st.noise_stream_replay(0, 5, 0)
    st.set_state(np.zeros((B, b.nc)), np.zeros((B, b.nc)), 0)
    st.set_history(0, None)
    st.run(20)
    st.sync()
    assert st.get_history(0).shape == (B, 2, b.nc)
    st.noise_stream_retain_cap(None)
    st.noise_stream_plan(0, Nz.stream_factor_plan(b, chunk=16), False, seed=5, traj_offset=0, max_chunk=16)
    assert st.noise_stream_retained(0) > 0 and np.array_equal(st.get_noise(0), want)
    st.close()

    dyn, axyz, baths, meta = synthetic.junction("C5", natom=12, ml=8, nmd=nmd, nw=60, seed=8)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=B, seed=3, noise_mode="device",
              verbose=False)
    m.noise_stream_bytes = 0  # force the streamed path
    for bb in baths:
        m.AddBath(bb)
    m.initialise()
    m._ensure_device().noise_stream_retain_cap(0)
    m.gen_noise(0, 0)
    assert m._st.noise_stream_retained(0) == 0 and getattr(baths[0], "_stream_cache", None)
    m.gen_noise(0, 1)  # from the host factor cache
    m.close()
