"""Host-side logic of the product (setup code that runs on the CPU): noise factorisation and
reference-compatible draws, memory-kernel construction, bath matrix conventions, initial state,
post-processing, ensemble sharding -- each against the reference-generated golden fixtures."""
import os

import numpy as np
import pytest

from conftest import load_golden


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("tag", ["ph_q", "ph_c", "ph_nozp"])
def test_phonon_factor_and_draws(tag):
    from sclmd_amd import noise as N

    g = load_golden("noise")
    T, phcut, cl, zp = g["params_" + tag]
    f = N.NoiseFactor(N.phonon_spectrum(g["gam"], g["gwl"], T, phcut, float(g["dt"]), int(g["nmd"]),
                                        bool(cl), bool(zp)))
    assert np.array_equal(f.evals, g["eval_" + tag])
    np.random.seed(11)
    r = f.draws()
    assert rel(np.einsum("wij,wj->wi", f.evecs, r), g["amp_" + tag]) < 1e-14
    # device-mode factor U sqrt(lambda+) reproduces the PSD part of the spectrum
    m = f.scaled()
    spec = N.phonon_spectrum(g["gam"], g["gwl"], T, phcut, float(g["dt"]), int(g["nmd"]), bool(cl), bool(zp))
    psd = np.einsum("wik,wjk->wij", m, m)
    assert rel(psd, spec) < 1e-10


@pytest.mark.parametrize("tag", ["e_eq", "e_bias", "e_cold"])
def test_electron_factor_and_draws(tag):
    from sclmd_amd import noise as N
    from sclmd_amd.functions import antisymmetrize, symmetrize

    g = load_golden("noise")
    bias, T, ecut, cl, zp = g["params_" + tag]
    f = N.NoiseFactor(N.electron_spectrum(symmetrize(g["efric"]), antisymmetrize(g["exim"]),
                                          symmetrize(g["exip"]), bias, T, ecut, float(g["dt"]),
                                          int(g["nmd"]), bool(cl), bool(zp)))
    assert np.array_equal(f.evals, g["eval_" + tag])
    np.random.seed(12)
    r = f.draws()
    assert rel(np.einsum("wij,wj->wi", f.evecs, r), g["amp_" + tag]) < 1e-14


def test_gamt_and_gmem():
    from sclmd_amd import baths as B

    g = load_golden("gamt")
    for tag, eta in (("eta0", 0.0), ("eta1", 0.02)):
        b = B.phbath(300.0, list(range(4)), debye=0.2, nw=int(g["nw"]), dt=float(g["dt"]), nmd=64,
                     ml=int(g["ml"]), gamma=g["gam"].copy(), gwl=g["gwl"], eta_ad=eta)
        b.gmem()
        assert rel(b.kernel, g["kernel_" + tag]) < 1e-13
        assert rel(b.gamma, g["gamma_after_" + tag]) < 1e-13
    assert rel(B.gamt(g["gamt_tl"], g["gamt_wl"], g["gwl"], g["gam"]), g["gamt_direct"]) < 1e-13
    b = B.phbath(300.0, list(range(4)), debye=0.15, nw=40, dt=0.38, nmd=64, ml=8)
    b.gmem()
    assert b.ml == 1 and np.array_equal(b.kernel, g["kernel_debye"])


def test_gmem_coefficients_factor_gamt():
    """The device kernel build contracts W = scale C(t, w) . I(w -> gwl) with Gamma
    (gle_add_bath_gmem); W . Gamma must equal the reference gamt (golden, both eta branches), and
    phbath.gmem(on_device=True) must leave the same kernel / updated gamma as the host path."""
    from sclmd_amd import baths as B

    g = load_golden("gamt")
    ml, nw, dt = int(g["ml"]), int(g["nw"]), float(g["dt"])
    for tag, eta in (("eta0", 0.0), ("eta1", 0.02)):
        b = B.phbath(300.0, list(range(4)), debye=0.2, nw=nw, dt=dt, nmd=64, ml=ml,
                     gamma=g["gam"].copy(), gwl=g["gwl"], eta_ad=eta)
        W = B.gmem_coefficients([dt * i for i in range(ml)], b.wl, g["gwl"], eta)
        assert W.shape == (ml, len(g["gwl"]))
        assert rel(np.einsum("ig,gab->iab", W, g["gam"]), g["kernel_" + tag]) < 1e-12
        b.gmem(on_device=True)
        assert b.gmem_recipe is not None and b.__dict__["_kernel"] is None
        assert rel(b.gamma, g["gamma_after_" + tag]) < 1e-12
        assert rel(b.kernel, g["kernel_" + tag]) < 1e-12      # lazy host evaluation of W . gamma
    W = B.gmem_coefficients(g["gamt_tl"], g["gamt_wl"], g["gwl"])
    assert rel(np.einsum("ig,gab->iab", W, g["gam"]), g["gamt_direct"]) < 1e-12
    # assigning a kernel drops the device recipe (the explicit kernel wins)
    b.kernel = g["kernel_eta0"]
    assert b.gmem_recipe is None


def test_ebath_conventions():
    from sclmd_amd.baths import ebath

    rng = np.random.default_rng(0)
    m = rng.normal(size=(4, 4))
    b = ebath([0, 1, 2, 3], 300.0, 0.38, 16, wmax=1.0, nw=10, bias=0.3, efric=m, exim=m, zeta1=m, zeta2=m)
    assert np.allclose(b.efric, b.efric.T) and np.allclose(b.zeta1, b.zeta1.T)
    assert np.allclose(b.exim, -b.exim.T) and np.allclose(b.zeta2, -b.zeta2.T)
    assert b.biased() and b.ml == 1 and b.kernel.shape == (1, 4, 4)
    b2 = ebath([0, 1, 2, 3], 300.0, 0.38, 16, bias=0.3, efric=m, exim=m)  # zeta None: inactive
    assert not b2.biased()
    with pytest.raises(ValueError):
        ebath([0, 1, 2], 300.0, 0.38, 16, efric=m)


def test_initialise_matches_reference():
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    g = load_golden("run_seeded")
    natom = int(g["natom"])
    m = MD.md(float(g["dt"]), int(g["nmd"]), float(g["T"]), axyz=synthetic.axyz_chain(natom),
              dyn=g["dyn"], verbose=False)
    assert rel(m.dyn, g["dyn_md"]) < 1e-14
    m.AddConstr([range(6, 8)])
    np.random.seed(int(g["seed"]))
    m.initialise()
    assert rel(m.p, g["p0"]) < 1e-14 and rel(m.q, g["q0"]) < 1e-14


def test_tools_files(tmp_path, monkeypatch):
    from sclmd_amd import tools

    g = load_golden("tools")
    kb, T = g["kb"], int(g["T"])
    monkeypatch.chdir(tmp_path)
    for i in range(3):
        for j in range(int(g["nrun"])):
            with open("kappa.%d.bath%d.run%d.dat" % (T, i, j), "w") as f:
                f.write("%i %f    %f \n" % (j, float(T), kb[i, j]))
    tools.calHF(dlist=2, bathnum=2)
    tools.calTC(delta=0.1, dlist=2, bathnum=2, L=10.0, A=4.0)
    np.testing.assert_allclose(np.loadtxt("heatflux.%d.dat" % T), g["heatflux_2"], rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt("thermalconductance.%d.dat" % T), g["tc_2"], rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt("thermalconductivity.%d.dat" % T), g["tcy_2"], rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt("heatflux-between-baths.%d.dat" % T), g["hfb_2"], rtol=1e-12)
    tools.calHF(dlist=1, bathnum=3)
    tools.calTC(delta=0.1, dlist=1, bathnum=3)
    np.testing.assert_allclose(np.loadtxt("heatflux.%d.dat" % T), g["heatflux_3"], rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt("thermalconductance.%d.dat" % T), g["tc_3"], rtol=1e-12)
    np.testing.assert_allclose(np.loadtxt("heatflux-between-baths.%d.dat" % T), g["hfb_3"], rtol=1e-12)


@pytest.mark.parametrize("n,w", [(64, 1), (64, 8), (512, 8), (7, 3), (3, 8)])
def test_shard_covers_ensemble(n, w):
    from sclmd_amd.ensemble import shard

    seen = []
    for r in range(w):
        off, cnt = shard(n, r, w)
        seen.extend(range(off, off + cnt))
    assert seen == list(range(n))


def test_synthetic_junction_shapes():
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", ml=16, nmd=64, natom=30, nw=50)
    assert dyn.shape == (90, 90) and len(axyz) == 30
    assert [b.nc for b in baths] == [30, 30] and baths[0].kernel.shape == (16, 30, 30)
    assert np.allclose(dyn, dyn.T) and np.linalg.eigvalsh(dyn).min() > 0
    dyn, axyz, baths, meta = synthetic.junction("C5", ml=8, nmd=32, natom=30, nw=50)
    assert len(baths) == 3 and baths[2].kind == "ebath" and baths[2].biased()


def test_checkpoint_netcdf_roundtrip(tmp_path):
    """MD{j}.nc helpers (md.py:768-783): record (unlimited) and fixed dimensions, float64 exact,
    atomic replace."""
    from sclmd_amd import checkpoint as C

    fn = str(tmp_path / "MD0.nc")
    rng = np.random.default_rng(0)
    ps, phis = rng.normal(size=(8, 5)), rng.normal(size=(3, 5))
    f, tmp = C.open_for_write(fn)
    f.createDimension("nnmd", None)
    f.createDimension("nph", 5)
    f.createDimension("one", 1)
    f.createDimension("mem", 3)
    C.Write2NetCDFFile(f, ps, "ps", ("nnmd", "nph"), units="")
    C.Write2NetCDFFile(f, phis, "phis", ("mem", "nph"), units="")
    C.Write2NetCDFFile(f, [42], "t", ("one",), units="")
    assert not os.path.exists(fn)
    C.commit(f, tmp, fn)
    assert os.path.exists(fn) and not os.path.exists(tmp)
    assert np.array_equal(C.ReadNetCDFVar(fn, "ps"), ps)
    assert np.array_equal(C.ReadNetCDFVar(fn, "phis"), phis)
    assert C.ReadNetCDFVar(fn, "t")[0] == 42 and C.has_var(fn, "ps") and not C.has_var(fn, "qs")


def test_read_history_both_layouts(tmp_path):
    """checkpoint.read_history: the ('traj', 'mem', 'nph') layout and the record layout md.dump
    uses for ensemble histories above a classic-format variable's size give the same array."""
    from sclmd_amd import checkpoint as C

    rng = np.random.default_rng(1)
    ph = rng.normal(size=(3, 4, 5))  # (traj, ml, nph)
    for lay in ("mem", "rec", "groups"):
        fn = str(tmp_path / (lay + ".nc"))
        f, tmp = C.open_for_write(fn)
        f.createDimension("nnmd", None)
        f.createDimension("nph", 5)
        f.createDimension("mem", 4)
        f.createDimension("traj", 3)
        C.Write2NetCDFFile(f, rng.normal(size=(9, 5)), "ps", ("nnmd", "nph"), units="")  # 9 records > ml
        if lay == "rec":  # round-4 files
            C.Write2NetCDFFile(f, np.transpose(ph, (1, 0, 2)), "phis", ("nnmd", "traj", "nph"), units="")
        elif lay == "groups":  # md.dump's trajectory groups: 2 + 1 trajectories
            for k, (a, b) in enumerate(((0, 2), (2, 3))):
                f.createDimension("trajg%d" % k, b - a)
                C.Write2NetCDFFile(f, ph[a:b], "phis_g%d" % k, ("trajg%d" % k, "mem", "nph"), units="")
        else:
            C.Write2NetCDFFile(f, ph, "phis", ("traj", "mem", "nph"), units="")
        C.commit(f, tmp, fn)
        assert np.array_equal(C.read_history(fn, "phis", 4), ph), lay


def _cpu_md():
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=4, ml=4, nmd=8, nw=20)
    return MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, verbose=False, ntraj=2)


def test_background_dump_writes_and_raises_on_the_callers_thread(tmp_path, monkeypatch):
    """md.dump with async_dump: the snapshot is taken on the caller's thread and written by a
    background thread; the next join (next dump, Run end, close) sees the file, and a failed write
    leaves no partial file and raises there."""
    m = _cpu_md()
    monkeypatch.chdir(tmp_path)
    from sclmd_amd import checkpoint as C

    good = {"fn": "MD0.nc", "dims": [("nnmd", None), ("nph", 3)], "t": 5, "ipie": 0, "savep": False,
            "vars": [("ps", np.arange(12.0).reshape(4, 3), ("nnmd", "nph")), ("t", np.array([5.0]), ("nph",))]}
    monkeypatch.setattr(m, "_dump_snapshot", lambda ipie, id: good)
    m.dump(0, 0)
    m._join_dump()
    assert np.array_equal(C.ReadNetCDFVar("MD0.nc", "ps"), np.arange(12.0).reshape(4, 3))
    bad = dict(good, fn="MD1.nc", vars=[("ps", np.zeros((2, 7)), ("nph", "nnmd"))])  # wrong shape
    monkeypatch.setattr(m, "_dump_snapshot", lambda ipie, id: bad)
    m.dump(0, 1)
    with pytest.raises(RuntimeError, match="MD1.nc"):
        m._join_dump()
    assert not os.path.exists("MD1.nc") and not os.path.exists("MD1.nc.tmp")
    m._join_dump()  # the error is raised once


def test_rmnc_removes_previous_file_only_after_the_new_one_is_committed(tmp_path, monkeypatch):
    """md.Run with RemoveNC: MD{j-1}.nc goes only once MD{j}.nc is on disk (md.py:596, 676-679), also
    while MD{j}.nc is still being written by the background dump: at every moment one of the two
    files is a complete checkpoint."""
    import threading

    m = _cpu_md()
    monkeypatch.chdir(tmp_path)
    from sclmd_amd import checkpoint as C

    snap = {"fn": "MD0.nc", "dims": [("nnmd", None), ("nph", 3)], "t": 5, "ipie": 0, "savep": False,
            "vars": [("ps", np.arange(12.0).reshape(4, 3), ("nnmd", "nph"))]}
    monkeypatch.setattr(m, "_dump_snapshot", lambda ipie, id: dict(snap, fn="MD%d.nc" % id))
    m.dump(0, 0)
    m._join_dump()
    gate, seen = threading.Event(), []
    real_commit = C.commit

    def slow_commit(f, tmp, fn):  # MD1.nc's commit waits until the removal has been requested
        gate.wait(10)
        seen.append(os.path.exists("MD0.nc"))
        real_commit(f, tmp, fn)

    monkeypatch.setattr(C, "commit", slow_commit)
    m.dump(0, 1)
    m.remove_after_dump("MD0.nc")
    assert os.path.exists("MD0.nc")  # MD1.nc is not committed yet
    gate.set()
    m._join_dump()
    assert seen == [True] and os.path.exists("MD1.nc") and not os.path.exists("MD0.nc")
    m.remove_after_dump("MD1.nc")  # nothing pending: at once
    assert not os.path.exists("MD1.nc")


def test_noise_key_follows_content():
    """The noise-factor cache key changes when a spectrum array is edited in place (an id() key
    would not) and is equal for equal content in a different array."""
    from sclmd_amd import synthetic

    _, _, baths, _ = synthetic.junction("C3", seed=5, natom=4, ml=4, nmd=8, nw=20)
    b = baths[0]
    k0 = b._noise_key()
    b.gamma = np.array(b.gamma)  # new object, same content
    assert b._noise_key() == k0
    b.gamma[3, 0, 0] += 1e-12
    assert b._noise_key() != k0


@pytest.mark.parametrize("kind", ["ph", "e_bias", "e_eq"])
def test_streamed_noise_factors_cover_the_positive_part(kind):
    """noise.stream_factor_chunks (the C5 path: factors streamed to the device by frequency chunk)
    gives, at every frequency, M M^H = A(w)_+ -- the covariance vargau draws from -- including the
    shared-factor regimes (flat flinterp half-cells, single-coefficient electron regimes) and the
    Cholesky path."""
    from sclmd_amd import noise as N
    from sclmd_amd import synthetic

    rng = np.random.default_rng(3)
    dt, nmd = synthetic.DT, 64
    if kind == "ph":
        b = synthetic.make_phbath(300.0, list(range(6)), 16, nmd, rng, nw=40)
    else:
        b = synthetic.make_biased_ebath(300.0, list(range(5)), nmd, rng, bias=1.0 if kind == "e_bias" else 0.0)
    ref = b.noise_factor().scaled()  # U diag(sqrt(lambda_+)) for every frequency
    kinds = set()
    for w0, m in N.stream_factor_chunks(b, chunk=7, workers=3):
        for j in range(m.shape[0]):
            kinds.add(b._spectrum_term(w0 + j)[0])
            got = m[j] @ np.conj(m[j]).T
            want = ref[w0 + j] @ np.conj(ref[w0 + j]).T
            assert np.max(np.abs(got - want)) <= 1e-12 * max(np.max(np.abs(want)), 1e-300) + 1e-300
    assert "dense" in kinds and ("shared" in kinds or "zero" in kinds), kinds


@pytest.mark.parametrize("layout", ["build", "reference"])
def test_poweratomlist_resume_reads_either_layout(tmp_path, layout):
    """md._read_poweratomlist: this build writes ('nnmd', 'atomlist', 'two'), the
    reference ('atomlist', 'nnmd', 'two') (md.py:742-744); both read back as (natomlist, nmd, 2)."""
    from sclmd_amd import checkpoint as C
    from sclmd_amd import md as MD

    nmd, na = 16, 3
    m = MD.md(0.38, nmd, 300.0, verbose=False)
    m.AddPowerSection([[0, 1], [2], [3, 4, 5]])
    want = np.random.default_rng(1).normal(size=(na, nmd, 2))
    fn = str(tmp_path / "MD0.nc")
    f, tmp = C.open_for_write(fn)
    # NetCDF classic allows only a leading record dimension: the reference-layout file (written by
    # netCDF4 there) gets a fixed nnmd here
    f.createDimension("nnmd", None if layout == "build" else nmd)
    f.createDimension("atomlist", na)
    f.createDimension("two", 2)
    if layout == "build":
        C.Write2NetCDFFile(f, np.transpose(want, (1, 0, 2)), "poweratomlist", ("nnmd", "atomlist", "two"))
    else:
        C.Write2NetCDFFile(f, want, "poweratomlist", ("atomlist", "nnmd", "two"))
    C.commit(f, tmp, fn)
    assert np.array_equal(m._read_poweratomlist(fn), want)


def test_cpu_baseline_times_a_biased_electron_bath():
    """bench.cpu_baseline builds electron baths as electron baths: the biased
    C5 ebath's bias terms are part of the timed reference-shaped step."""
    import bench
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C5", natom=24, ml=8, nmd=32, nw=40)
    rng = np.random.default_rng(0)
    bh = []
    for b in baths:
        n = rng.normal(size=(32, b.nc)) * 1e-3
        if b.kind == "ebath":
            bh.append(("e", b.cids, b.kernel, n, dict(bias=b.bias, exim=b.exim, zeta1=b.zeta1, zeta2=b.zeta2)))
        else:
            bh.append(("ph", b.cids, b.kernel, n, {}))
    assert [k for k, *_ in bh] == ["ph", "ph", "e"]
    r = bench.cpu_baseline(bh, dyn, meta["nph"], meta["dt"], 32, budget_s=0.3, nsample=3)
    assert r["value"] > 0 and r["kind"] == "port" and len(r["samples"]) == 3
