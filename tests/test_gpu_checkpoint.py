"""GPU tests of md.Run's MD{j}.nc checkpoints (md.dump, md.py:684-764) and resume logic
(md.py:506-567): continuing from the previous run's file and resuming an unfinished run reproduce
the uninterrupted run.

Tolerance 1e-10 relative (a resumed run re-derives the memory sum from the stored history with the
priming contraction instead of the ladder blocks: rounding only)."""
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _md(nstart, nstop, npie=2, save=True, ntraj=1):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=10, ml=16, nmd=64, nw=60)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, nstart=nstart, nstop=nstop,
              npie=npie, seed=11, noise_mode="device", verbose=False, ntraj=ntraj)
    for b in baths:
        m.AddBath(b)
    m.AddConstr([range(0, 3)])
    if save:
        m.CalPowerSpec()
        m.CalAveStruct()
        m.SaveAll()
    return m


def _final(m):
    return np.array(m.p), np.array(m.q), int(m.t), np.array(m.kappa_runs)


@pytest.fixture
def uninterrupted(tmp_path_factory):
    d = tmp_path_factory.mktemp("full")
    cwd = os.getcwd()
    os.chdir(d)
    try:
        m = _md(0, 2)
        m.Run()
        res = _final(m)
        m.close()
    finally:
        os.chdir(cwd)
    return d, res


def test_dump_files(uninterrupted):
    from sclmd_amd.checkpoint import ReadNetCDFVar, has_var

    d, (p, q, t, kap) = uninterrupted
    fn = str(d / "MD1.nc")
    for v in ("energy", "p", "q", "t", "ipie", "phis", "qhis", "power", "noise0", "noise1", "ps", "qs"):
        assert has_var(fn, v), v
    assert int(ReadNetCDFVar(fn, "ipie")[0]) == 1 and int(ReadNetCDFVar(fn, "t")[0]) == t == 128
    assert rel(ReadNetCDFVar(fn, "p"), p) == 0.0 and rel(ReadNetCDFVar(fn, "q"), q) == 0.0
    assert ReadNetCDFVar(fn, "phis").shape == (16, 30) and ReadNetCDFVar(fn, "noise0").shape == (64, 9)


def test_continue_from_previous_run(uninterrupted, tmp_path, monkeypatch):
    d, (p, q, t, kap) = uninterrupted
    shutil.copy(d / "MD0.nc", tmp_path / "MD0.nc")
    monkeypatch.chdir(tmp_path)
    m = _md(1, 2)
    m.Run()
    p2, q2, t2, kap2 = _final(m)
    m.close()
    assert t2 == t
    assert rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10
    assert rel(kap2[-1], kap[-1]) < 1e-9


def test_resume_unfinished_run(uninterrupted, tmp_path, monkeypatch):
    from sclmd_amd import md as MD

    d, (p, q, t, kap) = uninterrupted
    monkeypatch.chdir(tmp_path)
    # interrupted process: run 0 complete, run 1 stops after its first piece (ipie = 0 on disk)
    real_dump = MD.md.dump

    class Stop(Exception):
        pass

    def dump_then_stop(self, ipie, id):
        real_dump(self, ipie, id)
        if id == 1 and ipie == 0:
            raise Stop()

    monkeypatch.setattr(MD.md, "dump", dump_then_stop)
    m = _md(0, 2)
    with pytest.raises(Stop):
        m.Run()
    m.close()
    monkeypatch.setattr(MD.md, "dump", real_dump)
    from sclmd_amd.checkpoint import ReadNetCDFVar

    assert int(ReadNetCDFVar("MD1.nc", "ipie")[0]) == 0
    # new process: run 0 is found finished, run 1 resumes at its second piece
    m = _md(0, 2)
    m.Run()
    p2, q2, t2, _ = _final(m)
    m.close()
    assert t2 == t
    assert rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10


def test_unfinished_run_needs_saveall(uninterrupted, tmp_path, monkeypatch):
    from sclmd_amd.checkpoint import ReadNetCDFVar  # noqa: F401

    d, _ = uninterrupted
    monkeypatch.chdir(tmp_path)
    m = _md(0, 1, save=False)
    m.Run()                       # writes MD0.nc with ipie = 1 (finished, npie = 2)
    m.close()
    m = _md(0, 1, npie=4, save=False)   # same file read as unfinished (ipie + 1 < npie)
    with pytest.raises(RuntimeError, match="saveall"):
        m.Run()
    m.close()


def test_background_dump_files_identical_to_synchronous(tmp_path, monkeypatch):
    """md.Run's MD{j}.nc written on the background thread (async_dump, the default) are byte for
    byte the files of the synchronous writer, and a run continued from such a file reproduces the
    uninterrupted run."""
    from sclmd_amd import md as MD

    outs = {}
    for mode in (True, False):
        d = tmp_path / ("async" if mode else "sync")
        d.mkdir()
        monkeypatch.chdir(d)
        monkeypatch.setattr(MD.md, "async_dump", mode)
        m = _md(0, 2, npie=2, ntraj=2)
        m.Run()
        outs[mode] = _final(m)
        m.close()
    for fn in ("MD0.nc", "MD1.nc"):
        a = (tmp_path / "async" / fn).read_bytes()
        b = (tmp_path / "sync" / fn).read_bytes()
        assert a == b, fn
    assert rel(outs[True][0], outs[False][0]) == 0.0 and rel(outs[True][1], outs[False][1]) == 0.0
    # resume from the background-written file of run 0
    cont = tmp_path / "cont"
    cont.mkdir()
    shutil.copy(tmp_path / "async" / "MD0.nc", cont / "MD0.nc")
    monkeypatch.chdir(cont)
    monkeypatch.setattr(MD.md, "async_dump", True)
    m = _md(1, 2, npie=2, ntraj=2)
    m.Run()
    p2, q2, t2, kap2 = _final(m)
    m.close()
    p, q, t, kap = outs[True]
    assert t2 == t and rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10 and rel(kap2[-1], kap[-1]) < 1e-9


def test_ensemble_history_record_layout_continues(tmp_path, monkeypatch):
    """An ensemble whose p / q histories exceed a classic-format variable (C5: 32 x 4096 x 3000
    doubles) stores them as fixed-size trajectory groups (exactly ml rows each); continuing from that file reproduces the
    uninterrupted run (the limit is lowered here so a small ensemble takes that layout)."""
    from sclmd_amd import md as MD
    from sclmd_amd.checkpoint import read_history, var_dims

    monkeypatch.setattr(MD.md, "nc_var_limit", 0)
    full = tmp_path / "full"
    full.mkdir()
    monkeypatch.chdir(full)
    m = _md(0, 2, ntraj=3)
    m.Run()
    p, q, t, kap = _final(m)
    ph = np.array(m.phis)
    m.close()
    # one fixed-size variable per trajectory group (the limit of 0 puts one trajectory in each)
    from sclmd_amd.checkpoint import has_var

    assert not has_var(str(full / "MD0.nc"), "phis")
    assert [var_dims(str(full / "MD0.nc"), "phis_g%d" % k) for k in range(3)] == \
        [("trajg%d" % k, "mem", "nph") for k in range(3)]
    assert rel(read_history(str(full / "MD1.nc"), "phis", 16), ph) == 0.0
    cont = tmp_path / "cont"
    cont.mkdir()
    shutil.copy(full / "MD0.nc", cont / "MD0.nc")
    monkeypatch.chdir(cont)
    m = _md(1, 2, ntraj=3)
    m.Run()
    p2, q2, t2, kap2 = _final(m)
    m.close()
    assert t2 == t and rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10 and rel(kap2[-1], kap[-1]) < 1e-9


def test_full_history_getter_matches_host_composition(tmp_path, monkeypatch):
    """gle_get_full_history (the dump's one device read: recorded p / q histories with every bath's
    own ring on its DOFs, transposed on the device, optionally into page-locked buffers) equals the
    host composition md.phis / md.qhis make from gle_get_record_history and gle_get_history --
    before md.Run (no recording: bath rings only), and after it (recorded), with an extra bath of
    shorter memory overlapping another's DOFs (the later bath wins on its rows)."""
    from sclmd_amd import synthetic

    monkeypatch.chdir(tmp_path)
    m = _md(0, 1, npie=1, ntraj=3)
    b0 = m.baths[0]
    extra = synthetic.make_phbath(m.T, sorted({int(c) for c in b0.cids[:6]} | {0, 1}), 4, m.nmd, np.random.default_rng(3),
                                  dt=m.dt, nw=60)
    m.AddBath(extra)
    m.initialise()
    m.ResetHis()
    for i in range(len(m.baths)):
        m.gen_noise(i, 0)
    m.steps(40)
    for pinned in (False, True):
        ph, qh = m._histories(pinned=pinned)
        assert np.array_equal(ph, m.phis) and np.array_equal(qh, m.qhis)
    assert np.abs(qh).max() == 0.0 and np.abs(ph).max() > 0.0
    m.Run()
    for pinned in (False, True):
        ph, qh = m._histories(pinned=pinned)
        assert np.array_equal(ph, m.phis) and np.array_equal(qh, m.qhis)
    assert np.abs(qh).max() > 0.0
    m.close()


def test_wide_ensemble_continue_and_resume(tmp_path, monkeypatch):
    """40 trajectories (partial column tiles of every product width): continuing from the previous run's
    MD0.nc and resuming an unfinished run 1 both reproduce the uninterrupted run."""
    from sclmd_amd import md as MD

    full = tmp_path / "full"
    full.mkdir()
    monkeypatch.chdir(full)
    m = _md(0, 2, ntraj=40)
    m.Run()
    p, q, t, kap = _final(m)
    m.close()
    cont = tmp_path / "cont"
    cont.mkdir()
    shutil.copy(full / "MD0.nc", cont / "MD0.nc")
    monkeypatch.chdir(cont)
    m = _md(1, 2, ntraj=40)
    m.Run()
    p2, q2, t2, kap2 = _final(m)
    m.close()
    assert t2 == t and rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10 and rel(kap2[-1], kap[-1]) < 1e-9

    res = tmp_path / "resume"
    res.mkdir()
    monkeypatch.chdir(res)
    real_dump = MD.md.dump

    class Stop(Exception):
        pass

    def dump_then_stop(self, ipie, id):
        real_dump(self, ipie, id)
        if id == 1 and ipie == 0:
            raise Stop()

    monkeypatch.setattr(MD.md, "dump", dump_then_stop)
    m = _md(0, 2, ntraj=40)
    with pytest.raises(Stop):
        m.Run()
    m.close()
    monkeypatch.setattr(MD.md, "dump", real_dump)
    m = _md(0, 2, ntraj=40)
    m.Run()
    p3, q3, t3, _ = _final(m)
    m.close()
    assert t3 == t and rel(q3, q) < 1e-10 and rel(p3, p) < 1e-10
