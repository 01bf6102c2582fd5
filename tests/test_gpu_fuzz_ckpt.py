"""Seeded random md.Run checkpoint / resume cases (md.dump, md.py:684-764; resume, md.py:506-567): a
run interrupted right after the dump of a random piece of a random run, then a new process (a new
md) started in the same directory, ends where the uninterrupted run ends (1e-10 on p and q, 1e-9 on
every run's kappa).  Each case draws the junction size, the ensemble width (composed and two-launch
plans), the baths (memory lengths, a biased electron bath), constraints, npie and the number of
runs; device noise (trajectory-keyed, so the resumed run regenerates the same realisations)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NCASE = int(os.environ.get("SCLMD_FUZZ_CKPT", "8"))  # a wider sweep: SCLMD_FUZZ_CKPT=40


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _case(seed):
    r = np.random.default_rng(9000 + seed)
    return dict(natom=int(r.integers(6, 16)), ntraj=int(r.choice([1, 3, 40])), ml=int(r.choice([1, 8, 24])),
                ebath=bool(r.random() < 0.5), constr=bool(r.random() < 0.6), npie=int(r.choice([2, 4])),
                nrun=int(r.integers(2, 4)), stop_run=None, stop_piece=None, seed=seed, r=r)


def _md(c, nstart=0):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    cfg = "C5" if c["ebath"] else "C3"
    dyn, axyz, baths, meta = synthetic.junction(cfg, seed=5 + c["seed"], natom=c["natom"], ml=max(c["ml"], 1),
                                                nmd=64, nw=60)
    m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, nstart=nstart, nstop=c["nrun"],
              npie=c["npie"], ntraj=c["ntraj"], seed=3, noise_mode="device", verbose=False)
    for b in baths:
        m.AddBath(b)
    if c["constr"]:
        m.AddConstr([range(0, 3)])
    m.CalPowerSpec()
    m.CalAveStruct()
    m.SaveAll()
    return m


@pytest.mark.parametrize("seed", range(NCASE))
def test_random_interrupt_and_resume(seed, tmp_path, monkeypatch):
    from sclmd_amd import md as MD

    c = _case(seed)
    r = c["r"]
    stop_run, stop_piece = int(r.integers(0, c["nrun"])), int(r.integers(0, c["npie"]))
    full = tmp_path / "full"
    full.mkdir()
    monkeypatch.chdir(full)
    m = _md(c)
    m.Run()
    p, q, kap = np.array(m.p), np.array(m.q), np.array(m.kappa_runs)
    m.close()

    part = tmp_path / "part"
    part.mkdir()
    monkeypatch.chdir(part)
    real_dump = MD.md.dump

    class Stop(Exception):
        pass

    def dump_then_stop(self, ipie, id):
        real_dump(self, ipie, id)
        if id == stop_run and ipie == stop_piece:
            raise Stop()

    monkeypatch.setattr(MD.md, "dump", dump_then_stop)
    m = _md(c)
    with pytest.raises(Stop):
        m.Run()
    m.close()
    monkeypatch.setattr(MD.md, "dump", real_dump)
    m = _md(c)
    m.Run()
    p2, q2, kap2 = np.array(m.p), np.array(m.q), np.array(m.kappa_runs)
    m.close()
    desc = "case %s stop run %d piece %d" % ({k: v for k, v in c.items() if k != "r"}, stop_run, stop_piece)
    last = c["nrun"] - 1
    if stop_run == last and stop_piece == c["npie"] - 1:
        # every run was finished: the new process only finds the files (md.py:537-544) and steps
        # nothing; the last file holds the uninterrupted final state
        from sclmd_amd.checkpoint import ReadNetCDFVar

        fn = "MD%d.nc" % last
        assert len(kap2) == 0, desc
        assert rel(ReadNetCDFVar(str(part / fn), "q"), ReadNetCDFVar(str(full / fn), "q")) == 0.0, desc
        assert rel(ReadNetCDFVar(str(part / fn), "p"), ReadNetCDFVar(str(full / fn), "p")) == 0.0, desc
        return
    assert rel(q2, q) < 1e-10 and rel(p2, p) < 1e-10, (desc, rel(q2, q), rel(p2, p))
    # kappa of the resumed run covers only the steps this process ran (the reference keeps no
    # bath.cur in MD{j}.nc, md.py:506-535, 684-764); runs after it are whole and equal
    if stop_run < last:
        assert rel(kap2[-1], kap[-1]) < 1e-9, desc
