"""The ensemble reduce on the device (SURVEY.md 8b gle_reduce_current, 8e), both implementations:

* the C-ABI's own RCCL communicator: gle_comm_unique_id -> gle_comm_init(1 rank) ->
  gle_reduce_current / gle_comm_allreduce, and md.Run with comm = that communicator;
* torch.distributed with the nccl backend (RCCL) at world size 1, in-process, md.Run with
  comm = None inside the initialised default group.

At one rank every all-reduce is the identity, so each result must equal the handle's own
gle_current_sums / the comm-free run exactly (fp64 sums of one addend).  Multi-rank semantics of the
same code paths are covered by tests/test_distributed_gloo.py (2 gloo ranks) and the sharding
invariance test in test_gpu_md.py.  Replaces the reference's sequential ensemble and post-hoc
average: md.py:506, 657-664; tools.py:191-201."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _small_stepper(N, steps=40):
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C5", natom=12, ml=32, nmd=64, nw=40, seed=3)
    st = N.Stepper(meta["nph"], 4, meta["nmd"], meta["dt"], 0)
    for b in baths:
        if b.kind == "ebath":
            st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
        else:
            st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    rng = np.random.default_rng(9)
    st.set_state(rng.normal(size=(4, meta["nph"])) * 1e-3, rng.normal(size=(4, meta["nph"])) * 1e-3, 0)
    for i, b in enumerate(baths):
        st.set_history(i, None)
        st.set_noise(i, rng.normal(size=(4, meta["nmd"], b.nc)) * 1e-3)
    st.run(steps)
    return st, len(baths)


def test_gle_comm_single_rank_reduce():
    from sclmd_amd import _native as N

    uid = N.comm_unique_id()
    assert isinstance(uid, bytes) and len(uid) == N.COMM_ID_BYTES
    comm = N.Comm(1, 0, 0, uid)
    st, nb = _small_stepper(N)
    try:
        own = st.current_sums()
        assert own.shape == (nb, 3) and np.all(own[:, 2] == 4) and np.all(np.isfinite(own))
        assert np.any(own[:, 0] != 0.0)
        red = st.reduce_current(comm)          # gle_reduce_current over the 1-rank communicator
        alone = st.reduce_current(None)         # no communicator: this handle's sums
        assert np.array_equal(red, own) and np.array_equal(alone, own)
        v = np.linspace(-1.0, 2.0, 37)
        assert np.array_equal(st.comm_allreduce(comm, v), v)
        assert np.array_equal(st.comm_allreduce(None, v), v)
    finally:
        st.close()
        comm.close()
    assert comm.c is None


def _run_md(tmp_path, comm, tag):
    from sclmd_amd import md as MD
    from sclmd_amd import synthetic

    d = tmp_path / tag
    d.mkdir()
    cwd = os.getcwd()
    os.chdir(d)
    try:
        dyn, axyz, baths, meta = synthetic.junction("C3", seed=5, natom=12, ml=64, nmd=128, nw=80)
        m = MD.md(meta["dt"], meta["nmd"], meta["T"], axyz=axyz, dyn=dyn, ntraj=8, seed=41, nstart=0, nstop=2,
                  noise_mode="device", comm=comm, verbose=False)
        for b in baths:
            m.AddBath(b)
        m.AddPowerSection([[0, 1, 2], [3, 4, 5]])
        m.CalPowerSpec()
        m.Run()
        kap = np.array(m.kappa_runs)
        p, q = np.array(m.p), np.array(m.q)
        power, rows = m.power_spectra()
        files = sorted(os.listdir("."))
        m.close()
    finally:
        os.chdir(cwd)
    return kap, p, q, power, rows, files


def test_md_run_with_gle_comm_matches_plain(tmp_path):
    """md.Run with comm = the C-ABI's RCCL communicator: the per-run reduce goes through
    gle_reduce_current and the power-spectrum average through gle_comm_allreduce; one rank gives the
    comm-free run bit for bit."""
    from sclmd_amd import _native as N

    comm = N.Comm(1, 0, 0, N.comm_unique_id())
    try:
        a = _run_md(tmp_path, comm, "gle")
    finally:
        comm.close()
    b = _run_md(tmp_path, None, "plain")
    assert a[0].shape == (2, 2) and np.all(np.isfinite(a[0]))
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(x, y)
    assert all(np.array_equal(x, y) for x, y in zip(a[4], b[4]))
    assert a[5] == b[5] and "kappa.300.0.bath0.run1.dat" in a[5]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_md_run_torch_nccl_world1_matches_plain(tmp_path):
    """torch.distributed nccl (RCCL) process group of one rank: md.Run's reduce is a real RCCL
    all-reduce on the stepper's device (ensemble.allreduce_sums), equal to the run without a group.
    Run in a child process that initialises torch's HIP context before the library's (as a torchrun
    rank does); the parent runs the same md without a group and compares."""
    import json
    import subprocess
    import sys

    b = _run_md(tmp_path, None, "plain")
    out = tmp_path / "nccl.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "nccl_child.py"), str(tmp_path),
                        str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["backend"] == "nccl" and info["world"] == 1 and info["allreduce_identity"]
    a = np.load(out)
    for k, y in zip(["kap", "p", "q", "power"], b[:4]):
        assert np.array_equal(a[k], y), k
    assert all(np.array_equal(a["row%d" % i], y) for i, y in enumerate(b[4]))
    assert json.loads(str(a["files"])) == b[5]
