"""The benched configurations themselves against the oracle (VERDICT r01 "benched but never tested").

C3 as benched: 300-atom junction, 2 phonon baths nc = 300, ml = 1024, 64 trajectories with the
spectral ladder plan bench.py runs (levels P = 8 ... 256 at the default first block length, and
P = 4 ... 256 at block_len = 4; split-K cgemm items), started
at an unaligned t0 from a random nonzero history, run 540 steps so that every level's blocks are
computed from nonzero data (the P = 256 level fires at 256 and 512).  Reduced C5: three baths (two
phonon baths and a biased electron bath with exim, zeta1, zeta2 != 0, nc = 96-99), ml = 1024, 32
trajectories, same protocol.  Three trajectories of each batch are checked against the batched
oracle (oracle.GLEBatch, pinned to the reference-shaped oracle and the reference's fixtures):
1e-9 relative on q, p and the heat currents.  The noise period is 1024 (the period does not enter
the ladder plan; wrap-around is covered in test_gpu_md.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-9


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _obath(O, b, noise, dt, nmd):
    if b.kind == "ebath":
        return O.Bath("e", b.cids, b.kernel, noise, dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1,
                      zeta2=b.zeta2)
    return O.Bath("ph", b.cids, b.kernel, noise, dt, nmd)


def _run_vs_oracle(config, natom, B, check, t0=37, nst=540, nmd=1024, ml=1024, seed=1234, block_len=0):
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction(config, natom=natom, ml=ml, nmd=nmd, seed=seed)
    nph, dt = meta["nph"], meta["dt"]
    st = N.Stepper(nph, B, nmd, dt, 0, block_len, "auto", 0)
    try:
        for b in baths:
            if b.kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        rng = np.random.default_rng(seed + 1)
        p = rng.normal(size=(B, nph)) * 1e-3
        q = rng.normal(size=(B, nph)) * 1e-3
        st.set_state(p, q, t0)
        hist, noise = [], []
        for i, b in enumerate(baths):
            h = rng.normal(size=(B, b.ml, b.nc)) * 1e-3
            n = rng.normal(size=(B, nmd, b.nc)) * 1e-3
            st.set_history(i, h)
            st.set_noise(i, n)
            hist.append(h[check])
            noise.append(n[check])
        info = st.plan_info()
        assert info["far_mode"] == "spectral", info
        st.profile(True)
        st.run(nst)
        levels = st.profile_levels()
        pg, qg, t = st.get_state()
        cur = st.get_current()
        st.profile(False)
    finally:
        st.close()
    assert t == t0 + nst
    # every ladder level computed blocks inside the run (P = P0 ... 256 at ml = 1024)
    P0 = info["block_len"]
    assert P0 == (block_len or 8), info
    assert [P for P, _ in levels] == [P0 << k for k in range((256 // P0).bit_length())], levels
    assert all(bl >= 1.0 for _, bl in levels), levels
    ob = [_obath(O, b, noise[i], dt, nmd) for i, b in enumerate(baths)]
    sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=len(check))
    sim.p, sim.q, sim.t = p[check].T.copy(), q[check].T.copy(), t0
    for i in range(len(baths)):
        sim.set_history(i, hist[i])
    for _ in range(nst):
        sim.step()
    steps = (t0 + np.arange(nst)) % nmd
    for j, b_ in enumerate(check):
        assert rel(qg[b_], sim.q[:, j]) < TOL, (b_, rel(qg[b_], sim.q[:, j]))
        assert rel(pg[b_], sim.p[:, j]) < TOL, (b_, rel(pg[b_], sim.p[:, j]))
        for i in range(len(baths)):
            assert rel(cur[i, b_, steps], sim.cur[i][j, steps]) < TOL, (b_, i)
    return sim


@pytest.mark.parametrize("block_len", [0, 4])
def test_c3_bench_plan_vs_oracle(block_len):
    _run_vs_oracle("C3", None, 64, [0, 29, 63], block_len=block_len)


def test_c5_reduced_biased_vs_oracle():
    sim = _run_vs_oracle("C5", 96, 32, [0, 17, 31])
    assert sum(b.biased() for b in sim.baths) == 1
