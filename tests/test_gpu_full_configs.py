"""The benched configurations themselves against the oracle (VERDICT r01 "benched but never tested").

C3 as benched: 300-atom junction, 2 phonon baths nc = 300, ml = 1024, 64 trajectories with the
spectral ladder plan bench.py runs (levels P = 8 ... 256 at the default first block length, and
P = 4 ... 256 at block_len = 4; far-field GEMM chunks of 2 workgroups per CU), started
at an unaligned t0 from a random nonzero history, run 540 steps so that every level's blocks are
computed from nonzero data (the P = 256 level fires at 256 and 512).  Reduced C5: three baths (two
phonon baths and a biased electron bath with exim, zeta1, zeta2 != 0, nc = 96-99), ml = 1024, 32
trajectories, same protocol.  Three trajectories of each batch are checked against the batched
oracle (oracle.GLEBatch, pinned to the reference-shaped oracle and the reference's fixtures):
1e-9 relative on q, p and the heat currents.  The noise period is 1024 (the period does not enter
the ladder plan; wrap-around is covered in test_gpu_md.py).

The large-bath plan (any bath with nc > 512: first block length 4 with a direct P = 4 level, the
8-wave fused velocity stage, the fpot launch, split-K far-field GEMM chunks of 4 workgroups per CU)
is what bench.py runs at C5 (nc = 999 / 1002).  It is checked twice against the oracle: at nc = 522
(natom 522, ml = 512,
picked by the automatic rule), and at the reduced C5 size with the plan class forced through the
ABI (gle_set_plan_class), so both plan classes meet the same biased three-bath junction."""
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


def _expected_levels(P0, ml, pmax=256):
    """The ladder's block lengths: P = P0 2^l while 2P < ml, the last one at 4P >= ml or P = pmax."""
    out, P = [], P0
    while 2 * P < ml:
        out.append(P)
        if P >= pmax or 4 * P >= ml:
            break
        P *= 2
    return out


def _run_vs_oracle(config, natom, B, check, t0=37, nst=540, nmd=1024, ml=1024, seed=1234, block_len=0,
                   plan_class="auto", expect_class="small"):
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
        st.set_plan_class(plan_class)
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
        detail = st.plan_detail()
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
    # the plan class and what it sets: first block length, fused-stage waves, GEMM chunking
    assert detail["plan_class"] == expect_class, detail
    P0 = info["block_len"]
    assert P0 == (block_len or (8 if expect_class == "small" else 4)), info
    assert detail["fused_waves"] == (4 if expect_class == "small" else 8), detail
    assert detail["fpot_launch"] == (expect_class == "large"), detail
    assert detail["cg_per_cu"] == (2.0 if expect_class == "small" else 4.0), detail
    # every ladder level computed blocks inside the run (P = P0 ... 256 at ml = 1024)
    assert [P for P, _ in levels] == _expected_levels(P0, ml), levels
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


def test_c5_reduced_large_plan_forced_vs_oracle():
    """The large-bath plan at nc ~ 96: P0 = 4 (direct P = 4 level, spectral P = 8 ... 256), 8-wave
    fused stage, 2 GEMM workgroups per CU per chunk."""
    sim = _run_vs_oracle("C5", 96, 32, [0, 17, 31], plan_class="large", expect_class="large")
    assert sum(b.biased() for b in sim.baths) == 1


def test_c5_nc522_large_plan_vs_oracle():
    """nc = 522 > 512 on all three baths (two phonon baths and the biased electron bath): the plan
    class the automatic rule picks at C5 (nc = 999 / 1002), ml = 512 (levels P = 4 ... 128, the P =
    128 level fires at 128 and 256), 300 steps from an unaligned t0 and a random history."""
    sim = _run_vs_oracle("C5", 522, 32, [0, 17, 31], ml=512, nst=300, expect_class="large")
    assert [b.nc for b in sim.baths] == [522, 522, 522]
    assert sum(b.biased() for b in sim.baths) == 1


def test_c3_small_plan_forced_matches_auto_expectation():
    """Forcing the small-bath class where it is already the automatic choice changes nothing."""
    _run_vs_oracle("C3", 48, 16, [0, 15], nst=540, plan_class="small", expect_class="small")
