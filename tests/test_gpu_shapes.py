"""Plan classes x ensemble widths against the oracle.  The plans pick tile widths from B (16-, 32- and
64-column products, partial last column tiles, split DOF tiles below 128 tiles, audit words of 16
trajectories) and from the bath size (small- or large-bath plan); the benched shapes are B = 64 (C3)
and B = 32 (C5).  A 40-trajectory ensemble once planned a 48-column product width that the kernels
do not have (profiles/r06/bwidth), so every plan class runs here at widths across those boundaries:
composed or two-launch steps, a segment with a host force (md.potforce on the host), constraints,
levels firing at ml = 96, against oracle.GLEBatch at 1e-10."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-10


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _run(B, plan_class, far_mode="auto", constr=None, natom=40, ml=96, nmd=256, seed=11, config="C3",
         trim=None, scatter=None):
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction(config, natom=natom, ml=ml, nmd=nmd, nw=60, seed=seed)
    nph, dt = meta["nph"], meta["dt"]
    if scatter is not None:  # phonon baths on scattered DOF sets (non-affine DOF maps in the tiles)
        r = np.random.default_rng(seed + 7)
        perm = r.permutation(nph)
        d0, d1 = np.sort(perm[:37]), np.sort(perm[37:66])
        if scatter == "overlap":
            d1 = np.sort(np.concatenate([d1[:20], d0[:9]]))
        elif scatter == "unsorted":
            d0, d1 = perm[:37], perm[37:66]
        baths = [synthetic.make_phbath(300.0, list(map(int, d)), ml, nmd, r, nw=60) for d in (d0, d1)]
    if trim is not None:  # bath i's memory kernel cut to its first m lags
        i, m = trim
        baths[i].kernel = np.ascontiguousarray(baths[i].kernel[:m])
    st = N.Stepper(nph, B, nmd, dt, 0, 0, far_mode, 0)
    try:
        for b in baths:
            if b.kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        if constr is not None:
            st.set_constraint(constr)
        st.set_plan_class(plan_class)
        rng = np.random.default_rng(seed)
        p = rng.normal(size=(B, nph)) * 1e-2
        q = rng.normal(size=(B, nph)) * 1e-2
        if constr is not None:
            p[:, constr] = 0.0
            q[:, constr] = 0.0
        noise = [rng.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
        hist = [rng.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
        st.set_state(p, q, 5)
        for i in range(len(baths)):
            st.set_history(i, hist[i])
            st.set_noise(i, noise[i])
        ob = [O.Bath("e", b.cids, b.kernel, noise[i], dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1, zeta2=b.zeta2)
              if b.kind == "ebath" else O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)]
        sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=B,
                         constr=None if constr is None else [range(int(c), int(c) + 1) for c in constr])
        sim.p, sim.q, sim.t = p.T.copy(), q.T.copy(), 5
        for i in range(len(baths)):
            sim.set_history(i, hist[i])
        detail = st.plan_detail()
        st.run(37)
        for _ in range(37):
            sim.step()
        for _ in range(3):  # host force: the two-launch path
            qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
            st.step_end(-(qt @ dyn.T))
            sim.step()
        st.run(61)
        for _ in range(61):
            sim.step()
        pg, qg, t = st.get_state()
        cur = st.get_current()
        audit = st.cache_audit()
    finally:
        st.close()
    assert t == 5 + 101
    assert rel(qg, sim.q.T) < TOL and rel(pg, sim.p.T) < TOL, (rel(qg, sim.q.T), rel(pg, sim.p.T))
    steps = (5 + np.arange(101)) % nmd
    want = np.stack([c[:, steps] for c in sim.cur])
    assert rel(cur[:, :, steps], want) < 1e-9
    assert audit == (0, 0)
    return detail


@pytest.mark.parametrize("B", [1, 3, 8, 17, 40, 64, 100])
def test_large_bath_plan_widths_vs_oracle(B):
    """The large-bath plan (C5's: first block length 4, the potential-force launch between A and the
    fused velocity stage, split far-field GEMMs) forced on a small junction at several widths."""
    d = _run(B, "large")
    assert d["plan_class"] == "large" and d["fpot_launch"] and not d["composed_step"], d


@pytest.mark.parametrize("B", [24, 40, 96])
def test_small_bath_plan_widths_with_constraints_vs_oracle(B):
    """The small-bath plan (composed step) with constrained DOFs inside and outside the baths."""
    d = _run(B, "small", constr=[0, 1, 2, 60, 61, 119])
    assert d["plan_class"] == "small" and d["composed_step"], d


@pytest.mark.parametrize("B", [8, 40])
def test_direct_ladder_widths_vs_oracle(B):
    """far_mode direct: every ladder level a contraction (the spectral levels' transforms and GEMMs
    out of the plan)."""
    d = _run(B, "auto", far_mode="direct")
    assert d["composed_step"], d


@pytest.mark.parametrize("plan_class", ["small", "large"])
@pytest.mark.parametrize("B", [8, 40])
def test_biased_electron_bath_widths_vs_oracle(plan_class, B):
    """C5's bath mix at a small size: two phonon baths and a biased electron bath (exim, zeta1, zeta2
    != 0: the baths.py:233 bias terms), both plan classes (the biased bath keeps the two-launch path)."""
    d = _run(B, plan_class, config="C5")
    assert d["plan_class"] == plan_class and not d["composed_step"], d


@pytest.mark.parametrize("plan_class", ["small", "large"])
@pytest.mark.parametrize("ml", [1, 2, 3, 7, 17, 40])
def test_memory_lengths_vs_oracle(plan_class, ml):
    """Short memory kernels: ml = 1 (no memory: c = 1, baths.py:454-457), lengths inside the near field
    (ml < 2 P0: no ladder level) and just past the first levels, both plan classes, B = 8 and 40."""
    for B in (8, 40):
        _run(B, plan_class, ml=ml)


@pytest.mark.parametrize("plan_class", ["small", "large"])
@pytest.mark.parametrize("trim", [(0, 1), (1, 5), (0, 33)])
def test_mixed_memory_lengths_vs_oracle(plan_class, trim):
    """Baths of different memory lengths in one plan (one without memory, one inside the near field,
    one with ladder levels the other lacks)."""
    for B in (8, 40):
        _run(B, plan_class, trim=trim)


@pytest.mark.parametrize("plan_class", ["small", "large"])
@pytest.mark.parametrize("scatter", ["disjoint", "overlap", "unsorted"])
def test_scattered_bath_dofs_vs_oracle(plan_class, scatter):
    """Baths on scattered DOF sets: sorted and disjoint (composed step with non-affine DOF maps), two
    baths sharing 9 DOFs (the two-launch path; exlist / mf of noise.py), and cids in no order."""
    for B in (8, 40):
        d = _run(B, plan_class, scatter=scatter)
        assert d["composed_step"] == (plan_class == "small" and scatter != "overlap"), d


@pytest.mark.parametrize("B", [1008, 1009])
def test_widest_composed_ensembles_vs_oracle(B):
    """The composed step's audit holds ceil(B / 16) words and the stop word in one wave's 64 lanes, so
    B = 1008 is the widest composed plan and B = 1009 takes the two-launch plan."""
    d = _run(B, "small")
    assert d["composed_step"] == (B <= 1008), d


def test_widest_composed_audit_replays_vs_oracle():
    """B = 1008 with near-rest trajectories in the first and the last audit word (lanes 0 and 62; the
    stop word in lane 63): the run stops at the kick and is replayed on the two-launch path."""
    import test_gpu_composed as C

    st, sim = C._at_rest_setup(1008, kick=31, rest=[3, 1007])
    assert st.plan_detail()["composed_step"]
    st.run(45)
    for _ in range(45):
        sim.step()
    C._check(st, sim, 45)
    assert st.cache_audit()[0] >= 2
    st.close()


@pytest.mark.parametrize("plan_class,scatter", [("small", "overlap"), ("large", "overlap"), ("small", None),
                                                ("large", None)])
def test_device_steps_after_host_force_with_constraints(plan_class, scatter):
    """Device steps after steps with a host force, with constrained DOFs: md.potforce's cache then holds
    the host's force at q~, and the next device step's id0 call at q_{t+1} (q~ with the constrained
    DOFs zeroed) must miss it.  The velocity stage used to leave that step's cache distance unwritten
    after a host force, so the device reused the force at q~ (1e-5 error; found by
    tests/test_gpu_fuzz.py).  Three-launch (overlapping baths), fused and composed plans."""
    for B in (3, 40):
        _run(B, plan_class, constr=[0, 1, 2, 60, 61, 119], scatter=scatter)


@pytest.mark.parametrize("plan_class", ["small", "large"])
def test_three_baths_in_one_tile_vs_oracle(plan_class):
    """A tiny junction (24 DOFs) whose DOF tiles meet all three baths, each a few k-steps wide: more
    short product runs per tile than the even wave split holds (it failed to plan, 'too many k-step
    runs per wave', found by tests/test_gpu_fuzz_ckpt.py); the waves then take whole runs."""
    for B in (3, 40):
        _run(B, plan_class, config="C5", natom=8, ml=24)


@pytest.mark.parametrize("plan_class", ["small", "large"])
def test_memory_longer_than_run_vs_oracle(plan_class):
    """ml > nmd (a memory kernel longer than the noise period; nothing in the reference forbids it):
    the history ring is sized by ml, the noise index wraps by nmd."""
    for B in (3, 40):
        _run(B, plan_class, ml=200, nmd=64)
