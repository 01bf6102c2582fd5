"""The composed one-launch step (GLE_PLAN_COMPOSED_STEP, gle_internal.h): small-bath harmonic plans
run md.vv (md.py:367-411) as ONE chain launch per step -- p_{t+1} from precomputed composed operators,
q_{t+1} = q~ from the step's own K0.p_t and dyn.q_t.  Checked against the batched oracle
(oracle.GLEBatch, pinned to the reference-shaped oracle and the reference's fixtures) at 1e-10 on q,
p and the heat currents, across the switches the plan has to survive: steps with a host force in
between (the two-launch path, then back), a new noise realisation mid-run, constraints, and a history
ring / ladder that every level fires on.  md.potforce's 1e-9 cache reuse (md.py:767-779) is counted
by gle_cache_audit: zero on these runs, nonzero on a system at rest."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-10


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _setup(B, natom=40, ml=96, nmd=256, seed=3, constr=None):
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C3", natom=natom, ml=ml, nmd=nmd, nw=60, seed=seed)
    nph, dt = meta["nph"], meta["dt"]
    st = N.Stepper(nph, B, nmd, dt, 0)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    if constr is not None:
        st.set_constraint(constr)
    rng = np.random.default_rng(seed)
    p = rng.normal(size=(B, nph)) * 1e-2
    q = rng.normal(size=(B, nph)) * 1e-2
    noise = [rng.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
    hist = [rng.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
    st.set_state(p, q, 0)
    for i in range(len(baths)):
        st.set_history(i, hist[i])
        st.set_noise(i, noise[i])
    ob = [O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd) for i, b in enumerate(baths)]
    sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=B,
                     constr=None if constr is None else [range(int(c), int(c) + 1) for c in constr])
    sim.p, sim.q = p.T.copy(), q.T.copy()
    for i in range(len(baths)):
        sim.set_history(i, hist[i])
    return st, sim, baths, ob, meta, dyn, rng


def _check(st, sim, nst_total):
    p, q, t = st.get_state()
    assert t == nst_total
    assert rel(q, sim.q.T) < TOL and rel(p, sim.p.T) < TOL, (rel(q, sim.q.T), rel(p, sim.p.T))
    cur = st.get_current()[:, :, :nst_total]
    want = np.stack([c[:, :nst_total] for c in sim.cur])
    assert rel(cur, want) < 1e-9


def test_composed_plan_is_the_c3_bench_plan():
    """The benched C3 shape (B = 64, spectral ladder) plans the composed step."""
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    dyn, _, baths, meta = synthetic.junction("C3")
    st = N.Stepper(meta["nph"], 64, meta["nmd"], meta["dt"], 0)
    for b in baths:
        st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
    st.set_dyn(dyn)
    st.set_state(np.zeros((64, meta["nph"])), np.zeros((64, meta["nph"])), 0)
    d = st.plan_detail()
    st.close()
    assert d["composed_step"] and d["plan_class"] == "small" and not d["split_tiles"]


@pytest.mark.parametrize("B", [8, 3, 40, 50])
def test_composed_vs_oracle_with_path_switches(B):
    """Composed steps, then steps with a host force (the two-launch path), then composed steps again,
    a new noise realisation, more composed steps: every segment against the oracle.  B = 8 plans a
    spectral ladder, B = 3 a direct one; B = 40 and 50 a partial last column tile of the 64-column
    near-field and far-field products (B in (32, 48] once planned a 48-column width those products do
    not have)."""
    st, sim, baths, ob, meta, dyn, rng = _setup(B)
    assert st.plan_detail()["composed_step"]
    nst = 0
    st.run(37)
    for _ in range(37):
        sim.step()
    nst += 37
    _check(st, sim, nst)
    for _ in range(5):  # host driver steps: md.potforce evaluated on the host (-dyn.q)
        qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
        st.step_end(-(qt @ dyn.T))
        sim.step()
    nst += 5
    _check(st, sim, nst)
    st.run(70)  # crosses level boundaries (P up to 32 at ml = 96)
    for _ in range(70):
        sim.step()
    nst += 70
    _check(st, sim, nst)
    for i, b in enumerate(baths):  # a new run's noise (md.py:569-570)
        n = rng.normal(size=(B, meta["nmd"], b.nc)) * 1e-3
        st.set_noise(i, n)
        ob[i].noise = n
    st.run(41)
    for _ in range(41):
        sim.step()
    nst += 41
    _check(st, sim, nst)
    assert st.cache_audit() == (0, 0)
    st.close()


@pytest.mark.parametrize("B", [1, 2])
def test_split_tiles_vs_oracle(B):
    """Few DOF tiles (small B): each tile's products split over workgroups, the last arriver adding
    the slabs in fixed order (GLE_PLAN_SPLIT_TILES, xsub_combine in gle_chain.hip); 130 steps across
    level boundaries, a host-force segment and a new noise realisation, against the oracle."""
    st, sim, baths, ob, meta, dyn, rng = _setup(B, natom=120)
    d = st.plan_detail()
    assert d["composed_step"] and d["split_tiles"]
    st.run(61)
    for _ in range(61):
        sim.step()
    _check(st, sim, 61)
    for _ in range(3):
        qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
        st.step_end(-(qt @ dyn.T))
        sim.step()
    for i, b in enumerate(baths):
        n = rng.normal(size=(B, meta["nmd"], b.nc)) * 1e-3
        st.set_noise(i, n)
        ob[i].noise = n
    st.run(66)
    for _ in range(66):
        sim.step()
    _check(st, sim, 130)
    st.close()


def test_one_trajectory_split_valu_with_constraints_vs_oracle():
    """B = 1: split DOF tiles on the one-column VALU stage (chain stage 5) with constrained DOFs in and
    out of the baths (ApplyConstraint in the last arriver's epilogue), 150 steps against the oracle."""
    st, sim, *_ = _setup(1, natom=120, constr=[0, 1, 2, 150, 151, 300])
    d = st.plan_detail()
    assert d["composed_step"] and d["split_tiles"]
    st.run(150)
    for _ in range(150):
        sim.step()
    _check(st, sim, 150)
    st.close()


def test_composed_with_constraints_vs_oracle():
    """ApplyConstraint (md.py:407-408, 782-794) inside the composed step."""
    st, sim, *_ = _setup(8, constr=[0, 1, 2, 60, 61])
    assert st.plan_detail()["composed_step"]
    st.run(120)
    for _ in range(120):
        sim.step()
    _check(st, sim, 120)
    st.close()


def _at_rest_setup(B, constr=None, kick=None, rest=()):
    """Trajectories `rest` start at rest (p = q = 0, empty history) with zero noise, and from step
    `kick` on (None: from the start) their noise is 1e-16: |q~ - q| then stays below md.potforce's
    1e-9 and the reference reuses the force computed at another point (md.py:449-450, 767-779).
    The other trajectories move as in _setup."""
    st, sim, baths, ob, meta, dyn, rng = _setup(B, constr=constr)
    p, q, _ = st.get_state()
    p, q = p.copy(), q.copy()
    hist = [rng.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
    for r in rest:
        p[r] = 0.0
        q[r] = 0.0
        for h in hist:
            h[r] = 0.0
    if constr is not None:
        p[:, constr] = 0.0
        q[:, constr] = 0.0
    st.set_state(p, q, 0)
    sim.p, sim.q = p.T.copy(), q.T.copy()
    for i, b in enumerate(baths):
        n = rng.normal(size=(B, meta["nmd"], b.nc)) * 1e-3
        for r in rest:
            n[r] = 0.0
            n[r, (kick or 0):] = 1e-16
        st.set_history(i, hist[i])
        st.set_noise(i, n)
        sim.set_history(i, hist[i])
        ob[i].noise = n
    return st, sim


@pytest.mark.parametrize("constr", [None, [0, 1, 2, 60, 61]])
def test_potforce_cache_reuse_at_rest_vs_oracle(constr):
    """Every trajectory at rest under noise of 1e-16 (with and without constrained DOFs): each step
    hits md.potforce's cache at a point that is not q0, at q~ and (with constraints) at q_{t+1}.  Each
    composed run stops at its first step and is replayed on the two-launch path, which applies the
    rule per trajectory: p, q and the currents equal the oracle's (oracle.GLEBatch.potforce, sameq)."""
    B = 8
    st, sim = _at_rest_setup(B, constr=constr, rest=range(B))
    assert st.plan_detail()["composed_step"]
    nst = 0
    for k in (5, 1, 7):
        st.run(k)
        for _ in range(k):
            sim.step()
        nst += k
        _check(st, sim, nst)
    a = st.cache_audit()
    assert a[0] > 0 and (constr is None or a[1] > 0), a
    st.close()


@pytest.mark.parametrize("kick", [30, 31])
@pytest.mark.parametrize("constr", [None, [0, 1, 2, 60, 61]])
def test_potforce_cache_reuse_mid_run_vs_oracle(kick, constr):
    """Seven trajectories move; the eighth rests (exact zeros: its cache hits are at q0 itself, which
    the composed step reproduces) until its noise turns to 1e-16 at step `kick`.  The composed run
    stops there (an even and an odd step: the state it resumes from sits in either parity buffer),
    the rest of it is replayed on the two-launch path, and a later run goes back to composed steps:
    all against the oracle."""
    B = 8
    st, sim = _at_rest_setup(B, constr=constr, kick=kick, rest=[7])
    st.run(60)
    for _ in range(60):
        sim.step()
    _check(st, sim, 60)
    assert st.cache_audit()[0] > 0
    st.run(23)
    for _ in range(23):
        sim.step()
    _check(st, sim, 83)
    st.close()


@pytest.mark.parametrize("B,rest", [(40, [21, 38]), (64, [63]), (130, [5, 129])])
def test_potforce_cache_reuse_audit_words_vs_oracle(B, rest):
    """The audit packs a nibble per trajectory into ceil(B / 16) words, replicated 8 times up to B = 112
    and once above (XCheck in gle_chain.hip): near-rest trajectories in later words and nibbles (B = 64
    is the benched ensemble) stop the composed run at the kick and are replayed, against the oracle."""
    st, sim = _at_rest_setup(B, kick=31, rest=rest)
    assert st.plan_detail()["composed_step"]
    st.run(50)
    for _ in range(50):
        sim.step()
    _check(st, sim, 50)
    assert st.cache_audit()[0] >= len(rest)
    st.run(9)
    for _ in range(9):
        sim.step()
    _check(st, sim, 59)
    st.close()


def test_exact_rest_runs_composed_steps():
    """A trajectory at exact rest (zero noise, zero state): md.potforce hits its cache at q0 itself
    every step, which is the fresh evaluation -- no stop, no replay.  B = 3 plans the direct ladder,
    whose products keep an all-zero trajectory exactly zero (the spectral levels' transforms leave
    roundoff of the other trajectories' size in it, ~1e-18 here, which is then a near hit and is
    replayed like one)."""
    B = 3
    st, sim = _at_rest_setup(B, kick=10 ** 9, rest=[1])
    st.run(40)
    for _ in range(40):
        sim.step()
    _check(st, sim, 40)
    assert st.cache_audit() == (0, 0)
    st.close()
