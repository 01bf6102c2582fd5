"""Seeded random configurations against the oracle: the plan space has many switches (bath size class,
ensemble width, memory lengths, DOF maps, bath kinds and bias, constraints, far mode, first block
length, composed or two-launch steps, host-force segments), and a fixed list of cases samples their
combinations.  Each case draws a junction (chain or chain + long-range couplings), 1-3 baths on
random DOF sets (contiguous, scattered, overlapping), B in [1, 70], ml in [1, 130], sometimes
near-rest trajectories (md.potforce's 1e-9 cache reuse), then runs a random sequence of device runs,
host-force steps and new noise realisations over more than nmd steps (noise wrap-around) from a
nonzero t0 and history, against oracle.GLEBatch at 1e-9 on p, q, the heat currents, the kinetic
energy and the recordings (ps, qs, each bath's id0 force).  A failing
case prints its parameters (case index = seed)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-9
NCASE = int(os.environ.get("SCLMD_FUZZ_CASES", "60"))  # a wider sweep: SCLMD_FUZZ_CASES=300


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _case(seed):
    from sclmd_amd import synthetic

    r = np.random.default_rng(1000 + seed)
    tiny = r.random() < 0.3  # a few DOF tiles meeting several small baths (many short product runs)
    natom = int(r.integers(4, 11)) if tiny else int(r.integers(5, 60))
    nph = 3 * natom
    dyn = synthetic.chain_dyn(natom)
    if r.random() < 0.5:  # long-range couplings: the block-sparse dyn with scattered blocks
        n = int(r.integers(1, 3 * natom))
        i, j = r.integers(0, nph, n), r.integers(0, nph, n)
        v = r.normal(size=n) * 1e-3
        add = np.zeros((nph, nph))
        add[i, j] += v
        add = add + add.T
        dyn = dyn + add + np.eye(nph) * 2 * np.abs(add).sum(axis=1).max()
    nmd = int(r.choice([64, 128, 256]))
    B = int(r.choice([1, 2, 3, 5, 8, 13, 16, 17, 24, 31, 32, 33, 40, 48, 49, 63, 64, 70]))
    nb = 3 if tiny else int(r.integers(1, 4))
    baths, used = [], np.zeros(nph, bool)
    for k in range(nb):
        kind = "e" if (k == nb - 1 and r.random() < 0.4) else "ph"
        nc = int(r.integers(2, max(3, min(nph, 12 if tiny else 90))))
        mode = r.choice(["range", "scatter", "overlap"])
        if mode == "range":
            a = int(r.integers(0, nph - nc + 1))
            d = list(range(a, a + nc))
        elif mode == "scatter":
            d = sorted(int(x) for x in r.choice(nph, nc, replace=False))
        else:  # prefer DOFs already in a bath
            pool = np.nonzero(used)[0]
            take = min(len(pool), nc // 2)
            d = set(int(x) for x in r.choice(pool, take, replace=False)) if take else set()
            rest = [x for x in r.permutation(nph) if x not in d][: nc - len(d)]
            d = sorted(d | set(int(x) for x in rest))
        used[d] = True
        if kind == "e":
            b = synthetic.make_biased_ebath(300.0, d, nmd, r, bias=float(r.choice([0.0, 1.0])))
        else:
            ml = min(nmd, int(r.choice([1, 2, 3, 6, 17, 40, 96, 130])))
            b = synthetic.make_phbath(300.0 * (1 + 0.1 * k), d, ml, nmd, r, nw=60)
        baths.append(b)
    constr = None
    if r.random() < 0.4:
        constr = sorted(set(int(x) for x in r.choice(nph, int(r.integers(1, 8)), replace=False)))
    plan = str(r.choice(["auto", "small", "large"]))
    far = str(r.choice(["auto", "auto", "direct", "spectral"]))
    block_len = int(r.choice([0, 0, 1, 2, 4, 8]))
    segs = []
    total = 0
    while total < nmd + 40:
        u = r.random()
        if u < 0.2:
            k = int(r.integers(1, 4))
            segs.append(("host", k))
        elif u < 0.27:  # a new noise realisation (md.py:569-570)
            k = 0
            segs.append(("noise", 0))
        elif u < 0.31:  # a new state, history and step counter (a resumed run, md.py:506-567)
            k = 0
            segs.append(("restate", int(r.integers(0, 3 * nmd))))
        else:
            k = int(r.integers(1, 90))
            segs.append(("run", k))
        total += k
    # near-rest trajectories: zero state and history, noise 1e-16 from step `kick` on (md.potforce's
    # 1e-9 cache reuse at points that are not q0; the composed step's audit and replay)
    rest = []
    if r.random() < 0.25:
        rest = sorted(set(int(x) for x in r.choice(B, int(r.integers(1, min(B, 3) + 1)), replace=False)))
    kick = int(r.integers(0, nmd))
    if rest:  # host-force steps take the force as given; md.potforce's cache in front of a host driver is
        # the md layer's (md.py's per-trajectory sameq), so near-rest cases step on the device only
        segs = [("run", k) if kind == "host" else (kind, k) for kind, k in segs]
    t0 = int(r.integers(0, nmd))
    return dict(natom=natom, nph=nph, dyn=dyn, nmd=nmd, B=B, baths=baths, constr=constr, plan=plan, far=far,
                block_len=block_len, segs=segs, t0=t0, seed=seed, rest=rest, kick=kick)


def _rec_batch():
    """oracle.GLEBatch that also keeps md's recordings: ps / qs (md.py:374-377) and each bath's id0
    force fhis[i] (md.py:398), at slot t mod nmd."""
    from oracle import sclmd_oracle as O

    class RecBatch(O.GLEBatch):
        def step(self):
            t = int(self.t) % self.nmd
            if not hasattr(self, "rps"):
                self.rps = np.zeros((self.ntr, self.nmd, self.nph))
                self.rqs = np.zeros((self.ntr, self.nmd, self.nph))
                self.rf = [np.zeros((self.ntr, self.nmd, b.nc)) for b in self.baths]
            self.rps[:, t] = self.p.T
            self.rqs[:, t] = self.q.T
            self._seen = set()
            super().step()

        def _bath_force(self, i, t_noise, S, x, qarg):
            f = super()._bath_force(i, t_noise, S, x, qarg)
            if i not in self._seen:  # the step's first call per bath is md.force id0
                self._seen.add(i)
                self.rf[i][:, int(self.t) % self.nmd] = f.T
            return f

    return RecBatch


def _describe(c):
    return ("seed %d natom %d B %d nmd %d plan %s far %s block_len %d t0 %d constr %s rest %s kick %d baths %s" % (
        c["seed"], c["natom"], c["B"], c["nmd"], c["plan"], c["far"], c["block_len"], c["t0"], c["constr"], c["rest"],
        c["kick"],
        [(b.kind, b.nc, b.kernel.shape[0], getattr(b, "bias", None)) for b in c["baths"]]))


@pytest.mark.parametrize("seed", range(NCASE))
def test_random_configuration_vs_oracle(seed):
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N

    c = _case(seed)
    desc = _describe(c)
    B, nph, nmd, dyn, baths = c["B"], c["nph"], c["nmd"], c["dyn"], c["baths"]
    dt = baths[0].dt
    r = np.random.default_rng(seed)
    try:
        st = N.Stepper(nph, B, nmd, dt, 0, c["block_len"], c["far"], 0)
    except Exception as e:  # noqa: BLE001
        pytest.fail("%s: %s" % (desc, e))
    try:
        for b in baths:
            if b.kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        if c["constr"] is not None:
            st.set_constraint(c["constr"])
        st.set_plan_class(c["plan"])
        p = r.normal(size=(B, nph)) * 1e-2
        q = r.normal(size=(B, nph)) * 1e-2
        if c["constr"] is not None:
            p[:, c["constr"]] = 0.0
            q[:, c["constr"]] = 0.0
        def draw_noise():
            out = [r.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
            for n in out:
                n[c["rest"]] = 0.0
                for j in c["rest"]:
                    n[j, (c["t0"] + c["kick"]) % nmd:] = 1e-16
            return out

        noise = draw_noise()
        hist = [r.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
        p[c["rest"]] = 0.0
        q[c["rest"]] = 0.0
        for h in hist:
            h[c["rest"]] = 0.0
        st.set_state(p, q, c["t0"])
        for i in range(len(baths)):
            st.set_history(i, hist[i])
            st.set_noise(i, noise[i])
        ob = [O.Bath("e", b.cids, b.kernel, noise[i], dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1,
                     zeta2=b.zeta2) if b.kind == "ebath" else O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd)
              for i, b in enumerate(baths)]
        Rec = _rec_batch()
        sim = Rec(nph, dt, nmd, ob, dyn, ntr=B,
                  constr=None if c["constr"] is None else [range(x, x + 1) for x in c["constr"]])
        sim.p, sim.q, sim.t = p.T.copy(), q.T.copy(), c["t0"]
        st.record(N.REC_P | N.REC_Q | N.REC_F)
        for i in range(len(baths)):
            sim.set_history(i, hist[i])
        nst, t_start = 0, c["t0"]
        for kind, k in c["segs"]:
            if kind == "run":
                st.run(k)
                for _ in range(k):
                    sim.step()
            elif kind == "noise":
                noise = draw_noise()
                for i in range(len(baths)):
                    st.set_noise(i, noise[i])
                    ob[i].noise = noise[i]
            elif kind == "restate":
                p = r.normal(size=(B, nph)) * 1e-2
                q = r.normal(size=(B, nph)) * 1e-2
                p[c["rest"]] = 0.0
                q[c["rest"]] = 0.0
                if c["constr"] is not None:
                    p[:, c["constr"]] = 0.0
                    q[:, c["constr"]] = 0.0
                hist = [r.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
                for h in hist:
                    h[c["rest"]] = 0.0
                st.set_state(p, q, k)
                for i in range(len(baths)):
                    st.set_history(i, hist[i])
                sim = Rec(nph, dt, nmd, ob, dyn, ntr=B,
                          constr=None if c["constr"] is None else [range(x, x + 1) for x in c["constr"]])
                sim.p, sim.q, sim.t = p.T.copy(), q.T.copy(), k
                for i in range(len(baths)):
                    sim.set_history(i, hist[i])
                t_start, nst = k, 0
                continue
            else:
                for _ in range(k):
                    qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
                    st.step_end(-(qt @ dyn.T))
                    sim.step()
            nst += k
        pg, qg, t = st.get_state()
        cur = st.get_current()
        en = st.get_energy()
        rec = (st.get_record(N.REC_P), st.get_record(N.REC_Q), [st.get_record(N.REC_F, i) for i in range(len(baths))])
    finally:
        st.close()
    assert t == t_start + nst, desc
    assert rel(qg, sim.q.T) < TOL and rel(pg, sim.p.T) < TOL, (desc, rel(qg, sim.q.T), rel(pg, sim.p.T))
    # currents of the last nmd steps since the last restate (older ones are overwritten by the ring of
    # nmd entries; a restate starts a fresh oracle)
    steps = (t_start + np.arange(max(0, nst - nmd), nst)) % nmd
    if nst == 0:
        return
    want = np.stack([cc[:, steps] for cc in sim.cur])
    assert rel(cur[:, :, steps], want) < TOL, desc
    assert rel(en[:, steps], sim.etot[:, steps]) < TOL, desc
    # recordings (gle_record): ps / qs and the bath forces of md.force id0
    assert rel(rec[0][:, steps], sim.rps[:, steps]) < TOL and rel(rec[1][:, steps], sim.rqs[:, steps]) < TOL, desc
    for i in range(len(baths)):
        assert rel(rec[2][i][:, steps], sim.rf[i][:, steps]) < TOL, (desc, "fhis", i)


def test_interleaved_handles_vs_oracle():
    """Three live handles of different shapes (plan classes, widths, nmd) on one device, stepped in
    interleaved calls: no state leaks between handles (launch attributes, streams, audit words)."""
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N

    cases = [_case(s) for s in (3, 7, 11)]
    live = []
    try:
        for c in cases:
            B, nph, nmd, dyn, baths = c["B"], c["nph"], c["nmd"], c["dyn"], c["baths"]
            dt = baths[0].dt
            r = np.random.default_rng(c["seed"] + 99)
            st = N.Stepper(nph, B, nmd, dt, 0, c["block_len"], c["far"], 0)
            for b in baths:
                if b.kind == "ebath":
                    st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
                else:
                    st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
            st.set_dyn(dyn)
            st.set_plan_class(c["plan"])
            p = r.normal(size=(B, nph)) * 1e-2
            q = r.normal(size=(B, nph)) * 1e-2
            noise = [r.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
            st.set_state(p, q, 0)
            for i in range(len(baths)):
                st.set_noise(i, noise[i])
            ob = [O.Bath("e", b.cids, b.kernel, noise[i], dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1,
                         zeta2=b.zeta2) if b.kind == "ebath" else O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd)
                  for i, b in enumerate(baths)]
            sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=B)
            sim.p, sim.q = p.T.copy(), q.T.copy()
            live.append((st, sim, dyn))
        rr = np.random.default_rng(0)
        for _ in range(12):
            for st, sim, dyn in live:
                k = int(rr.integers(1, 40))
                if rr.random() < 0.2:
                    for _ in range(k % 3 + 1):
                        qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
                        st.step_end(-(qt @ dyn.T))
                        sim.step()
                else:
                    st.run(k)
                    for _ in range(k):
                        sim.step()
        for st, sim, _ in live:
            pg, qg, _ = st.get_state()
            assert rel(qg, sim.q.T) < TOL and rel(pg, sim.p.T) < TOL
    finally:
        for st, _, _ in live:
            st.close()


@pytest.mark.parametrize("seed", range(3))
def test_random_large_bath_vs_oracle(seed):
    """Baths above the small-bath limit (nc > 512: the large-bath plan picked by the automatic rule,
    first block length 4, the potential-force launch, dyn as ELL), random widths, memory lengths,
    constraints and host-force segments against the oracle."""
    from oracle import sclmd_oracle as O
    from sclmd_amd import _native as N
    from sclmd_amd import synthetic

    r = np.random.default_rng(7000 + seed)
    natom = int(r.integers(178, 200))
    nph = 3 * natom
    dyn = synthetic.chain_dyn(natom)
    nmd = 128
    B = int(r.choice([1, 8, 33]))
    nc = int(r.integers(513, 560))
    a0 = int(r.integers(0, nph - nc + 1))
    baths = [synthetic.make_phbath(300.0, list(range(a0, a0 + nc)), int(r.choice([2, 24])), nmd, r, nw=60)]
    if r.random() < 0.5:
        d = sorted(int(x) for x in r.choice(nph, 40, replace=False))
        baths.append(synthetic.make_biased_ebath(300.0, d, nmd, r))
    constr = sorted(set(int(x) for x in r.choice(nph, 4, replace=False))) if seed != 1 else None
    dt = baths[0].dt
    st = N.Stepper(nph, B, nmd, dt, 0)
    try:
        for b in baths:
            if b.kind == "ebath":
                st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
            else:
                st.add_bath(N.GLE_BATH_PHONON, b.cids, b.kernel)
        st.set_dyn(dyn)
        if constr is not None:
            st.set_constraint(constr)
        p = r.normal(size=(B, nph)) * 1e-2
        q = r.normal(size=(B, nph)) * 1e-2
        if constr is not None:
            p[:, constr] = 0.0
            q[:, constr] = 0.0
        noise = [r.normal(size=(B, nmd, b.nc)) * 1e-3 for b in baths]
        hist = [r.normal(size=(B, b.kernel.shape[0], b.nc)) * 1e-2 for b in baths]
        st.set_state(p, q, 11)
        for i in range(len(baths)):
            st.set_history(i, hist[i])
            st.set_noise(i, noise[i])
        assert st.plan_detail()["plan_class"] == "large"
        ob = [O.Bath("e", b.cids, b.kernel, noise[i], dt, nmd, bias=b.bias, exim=b.exim, zeta1=b.zeta1,
                     zeta2=b.zeta2) if b.kind == "ebath" else O.Bath("ph", b.cids, b.kernel, noise[i], dt, nmd)
              for i, b in enumerate(baths)]
        sim = O.GLEBatch(nph, dt, nmd, ob, dyn, ntr=B,
                         constr=None if constr is None else [range(x, x + 1) for x in constr])
        sim.p, sim.q, sim.t = p.T.copy(), q.T.copy(), 11
        for i in range(len(baths)):
            sim.set_history(i, hist[i])
        for kind, k in (("run", 47), ("host", 2), ("run", 70)):
            if kind == "run":
                st.run(k)
                for _ in range(k):
                    sim.step()
            else:
                for _ in range(k):
                    qt = st.step_begin(-(st.get_state()[1] @ dyn.T))
                    st.step_end(-(qt @ dyn.T))
                    sim.step()
        pg, qg, _ = st.get_state()
        cur = st.get_current()
    finally:
        st.close()
    assert rel(qg, sim.q.T) < TOL and rel(pg, sim.p.T) < TOL, (rel(qg, sim.q.T), rel(pg, sim.p.T))
    steps = (11 + np.arange(119)) % nmd
    want = np.stack([cc[:, steps] for cc in sim.cur])
    assert rel(cur[:, :, steps], want) < TOL
