#!/usr/bin/env python3
"""Full-size C5 properties on one MI355X (too large for the pytest suite: ~280 GB of device memory
per stepper, so the steppers run one after another).

C5 = 1000-atom chain, 2 phonon baths (nc = 999, ml = 4096) + 1 biased electron bath (nc = 1002,
exim/zeta1/zeta2 != 0), nmd = 8192, 32 trajectories (one GPU's share of the 256-trajectory ensemble).
Seeded random history, state and noise (the oracle would need ~12 s and 65 GB of host kernel per
step, so full-size parity is checked through size-independent properties):

  1. spectral ladder vs direct contraction of the same kernels: trajectories agree to 1e-10
     relative (two different far-field algorithms over all 4095 lags);
  2. linearity: state, history and noise x3 give the trajectory x3 and the heat current x9
     (1e-12 relative; x3 is not exact in binary, so rounding is exercised);
  3. determinism: a repeated run is bitwise identical.

Prints one JSON line with the measured deviations; exits non-zero on failure.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sclmd_amd import _native as N  # noqa: E402
from sclmd_amd import synthetic  # noqa: E402

NTRAJ, NSTEPS = 32, 40


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main():
    t0 = time.perf_counter()
    dyn, axyz, baths, meta = synthetic.junction("C5", seed=1234, gmem_device=True)
    nph, nmd, dt = meta["nph"], meta["nmd"], meta["dt"]
    rng = np.random.default_rng(99)
    p0 = rng.normal(size=(NTRAJ, nph)) * 1e-2
    q0 = rng.normal(size=(NTRAJ, nph)) * 1e-2
    hist = [rng.normal(size=(NTRAJ, b.ml, b.nc)) * 1e-2 if b.ml > 1 else None for b in baths]
    noise = [rng.normal(size=(NTRAJ, nmd, b.nc)) * 1e-3 for b in baths]
    log("[c5] inputs built (%.1fs)" % (time.perf_counter() - t0))

    def run(far_mode, scale=1.0):
        st = N.Stepper(nph, NTRAJ, nmd, dt, 0, 0, far_mode)
        try:
            for b in baths:
                if b.kind == "ebath":
                    st.add_bath(N.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
                else:
                    W, G = b.gmem_recipe
                    st.add_bath_gmem(b.cids, W, G)
            st.set_dyn(dyn)
            st.set_state(p0 * scale, q0 * scale, 0)
            for i, b in enumerate(baths):
                st.set_history(i, None if hist[i] is None else hist[i] * scale)
                st.set_noise(i, noise[i] * scale)
            st.run(NSTEPS)
            p, q, t = st.get_state()
            cur = st.get_current()[:, :, :NSTEPS]
            info = st.plan_info()
            log("[c5] %s x%g: %d steps, plan %s (%.1fs)" % (far_mode, scale, t, info, time.perf_counter() - t0))
            return p, q, cur, info
        finally:
            st.close()

    ps, qs, cs, info_s = run("spectral")
    ps2, qs2, cs2, _ = run("spectral")
    pl, ql, cl, _ = run("spectral", 3.0)
    pd, qd, cd, info_d = run("direct")
    res = {
        "config": "C5", "ntraj": NTRAJ, "steps": NSTEPS,
        "far_modes": [info_s["far_mode"], info_d["far_mode"]],
        "spectral_vs_direct_q": rel(qs, qd), "spectral_vs_direct_p": rel(ps, pd),
        "spectral_vs_direct_cur": rel(cs, cd),
        "linearity_q": rel(ql, 3.0 * qs), "linearity_cur": rel(cl, 9.0 * cs),
        "bitwise_repeat": bool(np.array_equal(qs, qs2) and np.array_equal(ps, ps2) and np.array_equal(cs, cs2)),
    }
    ok = (res["far_modes"] == ["spectral", "direct"] and res["spectral_vs_direct_q"] < 1e-10
          and res["spectral_vs_direct_p"] < 1e-10 and res["spectral_vs_direct_cur"] < 1e-9
          and res["linearity_q"] < 1e-12 and res["linearity_cur"] < 1e-11 and res["bitwise_repeat"])
    res["ok"] = ok
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
