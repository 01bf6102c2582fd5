import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def vv_cases():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("vv_") and f.endswith(".npz"))


def constr_from(g):
    rng = g["constr_ranges"]
    return [range(int(a), int(b)) for a, b in rng] if len(rng) else None


def oracle_from_golden(g):
    """Build the oracle GLE for a vv_* fixture (injected noise and kernels)."""
    from oracle import sclmd_oracle as O

    baths = []
    for i in range(int(g["nbath"])):
        kind = str(g["b%d_kind" % i])
        kw = {}
        if kind == "ebath":
            kw = dict(bias=float(g["b%d_bias" % i]), exim=g["b%d_exim" % i],
                      zeta1=g["b%d_zeta1" % i], zeta2=g["b%d_zeta2" % i])
        baths.append(O.Bath("e" if kind == "ebath" else "ph", g["b%d_cids" % i], g["b%d_kernel" % i],
                            g["b%d_noise" % i], float(g["dt"]), int(g["nmd"]), **kw))
    nph = 3 * int(g["natom"])
    sim = O.GLE(nph, float(g["dt"]), int(g["nmd"]), baths, dyn=g["dyn_md"], constr=constr_from(g))
    sim.p = g["p0"].copy()
    sim.q = g["q0"].copy()
    return sim


@pytest.fixture
def golden():
    return load_golden
