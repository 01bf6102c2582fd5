#!/usr/bin/env python3
"""GLE ensemble heat current vs the NEGF Landauer current (tests/test_gpu_negf.py's case) over a
few settings; one JSON line per setting on stdout (currents in nW)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_negf import landauer_case  # noqa: E402

for kw in (dict(), dict(zpmotion=True), dict(delta=0.2, ntraj=8192), dict(damp=300.0), dict(T=100.0)):
    os.chdir(tempfile.mkdtemp())
    t0 = time.time()
    r = landauer_case(**kw)
    r.update(case=kw, rel_anti=r["J_anti"] / r["J_negf"] - 1, rel_hot=r["J_hot"] / r["J_negf"] - 1,
             rel_cold=-r["J_cold"] / r["J_negf"] - 1, wall_s=round(time.time() - t0, 2))
    print(json.dumps(r), flush=True)
