#!/usr/bin/env python3
"""GLE ensemble heat current vs the NEGF Landauer current (tests/test_gpu_negf.py's case) over a
few settings; one JSON line per setting on stdout."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_negf import landauer_case  # noqa: E402

os.chdir(tempfile.mkdtemp())
for kw in (dict(), dict(delta=0.2, ntraj=1024), dict(damp=300.0), dict(T=100.0)):
    t0 = time.time()
    jh, jc, sh, sc, jn = landauer_case(**kw)
    print(json.dumps({"case": kw, "J_hot_nW": jh, "sem_hot": sh, "J_cold_nW": jc, "sem_cold": sc,
                      "J_landauer_nW": jn, "rel_hot": jh / jn - 1, "rel_cold": -jc / jn - 1,
                      "wall_s": round(time.time() - t0, 2)}), flush=True)
