"""INTEGRATION.md section 2's ctypes binding, executed as written.

CPU: the snippet loads libhipgle.so and its gle_config matches the C header field by field (sizes
and offsets from a gcc-compiled probe of include/hipgle.h).  GPU: its DeviceStepper steps the golden
vv_mixed / vv_biased trajectories (reference-generated) with the harmonic force and with a host
driver, against the golden q (1e-10 relative)."""
import ctypes
import os
import re
import subprocess
import types

import numpy as np
import pytest

from conftest import ROOT, constr_from, load_golden

LIB = os.path.join(ROOT, "sclmd_amd", "_lib", "libhipgle.so")


def snippet_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. Binding the C-ABI"):]
    m = re.search(r"```python\n(.*?)```", sec, re.S)
    assert m, "no python block in INTEGRATION.md section 2"
    return m.group(1)


def load_snippet(monkeypatch):
    monkeypatch.setenv("HIPGLE_LIB", LIB)
    mod = types.ModuleType("hipgle_snippet")
    exec(compile(snippet_source(), "INTEGRATION.md#2", "exec"), mod.__dict__)
    return mod


def c_layout(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "hipgle.h"\n'
                   "int main(void) { printf(\"%zu\", sizeof(gle_config));\n"
                   + "".join('  printf(" %%zu", offsetof(gle_config, %s));\n' % f
                             for f in ("nph", "ntraj", "nmd", "dt", "device", "block_len", "far_mode",
                                       "max_block"))
                   + "  return 0; }\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    return [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]


def test_snippet_config_matches_header(monkeypatch, tmp_path):
    mod = load_snippet(monkeypatch)
    cfg = mod.gle_config
    names = [f[0] for f in cfg._fields_]
    assert names == ["nph", "ntraj", "nmd", "dt", "device", "block_len", "far_mode", "max_block"]
    layout = c_layout(tmp_path)
    assert layout[0] == ctypes.sizeof(cfg)
    assert layout[1:] == [getattr(cfg, n).offset for n in names]
    # the binding's own error path: an odd nmd is rejected by gle_create with a message
    h = mod.H()
    bad = cfg(12, 1, 15, 0.38, 0, 0, 0, 0)
    assert mod._lib.gle_create(ctypes.byref(bad), ctypes.byref(h)) == -1
    assert b"even" in mod._lib.gle_last_error(None)


class _RefMd:
    """The attributes of a reference sclmd md object that the snippet reads (md.py:56-130)."""

    def __init__(self, g, driver=None):
        from oracle import sclmd_oracle as O

        self.nph, self.nmd, self.dt = 3 * int(g["natom"]), int(g["nmd"]), float(g["dt"])
        self.dyn = g["dyn_md"]
        self.constraint = constr_from(g)
        self.p, self.q, self.t = g["p0"].copy(), g["q0"].copy(), 0
        self.baths = []
        for i in range(int(g["nbath"])):
            b = types.SimpleNamespace(cids=g["b%d_cids" % i], kernel=g["b%d_kernel" % i], noise=g["b%d_noise" % i])
            if str(g["b%d_kind" % i]) == "ebath":
                b.efric = g["b%d_kernel" % i][0]
                b.bias = float(g["b%d_bias" % i])
                b.exim, b.zeta1, b.zeta2 = g["b%d_exim" % i], g["b%d_zeta1" % i], g["b%d_zeta2" % i]
            self.baths.append(b)
        self.pforce = driver
        self.q0, self.f0 = [], []
        self._same = O.same_q

    def potforce(self, q):  # md.potforce's cache (md.py:437-474)
        if self._same(q, self.q0):
            return self.f0
        f = self.pforce.force(q)
        self.q0, self.f0 = q, f
        return f


@pytest.mark.gpu
@pytest.mark.parametrize("case,driver", [("vv_mixed", False), ("vv_biased", False), ("vv_mixed", True)])
def test_snippet_steps_golden(monkeypatch, case, driver):
    from sclmd_amd import synthetic
    from sclmd_amd.drivers import HarmonicDriver

    mod = load_snippet(monkeypatch)
    g = load_golden(case)
    drv = HarmonicDriver(g["dyn_md"], synthetic.axyz_chain(int(g["natom"]))) if driver else None
    md = _RefMd(g, drv)
    if driver:
        md.dyn = None
    st = mod.DeviceStepper(md)
    try:
        qs = []
        for _ in range(int(g["nsteps"])):
            st.vv(md)
            qs.append(md.q.copy())
    finally:
        st.close()
    qs = np.array(qs)
    assert np.max(np.abs(qs - g["q"])) / np.max(np.abs(g["q"])) < 1e-10
    assert md.t == int(g["nsteps"])
