#!/usr/bin/env python3
"""Golden fixture for the NEGF / Landauer cross-check, made by running the REAL
reference's `sclmd.negf.bpt` (negf.py:8-273) once in the build container.

    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/make_golden_negf.py

Two things the reference module needs are absent here and neither is reached by what this script
calls:
  * `from lammps import lammps` (negf.py:5) -- only `bpt.getdynmat` (negf.py:41-97) uses it, to ask
    LAMMPS for the dynamical matrix.  A stub module satisfies the import; the object is built with
    `bpt.__new__` and its attributes (dynmat, natoms, damp, ...) are set as getdynmat would set them.
  * `np.complex_` (negf.py:167,175,183) was removed in numpy 2.0; it is aliased to np.complex128
    (the same type under its surviving name) for the duration of this script.
Nothing at test time, in smoke() or in bench.py reads /root/reference.

Output tests/golden/negf.npz:
  dynmat (full 3*natoms square, rad^2/ps^2), fixed / bath / bias DOF lists, damp (ps),
  maxomega (eV), intnum, tm_x / tm_y (gettm), current_T / current (thermalcurrent, nW),
  conductance, conductivity (L, A), ps_w / ps_T / ps_unbiased / ps_biased (bpt.ps), bias params.
"""
import contextlib
import io
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.modules["lammps"] = types.SimpleNamespace(lammps=None)
if not hasattr(np, "complex_"):
    np.complex_ = np.complex128

import sclmd.negf as RNEGF  # noqa: E402

RPC = 6.582119569e-4  # hbar in eV ps, as bpt.__init__ (negf.py:12)


def chain_dynmat(natom, k_md=0.01, onsite_md=1e-3):
    """Chain on every Cartesian axis in md units (eV^2), converted to rad^2/ps^2."""
    n = 3 * natom
    d = np.zeros((n, n))
    for a in range(natom):
        for x in range(3):
            i = 3 * a + x
            d[i, i] += onsite_md
            if a + 1 < natom:
                j = 3 * (a + 1) + x
                d[i, i] += k_md
                d[j, j] += k_md
                d[i, j] -= k_md
                d[j, i] -= k_md
    return d / RPC ** 2


def make_bpt(dynmat, natoms, maxomega, damp, bath, fixed, num):
    """A bpt as __init__ + getdynmat would leave it (negf.py:9-25, 68-86), LAMMPS call skipped."""
    b = RNEGF.bpt.__new__(RNEGF.bpt)
    b.rpc = 6.582119569e-4
    b.bc = 8.617333262e-5
    b.damp = damp
    b.maxomega = maxomega / b.rpc
    b.intnum = num
    b.dofatomfixed = fixed
    b.isbias = False
    b.dofatomofbias = []
    b.dofatomofbath = bath
    b.natoms = natoms
    d = (dynmat + dynmat.T) / 2
    d = np.delete(d, fixed[0], axis=0)
    d = np.delete(d, fixed[0], axis=1)
    sh = [dof - len(fixed[0]) for dof in fixed[1]]
    d = np.delete(d, sh, axis=0)
    d = np.delete(d, sh, axis=1)
    b.dynmat = d
    return b


def main():
    natom = 8
    dyn = chain_dynmat(natom)
    fixed = [list(range(0, 3)), list(range(21, 24))]
    bath = [list(range(3, 9)), list(range(15, 21))]
    bias_dofs = list(range(9, 15))
    maxomega, damp, num = 0.25, 0.1, 400
    b = make_bpt(dyn, natom, maxomega, damp, bath, fixed, num)
    with contextlib.redirect_stdout(io.StringIO()):
        cwd = os.getcwd()
        os.chdir("/tmp")  # gettm writes transmission.dat
        try:
            b.gettm(vector=True)
        finally:
            os.chdir(cwd)
    temps = np.array([0.0, 10.0, 100.0, 300.0, 1000.0])
    delta = 0.1
    cur = np.array([b.thermalcurrent(T, delta) for T in temps])
    cond = np.array([b.thermalconductance(T, delta) for T in temps[1:]])
    L, A = 12.0, 4.5
    kappa = np.array([b.thermalconductivity(T, delta, L, A) for T in temps[1:]])
    ps_w = np.linspace(0.0, maxomega / RPC, 9)[1:]
    ps_T = 300.0
    atomlist = np.array(bias_dofs)
    ps_unb = np.array([b.ps(w, ps_T, atomlist) for w in ps_w])
    rng = np.random.default_rng(7)
    nb = len(bias_dofs)
    bdamp = np.eye(nb) / 0.2 + 0.3 * np.diag(rng.random(nb))
    r = rng.standard_normal((nb, nb))
    chiplus = 0.05 * (r + r.T) / 2
    r = rng.standard_normal((nb, nb))
    chiminus = 0.05 * (r - r.T) / 2
    bias_eV = 0.6
    b.setbias(bias_eV, bdamp=bdamp, chiplus=chiplus, chiminus=chiminus, dofatomofbias=bias_dofs)
    ps_b = np.array([b.ps(w, ps_T, atomlist) for w in ps_w])
    np.savez(os.path.join(HERE, "negf.npz"), dynmat=dyn, natoms=natom, fixed0=fixed[0], fixed1=fixed[1],
             bath0=bath[0], bath1=bath[1], damp=damp, maxomega=maxomega, intnum=num,
             tm_x=b.tmnumber[:, 0], tm_y=b.tmnumber[:, 1], current_T=temps, delta=delta, current=cur,
             conductance=cond, L=L, A=A, conductivity=kappa, ps_w=ps_w, ps_T=ps_T, ps_atoms=atomlist,
             ps_unbiased=ps_unb, ps_biased=ps_b, bias=bias_eV, bias_dofs=bias_dofs, bdamp=bdamp,
             chiplus=chiplus, chiminus=chiminus)
    print("negf.npz: tm max %.4f, current(300K) %.6e nW" % (b.tmnumber[:, 1].max(), cur[3]))


if __name__ == "__main__":
    main()
