"""examples/runmd.py of sclmd (runmd.py:1-73) on the MI355X stepper.

Identical in shape to the reference script: two electron baths at T(1 +- delta/2) on DOF 60-209 and
393-542, constraints on atoms 0-19 and 181-200, 3 runs of nmd = 2**12 steps, then calHF/calTC.
LAMMPS/REBO is not installed in this image, so a harmonic driver with the lammpsdriver plugin
surface (.force(q) relative to f0, .axyz, .conv, .quit) stands in for it: a 201-atom C chain.
Set NMD=256 in the environment for a quick run.
"""
import os
import time

import numpy as np

from sclmd_amd.baths import ebath
from sclmd_amd.drivers import HarmonicDriver
from sclmd_amd.md import md
from sclmd_amd.synthetic import axyz_chain, chain_dyn
from sclmd_amd.tools import calHF, calTC

T = 300
delta = 0.1
nstart = 0
nstop = 3
dt = 0.25 / 0.658
nmd = int(os.environ.get("NMD", 2 ** 12))
lmp = HarmonicDriver(chain_dyn(201), axyz_chain(201))      # lammpsdriver(infile=lammpsinfile)
time_start = time.time()

fixatoms = [range(0 * 3, (19 + 1) * 3), range(181 * 3, (200 + 1) * 3)]
ecatsl = range(20 * 3, (69 + 1) * 3)
ecatsr = range(131 * 3, (180 + 1) * 3)
mdrun = md(dt, nmd, T, axyz=lmp.axyz, nstart=nstart, nstop=nstop)
mdrun.AddPotential(lmp)
damp = 100 / 0.658211814201041
etal = (1.0 / damp) * np.identity(len(ecatsl))
etar = (1.0 / damp) * np.identity(len(ecatsr))
ebl = ebath(ecatsl, T * (1 + delta / 2), mdrun.dt, mdrun.nmd, wmax=1., nw=500, bias=0.0, efric=etal,
            classical=False, zpmotion=True)
mdrun.AddBath(ebl)
ebr = ebath(ecatsr, T * (1 - delta / 2), mdrun.dt, mdrun.nmd, wmax=1., nw=500, bias=0.0, efric=etar,
            classical=False, zpmotion=True)
mdrun.AddBath(ebr)
mdrun.AddConstr(fixatoms)
mdrun.Run()
lmp.quit()
calHF()
calTC(delta=delta)
print("time cost", time.time() - time_start, "s.")
