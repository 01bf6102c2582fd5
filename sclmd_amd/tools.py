"""Post-processing of the per-run heat currents (sclmd/tools.py:132-215): calHF writes running
means, calTC the thermal conductance, from the kappa.{T}.bath{i}.run{j}.dat files md.Run writes."""
import glob

import numpy as np

from . import units as U


def _read_table(bathnum):
    temperature = None
    for fn in glob.glob("kappa.*.bath0.run0.dat"):
        with open(fn) as f:
            for line in f:
                temperature = float(line.split()[1])
    if temperature is None:
        raise FileNotFoundError("no kappa.*.bath0.run0.dat in the working directory")
    nrun = len(glob.glob("kappa.*.bath0.run*.dat"))
    kb = np.empty((bathnum, nrun))
    for i in range(bathnum):
        for j in range(nrun):
            for fn in glob.glob("kappa.%d.bath%d.run%d.dat" % (int(temperature), i, j)):
                with open(fn) as f:
                    for line in f:
                        kb[i][j] = line.split()[2]
    return temperature, kb


def calHF(dlist=1, bathnum=2):
    """Cumulative mean heat flux per bath after dropping the first dlist runs (tools.py:132-163)."""
    T, kb = _read_table(bathnum)
    kept = kb[:, dlist:]
    run = np.cumsum(kept, axis=1) / np.arange(1, kept.shape[1] + 1)
    np.savetxt("heatflux." + str(int(T)) + ".dat", np.transpose(run))
    return run


def calTC(delta, dlist=1, bathnum=2, L=None, A=None):
    """Thermal conductance (J0-J1)/2/(delta*T) [(J0+J1-J2)/4 for 3 baths] (tools.py:166-215)."""
    T, kb = _read_table(bathnum)
    out = {}
    if delta != 0:
        if bathnum == 2:
            kappa = (kb[0] - kb[1]) / 2 / (delta * T)
        elif bathnum == 3:
            kappa = (kb[0] + kb[1] - kb[2]) / 4 / (delta * T)
        else:
            raise ValueError("calTC supports 2 or 3 baths")
        kappa = kappa[dlist:]
        out["conductance"] = (np.mean(kappa), np.std(kappa))
        np.savetxt("thermalconductance." + str(int(T)) + ".dat", out["conductance"],
                   header="Mean(nW/K) Std(nW/K)")
        if L is not None and A is not None:
            out["conductivity"] = (np.mean(kappa * L / A * 10), np.std(kappa * L / A * 10))
            np.savetxt("thermalconductivity." + str(int(T)) + ".dat", out["conductivity"],
                       header="Mean(W/m-K) Std(W/m-K)")
    if bathnum == 2:
        flux = (kb[0] - kb[1]) / 2
    else:
        flux = -(kb[0] + kb[1] - kb[2]) / 4
    flux = flux[dlist:]
    out["flux"] = (np.mean(flux), np.std(flux))
    np.savetxt("heatflux-between-baths." + str(int(T)) + ".dat", out["flux"], header="Mean(nW) Std(nW)")
    return out


def get_atomname(mass):
    for k, v in U.AtomicMassTable.items():
        if abs(mass - v) < 0.01:
            return k


def get_atommass(name):
    return U.AtomicMassTable.get(name)
