"""sclmd_amd -- MI355X-native generalized-Langevin MD stepper with sclmd's API.

The per-step hot path (md.vv, the bath forces and the coloured-noise generator of sclmd) runs in
hand-written HIP kernels for gfx950 behind the C-ABI in include/hipgle.h (library
sclmd_amd/_lib/libhipgle.so).  The Python modules mirror sclmd's md / ebath / phbath / tools API
so scripts written for sclmd (examples/runmd.py) run unchanged apart from the import line.
"""
__version__ = "0.1.0"
