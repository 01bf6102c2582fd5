"""MD{j}.nc checkpoint files of md.Run (sclmd/md.py:684-764 dump, :506-567 resume, :768-783 helpers).

The reference writes them with netCDF4 (HDF5-based NETCDF4 format, zlib).  netCDF4 is not installed
here, so the files are written in the NetCDF classic (64-bit offset) format with scipy.io -- the same
dimension names, variable names, shapes and float64 data, readable by netCDF4.Dataset and by
ReadNetCDFVar below.  Deviations (documented in md.dump): no zlib compression; with ntraj > 1 every
per-trajectory variable gains a leading 'traj' dimension; with several ranks each rank writes its
own shard to MD{j}.r{rank}.nc.
"""
import os

import numpy as np
from scipy.io import netcdf_file


# fixed-size variables at least this large take the fast fill (parallel byte swap, no second copy)
FAST_FILL_BYTES = 64 << 20


class _WriteView(np.ndarray):
    """A variable's big-endian buffer whose tobytes() is a view of itself: scipy's classic-format
    writer (fp.write(var.data.tobytes())) then writes the filled buffer without copying GBs again."""

    def tobytes(self, order="C"):
        return memoryview(self.view(np.ndarray)).cast("B")


def _fill_big_endian(dst, src, workers=8):
    """dst[...] = src (little- to big-endian) on a thread pool (numpy's casting copy releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    d, s_ = dst.reshape(-1), np.ascontiguousarray(src).reshape(-1)
    edges = np.linspace(0, d.size, workers + 1).astype(np.int64)
    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(lambda k: np.copyto(d[edges[k]:edges[k + 1]], s_[edges[k]:edges[k + 1]]), range(workers)))


def Write2NetCDFFile(ncfile, var, varLabel, dimensions, units=None, description=None):
    """Create a float64 variable and fill it (md.py:768-775).  Large fixed-size variables (C5's
    history groups, 3 GB) are byte-swapped into the file's buffer on a thread pool and written
    from it without scipy's second whole-array copy (same bytes on disk)."""
    v = np.asarray(var, dtype=np.float64)
    tmp = ncfile.createVariable(varLabel, "d", tuple(dimensions))
    if len(dimensions) and ncfile.dimensions.get(dimensions[0]) is None:
        tmp[: v.shape[0]] = v  # record (unlimited) dimension
    elif v.nbytes >= FAST_FILL_BYTES and tmp.data.shape == v.shape:
        buf = np.empty(v.shape, dtype=">f8").view(_WriteView)
        _fill_big_endian(buf, v)
        tmp.__dict__["data"] = buf
    else:
        tmp[:] = v
    if units:
        tmp.units = units
    if description:
        tmp.description = description


def ReadNetCDFVar(file, var):
    """Copy of one variable of an MD{j}.nc file (md.py:778-783)."""
    with netcdf_file(file, "r", mmap=False) as f:
        return np.array(f.variables[var].data, dtype=np.float64)


def read_history(file, var, ml):
    """phis / qhis of an MD{j}.nc file as (ml, nph) or (ntraj, ml, nph): the ('mem', ...) layout; the
    trajectory groups md.dump writes for ensembles whose history exceeds a classic-format variable
    (var_g0, var_g1, ... over ('trajg{k}', 'mem', 'nph'), joined in order); or the record layout of
    round-4 files (rows [0, ml) of ('nnmd', 'traj', 'nph'))."""
    with netcdf_file(file, "r", mmap=False) as f:
        if var not in f.variables and (var + "_g0") in f.variables:
            parts, k = [], 0
            while (var + "_g%d" % k) in f.variables:
                parts.append(np.array(f.variables[var + "_g%d" % k].data, dtype=np.float64))
                k += 1
            return np.concatenate(parts, axis=0)
        v = f.variables[var]
        dims = tuple(v.dimensions)
        if dims and dims[0] == "nnmd":
            a = np.array(v.data[:ml], dtype=np.float64)
            return np.transpose(a, (1, 0, 2)) if a.ndim == 3 else a
        return np.array(v.data, dtype=np.float64)


def var_dims(file, var):
    """Dimension names of one variable of an MD{j}.nc file."""
    with netcdf_file(file, "r", mmap=False) as f:
        return tuple(f.variables[var].dimensions)


def has_var(file, var):
    with netcdf_file(file, "r", mmap=False) as f:
        return var in f.variables


def open_for_write(path, title="Output from md.py"):
    tmp = path + ".tmp"
    f = netcdf_file(tmp, "w", version=2)
    f.title = title
    return f, tmp


def commit(f, tmp, path):
    """Close and atomically move into place (a crash never leaves a half-written checkpoint)."""
    f.close()
    os.replace(tmp, path)


def abandon(f, tmp):
    """A write that failed: close what can be closed and remove the partial file."""
    try:
        f.close()
    except Exception:
        pass
    try:
        os.remove(tmp)
    except OSError:
        pass
