"""MD{j}.nc writer (sclmd_amd.checkpoint, md.py:768-775): the fast fill of large fixed-size
variables (parallel byte swap into the file's buffer, written without scipy's second copy) writes
exactly the bytes of scipy's own path, next to record variables and small variables."""
import numpy as np


def _write(path, arrays, fast):
    from sclmd_amd import checkpoint as C

    old = C.FAST_FILL_BYTES
    C.FAST_FILL_BYTES = 0 if fast else 1 << 62
    try:
        f, tmp = C.open_for_write(path)
        for name, size in (("nnmd", None), ("traj", 3), ("mem", 50), ("nph", 31), ("two", 2), ("one", 1)):
            f.createDimension(name, size)
        for name, a, dims in arrays:
            C.Write2NetCDFFile(f, a, name, dims, units="")
        C.commit(f, tmp, path)
    finally:
        C.FAST_FILL_BYTES = old
    return open(path, "rb").read()


def test_fast_fill_bytes_identical_to_scipy(tmp_path):
    from sclmd_amd.checkpoint import ReadNetCDFVar

    rng = np.random.default_rng(0)
    arrays = [("energy", rng.normal(size=(40, 3)), ("nnmd", "traj")),
              ("phis_g0", rng.normal(size=(3, 50, 31)), ("traj", "mem", "nph")),
              ("power", rng.normal(size=(40, 2)), ("nnmd", "two")),
              ("qhis_g0", np.asfortranarray(rng.normal(size=(3, 50, 31))), ("traj", "mem", "nph")),
              ("t", np.array([7.0]), ("one",))]
    a = _write(str(tmp_path / "a.nc"), arrays, fast=False)
    b = _write(str(tmp_path / "b.nc"), arrays, fast=True)
    assert a == b
    for name, arr, _ in arrays:
        assert np.array_equal(ReadNetCDFVar(str(tmp_path / "b.nc"), name), arr)
