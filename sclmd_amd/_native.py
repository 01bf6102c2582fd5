"""ctypes binding of the hipgle C-ABI (include/hipgle.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) into sclmd_amd/_lib/.
There is no CPU fallback: every compute call goes through this library and raises when it is
missing or when no HIP device is present.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCLMD_AMD_LIB", os.path.join(_HERE, "_lib", "libhipgle.so"))

GLE_BATH_PHONON = 0
PROFILE_EVENTS = 1  # hipgle.h GLE_PROFILE_EVENTS
PROFILE_COUNT = 2   # hipgle.h GLE_PROFILE_COUNT
PROFILE_CHAIN = 4   # hipgle.h GLE_PROFILE_CHAIN
GLE_BATH_ELECTRON = 1

_ERRNAMES = {-1: "GLE_ERR_ARG", -2: "GLE_ERR_HIP", -3: "GLE_ERR_STATE", -4: "GLE_ERR_NOMEM",
             -5: "GLE_ERR_UNSUP"}

# every symbol include/hipgle.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "gle_abi_version", "gle_create", "gle_destroy", "gle_last_error", "gle_device_count",
    "gle_add_bath", "gle_set_dyn", "gle_set_constraint", "gle_set_state", "gle_get_state",
    "gle_set_history", "gle_get_history", "gle_get_force", "gle_set_noise", "gle_get_noise",
    "gle_noise_factors", "gle_noise_generate", "gle_step_begin", "gle_step_end", "gle_run",
    "gle_sync", "gle_get_current", "gle_get_energy", "gle_current_sums", "gle_profile",
    "gle_profile_read", "gle_profile_read_device", "gle_profile_read_chain", "gle_plan_info", "gle_add_bath_gmem", "gle_get_kernel", "gle_gamt",
    "gle_profile_levels", "gle_step_work", "gle_reduce_current", "gle_comm_unique_id", "gle_comm_init",
    "gle_comm_destroy", "gle_record", "gle_record_zero", "gle_get_record", "gle_get_record_history",
    "gle_power_spectrum", "gle_set_record", "gle_set_record_history", "gle_noise_stream_begin",
    "gle_noise_stream_chunk", "gle_noise_stream_end", "gle_set_plan_class", "gle_plan_detail", "gle_plan_flags",
    "gle_comm_allreduce", "gle_noise_stream_abort", "gle_device_mem_info", "gle_noise_stream_shared",
    "gle_noise_stream_retain", "gle_noise_stream_retained", "gle_noise_stream_replay", "gle_get_full_history",
    "gle_host_alloc", "gle_host_free", "gle_cache_audit", "gle_noise_stream_retain_cap", "gle_chain_work",
]

REC_P, REC_Q, REC_F, REC_HIST = 1, 2, 4, 8


class GLEError(RuntimeError):
    pass


class gle_config(ctypes.Structure):
    _fields_ = [("nph", ctypes.c_int64), ("ntraj", ctypes.c_int64), ("nmd", ctypes.c_int64),
                ("dt", ctypes.c_double), ("device", ctypes.c_int32), ("block_len", ctypes.c_int32),
                ("far_mode", ctypes.c_int32), ("max_block", ctypes.c_int32)]

FAR_AUTO, FAR_DIRECT, FAR_SPECTRAL = 0, 1, 2
FAR_MODES = {"auto": FAR_AUTO, "direct": FAR_DIRECT, "spectral": FAR_SPECTRAL}
PLAN_AUTO, PLAN_SMALL_BATHS, PLAN_LARGE_BATHS = 0, 1, 2
PLAN_CLASSES = {"auto": PLAN_AUTO, "small": PLAN_SMALL_BATHS, "large": PLAN_LARGE_BATHS}


_P = ctypes.c_void_p
_D = ctypes.POINTER(ctypes.c_double)
_I64 = ctypes.POINTER(ctypes.c_int64)

_SIGS = {
    "gle_abi_version": (ctypes.c_int, []),
    "gle_create": (ctypes.c_int, [ctypes.POINTER(gle_config), ctypes.POINTER(_P)]),
    "gle_destroy": (ctypes.c_int, [_P]),
    "gle_last_error": (ctypes.c_char_p, [_P]),
    "gle_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32)]),
    "gle_device_mem_info": (ctypes.c_int, [ctypes.c_int32, _I64, _I64]),
    "gle_add_bath": (ctypes.c_int, [_P, ctypes.c_int32, _I64, ctypes.c_int64, ctypes.c_int64, _D,
                                    ctypes.c_double, _D, _D, _D, ctypes.POINTER(ctypes.c_int32)]),
    "gle_add_bath_gmem": (ctypes.c_int, [_P, _I64, ctypes.c_int64, ctypes.c_int64, _D, ctypes.c_int64, _D,
                                         ctypes.POINTER(ctypes.c_int32)]),
    "gle_get_kernel": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _D]),
    "gle_gamt": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _D, _D, _D]),
    "gle_set_dyn": (ctypes.c_int, [_P, _D]),
    "gle_set_constraint": (ctypes.c_int, [_P, _I64, ctypes.c_int64]),
    "gle_set_state": (ctypes.c_int, [_P, _D, _D, ctypes.c_int64]),
    "gle_get_state": (ctypes.c_int, [_P, _D, _D, _I64]),
    "gle_set_history": (ctypes.c_int, [_P, ctypes.c_int32, _D]),
    "gle_get_history": (ctypes.c_int, [_P, ctypes.c_int32, _D]),
    "gle_get_force": (ctypes.c_int, [_P, _D]),
    "gle_set_noise": (ctypes.c_int, [_P, ctypes.c_int32, _D]),
    "gle_get_noise": (ctypes.c_int, [_P, ctypes.c_int32, _D]),
    "gle_noise_factors": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, _D, _D]),
    "gle_noise_generate": (ctypes.c_int, [_P, ctypes.c_int32, _D, ctypes.c_uint64, ctypes.c_uint64]),
    "gle_step_begin": (ctypes.c_int, [_P, _D, _D]),
    "gle_step_end": (ctypes.c_int, [_P, _D]),
    "gle_run": (ctypes.c_int, [_P, ctypes.c_int64]),
    "gle_sync": (ctypes.c_int, [_P]),
    "gle_get_current": (ctypes.c_int, [_P, _D]),
    "gle_get_energy": (ctypes.c_int, [_P, _D]),
    "gle_current_sums": (ctypes.c_int, [_P, _D]),
    "gle_profile": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_profile_read": (ctypes.c_int, [_P, _I64, _D, _D, _D]),
    "gle_profile_read_device": (ctypes.c_int, [_P, _I64, _D]),
    "gle_profile_read_chain": (ctypes.c_int, [_P, _I64, _D, _D]),
    "gle_plan_info": (ctypes.c_int, [_P, _I64, _I64, _I64, ctypes.POINTER(ctypes.c_int32)]),
    "gle_profile_levels": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.POINTER(ctypes.c_int32), _D]),
    "gle_step_work": (ctypes.c_int, [_P, _D, _D]),
    "gle_chain_work": (ctypes.c_int, [_P, _D, _D]),
    "gle_set_plan_class": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_plan_detail": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), _D,
                                       ctypes.POINTER(ctypes.c_int32), _I64, ctypes.POINTER(ctypes.c_int32)]),
    "gle_plan_flags": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32)]),
    "gle_reduce_current": (ctypes.c_int, [_P, _P, _D]),
    "gle_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "gle_comm_init": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                     ctypes.POINTER(_P)]),
    "gle_comm_destroy": (ctypes.c_int, [_P]),
    "gle_comm_allreduce": (ctypes.c_int, [_P, _P, _D, ctypes.c_int64]),
    "gle_noise_stream_abort": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_record": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_record_zero": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_get_record": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _D]),
    "gle_get_record_history": (ctypes.c_int, [_P, _D, _D, _I64]),
    "gle_power_spectrum": (ctypes.c_int, [_P, ctypes.c_int32, _I64, _I64, _D]),
    "gle_set_record": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _D]),
    "gle_set_record_history": (ctypes.c_int, [_P, _D, _D]),
    "gle_noise_stream_begin": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]),
    "gle_noise_stream_chunk": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _D, _D,
                                              ctypes.c_uint64, ctypes.c_uint64]),
    "gle_noise_stream_end": (ctypes.c_int, [_P, ctypes.c_int32]),
    "gle_noise_stream_shared": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _D, _D, _D,
                                               ctypes.c_uint64, ctypes.c_uint64]),
    "gle_get_full_history": (ctypes.c_int, [_P, ctypes.c_int64, _D, _D]),
    "gle_host_alloc": (ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(_P)]),
    "gle_host_free": (ctypes.c_int, [_P]),
    "gle_cache_audit": (ctypes.c_int, [_P, _I64]),
    "gle_noise_stream_retain": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32]),
    "gle_noise_stream_retained": (ctypes.c_int, [_P, ctypes.c_int32, _I64]),
    "gle_noise_stream_retain_cap": (ctypes.c_int, [_P, ctypes.c_int64]),
    "gle_noise_stream_replay": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64]),
}

_lib = None


def load():
    """Load libhipgle.so (raises GLEError with the build hint when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GLEError("hipgle library not found at %s -- build it with `make` or "
                       "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older library (A/B experiments); build() checks the release one exports all
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(_D)


def _f64(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if shape is not None and a.shape != tuple(shape):
        a = a.reshape(shape)
    return a


def device_mem_info(device=0):
    """(free, total) bytes of HIP device `device` (gle_device_mem_info)."""
    lib = load()
    fr, tot = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.gle_device_mem_info(int(device), ctypes.byref(fr), ctypes.byref(tot))
    if rc != 0:
        raise GLEError("gle_device_mem_info failed: %s" % lib.gle_last_error(None).decode())
    return int(fr.value), int(tot.value)


class HostBuffer:
    """Page-locked host memory (gle_host_alloc) viewed as a float64 numpy array of `shape`: device
    reads into it run at the link's rate.  free() releases it; no view of .array may outlive that."""

    def __init__(self, shape):
        lib = load()
        n = int(np.prod(shape))
        p = _P()
        if lib.gle_host_alloc(n * 8, ctypes.byref(p)) != 0:
            raise GLEError("gle_host_alloc(%d bytes) failed: %s" % (n * 8, lib.gle_last_error(None).decode()))
        self._lib, self._p = lib, p.value
        self.array = np.ctypeslib.as_array((ctypes.c_double * max(n, 1)).from_address(self._p))[:n].reshape(shape)

    def free(self):
        if getattr(self, "_p", None):
            self.array = None
            self._lib.gle_host_free(self._p)
            self._p = None

    __del__ = free


def device_count():
    lib = load()
    n = ctypes.c_int32(0)
    rc = lib.gle_device_count(ctypes.byref(n))
    return int(n.value) if rc == 0 else 0


def gamt_device(W, G, device=0):
    """out[i] = sum_g W[i, g] G[g] on the device (the contraction of gamt, baths.py:19-52).
    W (ml, ngw); G (ngw, ...) -> (ml, ...)."""
    lib = load()
    W = _f64(W)
    G = np.asarray(G, dtype=np.float64)
    ml, ngw = W.shape
    if G.shape[0] != ngw:
        raise ValueError("gamt_device: W is (%d, %d) but G has %d rows" % (ml, ngw, G.shape[0]))
    tail = G.shape[1:]
    nel = int(np.prod(tail)) if tail else 1
    G2 = _f64(G, (ngw, nel))
    out = np.empty((ml, nel))
    rc = lib.gle_gamt(int(device), ml, ngw, nel, _ptr(W), _ptr(G2), _ptr(out))
    if rc != 0:
        raise GLEError("gle_gamt failed (%s): %s" % (_ERRNAMES.get(rc, rc), lib.gle_last_error(None).decode()))
    return out.reshape((ml,) + tail)


COMM_ID_BYTES = 128


def comm_unique_id():
    """RCCL unique id (bytes) for gle_comm_init; made by one rank, shared by the caller."""
    lib = load()
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    rc = lib.gle_comm_unique_id(buf)
    if rc != 0:
        raise GLEError("gle_comm_unique_id failed: %s" % lib.gle_last_error(None).decode())
    return buf.raw


class Comm:
    """RCCL communicator of the C-ABI (gle_comm_init): one rank per process and device."""

    def __init__(self, nranks, rank, device, uid):
        self.lib = load()
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("unique id must be %d bytes" % COMM_ID_BYTES)
        c = _P()
        rc = self.lib.gle_comm_init(int(nranks), int(rank), int(device), uid, ctypes.byref(c))
        if rc != 0:
            raise GLEError("gle_comm_init failed (%s): %s" % (_ERRNAMES.get(rc, rc),
                                                              self.lib.gle_last_error(None).decode()))
        self.c = c
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)

    def close(self):
        if getattr(self, "c", None):
            self.lib.gle_comm_destroy(self.c)
            self.c = None


class Stepper:
    """Owner of one gle_handle: a batch of ntraj trajectories of one system on one device."""

    def __init__(self, nph, ntraj, nmd, dt, device=0, block_len=0, far_mode="auto", max_block=0):
        self.lib = load()
        self.nph, self.ntraj, self.nmd, self.dt = int(nph), int(ntraj), int(nmd), float(dt)
        fm = FAR_MODES[far_mode] if isinstance(far_mode, str) else int(far_mode)
        cfg = gle_config(self.nph, self.ntraj, self.nmd, self.dt, int(device), int(block_len), fm,
                         int(max_block))
        h = _P()
        rc = self.lib.gle_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise GLEError("gle_create failed (%s): %s" % (_ERRNAMES.get(rc, rc),
                                                           self.lib.gle_last_error(None).decode()))
        self.h = h
        self.nbath = 0
        self.bath_nc = []
        self.bath_ml = []

    # --------------------------------------------------------------------------- helpers
    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.gle_last_error(self.h).decode() if self.h else ""
            raise GLEError("%s failed (%s): %s" % (what, _ERRNAMES.get(rc, rc), msg))

    def close(self):
        if getattr(self, "h", None):
            self.lib.gle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------------------- setup
    def add_bath(self, kind, cids, kernel, bias=0.0, exim=None, zeta1=None, zeta2=None):
        cids = np.ascontiguousarray(np.asarray(cids, dtype=np.int64))
        nc = len(cids)
        kernel = _f64(kernel)
        ml = kernel.shape[0]
        kernel = _f64(kernel, (ml, nc, nc))
        mats = [None if m is None else _f64(m, (nc, nc)) for m in (exim, zeta1, zeta2)]
        bid = ctypes.c_int32(-1)
        self._chk(self.lib.gle_add_bath(self.h, int(kind), cids.ctypes.data_as(_I64), nc, ml,
                                        _ptr(kernel), float(bias), _ptr(mats[0]), _ptr(mats[1]),
                                        _ptr(mats[2]), ctypes.byref(bid)), "gle_add_bath")
        self.nbath += 1
        self.bath_nc.append(nc)
        self.bath_ml.append(ml)
        return int(bid.value)

    def add_bath_gmem(self, cids, W, gamma):
        """Phonon bath whose memory kernel K_i = sum_g W[i, g] gamma[g] is built on the device
        (gle_add_bath_gmem)."""
        cids = np.ascontiguousarray(np.asarray(cids, dtype=np.int64))
        nc = len(cids)
        W = _f64(W)
        ml, ngw = W.shape
        gamma = _f64(gamma, (ngw, nc, nc))
        bid = ctypes.c_int32(-1)
        self._chk(self.lib.gle_add_bath_gmem(self.h, cids.ctypes.data_as(_I64), nc, ml, _ptr(W), ngw,
                                             _ptr(gamma), ctypes.byref(bid)), "gle_add_bath_gmem")
        self.nbath += 1
        self.bath_nc.append(nc)
        self.bath_ml.append(ml)
        return int(bid.value)

    def get_kernel(self, bath, i0=0, n=None):
        ml, nc = self.bath_ml[bath], self.bath_nc[bath]
        n = ml - i0 if n is None else n
        out = np.empty((n, nc, nc))
        self._chk(self.lib.gle_get_kernel(self.h, int(bath), int(i0), int(n), _ptr(out)), "gle_get_kernel")
        return out

    def set_dyn(self, dyn):
        d = _f64(dyn, (self.nph, self.nph))
        self._chk(self.lib.gle_set_dyn(self.h, _ptr(d)), "gle_set_dyn")

    def set_constraint(self, dofs):
        d = np.ascontiguousarray(np.asarray(sorted(set(int(x) for x in dofs)), dtype=np.int64))
        self._chk(self.lib.gle_set_constraint(self.h, d.ctypes.data_as(_I64), len(d)),
                  "gle_set_constraint")

    def set_state(self, p, q, t):
        p = _f64(p, (self.ntraj, self.nph))
        q = _f64(q, (self.ntraj, self.nph))
        self._chk(self.lib.gle_set_state(self.h, _ptr(p), _ptr(q), int(t)), "gle_set_state")

    def get_state(self):
        p = np.empty((self.ntraj, self.nph))
        q = np.empty((self.ntraj, self.nph))
        t = ctypes.c_int64(0)
        self._chk(self.lib.gle_get_state(self.h, _ptr(p), _ptr(q), ctypes.byref(t)), "gle_get_state")
        return p, q, int(t.value)

    def set_history(self, bath, phis=None):
        if phis is not None:
            phis = _f64(phis, (self.ntraj, self.bath_ml[bath], self.bath_nc[bath]))
        self._chk(self.lib.gle_set_history(self.h, int(bath), _ptr(phis)), "gle_set_history")

    def get_history(self, bath):
        out = np.empty((self.ntraj, self.bath_ml[bath], self.bath_nc[bath]))
        self._chk(self.lib.gle_get_history(self.h, int(bath), _ptr(out)), "gle_get_history")
        return out

    def get_force(self):
        out = np.empty((self.ntraj, self.nph))
        self._chk(self.lib.gle_get_force(self.h, _ptr(out)), "gle_get_force")
        return out

    def set_noise(self, bath, noise):
        n = _f64(noise, (self.ntraj, self.nmd, self.bath_nc[bath]))
        self._chk(self.lib.gle_set_noise(self.h, int(bath), _ptr(n)), "gle_set_noise")

    def get_noise(self, bath):
        out = np.empty((self.ntraj, self.nmd, self.bath_nc[bath]))
        self._chk(self.lib.gle_get_noise(self.h, int(bath), _ptr(out)), "gle_get_noise")
        return out

    def noise_factors(self, bath, m):
        """m: (nfreq, nc, nc) real or complex spectral factors."""
        m = np.asarray(m)
        nf = m.shape[0]
        mre = _f64(np.real(m))
        mim = _f64(np.imag(m)) if np.iscomplexobj(m) else None
        self._chk(self.lib.gle_noise_factors(self.h, int(bath), nf, _ptr(mre), _ptr(mim)),
                  "gle_noise_factors")

    def noise_generate(self, bath, x=None, seed=0, traj_offset=0):
        if x is not None:
            x = _f64(x)
        self._chk(self.lib.gle_noise_generate(self.h, int(bath), _ptr(x), int(seed) & (2**64 - 1),
                                              int(traj_offset)), "gle_noise_generate")

    def noise_stream(self, bath, factor_chunks, is_complex, seed, traj_offset=0, max_chunk=64):
        """Streamed device noise: factor_chunks yields (w0, M) with M (nw, nc, nc) real or complex."""
        self._chk(self.lib.gle_noise_stream_begin(self.h, int(bath), 1 if is_complex else 0, int(max_chunk)),
                  "gle_noise_stream_begin")
        try:
            for w0, m in factor_chunks:
                mre = _f64(np.real(m))
                mim = _f64(np.imag(m)) if is_complex else None
                self._chk(self.lib.gle_noise_stream_chunk(self.h, int(bath), int(w0), int(m.shape[0]), _ptr(mre),
                                                          _ptr(mim), int(seed) & (2**64 - 1), int(traj_offset)),
                          "gle_noise_stream_chunk")
        except BaseException:
            # a failed chunk or factor generator (e.g. LinAlgError) must not leave the spectrum
            # scratch (1-2 GB per C5 bath) on the device
            self.lib.gle_noise_stream_abort(self.h, int(bath))
            raise
        self._chk(self.lib.gle_noise_stream_end(self.h, int(bath)), "gle_noise_stream_end")

    def noise_stream_plan(self, bath, segments, is_complex, seed, traj_offset=0, max_chunk=64):
        """Streamed device noise from work segments (noise.stream_factor_plan): ("dense", w0, M) with
        M (nw, nc, nc) per-frequency factors, ("shared", w0, nw, scale, F) one factor F times
        scale[w] for frequencies [w0, w0 + nw); frequencies in no segment get no noise."""
        self._chk(self.lib.gle_noise_stream_begin(self.h, int(bath), 1 if is_complex else 0, int(max_chunk)),
                  "gle_noise_stream_begin")
        sd = int(seed) & (2**64 - 1)
        try:
            for seg in segments:
                if seg[0] == "dense":
                    _, w0, m = seg
                    # complex factors arrive as (Re, Im) planes (noise.stream_factor_plan) or complex
                    mr, mi = m if isinstance(m, tuple) else (np.real(m), np.imag(m) if is_complex else None)
                    for o in range(0, mr.shape[0], max_chunk):
                        mre = _f64(mr[o:o + max_chunk])
                        mim = _f64(mi[o:o + max_chunk]) if is_complex else None
                        self._chk(self.lib.gle_noise_stream_chunk(self.h, int(bath), int(w0 + o), int(mre.shape[0]),
                                                                  _ptr(mre), _ptr(mim), sd, int(traj_offset)),
                                  "gle_noise_stream_chunk")
                else:
                    _, w0, nw, scale, f = seg
                    sc = _f64(scale)
                    fre = _f64(np.real(f))
                    fim = _f64(np.imag(f)) if is_complex else None
                    self._chk(self.lib.gle_noise_stream_shared(self.h, int(bath), int(w0), int(nw), _ptr(sc),
                                                               _ptr(fre), _ptr(fim), sd, int(traj_offset)),
                              "gle_noise_stream_shared")
        except BaseException:
            self.lib.gle_noise_stream_abort(self.h, int(bath))
            raise
        self._chk(self.lib.gle_noise_stream_end(self.h, int(bath)), "gle_noise_stream_end")

    def noise_stream_retain(self, bath, retain=True):
        """Keep the next complete streamed plan's factors on the device (False frees them)."""
        self._chk(self.lib.gle_noise_stream_retain(self.h, int(bath), 1 if retain else 0), "gle_noise_stream_retain")

    def noise_stream_retain_cap(self, max_bytes):
        """Cap on the retained plans' device bytes over all baths (None: no cap)."""
        self._chk(self.lib.gle_noise_stream_retain_cap(self.h, -1 if max_bytes is None else int(max_bytes)),
                  "gle_noise_stream_retain_cap")

    def noise_stream_retained(self, bath):
        """Device bytes of the retained complete plan of `bath` (0: none)."""
        n = ctypes.c_int64(0)
        self._chk(self.lib.gle_noise_stream_retained(self.h, int(bath), ctypes.byref(n)), "gle_noise_stream_retained")
        return n.value

    def noise_stream_replay(self, bath, seed, traj_offset=0):
        """New noise from the retained plan (= streaming that plan again with this seed)."""
        self._chk(self.lib.gle_noise_stream_replay(self.h, int(bath), int(seed) & (2**64 - 1), int(traj_offset)),
                  "gle_noise_stream_replay")

    # --------------------------------------------------------------------------- stepping
    def step_begin(self, fpot=None, want_qt=True):
        f = None if fpot is None else _f64(fpot, (self.ntraj, self.nph))
        qt = np.empty((self.ntraj, self.nph)) if want_qt else None
        self._chk(self.lib.gle_step_begin(self.h, _ptr(f), _ptr(qt)), "gle_step_begin")
        return qt

    def step_end(self, fpot_qt=None):
        f = None if fpot_qt is None else _f64(fpot_qt, (self.ntraj, self.nph))
        self._chk(self.lib.gle_step_end(self.h, _ptr(f)), "gle_step_end")

    def run(self, nsteps):
        self._chk(self.lib.gle_run(self.h, int(nsteps)), "gle_run")

    def sync(self):
        self._chk(self.lib.gle_sync(self.h), "gle_sync")

    # --------------------------------------------------------------------------- outputs
    def get_current(self):
        out = np.empty((self.nbath, self.ntraj, self.nmd))
        self._chk(self.lib.gle_get_current(self.h, _ptr(out)), "gle_get_current")
        return out

    def get_energy(self):
        out = np.empty((self.ntraj, self.nmd))
        self._chk(self.lib.gle_get_energy(self.h, _ptr(out)), "gle_get_energy")
        return out

    def current_sums(self):
        out = np.empty((self.nbath, 3))
        self._chk(self.lib.gle_current_sums(self.h, _ptr(out)), "gle_current_sums")
        return out

    # --------------------------------------------------------------------------- recordings
    def record(self, flags):
        """Record REC_P / REC_Q / REC_F / REC_HIST on the device from the next step on (gle_record)."""
        self._chk(self.lib.gle_record(self.h, int(flags)), "gle_record")

    def record_zero(self, flags):
        self._chk(self.lib.gle_record_zero(self.h, int(flags)), "gle_record_zero")

    def get_record(self, what, bath=0):
        """REC_P / REC_Q: (ntraj, nmd, nph); REC_F: (ntraj, nmd, nc) of `bath`."""
        cols = self.bath_nc[bath] if what == REC_F else self.nph
        out = np.empty((self.ntraj, self.nmd, cols))
        self._chk(self.lib.gle_get_record(self.h, int(what), int(bath), _ptr(out)), "gle_get_record")
        return out

    def get_record_history(self):
        """(phis, qhis) on every DOF, newest first: (ntraj, ml, nph) each."""
        ml = ctypes.c_int64(0)
        self._chk(self.lib.gle_get_record_history(self.h, None, None, ctypes.byref(ml)), "gle_get_record_history")
        ph = np.empty((self.ntraj, ml.value, self.nph))
        qh = np.empty((self.ntraj, ml.value, self.nph))
        self._chk(self.lib.gle_get_record_history(self.h, _ptr(ph), _ptr(qh), ctypes.byref(ml)),
                  "gle_get_record_history")
        return ph, qh

    def get_full_history(self, ml, out_p=None, out_q=None):
        """(phis, qhis) as MD{j}.nc stores them: (ntraj, ml, nph) each, recorded rows with the baths'
        own rings on their DOFs (gle_get_full_history); written into out_p / out_q when given
        (C-contiguous float64 of that shape, e.g. HostBuffer arrays)."""
        shp = (self.ntraj, int(ml), self.nph)
        outs = []
        for o in (out_p, out_q):
            if o is None:
                o = np.empty(shp)
            elif o.shape != shp or o.dtype != np.float64 or not o.flags.c_contiguous:
                raise ValueError("history output must be C-contiguous float64 %s" % (shp,))
            outs.append(o)
        self._chk(self.lib.gle_get_full_history(self.h, int(ml), _ptr(outs[0]), _ptr(outs[1])), "gle_get_full_history")
        return outs[0], outs[1]

    def set_record(self, what, arr, bath=0):
        cols = self.bath_nc[bath] if what == REC_F else self.nph
        a = _f64(np.broadcast_to(np.asarray(arr, dtype=np.float64), (self.ntraj, self.nmd, cols)))
        self._chk(self.lib.gle_set_record(self.h, int(what), int(bath), _ptr(a)), "gle_set_record")

    def set_record_history(self, phis=None, qhis=None):
        ml = ctypes.c_int64(0)
        self._chk(self.lib.gle_get_record_history(self.h, None, None, ctypes.byref(ml)), "gle_get_record_history")
        shp = (self.ntraj, ml.value, self.nph)
        ph = None if phis is None else _f64(np.broadcast_to(np.asarray(phis, dtype=np.float64), shp))
        qh = None if qhis is None else _f64(np.broadcast_to(np.asarray(qhis, dtype=np.float64), shp))
        self._chk(self.lib.gle_set_record_history(self.h, _ptr(ph), _ptr(qh)), "gle_set_record_history")

    def power_spectrum(self, groups):
        """sum_{k in group} |DFT_t ps[:, k]|^2 for each DOF group: (ngroup, ntraj, nmd)."""
        lens = np.ascontiguousarray([len(g) for g in groups], dtype=np.int64)
        dofs = np.ascontiguousarray(np.concatenate([np.asarray(g, dtype=np.int64) for g in groups]) if len(groups)
                                    else np.zeros(0, dtype=np.int64), dtype=np.int64)
        out = np.empty((len(groups), self.ntraj, self.nmd))
        self._chk(self.lib.gle_power_spectrum(self.h, len(groups), lens.ctypes.data_as(_I64),
                                              dofs.ctypes.data_as(_I64), _ptr(out)), "gle_power_spectrum")
        return out

    def reduce_current(self, comm=None):
        """Ensemble current statistics [nbath][3] summed over the ranks of an RCCL Comm (None: this
        handle only) -- gle_reduce_current."""
        out = np.empty((self.nbath, 3))
        self._chk(self.lib.gle_reduce_current(self.h, None if comm is None else comm.c, _ptr(out)),
                  "gle_reduce_current")
        return out

    def comm_allreduce(self, comm, values):
        """Sum a float64 vector over the ranks of an RCCL Comm (None: unchanged) on this handle's
        stream -- gle_comm_allreduce."""
        buf = np.ascontiguousarray(np.asarray(values, dtype=np.float64)).copy()
        self._chk(self.lib.gle_comm_allreduce(self.h, None if comm is None else comm.c, _ptr(buf), buf.size),
                  "gle_comm_allreduce")
        return buf

    def profile(self, enable=True, events=True, chain=False):
        """enable: count ladder blocks; events: also HIP-event timing of the dominant kernel;
        chain: per-workgroup device stamps of the per-step chain's launches."""
        mode = (PROFILE_COUNT | (PROFILE_EVENTS if events else 0) | (PROFILE_CHAIN if chain else 0)) if enable else 0
        self._chk(self.lib.gle_profile(self.h, mode), "gle_profile")

    def profile_read(self):
        n = ctypes.c_int64(0)
        ms, fl, by = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_double(0)
        self._chk(self.lib.gle_profile_read(self.h, ctypes.byref(n), ctypes.byref(ms),
                                            ctypes.byref(fl), ctypes.byref(by)), "gle_profile_read")
        out = {"launches": int(n.value), "ms": ms.value, "flops": fl.value, "bytes": by.value}
        nd, msd = ctypes.c_int64(0), ctypes.c_double(0)
        self._chk(self.lib.gle_profile_read_device(self.h, ctypes.byref(nd), ctypes.byref(msd)),
                  "gle_profile_read_device")
        out["launches_device"], out["ms_device"] = int(nd.value), msd.value
        nc, msc, flc = ctypes.c_int64(0), ctypes.c_double(0), ctypes.c_double(0)
        self._chk(self.lib.gle_profile_read_chain(self.h, ctypes.byref(nc), ctypes.byref(msc), ctypes.byref(flc)),
                  "gle_profile_read_chain")
        out["chain_launches"], out["chain_ms"], out["chain_flops"] = int(nc.value), msc.value, flc.value
        return out

    def plan_info(self):
        a, b, c = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        m = ctypes.c_int32(0)
        self._chk(self.lib.gle_plan_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                         ctypes.byref(m)), "gle_plan_info")
        names = {v: k for k, v in FAR_MODES.items()}
        return {"block_len": int(a.value), "far_items": int(b.value), "device_bytes": int(c.value),
                "far_mode": names.get(int(m.value), int(m.value))}

    def set_plan_class(self, plan_class):
        """Force the plan class ("auto", "small", "large"; gle_set_plan_class) before set_state."""
        self._chk(self.lib.gle_set_plan_class(self.h, PLAN_CLASSES[plan_class]), "gle_set_plan_class")

    def plan_detail(self):
        """The built plan: class, fused-stage waves, far-field workgroups per CU, ladder levels."""
        c, w, n, ff = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        cu, dd = ctypes.c_double(0), ctypes.c_int64(0)
        self._chk(self.lib.gle_plan_detail(self.h, ctypes.byref(c), ctypes.byref(w), ctypes.byref(cu),
                                           ctypes.byref(n), ctypes.byref(dd), ctypes.byref(ff)), "gle_plan_detail")
        names = {v: k for k, v in PLAN_CLASSES.items()}
        fl = ctypes.c_int32(0)
        self._chk(self.lib.gle_plan_flags(self.h, ctypes.byref(fl)), "gle_plan_flags")
        return {"plan_class": names.get(int(c.value), int(c.value)), "fused_waves": int(w.value),
                "cg_per_cu": float(cu.value), "nlevel": int(n.value), "dyn_dropped": int(dd.value),
                "far_fused": bool(ff.value), "fpot_launch": bool(fl.value & 2),
                "composed_step": bool(fl.value & 8), "split_tiles": bool(fl.value & 16)}

    def cache_audit(self):
        """(at q~, at q_{t+1} after a constraint): composed steps at which md.potforce's cache rule
        would have reused a force within 1e-9 of a different point (gle_cache_audit)."""
        c = (ctypes.c_int64 * 2)()
        self._chk(self.lib.gle_cache_audit(self.h, c), "gle_cache_audit")
        return int(c[0]), int(c[1])

    def profile_levels(self):
        """[(P, blocks issued since profiling was enabled)] per ladder level."""
        n = ctypes.c_int32(0)
        self._chk(self.lib.gle_profile_levels(self.h, 0, ctypes.byref(n), None, None), "gle_profile_levels")
        P = (ctypes.c_int32 * max(1, n.value))()
        bl = np.zeros(max(1, n.value))
        self._chk(self.lib.gle_profile_levels(self.h, n.value, ctypes.byref(n), P, _ptr(bl)),
                  "gle_profile_levels")
        return [(int(P[i]), float(bl[i])) for i in range(n.value)]

    def step_work(self):
        """Algorithmic (flops, bytes) of one steady-state step of the plan (gle_step_work)."""
        fl, by = ctypes.c_double(0), ctypes.c_double(0)
        self._chk(self.lib.gle_step_work(self.h, ctypes.byref(fl), ctypes.byref(by)), "gle_step_work")
        return fl.value, by.value

    def chain_work(self):
        """Algorithmic (flops, bytes) of one step's chain launches (gle_chain_work)."""
        fl, by = ctypes.c_double(0), ctypes.c_double(0)
        self._chk(self.lib.gle_chain_work(self.h, ctypes.byref(fl), ctypes.byref(by)), "gle_chain_work")
        return fl.value, by.value
