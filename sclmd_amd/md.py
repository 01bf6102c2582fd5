"""Langevin MD engine with sclmd's md API (sclmd/md.py), stepping on the MI355X.

The constructor, setters and Run() follow sclmd/md.py:56-682 so examples/runmd.py only changes its
import line.  Extensions (keyword-only): ntraj (independent noise realisations batched on the
device), seed / traj_offset (per-trajectory RNG streams), noise_mode ("numpy": reference-compatible
legacy-RNG draws; "device": Philox draws on the GPU), device, block_len, comm.

State lives on the device after the first step; md.p / md.q / md.t read it back on access.
With ntraj == 1 arrays have the reference's shapes ((nph,), (nmd,)); with ntraj > 1 a leading
trajectory axis is added.
"""
import os
import sys
import time

import numpy as np

from . import _native
from . import units as U
from .functions import bose, chkShape, mdot, symmetrize


def sameq(q1, q2):
    """Cached-force test of md.potforce: same length and max|dq| < 1e-9 (md.py:767-779)."""
    if len(q1) != len(q2):
        return False
    return bool(np.max(np.abs(np.asarray(q1) - np.asarray(q2))) < 10e-10)


def ApplyConstraint(f, constr=None):
    """Zero the listed DOF index ranges on a copy (md.py:782-794)."""
    if constr is None:
        return f
    nf = np.array(f) * 1.0
    for c in constr:
        nf[..., list(c)] = 0
    return nf


class md:
    def __init__(self, dt, nmd, T, syslist=None, axyz=None, dyn=None, nstart=0, nstop=1, npie=1,
                 md2ang=0.06466, *, ntraj=1, seed=None, traj_offset=0, device=None,
                 noise_mode="numpy", block_len=0, far_mode="auto", max_block=0, comm=None, verbose=True):
        self.nstart, self.nstop = nstart, nstop
        self.dt, self.nmd = dt, nmd
        self.T = T
        self.npie = npie
        self.saveall = self.savep = self.saveq = self.rmnc = False
        self.nstep = None
        self.pforce = None
        self.constraint = None
        self.atomlist = None
        self.verbose = verbose
        self.ntraj = int(ntraj)
        self.seed = seed
        self.traj_offset = int(traj_offset)
        if noise_mode not in ("numpy", "device"):
            raise ValueError("noise_mode must be 'numpy' or 'device'")
        self.noise_mode = noise_mode
        self.device = device
        self.block_len = int(block_len)
        self.far_mode = far_mode
        self.max_block = int(max_block)
        self.comm = comm
        self.SetXyz(axyz)
        if syslist is not None:
            if len(syslist) > self.nta or min(syslist) < 0 or max(syslist) > self.nta - 1:
                raise ValueError("syslist out of range")
            self.syslist = np.array(syslist, dtype=int)
            self.na = len(syslist)
            self.nph = 3 * len(syslist)
        elif axyz is not None:
            self.syslist = np.arange(len(axyz))
            self.na = len(self.syslist)
            self.nph = 3 * self.na
        else:
            self.syslist = self.na = self.nph = None
        self.ml = 1
        self.cf = 0
        self._t = 0
        self._p = []
        self._q = []
        self.pinit, self.qinit = [], []
        self.q0, self.f0 = [], []
        self.baths = []
        self.fhis = []
        self.fbaths = []
        self.etot_host = np.zeros(nmd)
        self.initranvel = True
        self.setDyn(dyn)
        self.md2ang = md2ang
        self.mass = []
        self.get_atommass()
        if self.els is not None and len(self.mass) != len(self.els):
            raise ValueError("Wrong setting in els or mass")
        self.conv = (self.md2ang * np.array([3 * [1.0 / np.sqrt(m)] for m in self.mass]).flatten()
                     if self.mass else None)
        self._st = None            # device stepper
        self._dev_newer = False    # device holds newer p/q/t than the host mirrors
        self._host_newer = True
        self._noise_versions = {}
        self._rngs = None
        self.kappa_runs = []

    # ------------------------------------------------------------------------------ logging
    def _log(self, *a):
        if self.verbose:
            print(*a)

    # ------------------------------------------------------------------------------ state access
    def _pull(self):
        if self._st is not None and self._dev_newer:
            p, q, t = self._st.get_state()
            if self.ntraj == 1:
                p, q = p[0], q[0]
            self._p, self._q, self._t = p, q, t
            self._dev_newer = False

    @property
    def p(self):
        self._pull()
        return self._p

    @p.setter
    def p(self, v):
        self._pull()
        self._p = np.asarray(v, dtype=float)
        self._host_newer = True

    @property
    def q(self):
        self._pull()
        return self._q

    @q.setter
    def q(self, v):
        self._pull()
        self._q = np.asarray(v, dtype=float)
        self._host_newer = True

    @property
    def t(self):
        self._pull()
        return self._t

    @t.setter
    def t(self, v):
        self._pull()
        self._t = int(v)
        self._host_newer = True

    @property
    def etot(self):
        if self._st is None:
            return self.etot_host
        e = self._st.get_energy()
        return e[0] if self.ntraj == 1 else e

    # ------------------------------------------------------------------------------ setup API
    def get_atommass(self):
        if self.els is None:
            return
        for name in self.els:
            if name in U.AtomicMassTable:
                self.mass.append(U.AtomicMassTable[name])

    def info(self):
        self._log("--------------------------------------------")
        self._log("Basis information of the MD simulation:")
        self._log("System atom number:" + str(self.na))
        self._log("MD time step:" + str(self.dt))
        self._log("MD number of steps:" + str(self.nmd))
        self._log("MD memory kernel length:" + str(self.ml))
        self._log("Number of baths attached:" + str(len(self.baths)))
        self._log("Trajectories on this device:" + str(self.ntraj))

    def ResetSavepq(self):
        """Zero the recorded p / q series of the run (md.py:571-574 at a new run).  The series are
        recorded on the device by the step itself (gle_record), for every trajectory."""
        if self._st is not None:
            self._st.record_zero(_native.REC_P | _native.REC_Q)

    # ------------------------------------------------------------------------------ recordings
    def _rec_flags(self):
        f = 0
        if self.savep:
            f |= _native.REC_P
        if self.saveq:
            f |= _native.REC_Q
        if self.saveall:
            f |= _native.REC_F
        if getattr(self, "_in_run", False):
            f |= _native.REC_HIST  # md.phis / md.qhis on every DOF for the MD{j}.nc checkpoints
        return f

    def _apply_record(self):
        if self._st is not None:
            f = self._rec_flags()
            if f != getattr(self, "_rec_applied", None):
                self._st.record(f)
                self._rec_applied = f

    def _rec(self, what):
        st = self._ensure_device()
        self._apply_record()
        if not (self._rec_applied & what):
            return None
        return st.get_record(what)

    @property
    def ps(self):
        """md.ps (md.py:374-375): (nmd, nph), or (ntraj, nmd, nph); recorded on the device."""
        r = self._rec(_native.REC_P)
        if r is None:
            return None
        return r[0] if self.ntraj == 1 else r

    @ps.setter
    def ps(self, v):
        self._ensure_device()
        self._apply_record()
        self._st.set_record(_native.REC_P, np.asarray(v, dtype=float))

    @property
    def qs(self):
        """md.qs (md.py:376-377): (nmd, nph), or (ntraj, nmd, nph); recorded on the device."""
        r = self._rec(_native.REC_Q)
        if r is None:
            return None
        return r[0] if self.ntraj == 1 else r

    @qs.setter
    def qs(self, v):
        self._ensure_device()
        self._apply_record()
        self._st.set_record(_native.REC_Q, np.asarray(v, dtype=float))

    def fhis_of(self, i):
        """md.fhis[i] (md.py:398): bath i's id0 force of every step of the run on all DOFs, (nmd, nph)
        or (ntraj, nmd, nph); recorded on the device with SaveAll."""
        st = self._ensure_device()
        self._apply_record()
        if not (self._rec_applied & _native.REC_F):
            return None
        r = st.get_record(_native.REC_F, i)
        out = np.zeros((self.ntraj, self.nmd, self.nph))
        out[:, :, np.asarray(self.baths[i].cids)] = r
        return out[0] if self.ntraj == 1 else out

    def energy(self):
        """Kinetic energy 1/2 p.p (md.py:161-165)."""
        p = np.asarray(self.p)
        return 0.5 * np.sum(p * p, axis=-1)

    def AddBath(self, bath):
        if self.dt != bath.dt:
            raise ValueError("md.AddBath: md time step dt not consistent")
        if self.nmd != bath.nmd:
            raise ValueError("md.AddBath: number of md steps nmd not consistent")
        if self._st is not None:
            raise RuntimeError("md.AddBath: baths must be added before the first step")
        self.baths.append(bath)
        if bath.ml > self.ml:
            self.ml = bath.ml
        self.fbaths.append(np.zeros(self.nph))

    def AddPowerSection(self, atomlist):
        self.atomlist = atomlist
        self.poweratomlist = np.empty((len(self.atomlist), self.nmd, 2))

    def AddConstr(self, constr):
        self.constraint = constr

    def CalPowerSpec(self, cal=True):
        self.savep = cal
        self.power = np.empty((self.nmd, 2))

    def CalAveStruct(self, cal=True):
        self.saveq = cal

    def SaveAll(self, save=True):
        self.saveall = save

    def Savep(self, save=True):
        self.savep = save

    def Saveq(self, save=True):
        self.saveq = save

    def SaveTraj(self, nstep=100):
        self.nstep = nstep

    def RemoveNC(self, rmnc=True):
        self.rmnc = rmnc

    def SetT(self, T):
        self.T = T

    def SetMD(self, dt, nmd):
        self.dt, self.nmd = dt, nmd
        self.etot_host = np.zeros(nmd)

    def noranvel(self, rf=False):
        self.initranvel = rf

    def SetXyz(self, axyz):
        if axyz is not None:
            self.xyz = np.array([a[1:] for a in axyz], dtype="d").flatten()
            self.els = [a[0] for a in axyz]
            self.nta = len(axyz)
        else:
            self.xyz = self.els = self.nta = None

    def SetSyslist(self, syslist):
        self.syslist = np.array(syslist)
        self.na = len(syslist)
        self.nph = 3 * len(syslist)

    def setDyn(self, dyn=None):
        """Symmetrise, clip negative eigenvalues, keep U diag(w^2) U^T (md.py:250-292)."""
        if dyn is None:
            self.dyn, self.hw, self.U = None, [1.0], None
            return
        ndyn = np.array(dyn)
        n = chkShape(ndyn)
        if self.nph is not None and self.nph != n:
            raise ValueError("md.setDyn: the dimension of dynamical matrix is wrong")
        self.nph = n
        self.dyn = symmetrize(ndyn)
        av, au = np.linalg.eigh(self.dyn)
        if min(av) < 0:
            av = np.where(av < 0, 0.0, av)
        self.hw = np.array(list(map(np.real, list(map(np.sqrt, av)))))
        self.U = np.array(au)
        self.dyn = mdot(self.U, np.diag(np.array(av)), np.transpose(self.U))

    def AddPotential(self, pint):
        """Host force driver (md.py:481), or a list of drivers, one per trajectory of this rank's
        ensemble.  With a list, the trajectories' driver calls of a force phase run concurrently on
        a thread pool (LAMMPS / SIESTA / DeePMD release the GIL inside their engines), so an
        ensemble's host force phase costs about one driver call instead of ntraj of them.  A single
        driver instance is called for the trajectories one after another."""
        if isinstance(pint, (list, tuple)):
            if len(pint) != self.ntraj:
                raise ValueError("AddPotential: %d drivers for %d trajectories" % (len(pint), self.ntraj))
            self.pforces = list(pint)
            self.pforce = self.pforces[0]
        else:
            self.pforces = None
            self.pforce = pint

    def CompareForce(self, forcedriver):
        self.cf = 1
        self.forcedriver = forcedriver
        self.cflist = []

    # ------------------------------------------------------------------------------ RNG streams
    def _rng(self, b):
        """Trajectory b's random stream: the global numpy RNG (reference behaviour) when no seed is
        given, else RandomState(seed + traj_offset + b)."""
        if self.seed is None:
            return np.random
        if self._rngs is None:
            self._rngs = [np.random.RandomState(int(self.seed) + self.traj_offset + i)
                          for i in range(self.ntraj)]
        return self._rngs[b]

    def initialise(self):
        """Initial displacement and velocity from the modes of dyn (md.py:294-338)."""
        self._t = 0
        n = self.nph
        if self.dyn is None:
            p = np.zeros((self.ntraj, n))
            q = np.zeros((self.ntraj, n))
        else:
            av, au = self.hw, self.U
            p = np.zeros((self.ntraj, n))
            q = np.zeros((self.ntraj, n))
            for b in range(self.ntraj):
                rng = self._rng(b)
                dis = np.zeros(len(av))
                vel = np.zeros(len(av))
                for i in range(len(av)):
                    am = 0.0 if av[i] < 0.01 else ((bose(av[i], self.T) + 0.5) * 2.0 / av[i]) ** 0.5
                    r = rng.rand()
                    dis = dis + au[:, i] * am * np.cos(2.0 * np.pi * r)
                    vel = vel - av[i] * au[:, i] * am * np.sin(2.0 * np.pi * r)
                dis = ApplyConstraint(dis, self.constraint)
                vel = ApplyConstraint(vel, self.constraint)
                if self.initranvel:
                    p[b], q[b] = vel, dis
        if self.ntraj == 1:
            p, q = p[0], q[0]
        self._p, self._q = p, q
        self.pinit, self.qinit = p, q
        self._host_newer = True
        self._dev_newer = False

    def ResetHis(self):
        """Zero the friction-kernel history (md.py:340-349)."""
        if self.nph is None or self.ml is None:
            raise ValueError("self.nph and self.ml are not set")
        self._reset_his = True
        if self._st is not None:
            self._push_state()
            for i in range(len(self.baths)):
                self._st.set_history(i, None)
            self._reset_his = False

    # ------------------------------------------------------------------------------ device
    def _constr_dofs(self):
        if self.constraint is None:
            return []
        return sorted(set(int(d) for c in self.constraint for d in c))

    def _ensure_device(self):
        if self._st is not None:
            return self._st
        if self.nph is None:
            raise ValueError("md: the number of degrees of freedom is not set (axyz/dyn)")
        dev = self._device_ordinal()
        st = _native.Stepper(self.nph, self.ntraj, self.nmd, self.dt, dev, self.block_len, self.far_mode,
                             self.max_block)
        for b in self.baths:
            rec = getattr(b, "gmem_recipe", None)
            if rec is not None and b.__dict__.get("_kernel") is None:
                st.add_bath_gmem(b.cids, rec[0], rec[1])   # kernel built in HBM (phbath.gmem)
                continue
            if b.kernel is None:
                raise ValueError("md: bath %s has no kernel (call phbath.gmem())" % b)
            if b.kind == "ebath":
                if b.biased():
                    st.add_bath(_native.GLE_BATH_ELECTRON, b.cids, b.kernel, b.bias, b.exim, b.zeta1, b.zeta2)
                else:
                    st.add_bath(_native.GLE_BATH_ELECTRON, b.cids, b.kernel)
            else:
                st.add_bath(_native.GLE_BATH_PHONON, b.cids, b.kernel)
        if self.dyn is not None:
            st.set_dyn(self.dyn)
        c = self._constr_dofs()
        if c:
            st.set_constraint(c)
        self._st = st
        self._push_state()
        for i in range(len(self.baths)):
            st.set_history(i, None)
        self._reset_his = False
        return st

    def _push_state(self):
        if not self._host_newer:
            return
        p = np.asarray(self._p, dtype=float).reshape(self.ntraj, self.nph)
        q = np.asarray(self._q, dtype=float).reshape(self.ntraj, self.nph)
        self._st.set_state(p, q, self._t)
        self.q0, self.f0 = [], []
        self._host_newer = False

    def _sync_injected_noise(self):
        """Upload host-assigned bath.noise arrays that the device has not seen yet."""
        for i, b in enumerate(self.baths):
            if getattr(b, "_noise_src", None) is not None:
                continue
            v = getattr(b, "_noise_version", 0)
            if self._noise_versions.get(i) != v:
                n = b._noise_host
                if n is None:
                    raise RuntimeError("md: bath %d has no noise (call gnoi() or Run())" % i)
                n = np.asarray(n, dtype=float)
                if n.ndim == 2:
                    n = np.broadcast_to(n, (self.ntraj,) + n.shape)
                self._st.set_noise(i, n)
                self._noise_versions[i] = v

    # factors above this size are streamed to the device by frequency chunk instead of being held
    # there whole (C5: 4097 x 1000^2 doubles per bath beside ~200 GB of spectral kernels)
    noise_stream_bytes = 4 << 30
    # streamed baths keep their dense factors between runs (C5: ~11 GB for the three baths, against
    # ~46 s of factorisation per run without them): in device memory beside the plan when they fit
    # (gle_noise_stream_retain / _replay: no factor crosses PCIe after the first run), else on the host
    noise_factor_cache = True
    # largest fixed-size variable of an MD{j}.nc file (NetCDF classic format, scipy.io)
    nc_var_limit = 2**31 - 4096

    # device-mode baths whose spectrum is zero or one shared matrix at most of its frequencies (above
    # the cutoff: C3's phonon baths have 99 dense frequencies of 2049) take the streamed path too, which
    # factorises only the dense ones (the resident path decomposes, stores and uploads every frequency)
    stream_sparse_spectra = True

    def _sparse_spectrum(self, b):
        if not self.stream_sparse_spectra:
            return False
        key = b._noise_key()
        memo = getattr(b, "_sparse_memo", None)
        if memo is None or memo[0] != key:
            nfreq = int(self.nmd / 2) + 1
            ndense = sum(1 for i in range(nfreq) if b._spectrum_term(i, matrix=False)[0] == "dense")
            memo = b._sparse_memo = (key, 2 * ndense <= nfreq)
        return memo[1]

    # the ranks of one node split each streamed bath's factorisations and exchange the factors through
    # node-local shared memory (noise.NodeShare) instead of each factorising the whole spectrum
    share_factors = True

    def _node_share(self):
        """noise.NodeShare over this md's ranks, or None when it runs alone."""
        from . import ensemble
        from . import noise as _noise

        w = ensemble.world_size(self.comm)
        if w <= 1 or not self.share_factors:
            return None
        sh = getattr(self, "_share", None)
        if sh is None:
            r = ensemble.rank(self.comm)
            tok = float(int.from_bytes(os.urandom(6), "little")) if r == 0 else 0.0  # < 2^48: exact
            tok = int(np.asarray(self._allreduce(np.array([tok]))).reshape(-1)[0])
            sh = self._share = _noise.NodeShare(r, w, lambda: self._allreduce(np.zeros(1)), "%012x" % tok)
        return sh

    def _counted(self, plan, share):
        """The plan's segments, counting the dense factorisations this rank computes into
        md.noise_factorisations (with a NodeShare: its own block only)."""
        t0 = share.total if share is not None else 0
        n = 0
        for seg in plan:
            if seg[0] == "dense":
                m = seg[2][0] if isinstance(seg[2], tuple) else seg[2]
                n += m.shape[0]
            yield seg
        self.noise_factorisations = getattr(self, "noise_factorisations", 0) + (
            share.total - t0 if share is not None else n)

    def _noise_seed(self, i, run):
        base = 0 if self.seed is None else int(self.seed)
        return (base * 0x9E3779B97F4A7C15 + (run + 1) * 0xBF58476D1CE4E5B9 + (i + 1) * 0x94D049BB133111EB) % 2**64

    def gen_noise(self, i, run=0):
        """New noise realisation for bath i on the device (bath.gnoi, md.py:569-570)."""
        from . import noise as _noise

        st = self._ensure_device()
        b = self.baths[i]
        nfreq = int(self.nmd / 2) + 1
        fac_bytes = nfreq * b.nc * b.nc * 8 * (2 if b.kind == "ebath" else 1)
        if self.noise_mode == "device" and (fac_bytes > self.noise_stream_bytes or self._sparse_spectrum(b)):
            # zero frequencies skipped, shared-matrix frequencies as one factor and scales, dense
            # factors computed once and kept for the following runs (only the draws change per run,
            # md.py:569-570): on the device when they fit there (the stepper replays them with new
            # draws), else in host memory
            seed = self._noise_seed(i, run)
            share = self._node_share()
            if not self.noise_factor_cache:
                st.noise_stream_plan(i, self._counted(_noise.stream_factor_plan(b, share=share), share), b.kind == "ebath",
                                     seed, self.traj_offset)
            else:
                key = b._noise_key()
                dev = st.__dict__.setdefault("noise_plan_keys", {})  # bath -> key of its retained plan
                if dev.get(i) == key and st.noise_stream_retained(i):
                    st.noise_stream_replay(i, seed, self.traj_offset)
                else:
                    dev.pop(i, None)
                    if getattr(b, "_stream_cache_key", None) != key:
                        b._stream_cache, b._stream_cache_key = {}, key
                    st.noise_stream_retain(i, True)
                    fresh = not b._stream_cache.get("complete")
                    plan = _noise.stream_factor_plan(b, cache=b._stream_cache, share=share)
                    st.noise_stream_plan(i, self._counted(plan, share) if fresh else plan, b.kind == "ebath", seed,
                                         self.traj_offset)
                    if st.noise_stream_retained(i):
                        dev[i] = key
                        b._stream_cache, b._stream_cache_key = None, None  # the device copy serves
            b._noise_src = (st, i)
            b._noise_version = getattr(b, "_noise_version", 0) + 1
            self._noise_versions[i] = b._noise_version
            return
        fac = b.noise_factor(share=self._node_share())
        key = (self.noise_mode, b._fac_key)
        if getattr(self, "_fac_loaded", {}).get(i) != key:
            st.noise_factors(i, fac.evecs if self.noise_mode == "numpy" else fac.scaled())
            self._fac_loaded = getattr(self, "_fac_loaded", {})
            self._fac_loaded[i] = key
        if self.noise_mode == "numpy":
            x = np.stack([fac.draws(self._rng(bb)) for bb in range(self.ntraj)])
            st.noise_generate(i, x)
        else:
            st.noise_generate(i, None, seed=self._noise_seed(i, run), traj_offset=self.traj_offset)
        b._noise_src = (st, i)
        b._noise_version = getattr(b, "_noise_version", 0) + 1
        self._noise_versions[i] = b._noise_version

    # ------------------------------------------------------------------------------ forces
    def potforce(self, q):
        """Host potential force with md.potforce's cache (md.py:437-474); one trajectory."""
        if sameq(q, self.q0):
            return self.f0
        if self.pforce is not None:
            f = self.pforce.force(q)
        elif self.dyn is not None:
            f = -1.0 * mdot(self.dyn, q)
        else:
            raise RuntimeError("no driver, no md")
        self.q0, self.f0 = q, f
        return f

    def _host_forces(self, qs, cache):
        """Per-trajectory md.potforce with its sameq cache (md.py:437-474, 767-779)."""
        out = np.empty_like(qs)
        miss = []
        for b in range(self.ntraj):
            q0, f0 = cache[b]
            if len(q0) == len(qs[b]) and np.max(np.abs(qs[b] - q0)) < 10e-10:
                out[b] = f0
            else:
                miss.append(b)
        drivers = getattr(self, "pforces", None)
        if drivers is not None and len(miss) > 1:
            if getattr(self, "_pool", None) is None:
                from concurrent.futures import ThreadPoolExecutor

                nw = min(self.ntraj, int(os.environ.get("SCLMD_FORCE_WORKERS", os.cpu_count() or 1)))
                self._pool = ThreadPoolExecutor(max_workers=max(1, nw))
            qc = {b: qs[b].copy() for b in miss}
            futs = {b: self._pool.submit(drivers[b].force, qc[b]) for b in miss}
            for b in miss:  # collected in trajectory order: the cache update is deterministic
                f = np.asarray(futs[b].result(), dtype=float)
                cache[b] = (qc[b], f)
                out[b] = f
            return out
        for b in miss:
            drv = drivers[b] if drivers is not None else self.pforce
            q = qs[b].copy()
            f = np.asarray(drv.force(q), dtype=float)
            cache[b] = (q, f)
            out[b] = f
        return out

    # ------------------------------------------------------------------------------ stepping
    def vv(self, id=0):
        """One modified velocity-Verlet step (md.py:367-411) on the device."""
        st = self._ensure_device()
        self._push_state()
        if getattr(self, "_reset_his", False):
            for i in range(len(self.baths)):
                st.set_history(i, None)
            self._reset_his = False
        self._sync_injected_noise()
        self._apply_record()  # ps / qs / fhis / histories are recorded on the device by the step
        if self.cf:  # CompareForce: a host driver call per step (md.py:378-379), trajectory 0
            q = np.asarray(self.q)
            qq = q if self.ntraj == 1 else q[0]
            self.cflist.append(self.forcedriver.force(qq) + mdot(self.dyn, qq))
        if self.pforce is not None:
            if not hasattr(self, "_fcache") or len(self._fcache) != self.ntraj:
                self._fcache = [([], None)] * self.ntraj
            q = np.asarray(self._q_dev_host()).reshape(self.ntraj, self.nph)
            f = self._host_forces(q, self._fcache)
            qt = st.step_begin(f, want_qt=True)
            f2 = self._host_forces(qt, self._fcache)
            st.step_end(f2)
        else:
            st.step_begin(None, want_qt=False)
            st.step_end(None)
        self._dev_newer = True

    def _q_dev_host(self):
        return self.q

    @property
    def f(self):
        if self._st is None:
            return None
        f = self._st.get_force()
        return f[0] if self.ntraj == 1 else f

    def steps(self, n):
        """n steps; fully on the device when no host work is needed per step."""
        if self.pforce is None and not self.cf:
            st = self._ensure_device()
            self._push_state()
            self._sync_injected_noise()
            self._apply_record()
            st.run(n)
            self._dev_newer = True
        else:
            for _ in range(n):
                self.vv()

    # ------------------------------------------------------------------------------ Run
    def _reduce(self, sums):
        """Per-run current statistics of every rank: gle_reduce_current over the C-ABI's RCCL
        communicator when comm is a _native.Comm, else one torch.distributed all-reduce."""
        if isinstance(self.comm, _native.Comm):
            return self._ensure_device().reduce_current(self.comm)
        from . import ensemble

        return ensemble.allreduce_sums(sums, self.comm, device=self._device_ordinal())

    def _allreduce(self, values):
        """Sum a vector over the ensemble's ranks (gle_comm_allreduce or torch.distributed)."""
        if isinstance(self.comm, _native.Comm):
            return self._ensure_device().comm_allreduce(self.comm, values)
        from . import ensemble

        return ensemble.allreduce_sums(values, self.comm, device=self._device_ordinal())

    def _device_ordinal(self):
        if self.device is not None:
            return int(self.device)
        return int(os.environ.get("LOCAL_RANK", "0")) if _native.device_count() > 1 else 0

    def _is_root(self):
        from . import ensemble

        return ensemble.rank(self.comm) == 0

    # ------------------------------------------------------------------------------ checkpoints
    def _ncname(self, j):
        from . import ensemble

        w = ensemble.world_size(self.comm)
        return "MD%d.nc" % j if w == 1 else "MD%d.r%d.nc" % (j, ensemble.rank(self.comm))

    @property
    def phis(self):
        """Velocity history, newest first: (ml, nph), or (ntraj, ml, nph) (md.py:345-346, 386-387).
        The bath DOFs come from the bath history rings the friction reads; the other DOFs from the
        device recording of every DOF's history (md.Run records it; outside Run they read as
        zeros, as do rows past a bath's own ml)."""
        st = self._ensure_device()
        out = np.zeros((self.ntraj, self.ml, self.nph))
        if (getattr(self, "_rec_applied", 0) or 0) & _native.REC_HIST:
            ph, _ = st.get_record_history()
            n = min(self.ml, ph.shape[1])
            out[:, :n] = ph[:, :n]
        for i, b in enumerate(self.baths):
            h = st.get_history(i)                      # (ntraj, ml_b, nc_b)
            out[:, : h.shape[1], np.asarray(b.cids)] = h
        return out[0] if self.ntraj == 1 else out

    @property
    def qhis(self):
        """Position history (md.py:346, 387), newest first: (ml, nph) or (ntraj, ml, nph), from the
        device recording of every DOF's history (md.Run records it; zeros otherwise -- only its
        newest row, the current q, ever enters a force, baths.py:245-247)."""
        shp = (self.ntraj, self.ml, self.nph)
        out = np.zeros(shp)
        if self._st is not None and (getattr(self, "_rec_applied", 0) or 0) & _native.REC_HIST:
            _, qh = self._st.get_record_history()
            n = min(self.ml, qh.shape[1])
            out[:, :n] = qh[:, :n]
        return out[0] if self.ntraj == 1 else out

    def _histories(self, pinned=False):
        """(phis, qhis) as md.phis / md.qhis return them, in one device read (gle_get_full_history:
        the recorded histories with the baths' own rings on their DOFs, transposed on the device).
        pinned: into this md's page-locked snapshot buffers (reused by every dump; C5: 2 x 3.1 GB
        at the link's rate instead of pageable copies)."""
        st = self._ensure_device()
        t0 = time.perf_counter()
        outs = (None, None)
        if pinned:
            shp = (self.ntraj, self.ml, self.nph)
            bufs = getattr(self, "_snap_bufs", None)
            if bufs is None or bufs[0].array.shape != shp:
                self._free_snap_bufs()
                bufs = self._snap_bufs = (_native.HostBuffer(shp), _native.HostBuffer(shp))
            outs = (bufs[0].array, bufs[1].array)
        ph, qh = st.get_full_history(self.ml, *outs)
        self._tick("dump_histories", time.perf_counter() - t0)
        if self.ntraj == 1:
            return ph[0], qh[0]
        return ph, qh

    def _free_snap_bufs(self):
        """Release the dump's page-locked buffers (the background writer must be joined first)."""
        for b in getattr(self, "_snap_bufs", None) or ():
            b.free()
        self._snap_bufs = None

    def _load_phis(self, phis, qhis=None):
        st = self._ensure_device()
        self._push_state()  # history slots are relative to the device's t: set p, q, t first
        ph = np.asarray(phis, dtype=float)
        if ph.ndim == 2:
            ph = np.broadcast_to(ph, (self.ntraj,) + ph.shape)
        self._apply_record()
        if (self._rec_applied or 0) & _native.REC_HIST:
            qh = np.zeros_like(ph) if qhis is None else np.asarray(qhis, dtype=float)
            if qh.ndim == 2:
                qh = np.broadcast_to(qh, (self.ntraj,) + qh.shape)
            ml_r = st.get_record_history()[0].shape[1]
            full_p = np.zeros((self.ntraj, ml_r, self.nph))
            full_q = np.zeros((self.ntraj, ml_r, self.nph))
            n = min(ml_r, ph.shape[1])
            full_p[:, :n], full_q[:, :n] = ph[:, :n], qh[:, :n]
            st.set_record_history(full_p, full_q)
        for i, b in enumerate(self.baths):
            ml_b = st.bath_ml[i]
            h = np.zeros((self.ntraj, ml_b, len(b.cids)))
            n = min(ml_b, ph.shape[1])
            h[:, :n, :] = ph[:, :n, :][:, :, np.asarray(b.cids)]
            st.set_history(i, h)
        self._reset_his = False

    def _wrote_current(self, fn, ipie=None):
        """fn is the file this process wrote last, unchanged since, at the current t (and piece).  A
        file still being written by the background dump counts as written (its snapshot is the
        device state at that t; a write error surfaces at the next join)."""
        pend = getattr(self, "_dump_pending", None)
        if pend is not None and pend[0] == fn:
            return int(self.t) == pend[1] and (ipie is None or ipie == pend[2])
        ld = getattr(self, "_last_dump", None)
        if ld is None or ld[0] != fn or not os.path.isfile(fn):
            return False
        st_ = os.stat(fn)
        return (st_.st_mtime_ns, st_.st_size) == ld[1:3] and int(self.t) == ld[3] and (ipie is None or ipie == ld[4])

    # MD{j}.nc is written on a background thread from a host snapshot of the state (md.Run goes on
    # stepping the next piece / run meanwhile); False writes it before dump returns
    async_dump = True

    def dump(self, ipie, id):
        """Write MD{id}.nc (md.py:684-764): energy, p, q, t, ipie, phis, qhis, with SaveAll the noise
        series and fhis{i} (and ps / qs with savep / saveq), with savep the power spectra.  With
        ntraj > 1 a trajectory dimension is added.  Deviations: NetCDF classic format (netCDF4 is not
        installed; see sclmd_amd.checkpoint), where only the first dimension may be the unlimited
        'nnmd', so poweratomlist is stored as ('nnmd', 'atomlist', 'two') (transposed back on
        resume); ensemble histories above a classic-format variable's size are split into
        trajectory groups (phis_g{k} / qhis_g{k}, checkpoint.read_history joins them).

        The device state is copied to host memory here (the file holds exactly the state at this
        call); with async_dump the file itself is written on a background thread, joined before
        the next dump, before a checkpoint file is read or removed, at the end of Run and in
        close() -- a write error is raised there."""
        t0 = time.perf_counter()
        self._join_dump()
        t1 = time.perf_counter()
        snap = self._dump_snapshot(ipie, id)
        self._tick("dump_join", t1 - t0)
        self._tick("dump_snapshot", time.perf_counter() - t1)
        if not self.async_dump:
            self._apply_written(self._write_snapshot(snap))
            return
        import threading

        box = {"snap": snap, "lock": threading.Lock(), "committed": False, "remove": []}
        th = threading.Thread(target=self._write_snapshot_bg, args=(box,), name="sclmd-dump", daemon=True)
        self._dump_pending = (snap["fn"], int(self.t), ipie, th, box)
        th.start()

    @staticmethod
    def _write_snapshot_bg(box):
        # the writer thread touches only its box: what it wrote and its time are applied to the md by
        # _join_dump on the caller's thread
        try:
            box["written"] = md._write_snapshot(box["snap"])
            with box["lock"]:
                box["committed"] = True
                rm = list(box["remove"])
            for fn in rm:  # files to drop once this one is on disk (remove_after_dump)
                if os.path.exists(fn):
                    os.remove(fn)
        except BaseException as e:  # re-raised by _join_dump on the caller's thread
            box["error"] = e
        finally:
            box.pop("snap", None)   # the host copy is freed as soon as the file is written

    def _apply_written(self, written):
        last, dt = written
        self._last_dump = last
        self._tick("dump_write", dt)

    def _join_dump(self):
        """Wait for the background MD{j}.nc write, if any, and raise its error."""
        pend = getattr(self, "_dump_pending", None)
        if pend is None:
            return
        self._dump_pending = None
        pend[3].join()
        if "error" in pend[4]:
            raise RuntimeError("md.dump: writing %s failed" % pend[0]) from pend[4]["error"]
        self._apply_written(pend[4]["written"])

    def remove_after_dump(self, fn):
        """Remove fn once the newest MD{j}.nc is committed (md.py:676-679 removes MD{j-1}.nc after
        MD{j}.nc is on disk): at once when no dump is pending or it has committed, else by the writer
        thread right after its commit -- a checkpoint is on disk at every moment."""
        pend = getattr(self, "_dump_pending", None)
        if pend is not None:
            box = pend[4]
            with box["lock"]:
                if not box["committed"]:
                    box["remove"].append(fn)
                    return
        if os.path.exists(fn):
            os.remove(fn)

    def _dump_snapshot(self, ipie, id):
        """Host copy of everything MD{id}.nc holds: dimensions and (name, array, dims) variables."""
        multi = self.ntraj > 1
        tr = ("traj",) if multi else ()
        dims = [("nnmd", None), ("nph", self.nph), ("one", 1), ("two", 2), ("mem", self.ml), ("nmd", self.nmd)]
        if multi:
            dims.append(("traj", self.ntraj))
        if self.atomlist is not None:
            dims.append(("atomlist", len(self.atomlist)))
        for i, b in enumerate(self.baths):
            dims.append(("n" + str(i), b.nc))
        var = []

        def series(name, a):  # (nmd, X) or (ntraj, nmd, X) -> record dimension first
            a = np.asarray(a)
            if multi:
                var.append((name, np.transpose(a, (1, 0, 2)), ("nnmd", "traj", "nph")))
            else:
                var.append((name, a, ("nnmd", "nph")))

        if self.saveall:
            for i, b in enumerate(self.baths):
                nz = np.array(b.noise)
                if multi and nz.ndim == 2:  # one host-injected realisation shared by every trajectory
                    nz = np.broadcast_to(nz, (self.ntraj,) + nz.shape)
                if multi:  # (ntraj, nmd, nc) -> (nmd, ntraj, nc): the record dimension comes first
                    dims.append(("traj" + str(i), nz.shape[0]))
                    var.append(("noise" + str(i), np.transpose(nz, (1, 0, 2)), ("nnmd", "traj" + str(i), "n" + str(i))))
                else:
                    var.append(("noise" + str(i), nz, ("nnmd", "n" + str(i))))
                fh = self.fhis_of(i)
                if fh is not None:
                    series("fhis" + str(i), fh)
            if self.savep:
                series("ps", self.ps)
            if self.saveq:
                series("qs", self.qs)
        if self.savep:
            var.append(("power", np.array(self.power), ("nnmd", "two")))
            if self.atomlist is not None:
                var.append(("poweratomlist", np.transpose(np.array(self.poweratomlist), (1, 0, 2)),
                            ("nnmd", "atomlist", "two")))
        e = np.array(self.etot)
        var.append(("energy", e.T if multi else e, ("nnmd",) + tr))
        var.append(("p", np.array(self.p), tr + ("nph",)))
        var.append(("q", np.array(self.q), tr + ("nph",)))
        var.append(("t", np.array([self.t]), ("one",)))
        var.append(("ipie", np.array([ipie]), ("one",)))
        phis, qhis = self._histories(pinned=True)
        if multi and phis.nbytes >= self.nc_var_limit:
            # a classic-format variable holds < 2 GiB (C5: 32 x 4096 x 3000 doubles = 3.1 GB): the
            # ensemble's histories are split into fixed-size variables of whole trajectories,
            # phis_g{k} / qhis_g{k} over ('trajg{k}', 'mem', 'nph') -- exactly ml rows each, one
            # contiguous write per variable (checkpoint.read_history joins the groups)
            per = max(1, int(self.nc_var_limit // max(phis[0].nbytes, 1)))
            for k, a in enumerate(range(0, self.ntraj, per)):
                b_ = min(self.ntraj, a + per)
                dims.append(("trajg" + str(k), b_ - a))
                var.append(("phis_g" + str(k), phis[a:b_], ("trajg" + str(k), "mem", "nph")))
                var.append(("qhis_g" + str(k), qhis[a:b_], ("trajg" + str(k), "mem", "nph")))
        else:
            var.append(("phis", phis, tr + ("mem", "nph")))
            var.append(("qhis", qhis, tr + ("mem", "nph")))
        return {"fn": self._ncname(id), "dims": dims, "vars": var, "t": int(self.t), "ipie": ipie,
                "savep": bool(self.savep)}

    @staticmethod
    def _write_snapshot(snap):
        """Write the snapshot's file; returns ((fn, mtime, size, t, ipie, savep), seconds)."""
        from . import checkpoint as C

        t0 = time.perf_counter()
        fn = snap["fn"]
        f, tmp = C.open_for_write(fn)
        try:
            for name, size in snap["dims"]:
                f.createDimension(name, size)
            for name, a, d in snap["vars"]:
                C.Write2NetCDFFile(f, a, name, d, units="")
        except BaseException:
            C.abandon(f, tmp)
            raise
        C.commit(f, tmp, fn)
        st_ = os.stat(fn)
        # what this process wrote: the next run's start can skip reading its own file back, and an
        # unchanged second dump of the same piece need not be rewritten
        return (fn, st_.st_mtime_ns, st_.st_size, snap["t"], snap["ipie"], snap["savep"]), time.perf_counter() - t0

    def _tick(self, name, dt):
        """Wall time of the named host phase, accumulated (md.phase_times: where a Run's time goes)."""
        pt = self.__dict__.setdefault("phase_times", {})
        pt[name] = pt.get(name, 0.0) + dt

    def _read_poweratomlist(self, fn):
        """poweratomlist (natomlist, nmd, 2) from an MD{j}.nc file in either layout: this build's
        ('nnmd', 'atomlist', 'two') or the reference's ('atomlist', 'nnmd', 'two') (md.py:742-744),
        told apart by the variable's dimension names, and by its shape when those are unnamed."""
        from . import checkpoint as C

        arr = C.ReadNetCDFVar(fn, "poweratomlist")
        dims = C.var_dims(fn, "poweratomlist")
        na = len(self.atomlist)
        if dims and dims[0] == "nnmd":
            return np.transpose(arr, (1, 0, 2))
        if dims and dims[0] == "atomlist":
            return arr
        if arr.shape == (na, self.nmd, 2):
            return arr
        if arr.shape == (self.nmd, na, 2):
            return np.transpose(arr, (1, 0, 2))
        raise ValueError("poweratomlist in %s has shape %s, dims %s: not (%d, %d, 2) in either layout"
                         % (fn, arr.shape, dims, na, self.nmd))

    def _resume(self, j):
        """The reference's per-run file logic (md.py:506-567).  Returns the last finished piece
        (-1 for a new run) or None when run j is already complete."""
        from .checkpoint import ReadNetCDFVar, read_history

        fn, fnm = self._ncname(j), self._ncname(j - 1)
        pend = getattr(self, "_dump_pending", None)
        if pend is not None and not (pend[0] == fnm and self._wrote_current(fnm)):
            self._join_dump()  # a file this logic may read is still being written
        if os.path.isfile(fn):
            self._log("find file: " + fn)
            ipie = int(ReadNetCDFVar(fn, "ipie")[0])
            if ipie + 1 < self.npie:
                self._log("unfinished run: reading resume information")
                if not (self.saveall and self.saveq and self.savep):
                    raise RuntimeError("md.Run: saveall, savep and saveq must be set to continue an "
                                       "unfinished run (the reference exits here, md.py:531-533)")
                self.p = ReadNetCDFVar(fn, "p")
                self.q = ReadNetCDFVar(fn, "q")
                self.t = int(ReadNetCDFVar(fn, "t")[0])
                self._load_phis(read_history(fn, "phis", self.ml), read_history(fn, "qhis", self.ml))
                self.power = ReadNetCDFVar(fn, "power")
                if self.atomlist is not None:
                    self.poweratomlist = self._read_poweratomlist(fn)
                qs, ps = ReadNetCDFVar(fn, "qs"), ReadNetCDFVar(fn, "ps")
                self.qs = np.transpose(qs, (1, 0, 2)) if qs.ndim == 3 else qs
                self.ps = np.transpose(ps, (1, 0, 2)) if ps.ndim == 3 else ps
                for i, b in enumerate(self.baths):
                    nz = ReadNetCDFVar(fn, "noise" + str(i))
                    b.noise = np.transpose(nz, (1, 0, 2)) if nz.ndim == 3 else nz
                return ipie
            if ipie + 1 == self.npie:
                self._log("finished run")
                if self.savep:
                    self.power = ReadNetCDFVar(fn, "power")
                    if self.atomlist is not None:
                        self.poweratomlist = self._read_poweratomlist(fn)
                self.t = int(ReadNetCDFVar(fn, "t")[0])
                return None
            raise RuntimeError("md.Run: ipie error in %s (ipie = %d)" % (fn, ipie))
        if (os.path.isfile(fnm) or getattr(self, "_dump_pending", None) is not None) and self._wrote_current(fnm):
            # the previous run's file is the one this process just wrote from the device state it
            # still holds (same t, file unchanged): reading p, q and the histories back would only
            # return them (C5: 6 GB of phis / qhis)
            self._log("continuing from previous run (state on the device)")
        elif os.path.isfile(fnm):
            self._log("reading history from previous run")
            self.p = ReadNetCDFVar(fnm, "p")
            self.q = ReadNetCDFVar(fnm, "q")
            self.t = int(ReadNetCDFVar(fnm, "t")[0])
            ph = read_history(fnm, "phis", self.ml)
            qh = read_history(fnm, "qhis", self.ml)
            if ph.shape[-2:] == (self.ml, self.nph):
                self._load_phis(ph, qh if qh.shape == ph.shape else None)
        elif j != 0:
            raise RuntimeError("md.Run: no previous nc file exists (%s)" % fnm)
        for i in range(len(self.baths)):
            self.gen_noise(i, j)
        self.ResetSavepq()
        return -1

    def Run(self):
        """Independent runs nstart..nstop-1 (md.py:493-682): fresh noise per run, state and history
        carried over, per-run time-averaged heat current written to kappa.{T}.bath{i}.run{j}.dat,
        MD{j}.nc written after every piece and read back to resume an unfinished run or to continue
        from the previous run (md.py:506-567).  ps / qs / fhis and every DOF's p / q history are
        recorded on the device by the step itself; nothing crosses PCIe per step unless a host
        force driver or CompareForce needs it."""
        self.initialise()
        self.ResetHis()
        self.info()
        self._ensure_device()
        self._in_run = True
        self._apply_record()
        for j in range(self.nstart, self.nstop):
            self._log("\nMD run: " + str(j))
            ipie = self._resume(j)
            if ipie is None:
                continue
            traj = None
            if self.nstep is not None and self._is_root():
                traj = open("trajectories." + str(self.T) + ".run" + str(j) + ".ani", "w")
            piece = ipie
            for piece in range(ipie + 1, self.npie):
                nsteps = int(self.nmd / self.npie)
                if self.nstep is None:
                    self.steps(nsteps)
                else:
                    # frames at tt = 0 and tt % nstep == 0 (tt = t - 1 after the step, md.py:586-595):
                    # run on the device up to each frame step, then read that one state back
                    done = 0
                    while done < nsteps:
                        t = self.t
                        nxt = t if t == 0 else ((t + self.nstep - 1) // self.nstep) * self.nstep
                        k = min(nsteps - done, nxt - t + 1)
                        self.steps(k)
                        done += k
                        tt = self.t - 1
                        if traj is not None and (tt == 0 or tt % self.nstep == 0):
                            self._write_frame(traj, tt)
                self.dump(piece, j)  # md.py:596 (with savep written again after the power spectra)
            if traj is not None:
                traj.close()
            if self.cf:
                np.save("deltaforce.run" + str(j), np.array(self.cflist) / self.forcedriver.conv)
                self.cflist = []
            if self.savep:
                self._power(j)
                self.dump(piece, j)  # "dump again, to make sure power is all right" (md.py:654)
            cur = self._st.get_current()                      # (nbath, ntraj, nmd)
            sums = self._reduce(self._st.current_sums())      # (nbath, 3) over all ranks
            kap = sums[:, 0] / sums[:, 2] * U.curcof
            self.kappa_runs.append(kap)
            for ii, b in enumerate(self.baths):
                b.cur = cur[ii, 0] if self.ntraj == 1 else cur[ii]
            if self._is_root():
                for ii in range(len(self.baths)):
                    with open("kappa." + str(self.T) + ".bath" + str(ii) + ".run" + str(j) + ".dat", "w") as fk:
                        fk.write("%i %f    %f \n" % (j, self.T, kap[ii]))
                if self.saveq:
                    self._avestructure(j)
            # every rank removes its own shard of the previous run's file (md.py:676-679)
            if self.rmnc:
                pend = getattr(self, "_dump_pending", None)
                if pend is not None and pend[0] == self._ncname(j - 1):
                    self._join_dump()
                if os.path.exists(self._ncname(j - 1)):
                    self._log("Remove " + self._ncname(j - 1))
                    self.remove_after_dump(self._ncname(j - 1))  # once MD{j}.nc is committed
        # the last file is on disk (or its write error raised) when Run returns
        self._join_dump()
        self._in_run = False

    def _write_frame(self, fh, tt):
        q = self.q if self.ntraj == 1 else self.q[0]
        f = self.f if self.ntraj == 1 else self.f[0]
        s = self.xyz + self.conv * q
        fh.write(str(len(self.els)) + "\n" + str(tt) + "\n")
        for ip in range(len(self.els)):
            fh.write(str(self.els[ip]) + "    " + str(s[ip * 3]) + "   " + str(s[ip * 3 + 1]) + "   " +
                     str(s[ip * 3 + 2]) + "   " + str(f[ip * 3]) + "   " + str(f[ip * 3 + 1]) + "   " +
                     str(f[ip * 3 + 2]) + "\n")

    def power_spectra(self):
        """md.GetPower (md.py:351-360) on the device: functions.powerspecp of the recorded ps for all
        DOFs and for each AddPowerSection group, averaged over the whole ensemble: every trajectory
        of every rank of comm (one trajectory on one rank: exactly the reference's).  Returns
        (power (nmd, 2), [poweratomlist rows])."""
        st = self._ensure_device()
        self._apply_record()
        groups = [np.arange(self.nph)]
        if self.atomlist is not None:
            groups += [np.asarray(list(a), dtype=np.int64) for a in self.atomlist]
        spec = st.power_spectrum(groups)                  # (ngroup, ntraj, nmd): sum_k |DFT|^2
        # ensemble mean over every rank's trajectories (a no-op reduce alone)
        tot = self._allreduce(np.concatenate([spec.sum(axis=1).ravel(), [self.ntraj]]))
        mean = tot[:-1].reshape(len(groups), self.nmd) / tot[-1]
        dw = 2.0 * np.pi / self.dt / self.nmd
        w = dw * np.arange(self.nmd)
        rows = [np.stack([w, m * self.dt / self.nmd], axis=1) for m in mean]  # functions.py:233-236
        return rows[0], rows[1:]

    def _power(self, j):
        """Running average of the velocity power spectra over runs, power.*.dat and
        poweratomlist.*.dat files (md.py:604-653)."""
        prev = np.copy(self.power)
        prev_al = None if self.atomlist is None else np.copy(self.poweratomlist)
        power, al = self.power_spectra()
        k = j - self.nstart
        self.power = (prev * k + power) / float(k + 1) if k > 0 else power
        if self.atomlist is not None:
            al = np.array(al)
            self.poweratomlist = (prev_al * k + al) / float(k + 1) if k > 0 else al
        if self._is_root():
            def write(fn, pw):
                with open(fn, "w") as f:
                    for ni in range(len(pw)):
                        if self.hw is not None and pw[ni, 0] >= 1.5 * max(self.hw):
                            break
                        f.write("%f     %f \n" % (pw[ni, 0], pw[ni, 1]))

            write("power." + str(self.T) + ".run" + str(j) + ".dat", self.power)
            if self.atomlist is not None:
                for layer in range(len(self.atomlist)):
                    write("poweratomlist." + str(layer) + "." + str(self.T) + ".run" + str(j) + ".dat",
                          self.poweratomlist[layer])

    def _avestructure(self, j):
        """avestructure.{T}.run{j}.dat (md.py:665-675): time average of the recorded qs (and over this
        rank's trajectories)."""
        qs = np.asarray(self.qs)
        qm = qs.mean(axis=0) if qs.ndim == 2 else qs.mean(axis=(0, 1))
        ave = self.conv * qm + self.xyz
        with open("avestructure." + str(self.T) + ".run" + str(j) + ".dat", "w") as f:
            f.write(str(len(self.els)) + "\n" + "average structure" + "\n")
            for ip in range(len(self.els)):
                f.write(str(self.els[ip]) + "    " + str(ave[ip * 3]) + "   " + str(ave[ip * 3 + 1]) +
                        "   " + str(ave[ip * 3 + 2]) + "\n")

    def close(self):
        """Release the device stepper, the host driver pool and the host noise-factor caches of this
        md's streamed baths; a background MD{j}.nc write is joined first (its error raised after
        everything is released)."""
        err = None
        try:
            self._join_dump()
        except Exception as e:
            err = e
        if getattr(self, "_pool", None) is not None:
            self._pool.shutdown(wait=True)
            self._pool = None
        for b in self.baths:  # dense streamed factors (C5: ~11 GB of host memory)
            if getattr(b, "_stream_cache", None) is not None:
                b._stream_cache, b._stream_cache_key = None, None
        self._free_snap_bufs()  # after the join above: the writer reads them
        if self._st is not None:
            self._pull()
            self._st.close()
            self._st = None
        if err is not None:
            raise err
