"""Trajectory-ensemble data parallelism: one process per GPU, trajectories sharded in contiguous
blocks (global index = traj_offset + b, which also keys the RNG streams), one all-reduce of the
per-run heat-current statistics per run.

The reference runs its "ensemble" as a sequential chain of runs (md.py:506) averaged afterwards by
calTC (tools.py:191-201); independent trajectories share nothing but the bath/system parameters,
so there is no per-step communication.  torch.distributed is plumbing here: backend "nccl" is
RCCL over xGMI on the MI355X node, "gloo" is used for the CPU tests.
"""
import numpy as np


def _dist():
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover - torch always present in this image
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def _is_gle_comm(group):
    """An RCCL communicator of the C-ABI (sclmd_amd._native.Comm, gle_comm_init)."""
    return group is not None and hasattr(group, "nranks") and hasattr(group, "c")


def rank(group=None):
    if _is_gle_comm(group):
        return group.rank
    d = _dist()
    return d.get_rank(group) if d else 0


def world_size(group=None):
    if _is_gle_comm(group):
        return group.nranks
    d = _dist()
    return d.get_world_size(group) if d else 1


def shard(ntraj_total, rank_, world):
    """Contiguous block of trajectories for this rank: (offset, count)."""
    base, rem = divmod(int(ntraj_total), int(world))
    count = base + (1 if rank_ < rem else 0)
    offset = rank_ * base + min(rank_, rem)
    return offset, count


def allreduce_sums(sums, group=None, device=None):
    """Sum the per-rank [sum_b mean_t cur, sum_b (mean_t cur)^2, ntraj] rows over all ranks with a
    single collective (fp64).  A no-op without an initialised process group.  device: the HIP
    device of this rank's stepper; with the nccl backend (RCCL) the tensor goes there and it
    becomes torch's current device (a script that never called torch.cuda.set_device would
    otherwise put every rank's all-reduce on device 0).  A C-ABI communicator (md.comm given as a
    _native.Comm) reduces through the stepper instead (md._allreduce, gle_comm_allreduce)."""
    if _is_gle_comm(group):
        raise TypeError("a gle RCCL communicator reduces through its stepper (md._allreduce)")
    d = _dist()
    sums = np.asarray(sums, dtype=np.float64)
    if d is None:
        return sums
    import torch

    backend = d.get_backend(group)
    if backend == "nccl":
        if device is not None and torch.cuda.current_device() != int(device):
            torch.cuda.set_device(int(device))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(sums)).to(dev)
    d.all_reduce(t, op=d.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


def ensemble_stats(sums):
    """Per bath: ensemble mean and standard error of the time-averaged heat current (nW)."""
    from . import units as U

    s, s2, n = sums[:, 0], sums[:, 1], sums[:, 2]
    mean = s / n
    var = np.maximum(s2 / n - mean ** 2, 0.0)
    return mean * U.curcof, np.sqrt(var / np.maximum(n - 1, 1)) * U.curcof
