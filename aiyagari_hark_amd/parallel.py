"""Multi-GPU sharding, one process per GPU over torch.distributed.

Two ways the path shards:

* by calibration / shock stream (Table II sweep, bench.py): every rank solves its own
  economies; no collective in the data path.  ``split_calibrations`` assigns them.
* by agent population (configs[3], 1e8 agents): contiguous agent ranges per rank
  (``shard_range``); every rank holds a replica of the policy table; the per-period
  mean of end-of-period assets (``calc_R_and_W``, Aiyagari_Support.py:1868) becomes an
  RCCL all-reduce of one double, enqueued by libaiyagari on the compute stream between
  the per-period kernels (``bind_rccl`` + ``aiy_sim_periods``).  Philox shocks are
  keyed by the GLOBAL agent index, so a sharded history equals the single-GPU one up
  to the summation order of the mean.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous, balanced agent range of ``rank``: (offset, n_local), split on agent PAIRS
    so every offset is even (the Philox draw of a pair (2k, 2k + 1) then never straddles two
    shards, and the library's resident panel kernel takes every shard)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    pairs = (int(n_total) + 1) // 2
    base, rem = divmod(pairs, int(world))
    p_off = rank * base + min(rank, rem)
    p_loc = base + (1 if rank < rem else 0)
    offset = min(2 * p_off, int(n_total))
    n_local = max(0, min(2 * (p_off + p_loc), int(n_total)) - offset)
    return offset, n_local


def split_calibrations(items, world: int, rank: int):
    """Round-robin assignment of independent calibrations to ranks."""
    return [x for k, x in enumerate(items) if k % world == rank]


def initial_labor_states(n_total: int, n_lab: int, offset: int, n_local: int):
    """Even labour split of sim_birth (Aiyagari_Support.py:1203-1205) by global index
    (state = global index // (n_total / n_lab)); the reference permutes it with the
    agent RNG, which is immaterial for exchangeable agents and would need the whole
    population on every rank."""
    if n_total % n_lab:
        raise ValueError("AgentCount must be a multiple of LaborStatesNo (AS:757)")
    per = n_total // n_lab
    return (np.arange(offset, offset + n_local) // per).astype(np.uint8)


def torch_comm_ptr(group=None, device=None):
    """The ncclComm_t of torch.distributed's RCCL process group on ``device`` (an int), or
    None when the backend is not nccl or the communicator is not created yet.  torch's
    bundled librccl is the only RCCL in the process (libaiyagari's DT_NEEDED librccl.so.1
    resolves to the already-loaded copy), so the pointer is valid for the library."""
    import torch
    import torch.distributed as dist
    try:
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        if dist.get_backend(pg) != "nccl":
            return None
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        ptr = int(pg._get_backend(dev)._comm_ptr())
        return ptr or None
    except (AttributeError, RuntimeError, ValueError):
        return None


def bind_rccl(handle: "_lib.Handle", group=None, prefer_torch=True):
    """Bind an RCCL communicator over the ranks of ``group`` to the libaiyagari handle.

    prefer_torch: borrow torch.distributed's own communicator (aiy_comm_bind), so the
    process holds ONE communicator per device and the library's per-period all-reduces and
    torch's collectives are ordered on one comm; else (or when torch's is not available)
    create the library's own (rank 0 makes the ncclUniqueId, torch.distributed broadcasts it).
    Returns (world, rank, "torch" | "own")."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if prefer_torch:
        nccl = dist.get_backend(group) == "nccl"
        dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
        flag = torch.ones(1, dtype=torch.int32, device=dev)
        dist.all_reduce(flag, group=group)   # creates a lazily made communicator on every rank
        ptr = torch_comm_ptr(group)
        ok = ptr is not None and handle.lib.aiy_comm_bind(handle.h, ctypes.c_void_p(ptr)) == _lib.AIY_OK
        # every rank takes the same path: if any rank could not bind torch's communicator, the
        # ranks that did unbind it and all of them create the library's own below
        flag.fill_(1 if ok else 0)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) == 1:
            return world, rank, "torch"
        if ok:
            handle.check(handle.lib.aiy_comm_destroy(handle.h), "aiy_comm_destroy")
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        rc = handle.lib.aiy_comm_unique_id(buf)
        if rc != _lib.AIY_OK:
            raise _lib.AiyagariLibError("aiy_comm_unique_id failed")
    obj = [bytes(buf.raw) if rank == 0 else None]
    # src is a GLOBAL rank: the group's rank 0 (a subgroup need not contain global rank 0)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    uid = ctypes.create_string_buffer(obj[0], 128)
    handle.check(handle.lib.aiy_comm_init(handle.h, uid, world, rank), "aiy_comm_init")
    return world, rank, "own"


def unbind_rccl(handle: "_lib.Handle"):
    handle.check(handle.lib.aiy_comm_destroy(handle.h), "aiy_comm_destroy")


def torch_allreduce(group=None):
    """Caller-side all-reduce for DevicePanel.run(allreduce=...): sums a small device
    tensor over ``group`` in place.  With the nccl backend (RCCL on ROCm) the collective
    runs on the device tensor, ordered on the current stream; with gloo the value makes a
    round trip through the host (tests and CPU-rendezvous runs)."""
    import torch.distributed as dist

    backend = dist.get_backend(group)

    def reduce(t):
        if backend == "gloo":
            h = t.detach().to("cpu")
            dist.all_reduce(h, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=group)

    reduce.backend = backend
    return reduce
