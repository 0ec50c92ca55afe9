"""World-size-2 gloo tests of the sharding logic (CPU, no GPU).

The agent-sharded panel splits agents into contiguous global ranges, keys Philox by the
GLOBAL agent index and all-reduces the per-period asset sum.  Here each rank runs the
oracle panel on its shard with exactly that logic (aiyagari_hark_amd.parallel ranges and
labour initialisation, oracle Philox by global index, gloo all-reduce of the sum) and
the result must equal the unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aiyagari_hark_amd import parallel as par


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for n in (1, 7, 350, 1000006):
        for w in (1, 2, 3, 8):
            got = [par.shard_range(n, w, r) for r in range(w)]
            assert sum(nl for _, nl in got) == n
            assert got[0][0] == 0
            for (o1, n1), (o2, _) in zip(got, got[1:]):
                assert o1 + n1 == o2
            assert all(o % 2 == 0 for o, nl in got if nl)   # Philox pairs never straddle shards
            assert max(nl for _, nl in got) - min(nl for _, nl in got) <= 3   # one pair + the odd tail


def test_split_calibrations_cover():
    items = list(range(24))
    for w in (1, 2, 4, 8):
        parts = [par.split_calibrations(items, w, r) for r in range(w)]
        assert sorted(sum(parts, [])) == items
        assert all(len(p) == 24 // w for p in parts)


def _panel_history(a0, lab0, offset, T, seed, fx, allreduce, n_total):
    from oracle import hark_ks as H
    from oracle import philox as PX
    a, lab = a0.copy(), lab0.copy()
    emp = np.ones(a.size, dtype=bool)
    sow = dict(Mnow=float(fx["MSS"]), Mrkv=0, Rnow=float(fx["RSS"]), Wnow=float(fx["WSS"]))
    e = dict(H.INIT_ECONOMY)
    hist = []
    for t in range(T):
        u = PX.uniform(t, np.arange(offset, offset + a.size, dtype=np.uint64), seed)
        a, lab, _, _ = H.sim_one_period(a, lab, emp, u, sow["Rnow"], sow["Wnow"], sow["Mnow"], sow["Mrkv"],
                                        fx["LSStates"], fx["cdf"], fx["m"], fx["c"], fx["Mgrid"])
        total = allreduce(float(np.sum(a)))
        K = total / n_total
        Mrkv = int(fx["Mrkv_hist"][t])
        KtoL = K / 1.0
        R = 1.0 + 1.0 * (0.36 * KtoL ** (0.36 - 1.0)) - 0.08
        W = 1.0 * ((1.0 - 0.36) * KtoL ** 0.36)
        sow = dict(Mnow=R * K + W, Mrkv=Mrkv, Rnow=R, Wnow=W)
        hist.append(K)
    return np.array(hist), a, lab


def _worker(rank, world, port, out_q, n_total, T, seed):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "egm_cfg1.npz")))
        off, nl = par.shard_range(n_total, world, rank)
        lab0 = par.initial_labor_states(n_total, 7, off, nl).astype(np.int64)
        a0 = np.full(nl, float(fx["KSS"]))

        def allreduce(x):
            t = torch.tensor([x], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t.item())

        hist, a, lab = _panel_history(a0, lab0, off, T, seed, fx, allreduce, n_total)
        # gloo has no RCCL communicator to lend the library: bind_rccl creates its own there
        assert par.torch_comm_ptr() is None
        out_q.put((rank, hist, a, lab))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_panel_equals_single_shard():
    n_total, T, seed, world = 1400, 12, 77, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, n_total, T, seed)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, hist, a, lab = q.get(timeout=240)
        res[r] = (hist, a, lab)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fx = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "egm_cfg1.npz")))
    lab0 = par.initial_labor_states(n_total, 7, 0, n_total).astype(np.int64)
    hist1, a1, l1 = _panel_history(np.full(n_total, float(fx["KSS"])), lab0, 0, T, seed, fx, lambda x: x, n_total)
    assert np.allclose(res[0][0], hist1, rtol=1e-13, atol=0)
    assert np.allclose(res[1][0], hist1, rtol=1e-13, atol=0)
    assert np.array_equal(np.concatenate([res[0][2], res[1][2]]), l1)
    assert np.allclose(np.concatenate([res[0][1], res[1][1]]), a1, rtol=1e-12)


class _FakeLib:
    """Stand-in for libaiyagari's communicator entry points (host logic only)."""

    def __init__(self, bind_ok):
        self.bind_ok = bind_ok
        self.calls = []

    def aiy_comm_bind(self, h, ptr):
        self.calls.append("bind")
        return 0 if self.bind_ok else -5

    def aiy_comm_destroy(self, h):
        self.calls.append("destroy")
        return 0

    def aiy_comm_unique_id(self, buf):
        self.calls.append("uid")
        buf.raw = bytes(range(128))
        return 0

    def aiy_comm_init(self, h, uid, world, rank):
        self.calls.append(("init", bytes(uid.raw[:4]), world, rank))
        return 0


class _FakeHandle:
    def __init__(self, lib):
        self.lib = lib
        self.h = None

    def check(self, rc, what):
        assert rc == 0, what


def _bind_worker(rank, world, port, out_q, ok_ranks):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        par.torch_comm_ptr = lambda group=None, device=None: 0x1234   # a communicator to lend
        lib = _FakeLib(rank in ok_ranks)
        out = par.bind_rccl(_FakeHandle(lib))
        out_q.put((rank, out, lib.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("ok_ranks", [(0, 1), (0,)])
def test_bind_rccl_ranks_agree(ok_ranks):
    """bind_rccl: when one rank cannot bind torch's communicator, every rank takes the
    library's own (the ranks that bound unbind first), so no rank waits in a broadcast the
    others never join."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_bind_worker, args=(r, world, port, q, ok_ranks)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (o, c)) for r, o, c in (q.get(timeout=100) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    kinds = {res[r][0][2] for r in range(world)}
    assert len(kinds) == 1
    if len(ok_ranks) == world:
        assert kinds == {"torch"}
    else:
        assert kinds == {"own"}
        assert "destroy" in res[0][1] and "destroy" not in res[1][1]
        for r in range(world):
            assert ("init", bytes(range(4)), world, r) in res[r][1]
