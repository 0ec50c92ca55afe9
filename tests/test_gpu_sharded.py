"""GPU tests of the agent-sharded panel (SURVEY.md §8e.2, configs[3]): the library's
sharded period paths against the unsharded history.

The sharded form replaces np.mean(np.array(aNow)) (Aiyagari_Support.py:1868) by a sum
over ranks: per period aiy_sim_period_local (local agents, local sum in sow[6]) ->
caller all-reduce -> aiy_sim_period_prices.  Philox draws are keyed by the GLOBAL agent
index, so a sharded history equals the unsharded one except for the summation order
of the mean: labour states must match exactly, the K / M history to 1e-13 relative and
the assets to 1e-12 of the panel's scale.  A one-GPU box cannot host two RCCL ranks
(RCCL refuses two ranks on one device), so the multi-process test uses gloo for the
caller-side all-reduce, and the library's own RCCL path is exercised with a one-rank
communicator."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
MARKET = dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0))


def _fixture():
    return dict(np.load(os.path.join(GOLD, "egm_cfg1.npz")))


def _panel(dev, fx, n_local, T, offset=0, n_total=None, engine="grid"):
    from aiyagari_hark_amd.panel import DevicePanel
    p = DevicePanel(n_local, device=dev, act_T=T, agent_offset=offset, n_total=n_total, engine=engine)
    hist = np.resize(fx["Mrkv_hist"].astype(np.int32), T)
    p.bind_model(torch.as_tensor(fx["m"]).to(dev), torch.as_tensor(fx["c"]).to(dev),
                 torch.as_tensor(fx["Mgrid"]).to(dev), torch.as_tensor(fx["LSStates"]).to(dev),
                 torch.as_tensor(fx["cdf"]).to(dev), torch.as_tensor(hist).to(dev), MARKET)
    return p


def _reset(p, fx, lab0):
    p.reset(float(fx["KSS"]), lab0, float(fx["MSS"]), float(fx["KSS"]), 0, float(fx["RSS"]), float(fx["WSS"]))


def _unsharded(dev, fx, N, T, lab0, seed, U=None):
    p = _panel(dev, fx, N, T)
    _reset(p, fx, lab0)
    if U is None:
        p.run(0, T, shock_mode="philox", seed=seed, ge_iter=1)
    else:
        pos = {"t": 0}

        def src(n):
            o = U[pos["t"]:pos["t"] + n]
            pos["t"] += n
            return o
        p.run(0, T, shock_mode="numpy", u_host_source=src, chunk=16)
    torch.cuda.synchronize()
    return p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy()


def _check(got, ref):
    lab, a, hA, hM = got
    rlab, ra, rhA, rhM = ref
    assert np.array_equal(lab, rlab)
    assert np.max(np.abs(a - ra)) / np.max(np.abs(ra)) < 1e-12
    assert np.max(np.abs(hA - rhA) / np.abs(rhA)) < 1e-13
    assert np.max(np.abs(hM - rhM) / np.abs(rhM)) < 1e-13


@pytest.mark.parametrize("mode,split", [("philox", "pairs"), ("numpy", "pairs"), ("philox", "odd")])
def test_two_step_shards_equal_unsharded(gpu, mode, split):
    """Two shards in one process, summed between the two library steps, against the unsharded
    panel.  split "pairs": parallel.shard_range, which splits on agent pairs (offsets 0 and
    100 002 for N = 200 001: every shard takes the resident kernel); split "odd": hand-built
    shards (0, 100 001) and (100 001, 100 000) whose boundary cuts a Philox pair (2k, 2k + 1),
    so the second shard runs the per-period sim_period_kernel fallback of aiy_sim_period_local
    (ADVICE r5)."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.parallel import shard_range
    fx = _fixture()
    N, T, seed = 200_001, 40, 9
    lab0 = np.random.default_rng(4).integers(0, 7, N)
    U = np.random.default_rng(6).random((T, N)) if mode == "numpy" else None
    ref = _unsharded(gpu, fx, N, T, lab0, seed, U)
    h = _lib.handle(gpu.index)
    shards = []
    ranges = [shard_range(N, 2, r) for r in range(2)] if split == "pairs" else [(0, 100_001), (100_001, 100_000)]
    assert ranges[1][0] % 2 == (0 if split == "pairs" else 1)
    for off, nl in ranges:
        p = _panel(gpu, fx, nl, T, offset=off, n_total=N)
        _reset(p, fx, lab0[off:off + nl])
        shards.append((off, nl, p))
    sp = _lib.stream_ptr()
    for t in range(T):
        keep = []
        for off, nl, p in shards:
            pm = p._model[0]
            up = None
            if U is not None:
                ut = torch.as_tensor(np.ascontiguousarray(U[t, off:off + nl])).to(gpu)
                keep.append(ut)
                up = ut.data_ptr()
            h.check(h.lib.aiy_sim_period_local(h.h, ctypes.byref(pm), nl, off, _lib.ptr(p.a), _lib.ptr(p.lab), up,
                                               None, seed, 1, t, _lib.ptr(p.sow), sp), "local")
        total = shards[0][2].sow[6] + shards[1][2].sow[6]
        for off, nl, p in shards:
            p.sow[6] = total
            pm, mk = p._model[0], p._model[1]
            h.check(h.lib.aiy_sim_period_prices(h.h, ctypes.byref(pm), ctypes.byref(mk), N, t, _lib.ptr(p.sow),
                                                _lib.ptr(p.hist_A), _lib.ptr(p.hist_M), sp), "prices")
    torch.cuda.synchronize()
    got = (np.concatenate([p.lab.cpu().numpy() for _, _, p in shards]),
           np.concatenate([p.a.cpu().numpy() for _, _, p in shards]),
           shards[1][2].hist_A.cpu().numpy(), shards[1][2].hist_M.cpu().numpy())
    _check(got, ref)
    assert np.array_equal(shards[0][2].hist_A.cpu().numpy(), got[2])


def test_rccl_path_one_rank_equals_unsharded(gpu):
    """The library's own RCCL path (per-period kernel -> ncclAllReduce of the local sum
    -> price kernel, enqueued by aiy_sim_periods) with a one-rank communicator."""
    from aiyagari_hark_amd import _lib
    fx = _fixture()
    N, T, seed = 150_003, 30, 21
    lab0 = np.random.default_rng(8).integers(0, 7, N)
    ref = _unsharded(gpu, fx, N, T, lab0, seed)
    h = _lib.handle(gpu.index)
    uid = ctypes.create_string_buffer(128)
    assert h.lib.aiy_comm_unique_id(uid) == 0
    h.check(h.lib.aiy_comm_init(h.h, uid, 1, 0), "aiy_comm_init")
    try:
        p = _panel(gpu, fx, N, T)
        _reset(p, fx, lab0)
        p.run(0, T, shock_mode="philox", seed=seed, ge_iter=1)
        torch.cuda.synchronize()
        got = (p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy())
    finally:
        h.check(h.lib.aiy_comm_destroy(h.h), "aiy_comm_destroy")
    _check(got, ref)


def _torch_comm_rank(port, q, N, T, seed):
    """One rank of a torch.distributed RCCL ("nccl") group: the library borrows torch's own
    communicator (parallel.bind_rccl -> aiy_comm_bind) and runs the sharded-path panel."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from aiyagari_hark_amd import _lib
        from aiyagari_hark_amd.parallel import bind_rccl, unbind_rccl
        h = _lib.handle(0)
        world, rank, kind = bind_rccl(h)
        try:
            fx = _fixture()
            lab0 = np.random.default_rng(8).integers(0, 7, N)
            p = _panel(dev, fx, N, T)
            _reset(p, fx, lab0)
            p.run(0, T, shock_mode="philox", seed=seed, ge_iter=1)
            torch.cuda.synchronize()
            q.put((kind, p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy()))
        finally:
            unbind_rccl(h)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_torch_communicator_bound_equals_unsharded(gpu):
    """bind_rccl borrows torch.distributed's RCCL communicator (one communicator per device:
    torch's bundled librccl is the only RCCL in the process); with one rank the library's
    RCCL period path gives the unsharded history."""
    import multiprocessing as mp
    fx = _fixture()
    N, T, seed = 150_003, 30, 21
    lab0 = np.random.default_rng(8).integers(0, 7, N)
    ref = _unsharded(gpu, fx, N, T, lab0, seed)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_torch_comm_rank, args=(_free_port(), q, N, T, seed))
    proc.start()
    kind, *got = q.get(timeout=240)
    proc.join(timeout=60)
    assert proc.exitcode == 0
    assert kind == "torch"
    _check(tuple(got), ref)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_rank(rank, world, port, q, N, T, seed):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from aiyagari_hark_amd import build
        from aiyagari_hark_amd.parallel import shard_range, torch_allreduce
        build.build(verbose=False)
        dev = torch.device("cuda:0")
        fx = _fixture()
        lab0 = np.random.default_rng(12).integers(0, 7, N)
        off, nl = shard_range(N, world, rank)
        p = _panel(dev, fx, nl, T, offset=off, n_total=N)
        _reset(p, fx, lab0[off:off + nl])
        p.run(0, T, shock_mode="philox", seed=seed, ge_iter=1, allreduce=torch_allreduce())
        torch.cuda.synchronize()
        q.put((rank, p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_process_gloo_sharded_panel(gpu):
    """Two rank processes (both on GPU 0) drive the library's two-step sharded period,
    all-reducing the local sums over gloo (parallel.torch_allreduce): the concatenated
    shards equal the unsharded history."""
    import torch.multiprocessing as mp
    fx = _fixture()
    N, T, seed, world = 100_001, 30, 5, 2
    lab0 = np.random.default_rng(12).integers(0, 7, N)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, q, N, T, seed)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(world):
            r, *vals = q.get(timeout=240)
            res[r] = vals
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.is_alive():
                pr.kill()
    assert all(pr.exitcode == 0 for pr in procs)
    ref = _unsharded(gpu, fx, N, T, lab0, seed)
    got = (np.concatenate([res[0][0], res[1][0]]), np.concatenate([res[0][1], res[1][1]]), res[0][2], res[0][3])
    _check(got, ref)
    assert np.array_equal(res[0][2], res[1][2])


def test_run_past_history_is_refused(gpu):
    """a run past act_T is refused on the host (Python) and by the C ABI."""
    from aiyagari_hark_amd import _lib
    fx = _fixture()
    N, T = 7000, 12
    p = _panel(gpu, fx, N, T)
    _reset(p, fx, np.repeat(np.arange(7), N // 7))
    with pytest.raises(ValueError):
        p.run(5, T - 4, shock_mode="philox")
    h = _lib.handle(gpu.index)
    pm, mk = p._model[0], p._model[1]
    rc = h.lib.aiy_sim_periods(h.h, ctypes.byref(pm), ctypes.byref(mk), N, 0, N, _lib.ptr(p.a), _lib.ptr(p.lab), None,
                               0, None, 0, 1, 0, 5, T - 4, _lib.ptr(p.sow), _lib.ptr(p.hist_A), _lib.ptr(p.hist_M),
                               _lib.stream_ptr())
    assert rc == -1 and b"act_T" in h.lib.aiy_last_error(h.h)
    rc = h.lib.aiy_sim_period_local(h.h, ctypes.byref(pm), N, 0, _lib.ptr(p.a), _lib.ptr(p.lab), None, None, 0, 1,
                                    T, _lib.ptr(p.sow), _lib.stream_ptr())
    assert rc == -1
    p.run(0, T, shock_mode="philox")   # the full history is fine
    torch.cuda.synchronize()
    assert float(p.sow[7]) == T
