"""GPU parity: libaiyagari (HIP, gfx950) against the CPU oracle on identical inputs.

Tolerances (north_star): consumption policies within 1e-8 relative on the grid;
equilibrium r and K/Y within 1e-5 for the same grids and shocks.  Integer data
(labour states, cycle counts) must match exactly.  CRRA = 1 is expected bit-exact
(the kernels follow NumPy's operation order, see csrc/common.h)."""
import os

import numpy as np
import pytest
import torch

from oracle import hark_ks as H
from oracle import philox as PX

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
POLICY_RTOL = 1e-8


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def batch_from_fixture(fx, device):
    from aiyagari_hark_amd.egm import EgmBatch
    S = fx["P"].shape[0]
    lab = np.array([fx["LSStates"][sp // 4] for sp in range(S)])
    return EgmBatch.from_numpy(fx["aGrid"], fx["Mgrid"], fx["P"], fx["Rk"], fx["Wk"], fx["Mk"], lab,
                               float(fx["DiscFac"]), float(fx["CRRA"]), device=device)


@pytest.mark.parametrize("name", ["egm_cfg1", "egm_cfg1_afunc2", "egm_ckpt"])
def test_egm_single_steps(gpu, name):
    from aiyagari_hark_amd.egm import egm_step
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    b = batch_from_fixture(fx, gpu)
    crra = float(fx["CRRA"])
    mt = ct = None
    md = cd = None
    for step in range(4):
        mt, ct = H.egm_step(mt, ct, float(fx["DiscFac"]), crra, fx["aGrid"], fx["Mgrid"], fx["Rk"], fx["Wk"],
                            fx["Mk"], fx["LSStates"], fx["P"])
        md, cd = egm_step(b, md, cd)
        mh, ch = md[0].cpu().numpy(), cd[0].cpu().numpy()
        assert rel_err(ch, ct) <= (0.0 if crra == 1.0 else 1e-12), (step, rel_err(ch, ct))
        assert rel_err(mh, mt) <= (0.0 if crra == 1.0 else 1e-12)


@pytest.mark.parametrize("name", ["egm_cfg1", "egm_cfg1_afunc2", "egm_ckpt"])
def test_egm_solve_matches_golden(gpu, name):
    from aiyagari_hark_amd.egm import egm_solve
    fx = np.load(os.path.join(GOLD, name + ".npz"))
    b = batch_from_fixture(fx, gpu)
    m, c, cycles, dist = egm_solve(b, tol=1e-6, max_cycles=5000)
    assert int(cycles[0]) == int(fx["cycles"])
    assert rel_err(c[0].cpu().numpy(), fx["c"]) <= POLICY_RTOL
    assert rel_err(m[0].cpu().numpy(), fx["m"]) <= POLICY_RTOL
    assert dist[0] == pytest.approx(float(fx["dist"]), rel=1e-6)


def test_egm_batched_calibrations_independent(gpu):
    """Three calibrations in one launch == three separate solves (Table II batching)."""
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    fxs = [np.load(os.path.join(GOLD, n + ".npz")) for n in ("egm_cfg1", "egm_cfg1_afunc2", "egm_ckpt")]
    S = 28
    lab = [np.array([f["LSStates"][sp // 4] for sp in range(S)]) for f in fxs]
    b = EgmBatch.from_numpy(np.stack([f["aGrid"] for f in fxs]), np.stack([f["Mgrid"] for f in fxs]),
                            np.stack([f["P"] for f in fxs]), np.stack([f["Rk"] for f in fxs]),
                            np.stack([f["Wk"] for f in fxs]), np.stack([f["Mk"] for f in fxs]), np.stack(lab),
                            np.array([float(f["DiscFac"]) for f in fxs]), np.array([float(f["CRRA"]) for f in fxs]),
                            device=gpu)
    m, c, cycles, dist = egm_solve(b)
    for k, f in enumerate(fxs):
        assert int(cycles[k]) == int(f["cycles"])
        assert rel_err(c[k].cpu().numpy(), f["c"]) <= POLICY_RTOL


def test_egm_large_grid_step(gpu):
    """N_a = 2000 (config-2 law): one step from a converged-like table, HIP vs oracle."""
    from aiyagari_hark_amd.egm import egm_step
    m = H.KSModel(None, dict(aCount=2000))
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, 7, m.e)
    args = (0.96, 1.0, m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates, m.MrkvIndArray)
    mt, ct = H.egm_step(None, None, *args)
    mt, ct = H.egm_step(mt, ct, *args)
    m2, c2 = H.egm_step(mt, ct, *args)
    fx = dict(aGrid=m.aGrid, Mgrid=m.Mgrid, P=m.MrkvIndArray, LSStates=m.LSStates, Rk=Rk, Wk=Wk, Mk=Mk,
              DiscFac=0.96, CRRA=1.0)
    b = batch_from_fixture(fx, gpu)
    dm = torch.as_tensor(mt[None]).to(gpu)
    dc = torch.as_tensor(ct[None]).to(gpu)
    om, oc = egm_step(b, dm, dc)
    assert rel_err(oc[0].cpu().numpy(), c2) == 0.0
    assert rel_err(om[0].cpu().numpy(), m2) == 0.0


def test_policy_eval_matches_oracle(gpu):
    from aiyagari_hark_amd.egm import policy_eval
    fx = np.load(os.path.join(GOLD, "egm_cfg1_afunc2.npz"))
    rng = np.random.default_rng(0)
    n = 5000
    st = rng.integers(0, 28, n)
    mq = rng.uniform(0.0, 60.0, n)
    Mq = rng.uniform(0.3, 25.0, n)
    want = np.array([H.eval_policy_2d(fx["m"], fx["c"], fx["Mgrid"], int(s), np.array([q]), Q)[0]
                     for s, q, Q in zip(st, mq, Mq)])
    mt = torch.as_tensor(fx["m"]).to(gpu)
    ct = torch.as_tensor(fx["c"]).to(gpu)
    Mg = torch.as_tensor(fx["Mgrid"]).to(gpu)
    got = policy_eval(mt, ct, Mg, st, mq, Mq).cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    assert rel_err(got[ok], want[ok]) == 0.0


def _panel(gpu, fx, N, T, engine="grid"):
    from aiyagari_hark_amd.panel import DevicePanel
    p = DevicePanel(N, device=gpu, act_T=T, engine=engine)
    m = torch.as_tensor(fx["m"]).to(gpu)
    c = torch.as_tensor(fx["c"]).to(gpu)
    p.bind_model(m, c, torch.as_tensor(fx["Mgrid"]).to(gpu), torch.as_tensor(fx["LSStates"]).to(gpu),
                 torch.as_tensor(fx["cdf"]).to(gpu), torch.as_tensor(fx["Mrkv_hist"].astype(np.int32)).to(gpu),
                 dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
    return p


@pytest.mark.parametrize("engine", ["grid", "block"])
def test_panel_host_shocks_matches_golden(gpu, engine):
    """50 periods x 350 agents with a committed uniform stream: labour states exact,
    assets and the K/M history to 1e-12 (summation order of the mean differs)."""
    fx = np.load(os.path.join(GOLD, "egm_cfg1.npz"))
    pf = np.load(os.path.join(GOLD, "panel_cfg1.npz"))
    N, T = 350, int(pf["T"])
    p = _panel(gpu, fx, N, T, engine)
    p.reset(float(fx["KSS"]), pf["lab0"], float(fx["MSS"]), float(fx["KSS"]), 0, float(fx["RSS"]), float(fx["WSS"]))
    U = np.random.RandomState(int(pf["u_seed"])).random_sample((T, N))
    pos = {"t": 0}

    def src(n):
        out = U[pos["t"]:pos["t"] + n]
        pos["t"] += n
        return out

    p.run(0, T, shock_mode="numpy", u_host_source=src, chunk=7)
    torch.cuda.synchronize()
    assert np.array_equal(p.lab.cpu().numpy(), pf["lab_final"])
    assert rel_err(p.a.cpu().numpy(), pf["a_final"]) < 1e-12
    assert rel_err(p.hist_A.cpu().numpy(), pf["hist_A"]) < 1e-12
    assert rel_err(p.hist_M.cpu().numpy(), pf["hist_M"]) < 1e-12


@pytest.mark.parametrize("engine", ["grid", "block"])
def test_panel_philox_stream_matches_oracle(gpu, engine):
    """Device Philox uniforms == oracle Philox: labour draws of 3 periods agree exactly."""
    fx = np.load(os.path.join(GOLD, "egm_cfg1.npz"))
    N, T, seed, offset = 7000, 3, 2024, 0
    p = _panel(gpu, fx, N, T, engine)
    lab0 = np.repeat(np.arange(7), N // 7)
    p.reset(float(fx["KSS"]), lab0, float(fx["MSS"]), float(fx["KSS"]), 0, float(fx["RSS"]), float(fx["WSS"]))
    p.run(0, T, shock_mode="philox", seed=seed, ge_iter=1)
    torch.cuda.synchronize()
    lab = lab0.copy()
    for t in range(T):
        u = PX.uniform((1 << 20) + t, np.arange(N, dtype=np.uint64), seed)
        lab = H.draw_labor(lab, u, fx["cdf"])
    assert np.array_equal(p.lab.cpu().numpy(), lab)


@pytest.mark.parametrize("mode,shape", [("philox", 0), ("numpy", 0), ("philox", 1), ("philox", 2)])
def test_resident_panel_equals_per_period_kernel(gpu, mode, shape):
    """The persistent panel (one launch, agents in LDS, in-kernel grid barrier) against
    the one-launch-per-period kernel on 131 075 agents (odd: ragged last workgroup):
    labour states exact, assets (relative to the panel's scale) / history / market state
    to 1e-12 (the two differ only in the summation order of the mean); labour draws of the first periods against the
    oracle Philox exactly."""
    from aiyagari_hark_amd import _lib
    fx = np.load(os.path.join(GOLD, "egm_cfg1.npz"))
    N, T, seed = 131075, 150, 31
    rng = np.random.default_rng(5)
    lab0 = rng.integers(0, 7, N)
    U = rng.random((T, N))
    h = _lib.handle(gpu.index)
    out = {}
    h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT_SHAPE, shape), "aiy_set_option")
    for resident in (1, 0):
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT, resident), "aiy_set_option")
        try:
            p = _panel(gpu, fx, N, T, "grid")
            p.reset(float(fx["KSS"]), lab0, float(fx["MSS"]), float(fx["KSS"]), 0, float(fx["RSS"]),
                    float(fx["WSS"]))
            if mode == "philox":
                p.run(0, 2, shock_mode="philox", seed=seed, ge_iter=2)
                torch.cuda.synchronize()
                out[(resident, "lab2")] = p.lab.cpu().numpy()
                p.run(2, T - 2, shock_mode="philox", seed=seed, ge_iter=2)
            else:
                pos = {"t": 0}

                def src(n):
                    o = U[pos["t"]:pos["t"] + n]
                    pos["t"] += n
                    return o

                p.run(0, T, shock_mode="numpy", u_host_source=src, chunk=64)
            torch.cuda.synchronize()
            out[resident] = (p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy(),
                             p.sow.cpu().numpy())
        finally:
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT, 1), "aiy_set_option")
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT_SHAPE, 0), "aiy_set_option")
    res, ref = out[1], out[0]
    assert np.array_equal(res[0], ref[0])
    # assets near the borrowing limit come out of a cancellation (a = m - c), so they are
    # compared relative to the panel's scale; the aggregates elementwise
    assert np.max(np.abs(res[1] - ref[1])) / np.max(np.abs(ref[1])) < 1e-12
    for x, y in zip(res[2:4], ref[2:4]):
        assert rel_err(x, y) < 1e-12
    assert rel_err(res[4][:5], ref[4][:5]) < 1e-12
    assert res[4][7] == ref[4][7] == T
    if mode == "philox":
        lab = lab0.copy()
        for t in range(2):
            lab = H.draw_labor(lab, PX.uniform((2 << 20) + t, np.arange(N, dtype=np.uint64), seed), fx["cdf"])
        assert np.array_equal(out[(1, "lab2")], lab)


def test_batched_panel_equals_single_panels(gpu):
    """Three calibrations (different policies, shock seeds, odd population) in one block
    launch == three single-calibration grid-engine histories: labour exact, assets and
    the K/M history to 1e-12, final market state."""
    from aiyagari_hark_amd.panel import BatchedPanel
    names = ("egm_cfg1", "egm_cfg1_afunc2", "egm_ckpt")
    fxs = [np.load(os.path.join(GOLD, n + ".npz")) for n in names]
    N, T, seeds = 1001, 120, (5, 17, 99)
    mk = dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0))
    rng = np.random.default_rng(3)
    lab0 = rng.integers(0, 7, (3, N))
    bp = BatchedPanel(3, N, T, device=gpu)
    dv = lambda x: torch.as_tensor(np.ascontiguousarray(x)).to(gpu)  # noqa: E731
    bp.bind_models(dv(np.stack([f["m"] for f in fxs])), dv(np.stack([f["c"] for f in fxs])),
                   dv(np.stack([f["Mgrid"] for f in fxs])), dv(np.stack([f["LSStates"] for f in fxs])),
                   dv(np.stack([f["cdf"] for f in fxs])),
                   dv(np.stack([f["Mrkv_hist"][:T].astype(np.int32) for f in fxs])), [mk] * 3)
    bp.reset(np.array([float(f["KSS"]) for f in fxs]), lab0,
             [[float(f["MSS"]), float(f["KSS"]), 0, float(f["RSS"]), float(f["WSS"])] for f in fxs])
    bp.run(0, T // 2, shock_mode="philox", seeds=seeds, ge_iter=3)
    bp.run(T // 2, T - T // 2, shock_mode="philox", seeds=seeds, ge_iter=3)
    torch.cuda.synchronize()
    for k, f in enumerate(fxs):
        p = _panel(gpu, f, N, T, "grid")
        p.reset(float(f["KSS"]), lab0[k], float(f["MSS"]), float(f["KSS"]), 0, float(f["RSS"]), float(f["WSS"]))
        p.run(0, T, shock_mode="philox", seed=seeds[k], ge_iter=3)
        torch.cuda.synchronize()
        assert np.array_equal(bp.lab[k].cpu().numpy(), p.lab.cpu().numpy())
        assert rel_err(bp.a[k].cpu().numpy(), p.a.cpu().numpy()) < 1e-12
        assert rel_err(bp.hist_A[k].cpu().numpy(), p.hist_A.cpu().numpy()) < 1e-12
        assert rel_err(bp.hist_M[k].cpu().numpy(), p.hist_M.cpu().numpy()) < 1e-12
        assert rel_err(bp.sow[k, :5].cpu().numpy(), p.sow[:5].cpu().numpy()) < 1e-12


def test_economy_batch_matches_oracle(gpu):
    """Table II in the reference's algorithm: two calibrations solved to their KS fixed
    point in one EconomyBatch (batched EGM + one block-panel launch per GE iteration)
    reproduce each calibration's own oracle solve (numpy shock stream seeded per
    economy): same GE iteration count, coefficients within 1e-9, r and K/Y within 1e-5."""
    from aiyagari_hark_amd.sweep import EconomyBatch, build_economies
    cells = [dict(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), dict(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    econ_d = dict(act_T=1200, T_discard=400)
    agent_d = dict(AgentCount=350)
    econs = build_economies(cells, econ_d, agent_d, device=gpu, shock_mode="numpy", seed0=11)
    eb = EconomyBatch(econs)
    eb.solve()
    got = eb.results()
    for k, cell in enumerate(cells):
        ref = H.KSModel(dict(econ_d, **cell), dict(agent_d, **cell))
        log = []
        ref.solve(H.numpy_global_u_source(11 + k, 350), log=log)
        want = ref.results()
        g = econs[k].ge_log
        assert len(g) == len(log)
        for a, o in zip(g, log):
            assert a["cycles"] == o["cycles"]
            assert np.allclose(a["intercept"], o["intercept"], rtol=1e-9, atol=1e-12)
            assert np.allclose(a["slope"], o["slope"], rtol=1e-9, atol=1e-12)
        assert abs(got[k]["r"] - want["r"]) < 1e-5
        assert abs(got[k]["K_over_Y"] - want["saving_rate"] / 0.08) < 1e-5


def test_ge_fixed_point_matches_oracle(gpu):
    """Reduced Krusell-Smith fixed point (act_T = 1500, 350 agents) with the reference's
    global-RNG shock stream seeded identically: per-GE-iteration (intercept, slope) and
    the final r and K/Y agree (north_star: r and K/Y within 1e-5)."""
    from aiyagari_hark_amd.model import AiyagariEconomy, AiyagariType
    econ_d = dict(act_T=1500, T_discard=500, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0])
    agent_d = dict(AgentCount=350)
    ref = H.KSModel(dict(econ_d), dict(agent_d))
    log = []
    ref.solve(H.numpy_global_u_source(7, 350), log=log)
    want = ref.results()

    econ = AiyagariEconomy(**dict(econ_d, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0]))
    econ.verbose = False
    agent = AiyagariType(**agent_d)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    np.random.seed(7)
    econ.solve()
    assert len(econ.ge_log) == len(log)
    for g, o in zip(econ.ge_log, log):
        assert g["cycles"] == o["cycles"]
        assert np.allclose(g["intercept"], o["intercept"], rtol=1e-9, atol=1e-12)
        assert np.allclose(g["slope"], o["slope"], rtol=1e-9, atol=1e-12)
    r = econ.sow_state["Rnow"] - 1
    K = np.mean(econ.reap_state["aNow"][0])
    KtoY = K / (econ.sow_state["Mnow"] - (1 - 0.08) * K)
    assert abs(r - want["r"]) < 1e-5
    assert abs(KtoY - want["saving_rate"] / 0.08) < 1e-5
    # cFunc interop (Aiyagari-HARK.py:275)
    xi = agent.solution[0].cFunc[0].xInterpolators
    assert len(xi) == 15 and xi[0].x_list.shape == (33,)
    # .npz save/load: reloaded device tables evaluate identically
    import tempfile
    q_m = np.linspace(0.5, 40.0, 257)
    q_M = np.full(q_m.shape, float(econ.sow_state["Mnow"]))
    before = agent.solution[0].cFunc[5](q_m, q_M)
    afunc_before = [(f.intercept, f.slope) for f in agent.AFunc]
    with tempfile.TemporaryDirectory() as d:
        agent.save_solution(os.path.join(d, "sol.npz"))
        agent.solution = None
        agent.load_solution(os.path.join(d, "sol.npz"))
    assert agent.solution[0].m_tab.is_cuda
    np.testing.assert_array_equal(agent.solution[0].cFunc[5](q_m, q_M), before)
    assert [(f.intercept, f.slope) for f in agent.AFunc] == afunc_before


def test_search_index_equals_binary_search(gpu):
    """aiy_build_index + indexed lookup return exactly numpy searchsorted's bracket:
    evaluated through policy_eval-free path by comparing one EGM step with/without index."""
    from aiyagari_hark_amd import _lib
    fx = np.load(os.path.join(GOLD, "egm_cfg1_afunc2.npz"))
    h = _lib.handle(0)
    ipr = h.lib.aiy_index_ints_per_row()
    m = torch.as_tensor(fx["m"]).to(gpu).reshape(-1, fx["m"].shape[-1]).contiguous()
    idx = torch.empty((m.shape[0], ipr), dtype=torch.int32, device=gpu)
    h.check(h.lib.aiy_build_index(h.h, m.shape[0], m.shape[1], _lib.ptr(m), _lib.ptr(idx), _lib.stream_ptr()), "idx")
    torch.cuda.synchronize()
    H = idx.cpu().numpy()
    x = fx["m"].reshape(-1, fx["m"].shape[-1])
    shift = 44
    for r in range(0, x.shape[0], 37):
        xr = x[r, :-1]
        base = int(H[r, -1])
        assert base == int(np.float64(x[r, 1]).view(np.int64) >> shift)
        last = int(H[r, ipr - 2])
        for b in list(range(0, last + 2, 7)) + [last, last + 1]:
            edge = np.int64((base + b) << shift).view(np.float64)
            assert H[r, b] == np.searchsorted(xr, edge), (r, b)


def _brk_window(E, shift, n_buckets, n, q):
    """Host restatement of brk_window (csrc/common.h): the search window [lo, hi) of
    lower_bound(z[0..n), q) read from one bracket index E (uint64); lo == hi: resolved."""
    last, base = int(np.int64(E[n_buckets])), int(np.int64(E[n_buckets + 1]))
    bits = int(np.float64(q).view(np.uint64))
    key = (bits >> shift) - base
    lo_of = lambda e: int(e) >> 43  # noqa: E731
    if not q > 0 or key < 0:
        return 0, lo_of(E[0])
    if key >= n_buckets - 1:
        return (lo_of(E[n_buckets - 1]), n) if last == n_buckets - 1 else (n, n)
    if key > last:
        return n, n
    e = int(E[key])
    lo, cnt = lo_of(e), (e >> 40) & 7
    if cnt == 0:
        return lo, lo
    if cnt <= 3:
        w = min(40 // cnt, shift)
        mask = (1 << w) - 1
        qf = (bits >> (shift - w)) & mask
        xf = [(e >> (j * w)) & mask for j in range(cnt)]
        below = sum(x < qf for x in xf)
        upto = sum(x <= qf for x in xf)
        return (lo + below, lo + below) if w == shift else (lo + below, lo + upto)
    return (lo, lo + cnt) if cnt < 7 else (lo, lo_of(E[key + 1]))


def _tab_geom(n_lab, n_M, n_a):
    """Host restatement of panel_tab_geom (csrc/panel_common.h)."""
    up = lambda b: (b + 255) // 256 * 256  # noqa: E731
    Z, n_J = 2 * n_a, max(n_M - 1, 1)
    cells = 2 * n_lab * n_J
    lg = 4
    while lg < 13 and (1 << lg) < n_a:
        lg += 1
    buckets = 12 << lg
    rec_off = 0
    z_off = up(cells * 4 * (Z + 1) * 16)
    idx_off = up(z_off + cells * Z * 8)
    return dict(Z=Z, n_J=n_J, cells=cells, shift=52 - lg, buckets=buckets, z_off=z_off, idx_off=idx_off,
                bytes=up(idx_off + cells * (buckets + 2) * 8), rec_off=rec_off)


@pytest.mark.parametrize("name", ["egm_cfg1_afunc2", "big"])
def test_panel_tables_semantics(gpu, name):
    """aiy_panel_build: for every probed cell (labour l, aggregate state g, M interval j)
    z is the stable merge of the two rows' searched nodes; for queries across the cell
    (nodes, their ulp neighbours, random values, below / above the grid) the bracket
    index window contains searchsorted(z, q), and record k = searchsorted(z, q) holds
    exactly each row's HARK bracket nodes (max(searchsorted(x[:-1], q), 1) - 1, + 0)."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.panel import build_tables
    rng = np.random.default_rng(2)
    if name == "big":   # a 3000-node policy (config-2 density) built from one fixture row pair
        S, n_M, n_a = 28, 3, 3000
        base = np.sort(np.concatenate([[1e-7], 0.3 + np.cumsum(rng.exponential(0.004, n_a))]))
        m = np.stack([base * (1.0 + 0.01 * k) + 0.001 * s for s in range(S) for k in range(n_M)])
        m[:, 0] = 1e-7
        m = m.reshape(S, n_M, n_a + 1)
    else:
        fx = np.load(os.path.join(GOLD, name + ".npz"))
        m = np.ascontiguousarray(fx["m"])
        S, n_M, n1 = m.shape
        n_a = n1 - 1
    c = 0.5 * m + 0.01
    n_lab = S // 4
    h = _lib.handle(gpu.index)
    g = _tab_geom(n_lab, n_M, n_a)
    assert h.lib.aiy_panel_table_bytes(n_lab, n_M, n_a, 0) == g["bytes"]
    tab = build_tables(h, torch.as_tensor(m[None]).to(gpu), torch.as_tensor(c[None]).to(gpu), n_lab, gpu)
    torch.cuda.synchronize()
    raw = tab[0].cpu().numpy()
    Z, n_J = g["Z"], g["n_J"]
    rec = raw[g["rec_off"]:g["z_off"]].view(np.float64)[: g["cells"] * (Z + 1) * 8].reshape(g["cells"], Z + 1, 8)
    zz = raw[g["z_off"]:g["idx_off"]].view(np.float64)[: g["cells"] * Z].reshape(g["cells"], Z)
    E_all = raw[g["idx_off"]:].view(np.uint64)[: g["cells"] * (g["buckets"] + 2)].reshape(g["cells"], -1)
    resolved = total = 0
    for cell in sorted(set([0, 1, g["cells"] - 1] + list(rng.integers(0, g["cells"], 4)))):
        lgc, jc = divmod(cell, n_J)
        s = 4 * (lgc // 2) + 2 * (lgc % 2) + 1
        j0, j1 = (jc, jc + 1) if n_M > 1 else (0, 0)
        x0, x1 = m[s, j0], m[s, j1]
        y0, y1 = c[s, j0], c[s, j1]
        want_z = np.sort(np.concatenate([x0[:-1], x1[:-1]]), kind="stable")
        assert np.array_equal(zz[cell], want_z), cell
        rand = rng.uniform(x0[1], x0[-1], 300)
        qs = np.concatenate([rand, want_z, np.nextafter(want_z, np.inf), np.nextafter(want_z, -np.inf),
                             [-1.0, 0.0, 1e-9, 1e-7, 3 * x0[-1], 1e6]])
        for iq, q in enumerate(qs):
            k = int(np.searchsorted(want_z, q))
            lo, hi = _brk_window(E_all[cell], g["shift"], g["buckets"], Z, float(q))
            assert lo <= k <= hi, (cell, q, lo, hi, k)
            if iq < len(rand):
                resolved += lo == hi
                total += 1
            if k > 0 and k < Z and want_z[k - 1] == want_z[k]:
                continue   # empty segment, never selected
            i0 = max(int(np.searchsorted(x0[:-1], q)), 1)
            i1 = max(int(np.searchsorted(x1[:-1], q)), 1)
            want = [x0[i0 - 1], x0[i0], y0[i0 - 1], y0[i0], x1[i1 - 1], x1[i1], y1[i1 - 1], y1[i1]]
            assert np.array_equal(rec[cell, k], want), (cell, q, k)
    # random queries: at config-2 density most lookups resolve from the entry alone (at
    # N_a = 32 the two rows' nodes sit close together and often share a bucket)
    assert resolved > (0.95 if name == "big" else 0.5) * total


def test_stationary_capital_supply_matches_oracle(gpu):
    """E1/E2 at r = 4 %: stationary EGM tables bit-exact (CRRA 1), Young-lottery K to 1e-10."""
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    fx = np.load(os.path.join(GOLD, "stationary.npz"))
    b = StationaryBatch([Calibration()], fx["aGrid"], device=gpu)
    K, cycles, iters = b.capital_supply(np.array([float(fx["r"])]), egm_tol=1e-8, hist_tol=1e-12)
    m, c = b.last_tables
    assert int(cycles[0]) == int(fx["cycles"])
    assert rel_err(c[0, :, 0].cpu().numpy(), fx["c"]) == 0.0
    assert abs(K[0] - float(fx["K"])) / float(fx["K"]) < 1e-10
    assert abs(int(iters[0]) - int(fx["hist_iters"])) <= 2
    mass = b.mass[0].cpu().numpy()
    assert abs(mass.sum() - 1.0) < 1e-12
    assert np.max(np.abs(mass - fx["mass"])) < 1e-12


def test_stationary_bisection_matches_oracle(gpu):
    """GE bisection on r for a 3-calibration batch (mixed CRRA, Rouwenhorst row) vs the oracle."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    from oracle import stationary as ST
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=3.0),
            Calibration(LaborAR=0.3, LaborSD=0.2, CRRA=5.0)]
    res = solve_table2(cals, n_a=120, r_tol=1e-6, device=gpu)
    aGrid = ST.make_stationary_grid(0.001, 50.0, 120, 2)
    for k, cal in enumerate(cals):
        lab, P = ST.income_process(7, cal.LaborAR, cal.LaborSD, "tauchen")
        want = ST.ge_bisect(dict(DiscFac=0.96, CRRA=cal.CRRA, CapShare=0.36, DeprFac=0.08), aGrid, lab, P,
                            r_tol=1e-6)
        assert abs(res.r[k] - want["r"]) < 1e-5
        assert abs(res.KtoY[k] - want["KtoY"]) < 1e-5


def test_rouwenhorst_25_state_histogram(gpu):
    """Stress shape (25-state Rouwenhorst, S = 25 > 16): K_s(r) vs oracle."""
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    from oracle import stationary as ST
    cal = Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0, LaborStatesNo=25, income="rouwenhorst")
    aGrid = ST.make_stationary_grid(0.001, 50.0, 300, 2)
    b = StationaryBatch([cal], aGrid, device=gpu)
    K, cycles, iters = b.capital_supply(np.array([0.02]), egm_tol=1e-8, hist_tol=1e-12)
    lab, P = ST.income_process(25, 0.9, 0.4, "rouwenhorst")
    Kw, info = ST.capital_supply(0.02, dict(DiscFac=0.96, CRRA=5.0, CapShare=0.36, DeprFac=0.08), aGrid, lab, P)
    assert int(cycles[0]) == info["cycles"]
    assert abs(K[0] - Kw) / Kw < 1e-9


@pytest.mark.parametrize("S_lab,income,n_a,n_cal", [(7, "tauchen", 1000, 3), (25, "rouwenhorst", 700, 2),
                                                      (7, "tauchen", 5000, 2)])
def test_hist_fused_step_matches_push_mix(gpu, S_lab, income, n_a, n_cal):
    """Fused lottery step (hist_step_kernel, AIY_OPT_HIST_FUSED = 1) vs the default
    push/mix pair: same stationary mass to 1e-13, same iteration counts, and K_s(r)
    against the oracle's Young histogram (oracle/stationary.py)."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    from oracle import stationary as ST
    cals = [Calibration(LaborAR=0.9 - 0.3 * i, LaborSD=0.4, CRRA=1.0 + 2 * i, LaborStatesNo=S_lab, income=income)
            for i in range(n_cal)]
    aGrid = ST.make_stationary_grid(0.001, 50.0, n_a, 2)
    h = _lib.handle(gpu.index)
    r = np.array([0.02 + 0.004 * i for i in range(n_cal)])
    out = {}
    try:
        for fused in (0, 1):
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_FUSED, fused), "opt")
            b = StationaryBatch(cals, aGrid, device=gpu)
            K, cycles, iters = b.capital_supply(r, egm_tol=1e-8, hist_tol=1e-12)
            out[fused] = (K, iters, b.mass.cpu().numpy())
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_FUSED, 0), "opt")
    K0, it0, m0 = out[0]
    K1, it1, m1 = out[1]
    assert np.max(np.abs(it0 - it1)) <= 1          # atomics: summation order is not fixed in either path
    assert np.max(np.abs(m1 - m0)) < 1e-11
    assert np.max(np.abs(K1 - K0) / K0) < 1e-11
    for i, c in enumerate(cals):
        lab, P = ST.income_process(S_lab, c.LaborAR, c.LaborSD, income)
        Kw, _ = ST.capital_supply(r[i], dict(DiscFac=0.96, CRRA=c.CRRA, CapShare=0.36, DeprFac=0.08), aGrid, lab, P)
        assert abs(K1[i] - Kw) / Kw < 1e-9


def test_bisection_warm_histogram_same_equilibrium(gpu):
    """Warm-started distribution iteration between bisection steps (solve_table2's
    default) reaches the cold-started equilibrium: r and K/Y within 1e-9, identical
    bisection path."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0), Calibration(LaborAR=0.3, LaborSD=0.2, CRRA=1.0)]
    warm = solve_table2(cals, n_a=400, r_tol=1e-7, device=gpu, warm_hist=True)
    cold = solve_table2(cals, n_a=400, r_tol=1e-7, device=gpu, warm_hist=False)
    assert warm.bisection_steps == cold.bisection_steps
    assert np.max(np.abs(warm.r - cold.r)) < 1e-9
    assert np.max(np.abs(warm.KtoY - cold.KtoY)) < 1e-9
    assert sum(int(np.max(i)) for i in warm.hist_iters) < sum(int(np.max(i)) for i in cold.hist_iters)


def test_load_solution_resumes_ge_loop(gpu, tmp_path):
    """save after one GE iteration, load into a FRESH economy + agent with
    ``economy=``, resume econ.solve(): the resumed iterations reproduce iterations 1..k of
    the uninterrupted solve (same damping state intercept_prev / slope_prev, same saving
    rule, same Philox GE-iteration keys), bit for bit."""
    from aiyagari_hark_amd.model import AiyagariEconomy, AiyagariType

    def pair():
        econ = AiyagariEconomy(act_T=600, T_discard=200, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0])
        econ.verbose = False
        agent = AiyagariType(device=gpu, shock_mode="philox", shock_seed=3, AgentCount=700)
        agent.cycles = 0
        agent.get_economy_data(econ)
        econ.agents = [agent]
        econ.make_Mrkv_history()
        return econ, agent

    full, _ = pair()
    full.max_loops = 3
    full.solve()
    first, agent1 = pair()
    first.max_loops = 1
    first.solve()
    path = str(tmp_path / "ge1.npz")
    agent1.save_solution(path, economy=first)
    econ2, agent2 = pair()
    agent2.load_solution(path, economy=econ2)
    assert econ2.intercept_prev == first.intercept_prev and econ2.slope_prev == first.slope_prev
    econ2.max_loops = 2
    econ2.solve()
    for a, b in zip(econ2.ge_log, full.ge_log[1:]):
        assert a["intercept"] == b["intercept"] and a["slope"] == b["slope"]
        assert a["cycles"] == b["cycles"]
    assert econ2.sow_state["Rnow"] == full.sow_state["Rnow"]


def test_stationary_brent_warm_matches_oracle_bisection(gpu):
    """E1 with Brent's method and warm-started household + distribution solves (the bench's
    Table II settings) lands on the oracle's bisection root: r within 2e-7, K/Y within 1e-5,
    in fewer K_s evaluations."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    from oracle import stationary as ST
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.0, LaborSD=0.4, CRRA=3.0)]
    res = solve_table2(cals, n_a=150, r_tol=1e-8, device=gpu, method="brent")
    aGrid = ST.make_stationary_grid(0.001, 50.0, 150, 2)
    for k, cal in enumerate(cals):
        lab, P = ST.income_process(7, cal.LaborAR, cal.LaborSD, "tauchen")
        want = ST.ge_bisect(dict(DiscFac=0.96, CRRA=cal.CRRA, CapShare=0.36, DeprFac=0.08), aGrid, lab, P,
                            r_tol=1e-8)
        assert abs(res.r[k] - want["r"]) < 2e-7, (k, res.r[k], want["r"])
        assert abs(res.KtoY[k] - want["KtoY"]) < 1e-5
    assert res.bisection_steps < want["iters"]


def test_stationary_brent_many_states_matches_oracle(gpu):
    """E1 + E2 beyond 32 income states (36-state Rouwenhorst: the host-driven search over the
    pull-form BiCGSTAB's SMAX = 64 instantiation) lands on the oracle's bisection root."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    from oracle import stationary as ST
    cal = Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=3.0, LaborStatesNo=36, income="rouwenhorst")
    res = solve_table2([cal], n_a=150, r_tol=1e-8, device=gpu, method="brent")
    aGrid = ST.make_stationary_grid(0.001, 50.0, 150, 2)
    lab, P = ST.income_process(36, cal.LaborAR, cal.LaborSD, "rouwenhorst")
    want = ST.ge_bisect(dict(DiscFac=0.96, CRRA=cal.CRRA, CapShare=0.36, DeprFac=0.08), aGrid, lab, P, r_tol=1e-8)
    assert abs(res.r[0] - want["r"]) < 2e-7, (res.r[0], want["r"])
    assert abs(res.KtoY[0] - want["KtoY"]) < 1e-5


@pytest.mark.parametrize("method", ["bisect", "brent"])
def test_native_ge_search_equals_python_loop(gpu, method):
    """aiy_ge_stationary (the E1 search loop in C++) takes exactly the steps of
    the Python-driven loop: identical r (bit for bit) and step count.  The host-driven native
    loop is the one compared bit for bit; the device-resident search (one launch, its own
    cluster sizes and so its own reduction order) reaches the same root to the tolerance."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    nat = solve_table2(cals, n_a=300, r_tol=1e-8, device=gpu, method=method, engine="native", secant=False,
                       loose=False, extrapolate=False, groups=1, resident=False)
    py = solve_table2(cals, n_a=300, r_tol=1e-8, device=gpu, method=method, engine="python")
    assert nat.bisection_steps == py.bisection_steps
    assert np.array_equal(nat.r, py.r)
    assert np.array_equal(nat.KtoY, py.KtoY)
    if method == "brent":   # secant starts: other iterates, the same root to the search tolerance
        for sec_on, loose_on, ex_on, grp, res in ((True, False, False, 1, False), (True, True, False, 1, False),
                                                  (True, True, True, 1, False), (True, True, True, 3, False),
                                                  (False, False, False, 1, True), (True, True, True, 1, True)):
            sec = solve_table2(cals, n_a=300, r_tol=1e-8, device=gpu, method=method, engine="native",
                               secant=sec_on, loose=loose_on, extrapolate=ex_on, groups=grp, resident=res)
            assert np.max(np.abs(sec.r - py.r)) < 1e-7, (sec_on, loose_on, ex_on, grp, np.abs(sec.r - py.r))


@pytest.mark.parametrize("pull", [1, 0])
def test_distribution_solve_independent_of_launch_mates(gpu, pull):
    """One calibration's BiCGSTAB distribution solve (aiy_hist_solve, one cluster per
    calibration) gives the same K_s whether it shares its launch with other calibrations or
    runs alone, and with other work queued on the device: the clusters share no data, and a
    solve's result depends only on its own inputs (tools/hist_determinism.py).
    The pull form (AIY_OPT_HIST_PULL) has no atomics, so it is held bit for bit; the push
    form's LDS atomics from different waves add to a boundary destination in an order the
    hardware does not fix: a last-bit change in one matvec can move the Krylov path,
    so it is held to the stopping rule's own accuracy (K within ~4e5 hist_tol relative of the
    exact distribution, DESIGN.md §4c: 5e-7 here)."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    grid = sm.make_grid_exp_mult(0.001, 50.0, 300, 2)
    r = np.array([0.03, 0.02, float.fromhex("0x1.2a359f8a72972p-5")])
    h = _lib.handle(gpu.index)
    prev = h.set_options({_lib.AIY_OPT_HIST_PULL: pull})
    try:
        batch = StationaryBatch(cals, grid, device=gpu)
        K3, _, it3 = batch.capital_supply(r, accel=-1)
        assert np.all(np.isfinite(K3)) and np.all(it3 > 0)
        x = torch.randn(2048, 2048, device=gpu)
        for c in range(len(cals)):
            y = torch.tanh(x @ x * 1e-3)   # queued ahead of the solve's launches
            alone = StationaryBatch([cals[c]], grid, device=gpu)
            K1, _, _ = alone.capital_supply(r[c:c + 1], accel=-1)
            if pull:
                assert float(K1[0]).hex() == float(K3[c]).hex(), (c, K1[0], K3[c])
            else:
                assert abs(K1[0] - K3[c]) <= 5e-7 * abs(K3[c]), (c, K1[0], K3[c])
        assert torch.isfinite(y).all()
    finally:
        h.set_options(prev)
