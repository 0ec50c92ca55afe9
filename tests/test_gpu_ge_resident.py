"""GPU tests of the device-resident GE search (csrc/ge_resident.hip):
every calibration's cluster runs its whole root search -- EGM cycles, lottery, BiCGSTAB
distribution solve, K_s reduction, Brent / bisection update -- inside ONE launch.

* the same search as the host-driven loop (aiy_ge_stationary with AIY_OPT_GE_RESIDENT off):
  bisection takes the same steps and lands on the same r; Brent lands within the search
  tolerance of it (the two paths sum K_s in different orders, so a near-tie can take a
  different Brent step);
* the oracle's full-size Table II roots are pinned in test_gpu_benchsize.py (the bench's
  call, which takes this path by default).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cells(n):
    from aiyagari_hark_amd.stationary import table2_calibrations
    cals = table2_calibrations()
    return [cals[k] for k in np.linspace(0, len(cals) - 1, n).astype(int)]


def test_resident_plan_shapes(gpu):
    from aiyagari_hark_amd.stationary import resident_plan
    p = resident_plan(gpu, 24, 7, 10_000)
    assert p is not None
    G, nj, kc, blocks = p
    assert G * 24 <= torch.cuda.get_device_properties(gpu).multi_processor_count
    assert G * nj >= 10_000 and kc in (1, 2) and blocks % 8 == 0
    p3 = resident_plan(gpu, 3, 7, 10_000)
    assert p3 is not None and p3[0] >= G
    half = resident_plan(gpu, 24, 7, 10_000, cu_share=0.5)
    assert half is None or half[0] * 24 <= 128
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    from aiyagari_hark_amd import _lib
    h = _lib.handle(gpu.index)
    assert resident_plan(gpu, 3, 25, 50_000) is None     # configs[4]: the host-driven loop
    assert resident_plan(gpu, 3, 16, 50_000) is None     # every S > 8: the host-driven loop
    # clusters above 128 workgroups would escape the cluster reductions: the host loop runs
    assert resident_plan(gpu, 1, 7, 150_000) is None
    p1 = resident_plan(gpu, 1, 7, 120_000)
    assert p1 is None or p1[0] <= 128


@pytest.mark.parametrize("method", ["bisect", "brent"])
def test_resident_matches_host_search(gpu, method):
    from aiyagari_hark_amd.stationary import solve_table2
    cals = _cells(6)
    kw = dict(n_a=1500, device=gpu, method=method, accel=-1, warm_egm=True, groups=1)
    res = solve_table2(cals, resident=True, **kw)
    ref = solve_table2(cals, resident=False, **kw)
    print(f"\n{method}: resident r {res.r} steps {res.bisection_steps}; host r {ref.r} steps {ref.bisection_steps}")
    assert np.all(res.status == 0) and np.all(ref.status == 0)
    if method == "bisect":
        assert res.bisection_steps == ref.bisection_steps
        assert np.max(np.abs(res.r - ref.r)) <= 1e-12
    else:
        assert np.max(np.abs(res.r - ref.r)) <= 2e-7
    assert np.max(np.abs(res.KtoY - ref.KtoY) / ref.KtoY) <= 2e-6


def test_resident_default_sweep_and_stats(gpu):
    """solve_table2(method="brent") takes the resident path by default; its launch is
    counted by aiy_ge_launch_stats (the bench's roofline source)."""
    import ctypes

    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    h = _lib.handle(gpu.index)
    h.check(h.lib.aiy_ge_launch_stats(h.h, None, None, None, None, 1), "reset")
    res = solve_table2(table2_calibrations(), n_a=2000, device=gpu, method="brent")
    ms, n, pts, cyc = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
    h.check(h.lib.aiy_ge_launch_stats(h.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(pts), ctypes.byref(cyc), 1),
            "stats")
    print(f"\nresident sweep at N_a = 2000: {ms.value:.2f} ms in {n.value} launch(es), {pts.value:.3e} point-matvecs, "
          f"{cyc.value:.0f} EGM cycles; r = {np.round(100 * res.r, 5)}")
    assert 1 <= n.value <= 6 and ms.value > 0 and pts.value > 0 and cyc.value > 0   # rebalancing relaunches
    assert np.all(res.status == 0)
    ref = solve_table2(table2_calibrations(), n_a=2000, device=gpu, method="brent", resident=False)
    assert np.max(np.abs(res.r - ref.r)) <= 2e-7


def test_rebalancing_relaunches_match_one_launch(gpu):
    """AIY_OPT_GE_REBALANCE: clusters stop at evaluation boundaries once half the launch's
    calibrations have finished and the rest continue from their saved search state on larger
    clusters; the roots agree with the single launch to the search tolerance."""
    import ctypes

    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    h = _lib.handle(gpu.index)
    cals = table2_calibrations()
    kw = dict(n_a=3000, device=gpu, method="brent", resident=True)
    prior = h.get_option(_lib.AIY_OPT_GE_REBALANCE)
    try:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_REBALANCE, 0), "opt")
        one = solve_table2(cals, **kw)
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_REBALANCE, 50), "opt")
        reb = solve_table2(cals, **kw)
        launches, mid = ctypes.c_int32(), ctypes.c_int32()
        h.check(h.lib.aiy_ge_last_rounds(h.h, ctypes.byref(launches), ctypes.byref(mid)), "rounds")
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_REBALANCE, prior), "opt")
    print(f"\nsteps one {one.bisection_steps} rebalanced {reb.bisection_steps}; max |dr| {np.max(np.abs(reb.r - one.r)):.2e}; "
          f"{launches.value} launches, {mid.value} stops inside a distribution solve")
    # relaunches happened, and some clusters stopped inside a BiCGSTAB solve (resumed from x)
    assert launches.value >= 2 and mid.value >= 1
    assert np.all(reb.status == 0) and np.all(one.status == 0)
    assert np.max(np.abs(reb.r - one.r)) <= 2e-7
    assert np.max(np.abs(reb.KtoY - one.KtoY) / one.KtoY) <= 2e-6


def test_logsec_levels_same_roots(gpu):
    """AIY_OPT_GE_LOGSEC 0 / 1 / 2 (bisection bracketing and Brent in r; the two-point
    log-secant bracketing and Brent in log coordinates; also the one-point step): the same
    roots to the search tolerance on both the resident search and the host-driven loop, and
    the log-coordinate levels take fewer evaluations than bisection bracketing on the resident
    search (whose bisection_steps count each calibration's own evaluations)."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    h = _lib.handle(gpu.index)
    cals = table2_calibrations()
    with pytest.raises(RuntimeError):
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, 3), "opt")
    out = {}
    try:
        for lvl in (0, 1, 2):
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, lvl), "opt")
            for resident in (True, False):
                out[lvl, resident] = solve_table2(cals, n_a=2000, device=gpu, method="brent", resident=resident)
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, 2), "opt")
    base = out[0, False]
    for (lvl, resident), res in out.items():
        print(f"\nlogsec {lvl} resident {resident}: evaluations {int(np.sum(res.bisection_steps))}, "
              f"max |dr| {np.max(np.abs(res.r - base.r)):.2e}")
        assert np.all(res.status == 0)
        assert np.max(np.abs(res.r - base.r)) <= 2e-7
    assert np.sum(out[2, True].bisection_steps) < np.sum(out[0, True].bisection_steps)


@pytest.mark.parametrize("n_a", [3000, 10000])   # one and two columns per thread at 24 cells
def test_pull_matvec_sweep_deterministic(gpu, n_a):
    """AIY_OPT_HIST_PULL: the distribution solves of the resident search pull each
    destination's lottery sources in ascending order (no LDS atomics).  The same roots as
    the push form within the search tolerance, and -- in one launch (no rebalancing, whose
    stop points follow the wall clock and change the cluster sizes, i.e. the summation order of
    the cluster reductions) -- two sweeps bit-identical."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    h = _lib.handle(gpu.index)
    cals = table2_calibrations()
    kw = dict(n_a=n_a, device=gpu, method="brent", resident=True)
    prev = h.set_options({_lib.AIY_OPT_HIST_PULL: 0, _lib.AIY_OPT_GE_REBALANCE: 0})
    try:
        push = solve_table2(cals, **kw)
        h.set_options({_lib.AIY_OPT_HIST_PULL: 1})
        a = solve_table2(cals, **kw)
        b = solve_table2(cals, **kw)
    finally:
        h.set_options(prev)
    print(f"\npull vs push max |dr| {np.max(np.abs(a.r - push.r)):.2e}; pull runs equal: {np.array_equal(a.r, b.r)}")
    assert np.all(a.status == 0) and np.all(b.status == 0)
    assert np.array_equal(a.r, b.r) and np.array_equal(a.K_supply, b.K_supply)
    assert np.max(np.abs(a.r - push.r)) <= 2e-7


def test_final_ks_is_solved_at_hist_tol(gpu):
    """bracketing evaluations run loose (egm 1e-6, hist 1e-8) and Brent's at an
    adaptive distribution tolerance (up to the loose one), so a search that ENDS on such an
    evaluation evaluates that r once more at egm_tol / hist_tol before K_s is reported.  A
    coarse r_tol ends the searches while |K_s - K_d| is still large (during bracketing, or with
    the adaptive tolerance above hist_tol); Ks_out must then equal K_s at the last evaluated r
    solved cold at the full tolerances (the BiCGSTAB stopping rule leaves K ~4e5 tol relative
    off, DESIGN.md §4c: ~4e-7 at 1e-12, ~4e-3 at the loose 1e-8)."""
    import ctypes

    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import StationaryBatch, ge_stationary_native
    cals = _cells(4)
    aG = sm.make_grid_exp_mult(0.001, 50.0, 2000, 2)
    b = StationaryBatch(cals, aG, device=gpu)
    r, K, Ks, steps, cyc, its, status = ge_stationary_native(
        b, "brent", 3e-4, 1e-8, 1e-12, 60, True, True, -1, secant=True, loose=True, extrapolate=True, resident=True)
    assert np.all(status == 0)
    h = _lib.handle(gpu.index)
    ev = (ctypes.c_double * (len(cals) * 32 * 6))()
    assert h.lib.aiy_ge_last_eval_log(h.h, ev, len(cals)) == len(cals)
    ev = np.array(ev[:]).reshape(len(cals), 32, 6)
    r_last, adaptive = [], []
    for c in range(len(cals)):
        rows = ev[c][ev[c][:, 0] != 0.0]
        r_last.append(rows[-1, 0])
        fmin = np.min(np.abs(rows[:-1, 1])) if len(rows) > 1 else np.inf
        # a loose bracketing evaluation, or Brent's with ge_adapt_htol above hist_tol
        adaptive.append(rows[-1, 4] == 1.0 or 1e-9 * fmin > 1e-12)
    Kc, _, _ = StationaryBatch(cals, aG, device=gpu).capital_supply(np.array(r_last), egm_tol=1e-10, hist_tol=1e-12,
                                                                    accel=-1)
    rel = np.abs(Ks - Kc) / Kc
    print(f"\nsteps {steps}; last r {np.round(100 * np.array(r_last), 5)}; loose / adaptive final evaluation {adaptive}; "
          f"|Ks_out - K_s(hist_tol)| / K_s = {rel}")
    assert any(adaptive), "no search ended on a loose evaluation: the test does not exercise the final pass"
    # two solves at hist_tol = 1e-12 from different starts (the final pass warm, this one cold) stop
    # at different points of the same rule: near 1/beta - 1 (cell 0, r = 4.14 %) the stopping rule
    # leaves K a few 1e-6 relative off, against ~4e-3 for the loose evaluation
    assert np.max(rel) <= 2e-5
