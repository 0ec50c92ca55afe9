"""GPU tests of the device-resident Young-histogram iteration (csrc/hist_resident.hip,
build-defined row E2): one launch per aiy_hist_solve, a cluster of workgroups per
calibration, against the push/mix launch pair (AIY_OPT_HIST_RESIDENT = 0) and the CPU
oracle (oracle/stationary.py stationary_hist: mass' = P^T lottery_push(mass), stop at the
first iteration with max |mass' - mass| < tol).

Both device paths sum the lottery contributions with atomics (LDS or global), so their
masses agree to rounding (1e-13 absolute on masses of order 1e-5), the iteration counts
to +-1 (a sup-norm change within rounding of the tolerance), and K_s(r) to 1e-12."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(gpu, cals, aGrid, r, resident, cluster=0, accel=0):
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import StationaryBatch
    h = _lib.handle(gpu.index)
    h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_RESIDENT, int(resident)), "opt")
    h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, int(cluster)), "opt")
    try:
        b = StationaryBatch(cals, aGrid, device=gpu)
        K, cycles, iters = b.capital_supply(r, egm_tol=1e-8, hist_tol=1e-12, accel=accel)
        return K, iters, b.mass.cpu().numpy(), b
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_RESIDENT, 1), "opt")
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, 0), "opt")


def _launches(gpu, reset=True):
    import ctypes
    from aiyagari_hark_amd import _lib
    h = _lib.handle(gpu.index)
    ms, n = ctypes.c_double(), ctypes.c_int64()
    h.check(h.lib.aiy_hist_launch_stats(h.h, ctypes.byref(ms), ctypes.byref(n), int(reset)), "stats")
    return n.value


@pytest.mark.parametrize("shape", ["table2", "mixed", "rouwenhorst", "small_cluster", "tiny"])
def test_resident_histogram_equals_push_mix(gpu, shape):
    from aiyagari_hark_amd.stationary import Calibration, table2_calibrations
    from oracle import stationary as ST
    cluster = 0
    if shape == "table2":        # configs[2]: 24 calibrations x 7 states x 10 000 nodes, ONE launch
        cals, n_a = table2_calibrations(), 10000
    elif shape == "mixed":
        cals, n_a = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0), Calibration(LaborAR=0.0, LaborSD=0.2)], 3001
    elif shape == "rouwenhorst":  # S = 25 (stress shape, smaller grid)
        cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0, LaborStatesNo=25, income="rouwenhorst")]
        n_a = 2000
    elif shape == "small_cluster":   # 3 calibrations per GPU (Table II split over 8 GPUs), cluster of 4
        cals, n_a, cluster = table2_calibrations()[:3], 10000, 4
    else:
        cals, n_a = [Calibration(LaborAR=0.3, LaborSD=0.2, CRRA=3.0)], 40
    aGrid = ST.make_stationary_grid(0.001, 50.0, n_a, 2)
    r = np.linspace(0.02, 0.04, len(cals))
    _launches(gpu)
    K1, it1, m1, _ = _solve(gpu, cals, aGrid, r, True, cluster)
    assert _launches(gpu) >= 1, "the resident path did not run"
    K0, it0, m0, _ = _solve(gpu, cals, aGrid, r, False)
    assert np.max(np.abs(it1 - it0)) <= 1, (it1, it0)
    assert np.max(np.abs(m1 - m0)) < 1e-13
    assert np.max(np.abs(K1 - K0) / K0) < 1e-12
    assert np.all(np.abs(m1.reshape(len(cals), -1).sum(axis=1) - 1.0) < 1e-10)   # drift over ~1e4 iterations


def test_resident_histogram_matches_oracle(gpu):
    """Against the CPU oracle's lottery + distribution iteration on the same policy."""
    from aiyagari_hark_amd.stationary import Calibration
    from oracle import stationary as ST
    cal = Calibration(LaborAR=0.6, LaborSD=0.4, CRRA=3.0)
    aGrid = ST.make_stationary_grid(0.001, 50.0, 1500, 2)
    r = np.array([0.03])
    K, it, m, b = _solve(gpu, [cal], aGrid, r, True)
    lab, P = ST.income_process(7, cal.LaborAR, cal.LaborSD, "tauchen")
    w, _ = ST.prices(0.03, 0.36, 0.08)
    mt, ct = (x[0].cpu().numpy() for x in b.last_tables)
    lo, wlo, _ = ST.savings_lottery(mt[:, 0], ct[:, 0], aGrid, 1.03, w, lab)
    mass, iters, _ = ST.stationary_hist(lo, wlo, P, aGrid.size, tol=1e-12)
    assert abs(int(it[0]) - iters) <= 1
    assert np.max(np.abs(m[0] - mass)) < 1e-13
    Kw = float(np.sum(mass * aGrid[None, :]))
    assert abs(K[0] - Kw) / Kw < 1e-12


def test_resident_histogram_falls_back_when_spans_do_not_fit(gpu):
    """A cluster so large that the borrowing-constrained columns are covered by more than
    kHcCand workgroups' spans: the resident launch refuses the shape before iterating and
    the push/mix pair produces the answer (same as forcing push/mix)."""
    from aiyagari_hark_amd.stationary import Calibration
    from oracle import stationary as ST
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=1.0)]
    aGrid = ST.make_stationary_grid(0.001, 50.0, 2000, 2)
    r = np.array([0.035])
    K1, it1, m1, _ = _solve(gpu, cals, aGrid, r, True, cluster=128)
    K0, it0, m0, _ = _solve(gpu, cals, aGrid, r, False)
    assert np.max(np.abs(m1 - m0)) < 1e-13
    assert abs(K1[0] - K0[0]) / K0[0] < 1e-12


# ---------------------------------------------------------------------------------------
# BiCGSTAB mode (csrc/hist_krylov.hip, accel < 0): a different iteration to the same
# fixed point.  It stops at a mass T x whose x has max|T x - x| < tol (the plain rule),
# typically ~10x closer to the exact stationary distribution than the plain iterate (the
# plain iteration's own error is ~tol / (1 - lambda_2)), so it is compared with an
# over-converged oracle solution (K) and with the plain device iterate within the plain
# iterate's error.
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("shape", ["table2", "rouwenhorst", "tiny", "small_cluster"])
def test_bicgstab_histogram_matches_plain(gpu, shape):
    from aiyagari_hark_amd.stationary import Calibration, table2_calibrations
    from oracle import stationary as ST
    cluster = 0
    if shape == "table2":
        cals, n_a = table2_calibrations(), 10000
    elif shape == "rouwenhorst":
        cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
                for c in (1.0, 5.0)]
        n_a = 2000
    elif shape == "small_cluster":
        cals, n_a, cluster = table2_calibrations()[:3], 10000, 4
    else:
        cals, n_a = [Calibration(LaborAR=0.3, LaborSD=0.2, CRRA=3.0)], 40
    aGrid = ST.make_stationary_grid(0.001, 50.0, n_a, 2)
    r = np.linspace(0.02, 0.04, len(cals))
    _launches(gpu)
    Kb, itb, mb, _ = _solve(gpu, cals, aGrid, r, True, cluster, accel=-1)
    assert _launches(gpu) >= 1, "the resident BiCGSTAB path did not run"
    Kp, itp, mp, _ = _solve(gpu, cals, aGrid, r, True, cluster, accel=0)
    assert np.all(np.abs(mb.reshape(len(cals), -1).sum(axis=1) - 1.0) < 1e-10)
    assert np.max(np.abs(Kb - Kp) / Kp) < 1e-5, np.abs(Kb - Kp) / Kp
    assert np.max(np.abs(mb - mp)) < 1e-8
    if shape == "table2":
        assert itb.max() * 4 < itp.max(), (itb.max(), itp.max())


def test_bicgstab_histogram_matches_oracle(gpu):
    """The returned mass against the CPU oracle's transition on the same policy: its
    residual max|T m - m| is at the plain rule's level and K agrees with the over-converged
    oracle distribution to 1e-6 relative (the plain iterate's own K error at this tol is
    ~3e-6 on the slowest Table II cell, scratch study in DESIGN.md §4b)."""
    from aiyagari_hark_amd.stationary import Calibration
    from oracle import stationary as ST
    cal = Calibration(LaborAR=0.0, LaborSD=0.2, CRRA=1.0)    # the slowest Table II cell
    aGrid = ST.make_stationary_grid(0.001, 50.0, 1500, 2)
    r = np.array([0.0405])
    K, it, m, b = _solve(gpu, [cal], aGrid, r, True, accel=-1)
    lab, P = ST.income_process(7, cal.LaborAR, cal.LaborSD, "tauchen")
    w, _ = ST.prices(r[0], 0.36, 0.08)
    mt, ct = (x[0].cpu().numpy() for x in b.last_tables)
    lo, wlo, _ = ST.savings_lottery(mt[:, 0], ct[:, 0], aGrid, 1.0 + r[0], w, lab)
    res = np.max(np.abs(ST.hist_step_fast(m[0], lo, wlo, P) - m[0]))
    assert res < 1e-11, res
    exact, iters, _ = ST.stationary_hist(lo, wlo, P, aGrid.size, tol=1e-16, max_iter=400000,
                                         mass0=m[0], step=ST.hist_step_fast)
    Ke = float(np.sum(exact * aGrid[None, :]))
    assert abs(K[0] - Ke) / Ke < 1e-6, (K[0], Ke)
    plain, iters_p, _ = ST.stationary_hist(lo, wlo, P, aGrid.size, tol=1e-12, step=ST.hist_step_fast)
    assert int(it[0]) * 3 < iters_p, (int(it[0]), iters_p)


def test_pull_bicgstab_stress_size(gpu):
    """The pull form (csrc/hist_pull.h) that solves S > 8 calibrations: the three configs[4]
    cells (25-state Rouwenhorst, N_a = 50 000) in ONE launch near their roots.  Against the
    oracle's transition on the same policies: residual max|T m - m| at the plain rule's
    level, total mass 1; a second solve from the same start is bit-identical (no atomics)."""
    from aiyagari_hark_amd.stationary import Calibration
    from oracle import stationary as ST
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
            for c in (1.0, 3.0, 5.0)]
    aGrid = ST.make_stationary_grid(0.001, 50.0, 50000, 2)
    r = np.array([0.038, 0.028, 0.017])
    _launches(gpu)
    K, it, m, b = _solve(gpu, cals, aGrid, r, True, accel=-1)
    n = _launches(gpu)
    assert n == 1, f"{n} launches: the three clusters should be co-resident"
    K2, it2, m2, _ = _solve(gpu, cals, aGrid, r, True, accel=-1)
    assert np.array_equal(it, it2) and np.array_equal(m, m2), "pull-form solve not reproducible"
    for c, cal in enumerate(cals):
        lab, P = ST.income_process(25, cal.LaborAR, cal.LaborSD, "rouwenhorst")
        w, _ = ST.prices(r[c], 0.36, 0.08)
        mt, ct = (x[c].cpu().numpy() for x in b.last_tables)
        lo, wlo, _ = ST.savings_lottery(mt[:, 0], ct[:, 0], aGrid, 1.0 + r[c], w, lab)
        res = np.max(np.abs(ST.hist_step_fast(m[c], lo, wlo, P) - m[c]))
        print(f"\ncell {c}: {int(it[c])} matvecs, residual {res:.2e}, K {K[c]:.6f}")
        assert res < 1e-11, res
        assert abs(m[c].sum() - 1.0) < 1e-10


@pytest.mark.parametrize("n_states", [33, 49, 64])
def test_pull_bicgstab_many_states(gpu, n_states):
    """S > 32 (up to AIY_MAX_STATES = 64): the pull form's SMAX = 64 instantiation, its chunked
    LDS row sums at a small grid.  Against the oracle's transition on the same policy (residual
    at the plain rule's level, total mass 1) and the plain push/mix iteration's K (within the
    plain iterate's own error)."""
    from aiyagari_hark_amd.stationary import Calibration
    from oracle import stationary as ST
    cal = Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=3.0, LaborStatesNo=n_states, income="rouwenhorst")
    aGrid = ST.make_stationary_grid(0.001, 50.0, 1500, 2)
    r = np.array([0.025])
    _launches(gpu)
    K, it, m, b = _solve(gpu, [cal], aGrid, r, True, accel=-1)
    assert _launches(gpu) == 1, "the resident pull-form solve did not run"
    lab, P = ST.income_process(n_states, cal.LaborAR, cal.LaborSD, "rouwenhorst")
    w, _ = ST.prices(r[0], 0.36, 0.08)
    mt, ct = (x[0].cpu().numpy() for x in b.last_tables)
    lo, wlo, _ = ST.savings_lottery(mt[:, 0], ct[:, 0], aGrid, 1.0 + r[0], w, lab)
    res = np.max(np.abs(ST.hist_step_fast(m[0], lo, wlo, P) - m[0]))
    assert res < 1e-11, res
    assert abs(m[0].sum() - 1.0) < 1e-10
    Kp, itp, mp, _ = _solve(gpu, [cal], aGrid, r, False)   # plain push/mix launches
    assert abs(K[0] - Kp[0]) / Kp[0] < 1e-5, (K[0], Kp[0])
    assert int(it[0]) * 3 < int(itp[0]), (int(it[0]), int(itp[0]))


@pytest.mark.parametrize("cluster", [0, 24])
def test_pull_matvec_histogram_matches_push(gpu, cluster):
    """AIY_OPT_HIST_PULL on the standalone BiCGSTAB solve of the 24 Table II cells (two
    columns per thread at the default cluster, one at 24 workgroups): the same
    distribution as the push form to the solve tolerance, and a repeat bit-identical."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import table2_calibrations
    from oracle import stationary as ST
    h = _lib.handle(gpu.index)
    cals = table2_calibrations()
    aGrid = ST.make_stationary_grid(0.001, 50.0, 10000, 2)
    r = np.linspace(0.02, 0.04, len(cals))
    prev = h.set_options({_lib.AIY_OPT_HIST_PULL: 0})
    try:
        Kp, itp, mp, _ = _solve(gpu, cals, aGrid, r, True, cluster, accel=-1)
        h.set_options({_lib.AIY_OPT_HIST_PULL: 1})
        K1, it1, m1, _ = _solve(gpu, cals, aGrid, r, True, cluster, accel=-1)
        K2, it2, m2, _ = _solve(gpu, cals, aGrid, r, True, cluster, accel=-1)
    finally:
        h.set_options(prev)
    assert np.array_equal(m1, m2) and np.array_equal(it1, it2)
    assert np.max(np.abs(m1 - mp)) < 1e-8
    assert np.max(np.abs(K1 - Kp) / Kp) < 1e-5
