"""Stationary Aiyagari extensions (build-defined, no reference code).

``solve_table2`` solves many calibrations to general equilibrium at once:

  GE search on r (E1) -- per calibration, all searches advanced together (bisection,
                          or bisection to a sign change then Brent's method)
    w(r) = (1 - alpha) (alpha / (r + delta))^(alpha / (1 - alpha)),  R = 1 + r
    stationary EGM  -- aiy_egm_solve with one aggregate node (n_M = 1): the reference's
                       solve_Aiyagari arithmetic (Aiyagari_Support.py:1478-1504) with
                       constant prices, batched over calibrations
    Young lottery   -- aiy_hist_lottery + aiy_hist_solve (E2): stationary distribution
                       on the asset grid, K_s(r) = sum mass * a
    K_d(r) = (alpha / (r + delta))^(1 / (1 - alpha)); move the bracket toward K_s = K_d.

Income processes: the reference's Tauchen (Aiyagari_Support.py:885-887, 7 states) or
Rouwenhorst (E3, e.g. 25 states for the stress configuration), levels normalised by
their simple mean (quirk Q3).  Everything per grid point runs in libaiyagari; the
host only moves the brackets.
"""
from __future__ import annotations

import atexit
import ctypes
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import setup_math as sm
from .egm import EgmBatch, egm_solve

F64 = torch.float64

# Aiyagari (1994) Table II grid: rho x sigma x mu
TABLE2_RHO = (0.0, 0.3, 0.6, 0.9)
TABLE2_SIGMA = (0.2, 0.4)
TABLE2_CRRA = (1.0, 3.0, 5.0)


@dataclass
class Calibration:
    LaborAR: float = 0.6
    LaborSD: float = 0.2
    CRRA: float = 1.0
    DiscFac: float = 0.96
    CapShare: float = 0.36
    DeprFac: float = 0.08
    LaborStatesNo: int = 7
    income: str = "tauchen"       # or "rouwenhorst"

    def income_process(self):
        if self.income == "tauchen":
            y, P = sm.labor_tauchen(self.LaborStatesNo, self.LaborAR, self.LaborSD)
        elif self.income == "rouwenhorst":
            y, P = sm.rouwenhorst(self.LaborStatesNo, self.LaborAR, self.LaborSD)
        else:
            raise ValueError(self.income)
        return sm.labor_levels(y), P


def table2_calibrations(**kw):
    """The 24 calibrations of Aiyagari (1994) Table II (rho, sigma, CRRA)."""
    return [Calibration(LaborAR=r, LaborSD=s, CRRA=c, **kw)
            for s in TABLE2_SIGMA for r in TABLE2_RHO for c in TABLE2_CRRA]


def _resolve_device(device):
    """torch.device with an explicit index: None / "cuda" mean the current device (library
    handles are per device index, _lib.Handle(dev.index))."""
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError(f"stationary solves run on a GPU, not {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def firm_prices(r, alpha, delta):
    """(w, K_demand) with L = 1 (Cobb-Douglas firm of calc_R_and_W, AS:1886-1890).

    Element by element through libm's pow (math.pow), the function the native loops call
    (csrc/ge.hip: std::pow): numpy's vectorised power is not correctly rounded on every CPU
    (its AVX-512 form differs from libm in the last bit for ~10 % of rates), and a one-ulp
    difference in w or K_d makes the Python and native GE loops take different steps."""
    r, alpha, delta = np.broadcast_arrays(np.asarray(r, dtype=np.float64), np.asarray(alpha, dtype=np.float64),
                                          np.asarray(delta, dtype=np.float64))
    KtoL = np.empty(r.shape)
    w = np.empty(r.shape)
    for i in np.ndindex(r.shape):
        a = float(alpha[i])
        k = math.pow(a / (float(r[i]) + float(delta[i])), 1.0 / (1.0 - a))
        KtoL[i] = k
        w[i] = (1.0 - a) * math.pow(k, a)
    if KtoL.ndim == 0:
        return float(w), float(KtoL)
    return w, KtoL


@dataclass
class StationaryResult:
    r: np.ndarray
    K: np.ndarray
    K_supply: np.ndarray
    KtoY: np.ndarray
    saving_rate: np.ndarray
    bisection_steps: int
    egm_cycles: list = field(default_factory=list)
    hist_iters: list = field(default_factory=list)
    # per calibration (native engine): bit 1 a household solve stopped at its cycle cap,
    # bit 2 a distribution solve at its iteration cap, bit 4 the search at max_steps
    status: np.ndarray | None = None


class StationaryBatch:
    """Device buffers for one batch of stationary calibrations on a common grid size."""

    def __init__(self, cals, aGrid, device=None):
        self.cals = list(cals)
        self.device = _resolve_device(device)
        n_cal = len(self.cals)
        levels, Ps = zip(*(c.income_process() for c in self.cals))
        S = len(levels[0])
        if any(len(l) != S for l in levels):
            raise ValueError("all calibrations of a batch need the same number of income states")
        self.S = S
        self.n_a = int(np.asarray(aGrid).shape[-1])
        self.aGrid = np.broadcast_to(np.asarray(aGrid, dtype=np.float64), (n_cal, self.n_a)).copy()
        self.levels = np.stack(levels)
        self.P = np.stack(Ps)
        dev = self.device
        self.d_a = torch.as_tensor(self.aGrid).to(dev)
        self.d_P = torch.as_tensor(self.P).to(dev)
        self.d_lab = torch.as_tensor(self.levels).to(dev)
        self.d_beta = torch.as_tensor([c.DiscFac for c in self.cals], dtype=F64).to(dev)
        self.d_crra = torch.as_tensor([c.CRRA for c in self.cals], dtype=F64).to(dev)
        self.alpha = np.array([c.CapShare for c in self.cals])
        self.delta = np.array([c.DeprFac for c in self.cals])
        shp = (n_cal, S, self.n_a)
        self.lo = torch.empty(shp, dtype=torch.int32, device=dev)
        self.wlo = torch.empty(shp, dtype=F64, device=dev)
        self.mass = torch.empty(shp, dtype=F64, device=dev)
        self.work = torch.empty((2,) + shp, dtype=F64, device=dev)

    def capital_supply(self, r, egm_tol=1e-8, hist_tol=1e-12, max_hist=200000, warm=False, warm_egm=False,
                       accel=0):
        """K_s(r) for every calibration (r: array [n_cal]).  warm=True starts the
        distribution iteration from the previous call's stationary mass instead of the
        uniform one (same fixed point, to hist_tol; used between bisection steps, where r
        moves by half the bracket each step).  warm_egm=True starts the household solve
        from the previous call's converged policy (aiy_egm_solve_from): the fixed point
        moves by ~egm_tol / (1 - beta R), far inside the 1e-5 tolerance on r.  accel=E > 0
        lets the device-resident distribution iteration extrapolate along its slowest mode
        every E iterations (Aitken, AIY_OPT_HIST_ACCEL): the same fixed point to the
        iteration's own accuracy (~1e-7 relative in K), 1.5-3x fewer
        iterations; accel < 0 solves (I - T) mass = 0 by BiCGSTAB (AIY_OPT_HIST_KRYLOV,
        hist_krylov.hip): a mass T x with max|T x - x| < hist_tol, the plain iteration's
        stopping rule, in 10-20x fewer matvecs (counts are matvecs); 0 is the oracle's
        plain iteration."""
        n_cal, S = len(self.cals), self.S
        r = np.asarray(r, dtype=np.float64)
        w, _ = firm_prices(r, self.alpha, self.delta)
        R = 1.0 + r
        dev = self.device
        Rn = torch.as_tensor(np.repeat(R[:, None, None], S, axis=2)).to(dev)
        Wn = torch.as_tensor(np.repeat(w[:, None, None], S, axis=2)).to(dev)
        batch = EgmBatch(self.d_a, torch.zeros((n_cal, 1), dtype=F64, device=dev), self.d_P, Rn, Wn,
                         torch.zeros_like(Rn), self.d_lab, self.d_beta, self.d_crra)
        init = self.last_tables if (warm_egm and getattr(self, "last_tables", None) is not None) else None
        m, c, cycles, _ = egm_solve(batch, tol=egm_tol, init=init)
        h = _lib.handle(dev.index)
        dR = torch.as_tensor(R).to(dev)
        dw = torch.as_tensor(w).to(dev)
        sp = _lib.stream_ptr()
        h.check(h.lib.aiy_hist_lottery(h.h, n_cal, S, self.n_a, _lib.ptr(m), _lib.ptr(c), _lib.ptr(self.d_a),
                                       _lib.ptr(dR), _lib.ptr(dw), _lib.ptr(self.d_lab), _lib.ptr(self.lo),
                                       _lib.ptr(self.wlo), sp), "aiy_hist_lottery")
        if not (warm and getattr(self, "_mass_valid", False)):
            self.mass.fill_(1.0 / (S * self.n_a))
        K = (ctypes.c_double * n_cal)()
        iters = (ctypes.c_int32 * n_cal)()
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_ACCEL, max(int(accel), 0)), "aiy_set_option")
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_KRYLOV, int(accel < 0)), "aiy_set_option")
        try:
            h.check(h.lib.aiy_hist_solve(h.h, n_cal, S, self.n_a, _lib.ptr(self.lo), _lib.ptr(self.wlo),
                                         _lib.ptr(self.d_P), _lib.ptr(self.d_a), float(hist_tol), int(max_hist), 64,
                                         _lib.ptr(self.mass), _lib.ptr(self.work), K, iters, sp), "aiy_hist_solve")
        finally:
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_ACCEL, 0), "aiy_set_option")
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_KRYLOV, 0), "aiy_set_option")
        self.last_tables = (m, c)
        self._mass_valid = True
        return np.array(K[:]), np.array(cycles), np.array(iters[:])


class _Brent:
    """One calibration's root search on f(r) = K_s(r) - K_d(r) as a coroutine:
    ``propose()`` gives the next r to evaluate, ``update(f)`` takes f there.

    Until both signs of f have been evaluated it bisects the theoretical bracket
    [-delta / 2, 1 / beta - 1) (f < 0 below, f > 0 near 1 / beta - 1, where the household
    solve and the distribution converge slowly, so that endpoint is never evaluated).  It
    then runs Brent's method on the evaluated bracket (the scipy.optimize.brentq
    algorithm: secant / inverse quadratic steps, bisection safeguard), stopping within
    xtol of the root."""

    def __init__(self, lo, hi, xtol):
        self.lo, self.hi, self.flo, self.fhi, self.xtol = lo, hi, None, None, xtol
        self.brent = False
        self.done = False
        self.x = 0.5 * (lo + hi)

    def propose(self):
        return self.x

    def update(self, f):
        if self.done:
            return
        if not self.brent:
            if f > 0:
                self.hi, self.fhi = self.x, f
            else:
                self.lo, self.flo = self.x, f
            if self.hi - self.lo <= self.xtol:
                self.done, self.x = True, 0.5 * (self.lo + self.hi)
                return
            if self.flo is None or self.fhi is None:
                self.x = 0.5 * (self.lo + self.hi)
                return
            self.brent = True
            self.xpre, self.fpre, self.xcur, self.fcur = self.lo, self.flo, self.hi, self.fhi
            self.xblk = self.fblk = self.spre = self.scur = 0.0
            self._step()
            return
        self.xpre, self.fpre = self.xprev_eval, self.fprev_eval
        self.fcur = f
        self._step()

    def _step(self):
        xpre, fpre, xcur, fcur = self.xpre, self.fpre, self.xcur, self.fcur
        xblk, fblk, spre, scur = self.xblk, self.fblk, self.spre, self.scur
        if fpre * fcur < 0:
            xblk, fblk = xpre, fpre
            spre = scur = xcur - xpre
        if abs(fblk) < abs(fcur):
            xpre, xcur, xblk = xcur, xblk, xcur
            fpre, fcur, fblk = fcur, fblk, fcur
        delta = 0.5 * (self.xtol + 4 * np.finfo(float).eps * abs(xcur))
        sbis = 0.5 * (xblk - xcur)
        if fcur == 0 or abs(sbis) < delta:
            self.done, self.x = True, xcur
            return
        if abs(spre) > delta and abs(fcur) < abs(fpre):
            if xpre == xblk:
                stry = -fcur * (xcur - xpre) / (fcur - fpre)
            else:
                dpre = (fpre - fcur) / (xpre - xcur)
                dblk = (fblk - fcur) / (xblk - xcur)
                stry = -fcur * (fblk * dblk - fpre * dpre) / (dblk * dpre * (fblk - fpre))
            if 2 * abs(stry) < min(abs(spre), 3 * abs(sbis) - delta):
                spre, scur = scur, stry
            else:
                spre = scur = sbis
        else:
            spre = scur = sbis
        self.xprev_eval, self.fprev_eval = xcur, fcur
        xcur = xcur + (scur if abs(scur) > delta else (delta if sbis > 0 else -delta))
        self.xpre, self.fpre, self.xcur, self.fcur = xpre, fpre, xcur, fcur
        self.xblk, self.fblk, self.spre, self.scur = xblk, fblk, spre, scur
        self.x = xcur


def resident_plan(device, n_cal, S, n_a, cu_share=1.0):
    """(G, columns per workgroup, columns per thread, blocks) of the device-resident GE
    search (aiy_ge_resident_plan, csrc/ge_resident.hip) for this shape, or None when
    aiy_ge_stationary would run the host-driven loop instead."""
    dev = _resolve_device(device)
    h = _lib.handle(dev.index)
    prev = h.set_options({_lib.AIY_OPT_GE_RESIDENT: 1, _lib.AIY_OPT_CU_LIMIT: _cu_limit(dev, cu_share)})
    out = (ctypes.c_int32 * 4)()
    try:
        ok = h.lib.aiy_ge_resident_plan(h.h, int(n_cal), int(S), int(n_a), out)
    finally:
        h.set_options(prev)
    return tuple(out) if ok == 1 else None


def _cu_limit(dev, cu_share):
    return 0 if float(cu_share) >= 1.0 else _device_cus(dev, cu_share)


def ge_stationary_native(b, method, r_tol, egm_tol, hist_tol, max_steps, warm_hist, warm_egm, accel, r_lo=None,
                         r_hi=None, secant=False, loose=False, extrapolate=False, handle=None, stream=None,
                         resident=False, cu_share=1.0):
    """The whole E1 search in ONE library call (aiy_ge_stationary: the bracket updates run
    in C++ between device K_s evaluations, or -- resident=True, where the shape allows --
    the whole search of every calibration in one device-resident launch).  Returns (r, K,
    Ks, steps, egm_cycles_sum, hist_iters_sum, status).  handle / stream: a library handle
    and torch stream of the caller's (default: the device's shared handle, the current
    stream)."""
    n = len(b.cals)
    h = handle if handle is not None else _lib.handle(b.device.index)
    work = torch.empty(int(h.lib.aiy_ge_stationary_work_bytes(n, b.S, b.n_a)), dtype=torch.uint8, device=b.device)
    host = lambda x: (ctypes.c_double * n)(*[float(v) for v in x])  # noqa: E731
    alpha, delta = host(b.alpha), host(b.delta)
    disc = host([c.DiscFac for c in b.cals])
    model = _lib.StationaryModel(n, b.S, b.n_a, _lib.ptr(b.d_a), _lib.ptr(b.d_P), _lib.ptr(b.d_lab),
                                 _lib.ptr(b.d_beta), _lib.ptr(b.d_crra), ctypes.addressof(alpha),
                                 ctypes.addressof(delta), ctypes.addressof(disc))
    lo = host(np.broadcast_to(np.asarray(r_lo, float), (n,))) if r_lo is not None else None
    hi = host(np.broadcast_to(np.asarray(r_hi, float), (n,))) if r_hi is not None else None
    opt = _lib.GeOptions({"bisect": 0, "brent": 1}[method], float(r_tol), float(egm_tol), float(hist_tol),
                         int(max_steps), 5000, 200000, int(bool(warm_hist)), int(bool(warm_egm)), int(accel),
                         ctypes.addressof(lo) if lo is not None else None,
                         ctypes.addressof(hi) if hi is not None else None, int(bool(secant)), int(bool(loose)),
                         int(bool(extrapolate)), None)
    status = (ctypes.c_int32 * n)()
    opt.status_out = ctypes.addressof(status)
    r, K, Ks = (ctypes.c_double * n)(), (ctypes.c_double * n)(), (ctypes.c_double * n)()
    steps, cyc, its = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    prev = h.set_options({_lib.AIY_OPT_GE_RESIDENT: int(bool(resident)),
                          _lib.AIY_OPT_CU_LIMIT: _cu_limit(b.device, cu_share)})
    try:
        h.check(h.lib.aiy_ge_stationary(h.h, ctypes.byref(model), ctypes.byref(opt), _lib.ptr(work), r, K, Ks,
                                        ctypes.byref(steps), ctypes.byref(cyc), ctypes.byref(its),
                                        _lib.stream_ptr(stream)),
                "aiy_ge_stationary")
    finally:
        h.set_options(prev)
    return (np.array(r[:]), np.array(K[:]), np.array(Ks[:]), int(steps.value), int(cyc.value), int(its.value),
            np.array(status[:], dtype=np.int32))


_GROUP_CTX = {}   # (device, group) -> (library handle, torch stream), reused across sweeps
_GROUP_CARRY_OPTIONS = (_lib.AIY_OPT_GE_LOGSEC, _lib.AIY_OPT_GE_REBALANCE, _lib.AIY_OPT_GE_EXTRAP_PERIOD,
                        _lib.AIY_OPT_HIST_PULL, _lib.AIY_OPT_GE_LOOSE_HIST, _lib.AIY_OPT_GE_ANDERSON)


def _close_groups():
    """Destroy the group handles while the HIP runtime is up (as _lib.close_all does)."""
    while _GROUP_CTX:
        _, (h, _) = _GROUP_CTX.popitem()
        h.close()


atexit.register(_close_groups)


def _device_cus(dev, cu_share=1.0):
    """Compute units this process may fill with resident clusters: the device's, times
    cu_share (< 1 when several rank processes share one GPU, the bench's gloo rehearsal)."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    return max(1, int(cus * float(cu_share)))


def _solve_groups(cals, aGrid, dev, groups, method, r_tol, egm_tol, hist_tol, max_steps, warm_hist, warm_egm, accel,
                  r_lo, r_hi, secant, loose, extrapolate, cu_share=1.0):
    """Independent root searches for `groups` subsets of the calibrations, each on its own
    library handle and stream from its own host thread (the library releases the GIL):
    a batched search steps all its calibrations together and pays, at every step, for its
    slowest one; decoupled groups do not wait for each other's slow steps.  Every group's
    clusters must be co-resident with the others', so each calibration's cluster is capped
    at (compute units / calibrations) workgroups (and 32)."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(cals)
    # round-robin: on the Table II order this groups the cells by CRRA, i.e. cells whose
    # slow steps coincide (snake order, which mixes slow and fast cells in every group,
    # measured 177 GE solves/s, contiguous (sigma, rho) blocks 176, round-robin 204)
    idx = [list(range(g, n, groups)) for g in range(groups)]
    idx = [i for i in idx if i]
    cus = _device_cus(dev, cu_share)
    cap = max(1, min(32, cus // n))
    cur = torch.cuda.current_stream(dev)
    # the search options a caller set on the device's shared handle carry over to the groups
    shared = _lib.handle(dev.index)
    carry = {o: shared.get_option(o) for o in _GROUP_CARRY_OPTIONS}
    jobs = []
    for gi, ii in enumerate(idx):
        key = (dev.index, gi)
        if key not in _GROUP_CTX:
            _GROUP_CTX[key] = (_lib.Handle(dev.index), torch.cuda.Stream(dev))
        h, st = _GROUP_CTX[key]
        h.set_options({**carry, _lib.AIY_OPT_HIST_CLUSTER: cap})
        b = StationaryBatch([cals[i] for i in ii], aGrid, device=dev)
        sub = lambda x: None if x is None else np.broadcast_to(np.asarray(x, float), (n,))[ii]  # noqa: E731
        st.wait_stream(cur)
        jobs.append((ii, b, h, st, sub(r_lo), sub(r_hi)))

    def run(job):
        ii, b, h, st, lo, hi = job
        with torch.cuda.stream(st):
            return ge_stationary_native(b, method, r_tol, egm_tol, hist_tol, max_steps, warm_hist, warm_egm, accel,
                                        lo, hi, secant=secant, loose=loose, extrapolate=extrapolate, handle=h,
                                        stream=st)
    with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
        outs = list(ex.map(run, jobs))
    for _, _, _, st, _, _ in jobs:
        cur.wait_stream(st)
    r, K, Ks = np.zeros(n), np.zeros(n), np.zeros(n)
    status = np.zeros(n, dtype=np.int32)
    steps = cyc = its = 0
    for (ii, b, *_), (rg, Kg, Ksg, sg, cg, ig, stg) in zip(jobs, outs):
        r[ii], K[ii], Ks[ii], status[ii] = rg, Kg, Ksg, stg
        steps, cyc, its = max(steps, sg), cyc + cg, its + ig
    alpha = np.array([c.CapShare for c in cals])
    delta = np.array([c.DeprFac for c in cals])
    KtoY = K ** (1.0 - alpha)
    return StationaryResult(r=r, K=K, K_supply=Ks, KtoY=KtoY, saving_rate=delta * KtoY, bisection_steps=steps,
                            egm_cycles=[np.array([cyc])], hist_iters=[np.array([its])], status=status)


def solve_table2(cals=None, n_a=10000, aMin=0.001, aMax=50.0, aNestFac=2, r_tol=1e-7, egm_tol=1e-8,
                 hist_tol=1e-12, device=None, r_lo=None, r_hi=None, max_steps=60, log=None, warm_hist=True,
                 method="bisect", warm_egm=None, accel=None, engine="native", secant=None, loose=None,
                 extrapolate=None, groups=None, cu_share=1.0, resident=None):
    """GE on r (E1) for every calibration at once.  Returns StationaryResult.

    method: "bisect" -- bisection on K_s(r) - K_d(r) to bracket width r_tol (the oracle's
    ge_bisect, step for step); "brent" -- bisection until both signs are evaluated, then
    Brent's method per calibration to r_tol (about half the K_s evaluations; the same
    root to r_tol).
    warm_hist: each step's distribution iteration starts from the previous step's
    stationary mass (the oracle, oracle/stationary.py, starts from uniform; both converge
    to the same distribution to hist_tol).  warm_egm (default: on for "brent"): each
    step's household solve starts from the previous step's policy.  accel (default: -1 =
    BiCGSTAB for "brent", 0 = the plain iteration for "bisect"; E > 0: Aitken period) --
    the distribution solver (StationaryBatch.capital_supply).
    engine: "native" -- one aiy_ge_stationary call (C++ search loop); "python" -- the same
    search driven from Python step by step (per-step logs; identical iterates when
    secant=False).  secant (native only; default: on for "brent"): from the third
    evaluation on, the household and distribution solves start from the secant
    extrapolation of the last two evaluations' solutions (same fixed points to the same
    stopping rules, fewer cycles / matvecs).  loose (native only; default: on for
    "brent"): while a calibration is still bracketing its root, its evaluations stop at
    egm 1e-6 / hist 1e-10 and their sign is used only where |K_s - K_d| >= 5 % of K_d
    (else that r is evaluated again at the full tolerances).  The two bracket endpoints
    Brent's method starts from may be such loose evaluations (their sign is certain, their
    value good to ~1e-6 relative); Brent's points then run at an adaptive distribution
    tolerance between hist_tol and the loose one (about 1e-9 of the smallest |K_s - K_d| / K_d
    seen so far; a point whose |K_s - K_d| is not well above that evaluation's error is redone
    at hist_tol), and the evaluation the search ends on is re-solved at hist_tol before its
    K_s is reported; the root is still bracketed by the 5 % sign margin.  With loose bracketing the native
    search also brackets and runs Brent's method in log coordinates (log K_s/K_d against
    log(1/beta - 1 - r), where the excess supply is nearly linear; AIY_OPT_GE_LOGSEC,
    csrc/ge_search.h): the same root to r_tol in fewer evaluations.  extrapolate (native only;
    default: on for "brent"): the household solves extrapolate their cycle iterates
    geometrically where the distances fall at a steady rate (csrc/egm.hip; same stopping
    rule).  groups (native only; default: 3 for "brent" with >= 3 calibrations, else 1):
    the calibrations split round-robin into independent searches on their own handles,
    streams and host threads (_solve_groups; 3 groups fill the process's hardware queues
    beside the default stream -- 4 measured slower).  cu_share: the fraction of the
    device's compute units this process's resident clusters may hold (several rank
    processes on one GPU: 1 / ranks), so that every process's clusters stay co-resident.
    resident (native only; default: wherever resident_plan() has a plan, with the BiCGSTAB
    distribution solve): the whole search of every calibration in ONE device-resident
    launch (csrc/ge_resident.hip: each calibration's cluster runs its own EGM cycles,
    lottery, BiCGSTAB and root search, no host round trip, no waiting for other
    calibrations); groups are then 1."""
    cals = table2_calibrations() if cals is None else list(cals)
    device = _resolve_device(device)
    aGrid = sm.make_grid_exp_mult(aMin, aMax, n_a, aNestFac)
    if warm_egm is None:
        warm_egm = method == "brent"
    if accel is None:
        accel = -1 if method == "brent" else 0
    if secant is None:
        secant = method == "brent"
    if loose is None:
        loose = method == "brent"
    if extrapolate is None:
        extrapolate = method == "brent"
    if resident is None:
        resident = (engine == "native" and log is None and accel < 0 and
                    resident_plan(device, len(cals), cals[0].LaborStatesNo, n_a, cu_share) is not None)
    resident = bool(resident) and engine == "native" and log is None
    if resident:
        groups = 1
    if groups is None:
        groups = 3 if (method == "brent" and engine == "native" and log is None and len(cals) >= 3) else 1
    if groups > 1:
        # concurrent groups need every calibration's cluster resident at once: the smallest
        # cluster the grid allows (512-thread workgroups, 2 columns per thread for S <= 8)
        # times the calibrations must fit the compute units, else one batched search
        S0 = cals[0].LaborStatesNo
        g_min = -(-n_a // (512 * (2 if S0 <= 8 else 1)))
        if g_min * len(cals) > _device_cus(device, cu_share):
            groups = 1
    if engine == "native" and log is None and groups > 1 and len(cals) > 1:
        return _solve_groups(cals, aGrid, device, int(groups), method, r_tol, egm_tol,
                             hist_tol, max_steps, warm_hist, warm_egm, accel, r_lo, r_hi,
                             secant and warm_hist and warm_egm, loose, extrapolate, cu_share)
    b = StationaryBatch(cals, aGrid, device=device)
    n = len(cals)
    lo = np.full(n, -0.5 * b.delta) if r_lo is None else np.broadcast_to(np.asarray(r_lo, float), (n,)).copy()
    hi = (1.0 / np.array([c.DiscFac for c in cals]) - 1.0 - 1e-9) if r_hi is None else \
        np.broadcast_to(np.asarray(r_hi, float), (n,)).copy()
    steps = 0
    cyc_log, it_log = [], []
    Ks = np.zeros(n)
    if engine == "native" and log is None:
        r, K, Ks, steps, cyc_sum, it_sum, status = ge_stationary_native(b, method, r_tol, egm_tol, hist_tol, max_steps,
                                                                warm_hist, warm_egm, accel, r_lo if r_lo is not None
                                                                else None, r_hi if r_hi is not None else None,
                                                                secant=secant and warm_hist and warm_egm,
                                                                loose=loose, extrapolate=extrapolate,
                                                                resident=resident, cu_share=cu_share)
        KtoY = K ** (1.0 - b.alpha)
        return StationaryResult(r=r, K=K, K_supply=Ks, KtoY=KtoY, saving_rate=b.delta * KtoY, bisection_steps=steps,
                                egm_cycles=[np.array([cyc_sum])], hist_iters=[np.array([it_sum])], status=status)
    if method == "brent":
        search = [_Brent(lo[k], hi[k], r_tol) for k in range(n)]
        while not all(sr.done for sr in search) and steps < max_steps:
            x = np.array([sr.propose() for sr in search])
            Ks, cycles, iters = b.capital_supply(x, egm_tol=egm_tol, hist_tol=hist_tol, warm=warm_hist and steps > 0,
                                                 warm_egm=warm_egm and steps > 0, accel=accel)
            _, Kd = firm_prices(x, b.alpha, b.delta)
            for k, sr in enumerate(search):
                sr.update(float(Ks[k] - Kd[k]))
            steps += 1
            cyc_log.append(cycles)
            it_log.append(iters)
            if log is not None:
                log.append(dict(step=steps, r=x.copy(), Ks=Ks.copy(), Kd=Kd.copy()))
        r = np.array([sr.propose() for sr in search])
    elif method == "bisect":
        while np.any(hi - lo > r_tol) and steps < max_steps:
            mid = 0.5 * (lo + hi)
            Ks, cycles, iters = b.capital_supply(mid, egm_tol=egm_tol, hist_tol=hist_tol,
                                                 warm=warm_hist and steps > 0, warm_egm=warm_egm and steps > 0,
                                                 accel=accel)
            _, Kd = firm_prices(mid, b.alpha, b.delta)
            up = Ks > Kd
            hi = np.where(up, mid, hi)
            lo = np.where(up, lo, mid)
            steps += 1
            cyc_log.append(cycles)
            it_log.append(iters)
            if log is not None:
                log.append(dict(step=steps, r=mid.copy(), Ks=Ks.copy(), Kd=Kd.copy()))
        r = 0.5 * (lo + hi)
    else:
        raise ValueError(f"method {method!r}")
    _, K = firm_prices(r, b.alpha, b.delta)
    KtoY = K ** (1.0 - b.alpha)
    return StationaryResult(r=r, K=K, K_supply=Ks, KtoY=KtoY, saving_rate=b.delta * KtoY, bisection_steps=steps,
                            egm_cycles=cyc_log, hist_iters=it_log)
