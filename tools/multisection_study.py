"""CPU prototype: evaluations of the current root search (ge_search.h RootSearch, logsec 2)
vs rounds of a multisection search with M concurrent candidates, on the oracle's K_s(r)
(oracle/stationary.py) at a small grid.  Round counts only (no costs)."""
import math, sys, os, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import stationary as ST

NA = int(os.environ.get("NA", 600))
aGrid = ST.make_stationary_grid(0.001, 50.0, NA, 2)

def make_f(rho, sig, mu):
    cal = dict(DiscFac=0.96, CRRA=mu, CapShare=0.36, DeprFac=0.08)
    lab, P = ST.income_process(7, rho, sig, "tauchen")
    cache = {}
    def f(r):
        if r not in cache:
            Ks, _ = ST.capital_supply(r, cal, aGrid, lab, P, egm_tol=1e-8, hist_tol=1e-12, fast=True)
            _, Kd = ST.prices(r, 0.36, 0.08)
            cache[r] = (Ks - Kd, Kd)
        return cache[r]
    return f

class RootSearch:   # port of ge_search.h (method 1, logsec 2)
    def __init__(s, lo, hi, xtol, logsec=2):
        s.lo, s.hi, s.xtol = lo, hi, xtol
        s.logsec, s.logsec1 = logsec > 0, logsec >= 2
        s.nneg = 0; s.rtop = hi
        s.ua = s.ga = s.ub = s.gb = s.glo = s.ghi = 0.0
        s.logb = False; s.have_lo = s.have_hi = s.brent = False
        s.flo = s.fhi = 0.0
        s.xpre = s.fpre = s.xcur = s.fcur = s.xblk = s.fblk = s.spre = s.scur = 0.0
        s.xprev_eval = s.fprev_eval = 0.0
        s.x = 0.5 * (lo + hi); s.done = not (hi - lo > xtol)
    def update(s, f, Kd):
        if s.done: return
        tr = s.logsec and Kd > 0 and f > -Kd
        if not s.brent:
            if f > 0: s.hi, s.fhi, s.have_hi = s.x, f, True
            else: s.lo, s.flo, s.have_lo = s.x, f, True
            if tr:
                if f > 0: s.ghi = math.log1p(f / Kd)
                else: s.glo = math.log1p(f / Kd)
            if s.hi - s.lo <= s.xtol: s.done = True; s.x = 0.5 * (s.lo + s.hi); return
            if not s.have_lo or not s.have_hi:
                xe = s.x; s.x = 0.5 * (s.lo + s.hi)
                if s.logsec1 and not s.have_lo and tr and f > 0 and xe < s.rtop:
                    dc = s.rtop - xe; dn = 1.25 * math.exp(math.log(dc) + math.log1p(f / Kd))
                    dn = min(max(dn, 2 * dc), 16 * dc); xn = s.rtop - dn
                    if s.lo < xn < s.hi: s.x = xn
                if s.logsec and not s.have_hi and Kd > 0 and f > -Kd and xe < s.rtop:
                    s.ua, s.ga = s.ub, s.gb
                    s.ub, s.gb = math.log(s.rtop - xe), math.log1p(f / Kd)
                    s.nneg += 1
                    two = s.nneg >= 2 and s.gb > s.ga and s.ub < s.ua
                    us = s.ub - s.gb * (s.ub - s.ua) / (s.gb - s.ga) if two else s.ub + s.gb
                    dc = s.rtop - xe
                    if two or (s.nneg == 1 and s.logsec1 and math.exp(us) < dc / 4):
                        dn = 0.8 * math.exp(us); dn = min(max(dn, dc / 16), dc / 2); xn = s.rtop - dn
                        if s.lo < xn < s.hi: s.x = xn
                return
            s.brent = True
            if s.logsec and tr and s.hi < s.rtop:
                s.logb = True; s.xtol = s.xtol / (s.rtop - s.lo)
                s.xpre, s.fpre, s.xcur, s.fcur = math.log(s.rtop - s.lo), s.glo, math.log(s.rtop - s.hi), s.ghi
            else:
                s.xpre, s.fpre, s.xcur, s.fcur = s.lo, s.flo, s.hi, s.fhi
            s.xblk = s.fblk = s.spre = s.scur = 0.0
            s.step()
            if s.logb: s.x = s.rtop - math.exp(s.x)
            return
        s.xpre, s.fpre = s.xprev_eval, s.fprev_eval
        s.fcur = (math.log1p(f / Kd) if tr else (1e300 if f > 0 else -1e300)) if s.logb else f
        s.step()
        if s.logb: s.x = s.rtop - math.exp(s.x)
    def step(s):
        eps = 2.220446049250313e-16
        if s.fpre * s.fcur < 0: s.xblk, s.fblk = s.xpre, s.fpre; s.spre = s.scur = s.xcur - s.xpre
        if abs(s.fblk) < abs(s.fcur):
            xp, xc, fp, fc = s.xcur, s.xblk, s.fcur, s.fblk
            s.xpre, s.xcur, s.xblk = xp, xc, xp; s.fpre, s.fcur, s.fblk = fp, fc, fp
        delta = 0.5 * (s.xtol + 4 * eps * abs(s.xcur)); sbis = 0.5 * (s.xblk - s.xcur)
        if s.fcur == 0 or abs(sbis) < delta: s.done = True; s.x = s.xcur; return
        if abs(s.spre) > delta and abs(s.fcur) < abs(s.fpre):
            if s.xpre == s.xblk: stry = -s.fcur * (s.xcur - s.xpre) / (s.fcur - s.fpre)
            else:
                dpre = (s.fpre - s.fcur) / (s.xpre - s.xcur); dblk = (s.fblk - s.fcur) / (s.xblk - s.xcur)
                stry = -s.fcur * (s.fblk * dblk - s.fpre * dpre) / (dblk * dpre * (s.fblk - s.fpre))
            if 2 * abs(stry) < min(abs(s.spre), 3 * abs(sbis) - delta): s.spre = s.scur; s.scur = stry
            else: s.spre = s.scur = sbis
        else: s.spre = s.scur = sbis
        s.xprev_eval, s.fprev_eval = s.xcur, s.fcur
        s.xcur += s.scur if abs(s.scur) > delta else (delta if sbis > 0 else -delta)
        s.x = s.xcur

def run_current(f, lo, hi, xtol=1e-7):
    rs = RootSearch(lo, hi, xtol); n = 0
    while not rs.done and n < 60:
        fv, Kd = f(rs.x); rs.update(fv, Kd); n += 1
    return rs.x, n

def run_multi(f, lo, hi, M=3, xtol=1e-7):
    """Multisection in (u, g) = (log(rtop - r), log(K_s/K_d)): every round evaluates M points."""
    rtop = hi
    pts = []   # (r, f, Kd)
    rounds = 0
    def g_of(fv, Kd): return math.log1p(fv / Kd) if fv > -Kd else -50.0
    # round 1: the midpoint and points toward rtop, spread in log distance
    d0 = rtop - 0.5 * (lo + hi)
    cand = [rtop - d0 * q for q in [1.0, 1 / 8, 1 / 64, 1 / 512][:M]]
    while rounds < 30:
        rounds += 1
        for r in cand: pts.append((r,) + f(r))
        pts.sort()
        neg = [p for p in pts if p[1] < 0]; pos = [p for p in pts if p[1] > 0]
        a = max(neg)[0] if neg else lo
        b = min(pos)[0] if pos else rtop
        if pos and neg and b - a <= xtol: return 0.5 * (a + b), rounds
        # model: secant / quadratic in (u, g) through the points nearest the sign change
        if not pos:   # only K_s < K_d: extrapolate toward rtop
            (r1, f1, k1), (r2, f2, k2) = (neg[-1], neg[-2]) if len(neg) >= 2 else (neg[-1], None)
            u1, g1 = math.log(rtop - r1), g_of(f1, k1)
            if f2 is not None and r2 != r1:
                u2, g2 = math.log(rtop - r2), g_of(f2, k2)
                slope = (g1 - g2) / (u1 - u2) if u1 != u2 else -1.0
                if not slope < 0: slope = -1.0
            else: slope = -1.0
            us = u1 - g1 / slope
            spread = max(0.5, abs(g1 / slope) * 0.3)
            us_list = [us - spread, us, us + spread][:M]
            cand = [rtop - math.exp(min(u, u1 - 0.05)) for u in us_list]
            continue
        if not neg:   # only K_s > K_d: step away from rtop
            r1 = pos[0][0]
            cand = [r1 - (r1 - lo) * q for q in [0.25, 0.5, 0.75][:M]]
            continue
        # bracket (a, b): inverse interpolation in u through the bracketing points
        ua, ub = math.log(rtop - a), math.log(rtop - b)
        fa = [p for p in pts if p[0] == a][0]; fb = [p for p in pts if p[0] == b][0]
        ga, gb = g_of(fa[1], fa[2]), g_of(fb[1], fb[2])
        us = ua - ga * (ub - ua) / (gb - ga)
        width = abs(ua - ub)
        # spread: a fraction of the bracket, shrinking as the model gets better
        eps = width / (2 * (M + 1))
        us_list = sorted([us + (k - (M - 1) / 2) * eps for k in range(M)])
        lo_u, hi_u = min(ua, ub), max(ua, ub)
        us_list = [min(max(u, lo_u + 1e-3 * width), hi_u - 1e-3 * width) for u in us_list]
        cand = sorted(set(rtop - math.exp(u) for u in us_list))
    return None, rounds

if __name__ == "__main__":
    from aiyagari_hark_amd.stationary import table2_calibrations
    cells = [(c.LaborAR, c.LaborSD, c.CRRA) for c in table2_calibrations()]
    idx = [int(x) for x in sys.argv[1:]] or range(len(cells))
    for k in idx:
        rho, sig, mu = cells[k]
        f = make_f(rho, sig, mu)
        lo, hi = -0.04, 1 / 0.96 - 1 - 1e-9
        r0, n0 = run_current(f, lo, hi)
        r3, n3 = run_multi(f, lo, hi, 3)
        r2, n2 = run_multi(f, lo, hi, 2)
        print(json.dumps(dict(cell=k, rho=rho, sig=sig, mu=mu, r=r0, evals=n0, r3=r3, rounds3=n3, r2=r2, rounds2=n2)), flush=True)
