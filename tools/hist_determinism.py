#!/usr/bin/env python3
"""Run-to-run determinism of the standalone BiCGSTAB distribution solve (aiy_hist_solve,
hist_bicg_kernel): the same K_s(r) evaluation repeated, K printed bit for bit.  The library
is the one AIYAGARI_LIB names (default: the in-tree build).

    python tools/hist_determinism.py [n_a] [repeats]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def ge_mode():
    """The native host loop against the Python loop (test_native_ge_search_equals_python_loop)."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    out = {}
    for eng in ("native", "python", "native", "python"):
        kw = dict(secant=False, loose=False, extrapolate=False, groups=1, resident=False) if eng == "native" else {}
        res = solve_table2(cals, n_a=300, r_tol=1e-8, device=dev, method="brent", engine=eng, **kw)
        out.setdefault(eng, []).append([float(x).hex() for x in res.r] + [int(res.bisection_steps)])
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), **out)))
    # the first step after which the two loops' iterates differ (their r after k steps)
    for k in range(1, 13):
        rr = {}
        for eng in ("native", "python"):
            kw = dict(secant=False, loose=False, extrapolate=False, groups=1, resident=False) if eng == "native" else {}
            res = solve_table2(cals, n_a=300, r_tol=1e-8, device=dev, method="brent", engine=eng, max_steps=k, **kw)
            rr[eng] = [float(x).hex() for x in res.r]
        print(json.dumps(dict(steps=k, same=rr["native"] == rr["python"], **rr)), flush=True)


def noisy_mode(n_a):
    """The same evaluation with and without other work on a second stream (other wave timing
    on the CUs the solve's clusters share): a solve whose result depends on timing differs."""
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    b = StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, n_a, 2), device=dev)
    r = np.array([0.03, 0.02, 0.035])
    side = torch.cuda.Stream()
    x = torch.randn(4096, 4096, device=dev)
    out = {}
    for mode in ("quiet", "noisy", "quiet", "noisy", "noisy"):
        if mode == "noisy":
            with torch.cuda.stream(side):
                for _ in range(40):
                    x = torch.tanh(x @ x * 1e-3)
        K, cyc, it = b.capital_supply(r, accel=-1)
        torch.cuda.synchronize()
        out.setdefault(mode, []).append([float(v).hex() for v in K])
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), n_a=n_a, **out)))


def cross_mode():
    """One calibration's K at a fixed r while the others of the batch move: the calibrations'
    clusters share a launch (and nothing else), so the bits must not change."""
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    grid = sm.make_grid_exp_mult(0.001, 50.0, 300, 2)
    r3 = float.fromhex("0x1.2a359f8a72972p-5")
    rows = []
    for r1, r2 in ((0.03, 0.004), (0.04, 0.0038), (0.041, 0.0038), (0.02, 0.01), (0.041, 0.0038)):
        b = StationaryBatch(cals, grid, device=dev)
        K, _, it = b.capital_supply(np.array([r1, r2, r3]), accel=-1)
        rows.append([r1, r2, float(K[2]).hex(), int(it[2])])
    b = StationaryBatch(cals[2:], grid, device=dev)
    K, _, it = b.capital_supply(np.array([r3]), accel=-1)
    rows.append(["alone", None, float(K[0]).hex(), int(it[0])])
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), same=len({r[2] for r in rows}) == 1,
                          rows=rows)))


def warm_mode():
    """The Python loop's first five evaluations replayed (warm mass and policy between them),
    with and without other GPU work between the calls: step 5's K bits must not change."""
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch, solve_table2
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    grid = sm.make_grid_exp_mult(0.001, 50.0, 300, 2)
    log = []
    solve_table2(cals, n_a=300, r_tol=1e-8, device=dev, method="brent", engine="python", max_steps=5, log=log)
    rs = [e["r"] for e in log]
    ref = [float(v).hex() for v in log[-1]["Ks"]]
    other = StationaryBatch(cals, grid, device=dev)
    rows = {}
    b = StationaryBatch(cals, grid, device=dev)
    for k, r in enumerate(rs):
        b.capital_supply(r, warm=k > 0, warm_egm=k > 0, accel=-1)
        lo = b.lo.cpu().numpy().reshape(len(cals), -1, 300)
        dec = np.argwhere(np.diff(lo, axis=2) < 0)
        print(json.dumps(dict(step=k + 1, non_monotone=len(dec), where=dec[:8].tolist(),
                              lo_min=int(lo.min()), lo_max=int(lo.max()))), flush=True)
    big = torch.randn(8192, 8192, device=dev)
    for mode in ("plain",):
        b = StationaryBatch(cals, grid, device=dev)
        for k, r in enumerate(rs):
            if mode == "other_batch" and k > 0:
                other.capital_supply(r + 1e-3, accel=-1)
            if mode == "torch" and k > 0:
                x = torch.randn(2048, 2048, device=dev)
                (x @ x).sum().item()
            if mode == "busy" and k > 0:   # the queue busy when the solve's launches arrive
                for _ in range(3):
                    big = torch.tanh(big @ big * 1e-4)
            if mode == "busy_side" and k > 0:   # other work on the CUs while the solve runs
                side = torch.cuda.Stream()
                with torch.cuda.stream(side):
                    for _ in range(6):
                        big = torch.tanh(big @ big * 1e-4)
            K, _, it = b.capital_supply(r, warm=k > 0, warm_egm=k > 0, accel=-1)
        torch.cuda.synchronize()
        rows.setdefault(mode, []).append([float(v).hex() for v in K])
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), loop=ref, **rows)))


def counts_mode():
    """EGM cycles and distribution matvecs of the two loops after 4 and 5 steps."""
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    for k in (4, 5):
        for eng in ("native", "python"):
            kw = dict(secant=False, loose=False, extrapolate=False, groups=1, resident=False) if eng == "native" else {}
            res = solve_table2(cals, n_a=300, r_tol=1e-8, device=dev, method="brent", engine=eng, max_steps=k, **kw)
            print(json.dumps(dict(steps=k, eng=eng, K=[float(x).hex() for x in res.K_supply],
                                  cyc=[np.asarray(c).tolist() for c in res.egm_cycles],
                                  its=[np.asarray(c).tolist() for c in res.hist_iters])), flush=True)


def sweep_mode(rebalance):
    """The 24-cell Table II sweep (device-resident search) three times: r bit for bit.  With
    rebalance = 0 the launch sequence does not depend on timing, so any difference comes from
    the kernels."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    h = _lib.handle(0)
    h.set_options({_lib.AIY_OPT_GE_REBALANCE: rebalance})
    runs = []
    for _ in range(3):
        res = solve_table2(table2_calibrations(), n_a=10000, r_tol=1e-7, device=dev, method="brent", accel=-1)
        runs.append([float(x).hex() for x in res.r])
    same = all(r == runs[0] for r in runs)
    ndiff = [sum(a != b for a, b in zip(runs[0], r)) for r in runs[1:]]
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), rebalance=rebalance, identical=same,
                          cells_differing=ndiff, r0=runs[0][:4])))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        return sweep_mode(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    if len(sys.argv) > 1 and sys.argv[1] == "counts":
        return counts_mode()
    if len(sys.argv) > 1 and sys.argv[1] == "warm":
        return warm_mode()
    if len(sys.argv) > 1 and sys.argv[1] == "cross":
        return cross_mode()
    if len(sys.argv) > 1 and sys.argv[1] == "ge":
        return ge_mode()
    if len(sys.argv) > 1 and sys.argv[1] == "noisy":
        return noisy_mode(int(sys.argv[2]) if len(sys.argv) > 2 else 300)
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    n_a = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.6, LaborSD=0.2, CRRA=1.0), Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=5.0),
            Calibration(LaborAR=0.3, LaborSD=0.4, CRRA=3.0)]
    b = StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, n_a, 2), device=dev)
    r = np.array([0.03, 0.02, 0.035])
    seen = []
    for _ in range(reps):
        K, cyc, it = b.capital_supply(r, accel=-1)
        torch.cuda.synchronize()
        seen.append([float(x).hex() for x in K] + [int(x) for x in it])
    same = all(s == seen[0] for s in seen)
    # the same evaluations one calibration per call (other co-resident clusters, so other
    # wave timing; the same cluster shape)
    single = []
    for c in range(len(cals)):
        bc = StationaryBatch([cals[c]], sm.make_grid_exp_mult(0.001, 50.0, n_a, 2), device=dev)
        K, cyc, it = bc.capital_supply(r[c:c + 1], accel=-1)
        torch.cuda.synchronize()
        single.append(float(K[0]).hex())
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), n_a=n_a, deterministic=same,
                          single_equals_batch=single == seen[0][:len(cals)], single=single, runs=seen[:2])))


if __name__ == "__main__":
    main()
