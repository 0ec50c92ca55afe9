"""configs[4] (stress: rho 0.9, sigma 0.4, CRRA 1/3/5, 25-state Rouwenhorst, N_a = 50 000)
solved with each AIY_OPT_GE_LOGSEC level: median seconds per solve and K_s evaluations per
cell, to compare the root-search variants on cells whose roots lie far below 1/beta - 1.

    python tools/stress_logsec.py [--levels 0,1,2] [--reps 3]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--levels", default="0,1,2")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n-a", type=int, default=50_000)
    args = ap.parse_args()
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    dev = torch.device("cuda:0")
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst") for c in (1.0, 3.0, 5.0)]
    h = _lib.handle(0)
    try:
        for lvl in [int(x) for x in args.levels.split(",")]:
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, lvl), "opt")
            solve_table2(cals, n_a=args.n_a, device=dev, method="brent")
            ts = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                res = solve_table2(cals, n_a=args.n_a, device=dev, method="brent")
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            print(f"[stress] logsec {lvl}: {np.median(ts):.3f} s per solve ({len(cals) / np.median(ts):.2f} GE solves/s), "
                  f"evaluations {np.atleast_1d(np.asarray(res.bisection_steps)).astype(int).tolist()}, r % {np.round(100 * res.r, 5)}",
                  flush=True)
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, 2), "opt")


if __name__ == "__main__":
    main()
