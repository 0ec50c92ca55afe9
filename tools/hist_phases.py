#!/usr/bin/env python3
"""One K_s(r) evaluation of the 24 Table II calibrations (N_a = 10 000) through the
library named by AIYAGARI_LIB (e.g. the AIY_DIAG_PHASES variant, which prints per-phase
times of the resident histogram); prints wall time and iteration counts.
Arguments: [n_cal] [cluster cap] [accel: Aitken period, < 0 BiCGSTAB]."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.stationary import StationaryBatch, table2_calibrations
    n_cal = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    cluster = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    accel = int(sys.argv[3]) if len(sys.argv) > 3 else 32   # < 0: BiCGSTAB (hist_krylov.hip)
    dev = torch.device("cuda:0")
    h = _lib.handle(0)
    h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, cluster), "opt")
    if os.environ.get("STRESS"):   # configs[4]: 25-state Rouwenhorst, N_a = 50 000, near the roots
        from aiyagari_hark_amd.stationary import Calibration
        cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
                for c in (1.0, 3.0, 5.0)][:n_cal]
        b = StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, 50000, 2), device=dev)
        r = np.array([0.038, 0.028, 0.017])[:n_cal]
    else:
        cals = table2_calibrations()[:n_cal]
        b = StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, 10000, 2), device=dev)
        r = np.full(n_cal, 0.03)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        K, cyc, it = b.capital_supply(r, accel=accel)
        torch.cuda.synchronize()
        print(json.dumps(dict(n_cal=n_cal, cluster=cluster, rep=rep, seconds=time.perf_counter() - t0,
                              hist_iters_max=int(np.max(it)), egm_cycles_max=int(np.max(cyc)))), flush=True)


if __name__ == "__main__":
    main()
