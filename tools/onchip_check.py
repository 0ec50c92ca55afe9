"""On-chip vs HBM-vector pull solve (AIY_OPT_HIST_ONCHIP 1 / 0) on configs[4]'s three cells:
K_s, BiCGSTAB matvecs and the largest mass difference, at N_a given (default 50 000)."""
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
    from aiyagari_hark_amd.stationary import Calibration, StationaryBatch
    n_a = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    dev = torch.device("cuda:0")
    h = _lib.handle(0)
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst") for c in (1.0, 3.0, 5.0)]
    grid = sm.make_grid_exp_mult(0.001, 50.0, n_a, 2)
    r = np.array([0.038, 0.028, 0.017])
    out = {}
    for oc in (0, 1):
        h.set_options({_lib.AIY_OPT_HIST_ONCHIP: oc})
        b = StationaryBatch(cals, grid, device=dev)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            K, cyc, it = b.capital_supply(r, accel=-1, hist_tol=1e-11)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        out[oc] = (K, it, b.mass.cpu().numpy())
        print(json.dumps(dict(onchip=oc, n_a=n_a, seconds=el, K=[float(x) for x in K], iters=[int(x) for x in it])), flush=True)
    h.set_options({_lib.AIY_OPT_HIST_ONCHIP: 1})
    d = np.abs(out[0][2] - out[1][2]).reshape(3, -1).max(axis=1)
    print(json.dumps(dict(mass_maxdiff=[float(x) for x in d])), flush=True)


if __name__ == "__main__":
    main()
