"""Where the wall time of one Table II sweep (configs[2], the bench step) goes on the GPU
box: host setup (StationaryBatch: grids, income processes, device buffers) vs the native
search (aiy_ge_stationary); and, on the Python-driven search, the household solve, the
lottery + distribution solve and the host between them, per K_s(r) evaluation.
One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd import egm as egm_mod
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd import stationary as stn
    dev = torch.device("cuda:0")
    stn.solve_table2(n_a=1000, device=dev, max_steps=3)
    cals = stn.table2_calibrations()
    out = {}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b = stn.StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, 10000, 2), device=dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        stn.ge_stationary_native(b, "brent", 1e-7, 1e-8, 1e-12, 60, True, True, -1, secant=True, loose=True, extrapolate=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out.setdefault("setup_ms", []).append(1e3 * (t1 - t0))
        out.setdefault("native_ms", []).append(1e3 * (t2 - t1))
    # python engine, per phase
    acc = {"egm": 0.0}
    orig = egm_mod.egm_solve

    def timed(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = orig(*a, **k)
        torch.cuda.synchronize()
        acc["egm"] += time.perf_counter() - t
        return r
    stn.egm_solve = timed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = stn.solve_table2(device=dev, method="brent", engine="python")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    stn.egm_solve = orig
    out.update(python_total_ms=1e3 * el, python_egm_ms=1e3 * acc["egm"], steps=res.bisection_steps,
               egm_cycles_max_sum=int(sum(int(np.max(c)) for c in res.egm_cycles)),
               hist_matvecs_max_sum=int(sum(int(np.max(i)) for i in res.hist_iters)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
