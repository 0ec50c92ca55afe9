#!/usr/bin/env python3
"""Per-step cost profile of the Table II sweep (configs[2]) on the Python-driven search:
per K_s evaluation the max / mean distribution iterations and EGM cycles over the 24
calibrations, and the wall time split between the household solve and the distribution
iteration.  One JSON line per step, then a summary line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd.stationary import solve_table2
    dev = torch.device("cuda:0")
    method = sys.argv[1] if len(sys.argv) > 1 else "brent"
    accel = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    solve_table2(n_a=1000, device=dev, max_steps=3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = solve_table2(device=dev, method=method, accel=accel, engine="python")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for k, (it, cy) in enumerate(zip(res.hist_iters, res.egm_cycles)):
        it, cy = np.asarray(it), np.asarray(cy)
        print(json.dumps(dict(step=k, hist_max=int(it.max()), hist_mean=float(it.mean()), egm_max=int(cy.max()),
                              egm_mean=float(cy.mean()))))
    print(json.dumps(dict(method=method, accel=accel, seconds=el, steps=res.bisection_steps,
                          hist_max_sum=int(sum(int(np.max(i)) for i in res.hist_iters)),
                          egm_max_sum=int(sum(int(np.max(c)) for c in res.egm_cycles)))))


if __name__ == "__main__":
    main()
