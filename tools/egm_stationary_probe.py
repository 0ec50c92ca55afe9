"""Stationary EGM cycle (n_M = 1) latency on the GPU box: one cycle-kernel launch of the
Table II batch (24 calibrations) and of single calibrations, at N_a = 10 000 (converged
tables as input, hints from the solve), via aiy_egm_kernel_time; prints JSON lines."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    from aiyagari_hark_amd.stationary import StationaryBatch, firm_prices, table2_calibrations
    dev = torch.device("cuda:0")
    h = _lib.handle(0)
    for n_a in (10000, 1000):
        for sel in ("all", "crra1", "crra5"):
            allc = table2_calibrations()
            cals = allc if sel == "all" else [c for c in allc if c.CRRA == (1.0 if sel == "crra1" else 5.0)]
            b = StationaryBatch(cals, sm.make_grid_exp_mult(0.001, 50.0, n_a, 2), device=dev)
            n, S = len(cals), b.S
            r = np.full(n, 0.03)
            w, _ = firm_prices(r, b.alpha, b.delta)
            Rn = torch.as_tensor(np.repeat((1 + r)[:, None, None], S, axis=2)).to(dev)
            Wn = torch.as_tensor(np.repeat(w[:, None, None], S, axis=2)).to(dev)
            batch = EgmBatch(b.d_a, torch.zeros((n, 1), dtype=torch.float64, device=dev), b.d_P, Rn, Wn,
                             torch.zeros_like(Rn), b.d_lab, b.d_beta, b.d_crra)
            torch.cuda.synchronize()
            import time
            t0 = time.perf_counter()
            m, c, cycles, _ = egm_solve(batch, tol=1e-8)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            m0, c0 = m.contiguous(), c.contiguous()
            mo, co = torch.empty_like(m0), torch.empty_like(c0)
            d, i = batch._abi()
            ms = ctypes.c_float()
            h.check(h.lib.aiy_egm_kernel_time(h.h, ctypes.byref(d), ctypes.byref(i), _lib.ptr(m0), _lib.ptr(c0),
                                              _lib.ptr(mo), _lib.ptr(co), 50, ctypes.byref(ms), _lib.stream_ptr()),
                    "kernel_time")
            print(json.dumps(dict(n_a=n_a, cals=n, sel=sel, lib=os.environ.get("AIYAGARI_LIB", "in-tree"), cycle_us=1000.0 * ms.value / 50, solve_s=el,
                                  cycles_max=int(np.max(cycles)), us_per_solve_cycle=1e6 * el / int(np.max(cycles)))),
                  flush=True)


if __name__ == "__main__":
    main()
