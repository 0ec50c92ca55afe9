#!/usr/bin/env python3
"""Wall time of the configs[2] Table II stationary sweep (E1 + E2, 24 calibrations at
N_a = 10 000) with the resident histogram on / off and several cluster sizes, plus the
resident launches' own kernel time.  One JSON line per variant."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import solve_table2
    dev = torch.device("cuda:0")
    h = _lib.handle(0)
    variants = [dict(resident=1, cluster=0), dict(resident=1, cluster=16), dict(resident=1, cluster=64),
                dict(resident=0, cluster=0)]
    if len(sys.argv) > 1:
        variants = [json.loads(a) for a in sys.argv[1:]]
    solve_table2(n_a=1000, device=dev, max_steps=3)   # warm-up (allocations, kernels)
    for v in variants:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_RESIDENT, v.get("resident", 1)), "opt")
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, v.get("cluster", 0)), "opt")
        kw = {k: v[k] for k in ("method", "warm_egm", "accel") if k in v}
        ms, n = ctypes.c_double(), ctypes.c_int64()
        h.check(h.lib.aiy_hist_launch_stats(h.h, None, None, 1), "stats")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = solve_table2(n_a=v.get("n_a", 10000), device=dev, **kw)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        h.check(h.lib.aiy_hist_launch_stats(h.h, ctypes.byref(ms), ctypes.byref(n), 1), "stats")
        hist_iters = [int(max(i)) for i in res.hist_iters]
        egm = [int(max(c)) for c in res.egm_cycles]
        print(json.dumps(dict(variant=v, seconds=el, ge_solves_per_s=24 / el, steps=res.bisection_steps,
                              hist_iters_max_sum=sum(hist_iters), egm_cycles_max_sum=sum(egm),
                              hist_kernel_ms=ms.value, hist_launches=n.value,
                              us_per_hist_iter=1e3 * ms.value / max(1, sum(hist_iters)),
                              r_percent=[round(100 * x, 6) for x in res.r])), flush=True)


if __name__ == "__main__":
    main()
