"""Per-calibration phase profile of the device-resident GE search (csrc/ge_resident.hip)
on the Table II sweep: EGM / lottery / distribution solve / K + search microseconds of each
calibration's cluster (workgroup 0's clock), EGM cycles, matvecs, evaluations; and the
sweep's wall time beside the host-driven search.

    python tools/ge_resident_profile.py [--n-a 10000] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-a", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cells", type=int, default=24)
    ap.add_argument("--cluster-cap", type=int, default=0)
    ap.add_argument("--modes", default="resident,host")
    ap.add_argument("--rebalance", type=int, default=-1, help="AIY_OPT_GE_REBALANCE (-1: default)")
    ap.add_argument("--extrap", type=int, default=-1, help="AIY_OPT_GE_EXTRAP_PERIOD (-1: default)")
    ap.add_argument("--logsec", type=int, default=-1, help="AIY_OPT_GE_LOGSEC (-1: default)")
    ap.add_argument("--loose-hist", type=int, default=-1, help="AIY_OPT_GE_LOOSE_HIST (-1: default)")
    ap.add_argument("--stress", action="store_true", help="configs[4]'s 3 cells (25 states) instead of Table II")
    ap.add_argument("--all-evals", action="store_true", help="print every calibration's evaluation log")
    args = ap.parse_args()
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.stationary import Calibration, solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    if args.stress:
        cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
                for c in (1.0, 3.0, 5.0)]
        if args.n_a == 10_000:
            args.n_a = 50_000
    else:
        cals = table2_calibrations()[:args.cells]
    h = _lib.handle(0)
    if args.cluster_cap:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, args.cluster_cap), "opt")
    if args.rebalance >= 0:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_REBALANCE, args.rebalance), "opt")
    if args.logsec >= 0:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOGSEC, args.logsec), "opt")
    if args.loose_hist >= 0:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_LOOSE_HIST, args.loose_hist), "opt")
    if args.extrap >= 0:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_GE_EXTRAP_PERIOD, args.extrap), "opt")
    out = {}
    for mode in args.modes.split(","):
        kw = dict(n_a=args.n_a, device=dev, method="brent", resident=mode == "resident", groups=1)
        solve_table2(cals, **kw)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            res = solve_table2(cals, **kw)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        out[mode] = dict(ms=[round(1e3 * x, 2) for x in ts], r=[float(x) for x in res.r])
        print(f"[profile] {mode}: {np.median(ts) * 1e3:.1f} ms per sweep ({len(cals) / np.median(ts):.1f} GE solves/s)",
              file=sys.stderr, flush=True)
        if mode == "resident":
            prof = (ctypes.c_double * (8 * len(cals)))()
            n = h.lib.aiy_ge_last_profile(h.h, prof, len(cals))
            p = np.array(prof[:8 * n]).reshape(n, 8)
            rows = []
            for c in range(n):
                egm, lot, hist, k, tot, cyc, mv, ev = p[c]
                rows.append(dict(cell=c, egm_us=round(egm, 1), lottery_us=round(lot, 1), hist_us=round(hist, 1),
                                 k_us=round(k, 1), total_us=round(tot, 1), egm_cycles=int(cyc), matvecs=int(mv),
                                 evaluations=int(ev), us_per_cycle=round(egm / max(1, cyc), 2),
                                 us_per_matvec=round(hist / max(1, mv), 2)))
                print(f"[profile] cell {c:2d}: total {tot / 1e3:6.2f} ms  egm {egm / 1e3:6.2f} ms ({int(cyc):5d} cyc, "
                      f"{egm / max(1, cyc):5.2f} us)  lottery {lot / 1e3:5.2f} ms  hist {hist / 1e3:6.2f} ms "
                      f"({int(mv):5d} mv, {hist / max(1, mv):5.2f} us)  K {k / 1e3:5.2f} ms  evals {int(ev)}",
                      file=sys.stderr, flush=True)
            out["profile"] = rows
            ev = (ctypes.c_double * (32 * 6 * len(cals)))()
            ne = h.lib.aiy_ge_last_eval_log(h.h, ev, len(cals))
            e = np.array(ev[:32 * 6 * ne]).reshape(ne, 32, 6)
            out["evaluations"] = [[dict(r=float(x[0]), f_rel=float(x[1]), egm_cycles=int(x[2]), matvecs=int(x[3]),
                                        loose=int(x[4]), us=round(float(x[5]), 1)) for x in e[c] if x[2] > 0]
                                  for c in range(ne)]
            for c in (range(ne) if args.all_evals else ((0, 1, 2) if args.stress else (0, 11, 23))):
                if c < ne:
                    print(f"[evals] cell {c}: " + "; ".join(f"r={x['r']:.6f} f={x['f_rel']:+.1e} cyc={x['egm_cycles']} "
                                                            f"mv={x['matvecs']}{' L' if x['loose'] else ''} "
                                                            f"{x['us']:.0f}us"
                                                            for x in out["evaluations"][c]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
