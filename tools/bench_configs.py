"""Measurements of BASELINE.json configs[2..4] on one MI355X (the bench.py line covers
configs[1]); one JSON line per config on stdout, progress on stderr.

  table2  configs[2]: the 24 Aiyagari Table II calibrations (rho x sigma x CRRA), stationary
          mode (E1 bisection on r + stationary EGM + Young histogram E2), N_a = 10 000,
          7-state Tauchen, all 24 batched on ONE GPU (the 8-GPU run splits them 3 per rank).
  panel   configs[3] per-GPU shard: 12 499 998 agents (1e8 / 8, multiple of 7) x 1 000
          periods of the reference panel (Philox shocks) at N_a = 10 000 -- the population
          no longer fits in LDS, so this is the grid engine (one launch per period).
  table2_ref  configs[2] in the reference algorithm: 24 KS-form economies (notebook grids,
          350 agents, act_T = 11 000) to their AFunc fixed points in one EconomyBatch.
  stats   wealth statistics (HARK get_lorenz_shares) of a 12.5M-agent shard in HBM.
  stress  configs[4]: rho = 0.9, sigma = 0.4, CRRA in {1, 3, 5}, 25-state Rouwenhorst,
          N_a = 50 000, Young histogram 25 x 50 000 per calibration.

Kernel durations come from `rocprofv3 --kernel-trace --stats` of this script
(profiles/<tag>_configs_kernel_stats.csv); this script reports wall-clock rates.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print("[configs]", *a, file=sys.stderr, flush=True)


def table2(n_a, device):
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    cals = table2_calibrations()
    solve_table2(cals[:2], n_a=200, device=device)          # warm-up (module load, allocator)
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = solve_table2(cals, n_a=n_a, device=device)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    cyc = int(np.sum([np.max(c) for c in res.egm_cycles]))
    hit = int(np.sum([np.max(i) for i in res.hist_iters]))
    pts = int(np.sum([np.sum(i) for i in res.hist_iters])) * 7 * n_a
    return dict(config="configs[2] Table II stationary sweep", value=len(cals) / dt, unit="GE solves/s",
                seconds=dt, n_cal=len(cals), n_a=n_a, S=7, bisection_steps=res.bisection_steps,
                egm_cycles_max_sum=cyc, hist_iters_max_sum=hit, hist_point_iters=pts,
                r_percent=[round(100 * x, 6) for x in res.r], saving_rate_percent=[round(100 * x, 6) for x in res.saving_rate],
                calibrations=[(c.LaborAR, c.LaborSD, c.CRRA) for c in cals])


def stress(n_a, device):
    from aiyagari_hark_amd.stationary import Calibration, solve_table2
    cals = [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
            for c in (1.0, 3.0, 5.0)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = solve_table2(cals, n_a=n_a, device=device, method="brent")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    pts = int(np.sum([np.sum(i) for i in res.hist_iters])) * 25 * n_a
    return dict(config="configs[4] stress: rho 0.9, sigma 0.4, 25-state Rouwenhorst, Young histogram",
                value=len(cals) / dt, unit="GE solves/s", seconds=dt, n_cal=len(cals), n_a=n_a, S=25,
                bisection_steps=res.bisection_steps, hist_point_iters=pts, hist_point_iters_per_s=pts / dt,
                r_percent=[round(100 * x, 6) for x in res.r], saving_rate_percent=[round(100 * x, 6) for x in res.saving_rate])


def panel(n_agents, n_a, periods, device):
    from bench import make_economy
    econ, agent = make_economy(0, n_agents, n_a, periods, device, t_discard=periods // 10)
    econ.reset()
    agent.solve()
    torch.cuda.synchronize()
    econ.reset()
    econ.make_history()                      # warm-up history (tables, graph capture)
    torch.cuda.synchronize()
    p = agent.panel                          # time the device history alone (no host copy-back)
    p.reset(agent.kInit, agent.state_now["LaborSupplyState"], econ.sow_init["Mnow"], econ.sow_init["Aprev"],
            econ.sow_init["Mrkv"], econ.sow_init["Rnow"], econ.sow_init["Wnow"])
    torch.cuda.synchronize()
    t = time.perf_counter()
    p.run(0, periods, shock_mode="philox", seed=agent.shock_seed, ge_iter=1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ap = n_agents * periods
    return dict(config="configs[3] per-GPU shard of the 1e8-agent panel (grid engine, Philox)", value=ap / dt,
                unit="agent-periods/s", seconds=dt, agents=n_agents, periods=periods, n_a=n_a,
                us_per_period=1e6 * dt / periods, algorithmic_GBps=18.0 * ap / dt / 1e9,
                hbm_frac=18.0 * ap / dt / 8e12, K_last=float(p.hist_A[periods - 1].item()), engine=p._engine(_lib_handle()))


def wealth_stats(n, device):
    """Lorenz shares + percentiles of an n-agent wealth vector resident in HBM (the
    notebook's 15 pctiles), aiy_wealth_stats: device sort + scans + interpolation."""
    from aiyagari_hark_amd import stats
    g = torch.Generator(device=device)
    g.manual_seed(0)
    a = torch.exp(torch.randn(n, dtype=torch.float64, device=device, generator=g))
    pct = np.linspace(0.01, 0.999, 15)
    stats.get_lorenz_shares(a, percentiles=pct)
    torch.cuda.synchronize()
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        stats.get_lorenz_shares(a, percentiles=pct)
    dt = (time.perf_counter() - t) / reps
    return dict(config="wealth statistics (SURVEY §8f rank 1) of one GPU's panel shard", value=n / dt,
                unit="agents/s", seconds=dt, agents=n, ms_per_call=1e3 * dt)


def table2_reference(device, agents=350):
    """configs[2] in the reference's own algorithm: the 24 Table II cells, each a
    Krusell-Smith-form economy with the notebook's grids (32-point asset grid, 15 M nodes,
    350 agents, act_T = 11 000, T_discard = 1 000), solved to its AFunc fixed point by one
    EconomyBatch (batched EGM + one block-panel launch per GE iteration), Philox shocks."""
    from aiyagari_hark_amd.sweep import EconomyBatch, build_economies, table2_grid
    warm = build_economies(table2_grid()[:2], dict(act_T=300, T_discard=100), dict(AgentCount=agents),
                           device=device)
    EconomyBatch(warm).solve()
    torch.cuda.synchronize()
    econs = build_economies(table2_grid(), {}, dict(AgentCount=agents), device=device)
    eb = EconomyBatch(econs)
    t = time.perf_counter()
    loops = eb.solve()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    res = eb.results()
    return dict(config="configs[2] Table II in the reference algorithm (KS-form GE per cell, notebook grids)",
                value=len(econs) / dt, unit="GE solves/s", seconds=dt, n_cal=len(econs), agents=agents,
                act_T=econs[0].act_T, ge_iterations=list(loops),
                r_percent=[round(100 * r["r"], 4) for r in res],
                saving_rate_percent=[round(100 * r["saving_rate"], 4) for r in res])


def _lib_handle():
    from aiyagari_hark_amd import _lib
    return _lib.handle(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=["table2", "table2_ref", "panel", "stress", "stats"])
    ap.add_argument("--n-a", type=int, default=10000)
    ap.add_argument("--stress-n-a", type=int, default=50000)
    ap.add_argument("--agents", type=int, default=12_499_998)
    ap.add_argument("--periods", type=int, default=1000)
    ap.add_argument("--hist-fused", type=int, default=-1, help="AIY_OPT_HIST_FUSED (-1: library default)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    import threading
    t0 = time.time()

    def heartbeat():                        # gpurun treats 3 silent minutes as a hang
        while True:
            time.sleep(30)
            log(f"... {time.time() - t0:.0f}s")
    threading.Thread(target=heartbeat, daemon=True).start()
    from aiyagari_hark_amd import _lib
    _lib.load()
    if args.hist_fused >= 0:
        h = _lib.handle(0)
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_FUSED, args.hist_fused), "opt")
    for w in args.which:
        log("start", w)
        if w == "table2":
            r = table2(args.n_a, dev)
        elif w == "panel":
            r = panel(args.agents, args.n_a, args.periods, dev)
        elif w == "table2_ref":
            r = table2_reference(dev)
        elif w == "stats":
            r = wealth_stats(args.agents, dev)
        elif w == "stress":
            r = stress(args.stress_n_a, dev)
        else:
            raise SystemExit(f"unknown config {w}")
        log("done", w, f"{r['seconds']:.2f}s")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
