#!/usr/bin/env python3
"""Benchmark: the Aiyagari household block on MI355X (BASELINE.json configs[1]).

Workload (one "step" = one full general-equilibrium solve, the reference's
``A94economy.solve()``, Aiyagari-HARK.py:249): Krusell-Smith-form household with
rho = 0.6, sigma = 0.2, CRRA = 1 (BASELINE config 1 calibration), 7-state Tauchen x
4 KS sub-states = 28 discrete states, 15 aggregate-M nodes, a 10 000-point asset grid
(exp-mult law of Aiyagari_Support.py:880), 1 000 006 agents simulated for act_T =
11 000 periods (T_discard = 1 000), labour shocks from on-device Philox, GE = damped
log-linear saving-rule regression to tolerance 0.01 (Aiyagari_Support.py:1574).
Every step restarts from the reference's initial saving rule (intercept 0, slope 1).

Multi-GPU (``torchrun --nproc-per-node N``): the path shards by calibration / shock
stream -- each rank solves its own economy (Philox seed = rank) with no collective in
the data path; value = total GE solves per second over all ranks (weak scaling).

Prints ONE JSON line (rank 0).  Extra diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak, MI355X_MICROARCH.md chip table
PANEL_BYTES_PER_AGENT = 18     # a in/out 16 B + labour state in/out 2 B (Philox)
N_AGENTS = 1_000_006           # nearest multiple of 7 >= 1e6
N_A = 10_000
ACT_T = 11_000
T_DISCARD = 1_000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def make_economy(seed, n_agents, n_a, act_T, device, t_discard=T_DISCARD):
    from aiyagari_hark_amd.model import AiyagariEconomy, AiyagariType
    econ_d = dict(act_T=act_T, T_discard=t_discard, LaborAR=0.6, LaborSD=0.2, CRRA=1.0,
                  intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0])
    agent_d = dict(LaborAR=0.6, LaborSD=0.2, CRRA=1.0, aCount=n_a, AgentCount=n_agents)
    econ = AiyagariEconomy(**econ_d)
    econ.verbose = False
    agent = AiyagariType(device=device, shock_mode="philox", shock_seed=seed, **agent_d)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    return econ, agent


def reset_rule(econ, agent):
    econ.intercept_prev[:] = [0.0, 0.0]
    econ.slope_prev[:] = [1.0, 1.0]
    econ.update()
    agent.get_economy_data(econ)


class Probe:
    """Accumulates host wall time of the EGM solves and the panel histories."""

    def __init__(self):
        self.egm_s = 0.0
        self.panel_s = 0.0
        self.ge_iters = 0
        self.cycles = 0


def run_step(econ, agent, probe: Probe):
    reset_rule(econ, agent)
    solve_agents, make_history = econ.solve_agents, econ.make_history

    def timed_solve():
        t = time.perf_counter()
        solve_agents()
        torch.cuda.synchronize()
        probe.egm_s += time.perf_counter() - t
        probe.cycles += agent.completed_cycles + 1

    def timed_hist():
        t = time.perf_counter()
        make_history()
        probe.panel_s += time.perf_counter() - t
        probe.ge_iters += 1

    econ.solve_agents, econ.make_history = timed_solve, timed_hist
    try:
        econ.solve()
    finally:
        econ.solve_agents, econ.make_history = solve_agents, make_history


def panel_kernel_time(agent, n_periods):
    """Duration of ONE persistent panel launch covering a whole history of n_periods
    periods (the launch aiy_sim_periods makes for make_history), from the end-of-history
    population: HIP events on the launch's stream (aiy_sim_kernel_time)."""
    from aiyagari_hark_amd import _lib
    p = agent.panel
    h = _lib.handle(agent.device.index)
    a = p.a.clone()
    lab = p.lab.clone()
    sow = p.sow.clone()
    pm, mk = p._model[:2]
    ms = ctypes.c_float()
    stream = torch.cuda.current_stream()
    for n in (10, n_periods):   # warm, then the timed history launch
        h.check(h.lib.aiy_sim_kernel_time(h.h, ctypes.byref(pm), ctypes.byref(mk), p.n_local, _lib.ptr(a),
                                          _lib.ptr(lab), 99, 7, _lib.ptr(sow), n, ctypes.byref(ms),
                                          stream.cuda_stream), "timing")
    return ms.value


def egm_kernel_time(agent, n_launch=20):
    """Average duration of one EGM cycle kernel from the converged policy: HIP events
    on its stream (aiy_egm_kernel_time; the search-index build is outside)."""
    from aiyagari_hark_amd import _lib
    sol = agent.solution[0]
    b = agent.egm_batch
    m0 = sol.m_tab[None].contiguous()
    c0 = sol.c_tab[None].contiguous()
    mo, co = torch.empty_like(m0), torch.empty_like(c0)
    d, i = b._abi()
    h = _lib.handle(agent.device.index)
    ms = ctypes.c_float()
    for n in (2, n_launch):
        h.check(h.lib.aiy_egm_kernel_time(h.h, ctypes.byref(d), ctypes.byref(i), _lib.ptr(m0), _lib.ptr(c0),
                                          _lib.ptr(mo), _lib.ptr(co), n, ctypes.byref(ms),
                                          torch.cuda.current_stream().cuda_stream), "aiy_egm_kernel_time")
    return ms.value / n_launch


def table2_reference_leg(world, rank, dev, agents=350):
    """configs[2] in the reference's own algorithm, reported beside the headline: the 24
    Table II cells (rho x sigma x CRRA) as KS-form economies with the notebook's grids
    (32-point asset grid, 15 M nodes, 350 agents, act_T = 11 000), split round-robin over
    the ranks (parallel.split_calibrations; 3 per GPU at 8 GPUs), each rank solving its
    cells to their AFunc fixed points in one EconomyBatch; no collective in the data path.
    Value = 24 / (max over ranks of the wall time)."""
    from aiyagari_hark_amd.parallel import split_calibrations
    from aiyagari_hark_amd.sweep import EconomyBatch, build_economies, table2_grid
    cells = table2_grid()
    mine = split_calibrations(list(enumerate(cells)), world, rank)
    warm = build_economies(cells[:1], dict(act_T=300, T_discard=100), dict(AgentCount=agents), device=dev)
    EconomyBatch(warm).solve()
    econs = [build_economies([c], {}, dict(AgentCount=agents), device=dev, seed0=k)[0] for k, c in mine]
    barrier(world)
    t0 = time.perf_counter()
    loops = EconomyBatch(econs).solve() if econs else []
    barrier(world)
    el = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    return {"value": len(cells) / el, "unit": "GE solves/s", "seconds": el, "calibrations": len(cells),
            "per_rank": len(mine), "agents": agents, "act_T": 11000, "ge_iterations_rank0": list(loops),
            "workload": "configs[2] Table II, reference algorithm: KS-form GE per cell, notebook grids, "
                        "one EconomyBatch per rank"}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return float(d[kernel]["hbm_bytes_per_launch"])
    except Exception:
        return None


def cpu_baseline(n_ge, cycles_per_solve, budget_s=20.0):
    """The oracle (NumPy restatement of the reference path at HARK's vectorisation
    granularity) timed on this host on a bounded sample of the same workload: EGM cycles
    at N_a = 10 000 and panel periods of 1 000 006 agents; the GE solve time is then
    n_ge x (cycles x t_cycle + act_T x t_period) with the counts the GPU run took."""
    from oracle import hark_ks as H
    m = H.KSModel(dict(act_T=50), dict(aCount=N_A, AgentCount=N_AGENTS))
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, 7, m.e)
    args = (0.96, 1.0, m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates, m.MrkvIndArray)
    mt, ct = H.egm_step(None, None, *args)
    t0 = time.perf_counter()
    n_cyc = 0
    while n_cyc < 2 or (time.perf_counter() - t0 < budget_s / 2 and n_cyc < 8):
        mt, ct = H.egm_step(mt, ct, *args)
        n_cyc += 1
    t_cycle = (time.perf_counter() - t0) / n_cyc
    emp, lab = H.sim_birth_labor(N_AGENTS, 7, 0.0, seed=0)
    a = np.full(N_AGENTS, m.ss["KSS"])
    rng = np.random.RandomState(1)
    t0 = time.perf_counter()
    n_per = 0
    while n_per < 2 or (time.perf_counter() - t0 < budget_s / 2 and n_per < 40):
        a, lab, _, _ = H.sim_one_period(a, lab, emp, rng.random_sample(N_AGENTS), m.ss["RSS"], m.ss["WSS"],
                                        m.ss["MSS"], 0, m.LSStates, m.cdf_table, mt, ct, m.Mgrid)
        H.calc_R_and_W([a], [emp.astype(float)], 0, m.e)
        n_per += 1
    t_period = (time.perf_counter() - t0) / n_per
    ge_time = n_ge * (cycles_per_solve * t_cycle + ACT_T * t_period)
    return dict(value=1.0 / ge_time, unit="GE solves/s", cores=1, kind="port",
                sample=(f"oracle/hark_ks.py on this host: {n_cyc} EGM cycles at N_a=10000 "
                        f"({t_cycle:.3f} s each) + {n_per} panel periods of 1000006 agents ({t_period:.3f} s each), "
                        f"extrapolated to the GPU run's {n_ge:.1f} GE iterations x ({cycles_per_solve:.1f} EGM cycles "
                        f"+ 11000 periods); single thread (OMP/OPENBLAS=1); host {platform.processor() or platform.machine()}"),
                agent_periods_per_s=N_AGENTS / t_period, egm_cycle_s=t_cycle)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--agents", type=int, default=N_AGENTS)
    ap.add_argument("--grid", type=int, default=N_A)
    ap.add_argument("--act-T", type=int, default=ACT_T)
    ap.add_argument("--t-discard", type=int, default=T_DISCARD)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-table2", action="store_true", help="skip the Table II reference-algorithm leg")
    ap.add_argument("--no-kernel-diag", action="store_true",
                    help="skip the extra timing launches after the timed region (PMC passes)")
    args = ap.parse_args()

    world, rank, local = setup_dist()
    dev = torch.device("cuda", local)
    from aiyagari_hark_amd import build
    if rank == 0:
        build.build(verbose=False)
    barrier(world)

    econ, agent = make_economy(seed=rank, n_agents=args.agents, n_a=args.grid, act_T=args.act_T, device=dev,
                               t_discard=args.t_discard)
    for _ in range(args.warmup):
        run_step(econ, agent, Probe())
    probe = Probe()
    from aiyagari_hark_amd import _lib
    hnd = _lib.handle(dev.index)
    hnd.check(hnd.lib.aiy_panel_launch_stats(hnd.h, None, None, None, 1), "stats reset")
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step(econ, agent, probe)
    barrier(world)
    elapsed = time.perf_counter() - t0
    st_ms, st_n, st_per = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    hnd.check(hnd.lib.aiy_panel_launch_stats(hnd.h, ctypes.byref(st_ms), ctypes.byref(st_n), ctypes.byref(st_per), 1),
              "stats")
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    sow = econ.sow_state
    K = float(np.mean(econ.reap_state["aNow"][0]))
    r = sow["Rnow"] - 1.0
    KtoY = K / (sow["Mnow"] - (1 - econ.DeprFac) * K)
    n_ge = probe.ge_iters / args.steps
    cyc = probe.cycles / max(1, probe.ge_iters)

    # ---- dominant-kernel rooflines (live HIP events) ----
    # panel: one launch = one history (act_T periods of every agent); algorithmic bytes
    # 18 per agent-period; EGM: one launch = one cycle, 32 B per node
    # the timed region's own history launches (HIP events around each launch)
    t_launch_ms = st_ms.value / max(1, st_n.value)
    per_launch = st_per.value / max(1, st_n.value)
    t_panel_ms = t_launch_ms / max(1.0, per_launch)
    if args.no_kernel_diag:
        t_conv_ms, t_egm_ms = float("nan"), float("nan")
    else:
        t_conv_ms = panel_kernel_time(agent, args.act_T) / args.act_T   # converged-policy history, diagnostic
        t_egm_ms = egm_kernel_time(agent)
    panel_bytes = PANEL_BYTES_PER_AGENT * args.agents * per_launch
    egm_bytes = 32 * 28 * 15 * (args.grid + 1)
    panel_gbs = panel_bytes / (t_launch_ms * 1e-3) / 1e9
    egm_gbs = egm_bytes / (t_egm_ms * 1e-3) / 1e9
    panel_share = probe.panel_s / max(1e-9, probe.panel_s + probe.egm_s)

    solves_per_s = world * args.steps / elapsed
    agent_periods = world * args.steps * n_ge * args.act_T * args.agents / elapsed
    line = {
        "metric": "GE solves/sec (Table II sweep); agent-periods/sec; % HBM roofline",
        "value": solves_per_s,
        "unit": "GE solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (calibration of BASELINE config 1, on-device Philox labour shocks)",
        "config": {"workload": "BASELINE configs[1]: KS-form Aiyagari GE, 28 states x 15 M nodes x "
                               f"{args.grid}-pt asset grid, {args.agents} agents x {args.act_T} periods per GE "
                               "iteration, one independent economy per GPU",
                   "n_a": args.grid, "agents_per_gpu": args.agents, "act_T": args.act_T, "S": 28, "n_M": 15,
                   "parallelism": f"calibration/shock-stream sharding x{world}, no data-path collective"},
        "agent_periods_per_sec": agent_periods,
        "ge_iterations_per_solve": n_ge,
        "egm_cycles_per_ge_iteration": cyc,
        "time_share": {"panel": panel_share, "egm": 1 - panel_share},
        "result": {"r": r, "K_over_Y": KtoY, "saving_rate": econ.DeprFac * KtoY},
        "roofline": {"kernel": "sim_resident_kernel", "bound": "hbm", "achieved": panel_gbs,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": panel_gbs / HBM_PEAK_GBS,
                     "traffic": pmc_traffic("sim_resident_kernel"),
                     "algorithmic_bytes_per_launch": panel_bytes, "avg_launch_ms": t_launch_ms,
                     "launch": f"one history: {per_launch:.0f} periods x {args.agents} agents",
                     "launches_timed": st_n.value, "us_per_period": 1e3 * t_panel_ms,
                     "us_per_period_converged_policy": 1e3 * t_conv_ms},
        "roofline_other": {"kernel": "egm_cycle_kernel", "bound": "hbm", "achieved": egm_gbs, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": egm_gbs / HBM_PEAK_GBS, "traffic": pmc_traffic("egm_cycle_kernel"),
                           "algorithmic_bytes_per_launch": egm_bytes, "avg_launch_ms": t_egm_ms},
        "cpu_baseline": None,
    }
    if not args.no_table2:
        line["table2_reference"] = table2_reference_leg(world, rank, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        os.environ.setdefault("OMP_NUM_THREADS", "1")
        cb = cpu_baseline(n_ge, cyc)
        line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
        line["cpu_baseline"]["agent_periods_per_sec"] = cb["agent_periods_per_s"]
    log(f"[bench] rank {rank}: {args.steps} GE solves in {elapsed:.2f}s; GE iters/solve {n_ge:.1f}; "
        f"EGM cycles/iter {cyc:.1f}; egm {probe.egm_s:.2f}s panel {probe.panel_s:.2f}s; "
        f"panel kernel {t_panel_ms * 1e3:.1f}us ({panel_gbs:.0f} GB/s), egm kernel {t_egm_ms * 1e3:.1f}us "
        f"({egm_gbs:.0f} GB/s); r={r:.6f} K/Y={KtoY:.6f}")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
