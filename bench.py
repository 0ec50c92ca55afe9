#!/usr/bin/env python3
"""Benchmark of the MI355X Aiyagari household block against BASELINE.json's metric
"GE solves/sec (Table II sweep); agent-periods/sec; % HBM roofline".

Headline (``value``): configs[2], the Aiyagari (1994) Table II sweep -- the 24
calibrations rho in {0, .3, .6, .9} x sigma in {.2, .4} x CRRA in {1, 3, 5}, each solved
to general equilibrium in r (build-defined E1: root search on K_s(r) = K_d(r), Brent's
method after a sign change) with the stationary household on a 10 000-point asset grid
(7-state Tauchen; EGM of Aiyagari_Support.py:1423-1520 with one aggregate node) and its
stationary distribution by the Young lottery (E2).  One step = the whole 24-cell sweep
from cold buffers.  With N ranks the cells are split round-robin (3 per GPU at 8), no
collective in the data path; value = 24 / (max over ranks of the seconds per sweep):
STRONG scaling (the sweep's total work is fixed).

Secondary legs on the same line (each its own object):
  configs1  -- BASELINE configs[1]: the reference's own Krusell-Smith-form GE solve
               (Aiyagari-HARK.py:249) at 10 000 grid points x 1 000 006 agents x 11 000
               periods per GE iteration; one independent economy per rank.
  configs3  -- BASELINE configs[3]: 99 999 998 agents x 1 000 periods sharded over the
               ranks with a per-period RCCL all-reduce of the asset sum (the agent-sharded
               np.mean of Aiyagari_Support.py:1868); agent-periods/s.
  table2_reference -- configs[2] in the reference's own algorithm (KS form per cell,
               notebook grids: 32 points, 350 agents, act_T = 11 000).

Run ``python bench.py --gpus N``: without WORLD_SIZE in the environment it starts N rank
processes itself (torch.distributed.run on 127.0.0.1) before touching the GPU.  Prints
ONE JSON line (rank 0); diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak, MI355X_MICROARCH.md chip table
PANEL_BYTES_PER_AGENT = 18     # a in/out 16 B + labour state in/out 2 B (Philox)
HIST_BYTES_PER_POINT = 28      # mass in 8, lottery index 4, weight 8, mass out 8
# per (state, node) point and matvec of the BiCGSTAB distribution solve (hist_krylov.hip):
# the 28 B of the push/mix matvec plus half an iteration's iterate traffic (x read and
# written twice, p written and read: 48 B per iteration of two matvecs)
HIST_BYTES_PER_POINT_KRYLOV = 52
N_AGENTS = 1_000_006           # nearest multiple of 7 >= 1e6
N_AGENTS_C3 = 99_999_998       # 1e8 agents, multiple of 7
T_C3 = 1000
N_A = 10_000
ACT_T = 11_000
T_DISCARD = 1_000
N_TABLE2 = 24


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """Start n rank processes of this script (one per GPU) before any GPU call here, and
    exit with their status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def setup_dist():
    import torch
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
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(obj, world):
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def hist_stats(h, reset, dev=None):
    """Resident-histogram kernel milliseconds and launches since the last reset, summed
    over the device's shared handle and the handles of solve_table2's independent groups
    (stationary._GROUP_CTX): per-launch HIP events, so overlapping groups are counted launch
    by launch."""
    from aiyagari_hark_amd import stationary
    hs = [h] + [hg for (d, _), (hg, _) in stationary._GROUP_CTX.items() if dev is None or d == dev.index]
    tot_ms, tot_n = 0.0, 0
    for hh in hs:
        ms, n = ctypes.c_double(), ctypes.c_int64()
        hh.check(hh.lib.aiy_hist_launch_stats(hh.h, ctypes.byref(ms), ctypes.byref(n), int(reset)), "hist stats")
        tot_ms, tot_n = tot_ms + ms.value, tot_n + n.value
    return tot_ms, tot_n


# ------------------------------------------------------------------------------------
# headline: configs[2] Table II stationary sweep
# ------------------------------------------------------------------------------------
def table2_leg(args, world, rank, dev):
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.parallel import split_calibrations
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    cells = table2_calibrations()
    mine = split_calibrations(list(range(len(cells))), world, rank)
    cals = [cells[k] for k in mine]
    h = _lib.handle(dev.index)

    def sweep():
        return solve_table2(cals, n_a=args.grid, device=dev, method="brent")

    for _ in range(args.warmup):
        sweep()
    hist_stats(h, True, dev)
    point_iters = 0   # (state, node) points x matvecs of the distribution solves
    res = None
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = sweep()
        point_iters += sum(int(np.sum(it)) for it in res.hist_iters) * 7 * args.grid
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    hist_ms, hist_n = hist_stats(h, True, dev)
    # dominant kernel: the device-resident BiCGSTAB distribution solve (one launch per K_s(r)
    # evaluation); algorithmic bytes 52 per (state, node) point per matvec
    hist_bytes = HIST_BYTES_PER_POINT_KRYLOV * point_iters
    hist_gbs = hist_bytes / max(1e-12, hist_ms * 1e-3) / 1e9
    per_rank = gather_objects(dict(cells=mine, r=[float(x) for x in res.r], KtoY=[float(x) for x in res.KtoY],
                                   evaluations=res.bisection_steps), world)
    r = [None] * len(cells)
    kty = [None] * len(cells)
    for pr in per_rank:
        for k, rr, ky in zip(pr["cells"], pr["r"], pr["KtoY"]):
            r[k], kty[k] = rr, ky
    out = dict(seconds_per_sweep=el / args.steps, value=len(cells) * args.steps / el,
               hist_kernel_ms_per_sweep=hist_ms / args.steps, hist_launches_per_sweep=hist_n / args.steps,
               hist_gbs=hist_gbs, hist_bytes_per_launch=hist_bytes / max(1, hist_n),
               hist_avg_launch_ms=hist_ms / max(1, hist_n),
               evaluations_rank0=per_rank[0]["evaluations"], r_percent=[round(100 * x, 6) for x in r],
               saving_rate_percent=[round(100 * 0.08 * x, 5) for x in kty])
    log(f"[bench] table2: {el / args.steps:.3f} s per sweep ({out['value']:.2f} GE solves/s); "
        f"hist kernel {hist_ms / args.steps:.1f} ms per sweep, {hist_gbs:.0f} GB/s algorithmic; "
        f"hist_point_iters={point_iters} hist_launches={hist_n}")
    return out


# ------------------------------------------------------------------------------------
# configs[1]: the reference's KS-form GE solve at 10k x 1M
# ------------------------------------------------------------------------------------
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


def egm_kernel_time(agent, n_launch=20):
    """Average duration of one EGM cycle kernel from the converged policy (HIP events on
    its stream, aiy_egm_kernel_time; its row hints set by one untimed launch, as the
    cycle before sets them in a solve)."""
    import torch
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


def configs1_leg(args, world, rank, dev):
    import torch
    from aiyagari_hark_amd import _lib
    econ, agent = make_economy(seed=rank, n_agents=args.agents, n_a=args.grid, act_T=args.act_T, device=dev)
    stats = dict(egm_s=0.0, panel_s=0.0, ge_iters=0, cycles=0)
    solve_agents, make_history = econ.solve_agents, econ.make_history

    def timed_solve():
        t = time.perf_counter()
        solve_agents()
        torch.cuda.synchronize()
        stats["egm_s"] += time.perf_counter() - t
        stats["cycles"] += agent.completed_cycles + 1

    def timed_hist():
        t = time.perf_counter()
        make_history()
        stats["panel_s"] += time.perf_counter() - t
        stats["ge_iters"] += 1

    def step():
        reset_rule(econ, agent)
        econ.solve_agents, econ.make_history = timed_solve, timed_hist
        try:
            econ.solve()
        finally:
            econ.solve_agents, econ.make_history = solve_agents, make_history

    step()   # warm-up
    for k in stats:
        stats[k] = 0 if isinstance(stats[k], int) else 0.0
    h = _lib.handle(dev.index)
    h.check(h.lib.aiy_panel_launch_stats(h.h, None, None, None, 1), "stats reset")
    n_steps = max(1, args.c1_steps)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(n_steps):
        step()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    st_ms, st_n, st_per = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    h.check(h.lib.aiy_panel_launch_stats(h.h, ctypes.byref(st_ms), ctypes.byref(st_n), ctypes.byref(st_per), 1),
            "stats")
    sow = econ.sow_state
    K = float(np.mean(econ.reap_state["aNow"][0]))
    n_ge = stats["ge_iters"] / n_steps
    cyc = stats["cycles"] / max(1, stats["ge_iters"])
    t_launch_ms = st_ms.value / max(1, st_n.value)
    per_launch = st_per.value / max(1, st_n.value)
    panel_bytes = PANEL_BYTES_PER_AGENT * args.agents * per_launch
    panel_gbs = panel_bytes / max(1e-12, t_launch_ms * 1e-3) / 1e9
    t_egm_ms = egm_kernel_time(agent)
    egm_bytes = 32 * 28 * 15 * (args.grid + 1)
    egm_gbs = egm_bytes / (t_egm_ms * 1e-3) / 1e9
    out = dict(value=world * n_steps / el, unit="GE solves/s", steps=n_steps, seconds=el,
               agent_periods_per_sec=world * n_steps * n_ge * args.act_T * args.agents / el,
               ge_iterations_per_solve=n_ge, egm_cycles_per_ge_iteration=cyc,
               time_share={"panel": stats["panel_s"] / max(1e-9, stats["panel_s"] + stats["egm_s"]),
                           "egm": stats["egm_s"] / max(1e-9, stats["panel_s"] + stats["egm_s"])},
               result={"r": sow["Rnow"] - 1.0, "K_over_Y": K / (sow["Mnow"] - (1 - econ.DeprFac) * K),
                       "note": "the reference's market tolerance 0.01 stops this 1M-agent economy after 5 GE "
                               "iterations; at tolerance 1e-4 the same fixed point gives r = 4.092 % "
                               "(profiles/r02a_ks_tolerance_probe.jsonl, DESIGN.md §7)"},
               roofline={"kernel": "sim_resident_kernel", "bound": "hbm", "achieved": panel_gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": panel_gbs / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("sim_resident_kernel"), "algorithmic_bytes_per_launch": panel_bytes,
                         "avg_launch_ms": t_launch_ms, "us_per_period": 1e3 * t_launch_ms / max(1.0, per_launch),
                         "launch": f"one history: {per_launch:.0f} periods x {args.agents} agents",
                         "launches_timed": st_n.value},
               roofline_egm={"kernel": "egm_cycle_kernel", "bound": "hbm", "achieved": egm_gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": egm_gbs / HBM_PEAK_GBS, "traffic": pmc_traffic("egm_cycle_kernel"),
                             "algorithmic_bytes_per_launch": egm_bytes, "avg_launch_ms": t_egm_ms},
               workload="BASELINE configs[1]: KS-form Aiyagari GE (Aiyagari-HARK.py:249), 28 states x 15 M nodes x "
                        f"{args.grid}-pt grid, {args.agents} agents x {args.act_T} periods per GE iteration, Philox "
                        "labour shocks; one independent economy per GPU (weak)")
    log(f"[bench] configs1: {el / n_steps:.3f} s per GE solve; panel {1e3 * t_launch_ms / max(1.0, per_launch):.1f} "
        f"us/period ({panel_gbs:.0f} GB/s), egm {t_egm_ms * 1e3:.1f} us ({egm_gbs:.0f} GB/s)")
    return out, econ, agent


# ------------------------------------------------------------------------------------
# configs[3]: 1e8 agents x 1000 periods, agent-sharded, per-period RCCL all-reduce
# ------------------------------------------------------------------------------------
def configs3_leg(args, world, rank, dev, econ, agent):
    import torch
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.panel import DevicePanel
    from aiyagari_hark_amd.parallel import bind_rccl, initial_labor_states, shard_range, unbind_rccl
    h = _lib.handle(dev.index)
    n_total = args.c3_agents
    T = args.c3_periods
    off, nl = shard_range(n_total, world, rank)
    # the policy every rank simulates: the converged configs[1] household at the reference's
    # initial saving rule (deterministic, identical on every rank)
    reset_rule(econ, agent)
    agent.solve()
    sol = agent.solution[0]
    lab_level = torch.as_tensor(sm.labor_levels(agent.TauchenAux[0])).to(dev)
    lab_cdf = torch.as_tensor(sm.choice_cdf_table(agent.TauchenAux[1])).to(dev)
    hist = np.resize(np.asarray(econ.MrkvNow_hist, dtype=np.int32), T + 64)
    if world > 1:
        bind_rccl(h)
    try:
        p = DevicePanel(nl, device=dev, agent_offset=off, n_total=n_total, act_T=T + 64, engine="grid")
        p.bind_model(sol.m_tab, sol.c_tab, sol.M_grid, lab_level, lab_cdf, torch.as_tensor(hist).to(dev),
                     econ.market_constants())
        lab0 = initial_labor_states(n_total, 7, off, nl)

        def reset():
            p.reset(econ.KSS, lab0, econ.sow_init["Mnow"], econ.sow_init["Aprev"], 0, econ.sow_init["Rnow"],
                    econ.sow_init["Wnow"])

        reset()
        p.run(0, 64, shock_mode="philox", seed=11, ge_iter=0)   # warm-up
        reset()
        h.check(h.lib.aiy_panel_launch_stats(h.h, None, None, None, 1), "stats reset")
        barrier(world)
        t0 = time.perf_counter()
        p.run(0, T, shock_mode="philox", seed=11, ge_iter=0)
        barrier(world)
        el = max_over_ranks(time.perf_counter() - t0, world, dev)
        st_ms, st_n, st_per = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        h.check(h.lib.aiy_panel_launch_stats(h.h, ctypes.byref(st_ms), ctypes.byref(st_n), ctypes.byref(st_per), 1),
                "stats")
        K_T = float(p.hist_A[T - 1].item())
    finally:
        if world > 1:
            unbind_rccl(h)
    aps = n_total * T / el
    # dominant kernel: single rank -> the persistent panel streaming agents from HBM (HIP
    # events around the launch); sharded -> per-period kernel + RCCL all-reduce + price
    # kernel, timed on the wall clock of the whole period
    if world == 1 and st_n.value > 0:
        kern_ms = st_ms.value / st_n.value
        kern = "sim_resident_kernel (HBM-streaming form)"
    else:
        kern_ms = 1e3 * el
        kern = "sim_period_kernel + ncclAllReduce + period_price_kernel (wall clock of the periods)"
    bytes_launch = PANEL_BYTES_PER_AGENT * nl * T
    gbs = bytes_launch / max(1e-12, kern_ms * 1e-3) / 1e9
    out = dict(value=aps, unit="agent-periods/s", agents=n_total, periods=T, seconds=el, agents_per_rank=nl,
               us_per_period=1e6 * el / T, K_final=K_T,
               roofline={"kernel": kern, "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": bytes_launch,
                         "avg_launch_ms": kern_ms},
               workload=f"BASELINE configs[3]: {n_total} agents x {T} periods, agents sharded over {world} rank(s), "
                        "Philox by global agent index, per-period RCCL all-reduce of the asset sum when sharded")
    log(f"[bench] configs3: {el:.3f} s for {T} periods ({aps:.3e} agent-periods/s, {1e6 * el / T:.0f} us/period)")
    return out


# ------------------------------------------------------------------------------------
# configs[2] in the reference's own algorithm
# ------------------------------------------------------------------------------------
def table2_reference_leg(world, rank, dev, agents=350):
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
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    return {"value": len(cells) / el, "unit": "GE solves/s", "seconds": el, "calibrations": len(cells),
            "per_rank": len(mine), "agents": agents, "act_T": 11000, "ge_iterations_rank0": list(loops),
            "workload": "configs[2] Table II, reference algorithm: KS-form GE per cell, notebook grids, "
                        "one EconomyBatch per rank"}


def pmc_traffic(kernel, scale=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE
    passes of this bench, FETCH doubled per MI355X_MICROARCH.md), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))[kernel]
        if scale is not None and "hbm_bytes_per_point_iter" in d:
            return float(d["hbm_bytes_per_point_iter"]) * scale
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


# ------------------------------------------------------------------------------------
# CPU baseline: the oracle on this host (bounded sample of the headline workload)
# ------------------------------------------------------------------------------------
def _cpu_eval(args_tuple):
    """One complete K_s(r) evaluation (EGM to 1e-8 + lottery + distribution to 1e-12) of
    one Table II calibration at N_a = 10 000 with the vectorised NumPy oracle."""
    rho, sig, mu, r, n_a = args_tuple
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import stationary as ST
    aGrid = ST.make_stationary_grid(0.001, 50.0, n_a, 2)
    lab, P = ST.income_process(7, rho, sig, "tauchen")
    t = time.perf_counter()
    K, info = ST.capital_supply(r, dict(DiscFac=0.96, CRRA=mu, CapShare=0.36, DeprFac=0.08), aGrid, lab, P, fast=True)
    return time.perf_counter() - t, info["cycles"], info["hist_iters"]


def host_info():
    model = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return model, os.cpu_count(), usable


def cpu_baseline(n_a, r_star, budget_workers=16):
    """The oracle (oracle/stationary.py, vectorised NumPy: np.bincount lottery push, one
    thread) on this host, on complete units of the headline workload: K_s(r) evaluations of
    Table II calibrations at N_a = 10 000 (EGM to 1e-8, Young lottery to 1e-12).  A CPU GE
    solve is the oracle's own bisection: 20 evaluations of the bracket [-delta/2,
    1/beta - 1) to 1e-7, of which the first three lie far below the root (fast: the
    distribution converges quickly) and the other 17 within ~0.5 % of it (slow).  Single
    core, rho = 0.6 / sigma = 0.2 / CRRA = 1 cell (root r* from the GPU sweep): one
    evaluation at r* - 2 % for the far steps and three at r* - 0.25 %, r* - 0.03 %,
    r* + 0.005 % for the near ones; GE solve time = 3 t_far + 17 mean(t_near).  All cores:
    one near-root evaluation (r* - 0.03 %) of each of min(usable cores, 24) cells at once in
    a process pool, GE solves/s = cells / (20 x wall)."""
    import multiprocessing as mp
    model, n_cpu, usable = host_info()
    rs = r_star[6]   # the (0.6, 0.2, 1) cell
    far = _cpu_eval((0.6, 0.2, 1.0, rs - 0.02, n_a))
    near = [_cpu_eval((0.6, 0.2, 1.0, rs + dr, n_a)) for dr in (-0.0025, -0.0003, 0.00005)]
    t_ge = 3 * far[0] + 17 * float(np.mean([o[0] for o in near]))
    from aiyagari_hark_amd.stationary import table2_calibrations
    cells = table2_calibrations()
    workers = max(1, min(budget_workers, usable, len(cells)))
    jobs = [(c.LaborAR, c.LaborSD, c.CRRA, r_star[k] - 0.0003, n_a) for k, c in enumerate(cells[:workers])]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_cpu_eval, jobs)
    all_wall = time.perf_counter() - t0
    return {"value": 1.0 / t_ge, "unit": "GE solves/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/stationary.py (vectorised NumPy, one thread, OMP_NUM_THREADS=1) on this host: 4 "
                       f"complete K_s(r) evaluations of the rho=0.6 sigma=0.2 CRRA=1 Table II cell at N_a={n_a}: "
                       f"r*-2% {far[0]:.2f} s, near-root {[round(o[0], 2) for o in near]} s (histogram iterations "
                       f"{[far[2]] + [o[2] for o in near]}); GE solve = the oracle's 20 bisection evaluations "
                       f"(3 far + 17 near) = {t_ge:.1f} s"),
            "host": {"cpu_model": model, "nproc": n_cpu, "usable_cores": usable,
                     "threads": os.environ.get("OMP_NUM_THREADS", "unset")},
            "all_cores": {"value": workers / (20 * all_wall), "unit": "GE solves/s", "cores": workers,
                          "kind": "port",
                          "sample": f"{workers} Table II cells, one near-root K_s evaluation each (r* - 0.03 %), one "
                                    f"process per core: {all_wall:.2f} s wall (per cell {min(x[0] for x in res):.2f}-"
                                    f"{max(x[0] for x in res):.2f} s); GE solves/s = cells / (20 x wall)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--grid", type=int, default=N_A)
    ap.add_argument("--agents", type=int, default=N_AGENTS)
    ap.add_argument("--act-T", type=int, default=ACT_T)
    ap.add_argument("--c1-steps", type=int, default=1)
    ap.add_argument("--c3-agents", type=int, default=N_AGENTS_C3)
    ap.add_argument("--c3-periods", type=int, default=T_C3)
    ap.add_argument("--legs", default="table2,configs1,configs3,table2_reference")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)

    import torch
    world, rank, local = setup_dist()
    if args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting n_gpus={world}")
    dev = torch.device("cuda", local)
    from aiyagari_hark_amd import build
    if rank == 0:
        build.build(verbose=False)
    barrier(world)
    legs = set(args.legs.split(","))
    t2 = table2_leg(args, world, rank, dev)
    line = {
        "metric": "GE solves/sec (Table II sweep); agent-periods/sec; % HBM roofline",
        "value": t2["value"],
        "unit": "GE solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t2["seconds_per_sweep"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: Aiyagari (1994) Table II calibrations, no shocks drawn (stationary distribution)",
        "config": {"workload": "BASELINE configs[2]: Table II sweep, 24 calibrations (rho x sigma x CRRA), stationary "
                               f"Aiyagari GE in r (Brent on K_s = K_d), {args.grid}-pt asset grid, 7-state Tauchen, "
                               "Young-lottery stationary distribution; one step = the whole sweep",
                   "calibrations": N_TABLE2, "n_a": args.grid, "S": 7,
                   "parallelism": f"calibrations split round-robin over {world} GPU(s), no data-path collective; "
                                  "per GPU 3 independent root searches (own handle, stream, host thread)"},
        "roofline": {"kernel": "hist_bicg_kernel (device-resident BiCGSTAB solve of the Young-lottery "
                               "stationary distribution)", "bound": "hbm",
                     "achieved": t2["hist_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": t2["hist_gbs"] / HBM_PEAK_GBS,
                     "traffic": pmc_traffic("hist_bicg_kernel",
                                            scale=t2["hist_bytes_per_launch"] / HIST_BYTES_PER_POINT_KRYLOV),
                     "algorithmic_bytes_per_launch": t2["hist_bytes_per_launch"],
                     "avg_launch_ms": t2["hist_avg_launch_ms"],
                     "launch": "one K_s(r) evaluation of the rank's calibrations: every matvec of the solve "
                               "(52 B per state x node point per matvec: 28 B lottery push + mix, 24 B iterate "
                               "updates)",
                     "kernel_time_share": t2["hist_kernel_ms_per_sweep"] / (1e3 * t2["seconds_per_sweep"])},
        "table2": {k: t2[k] for k in ("seconds_per_sweep", "evaluations_rank0", "hist_launches_per_sweep",
                                      "hist_kernel_ms_per_sweep", "r_percent", "saving_rate_percent")},
        "cpu_baseline": None,
    }
    if "configs1" in legs or "configs3" in legs:
        c1, econ, agent = configs1_leg(args, world, rank, dev)
        if "configs1" in legs:
            line["configs1"] = c1
        if "configs3" in legs:
            line["configs3"] = configs3_leg(args, world, rank, dev, econ, agent)
    if "table2_reference" in legs:
        line["table2_reference"] = table2_reference_leg(world, rank, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.grid, [x / 100.0 for x in t2["r_percent"]])
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
