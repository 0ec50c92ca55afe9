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
EGM_BYTES_PER_NODE_CYCLE = 32  # SURVEY.md §8d stationary EGM: read (m, c) next + write (m, c) new per node
N_AGENTS = 1_000_006           # nearest multiple of 7 >= 1e6
N_AGENTS_C3 = 99_999_998       # 1e8 agents, multiple of 7
T_C3 = 1000
N_A = 10_000
ACT_T = 11_000
T_DISCARD = 1_000
N_TABLE2 = 24
# kernel templates the legs' dominant launches are expected to use (PMC entries are matched
# on them: a template the library no longer launches has no traffic figure)
C1_PANEL_TEMPLATE = "sim_resident_kernel<512, 8, true, true"
# configs[1]'s LDS-resident panel is not bound by HBM (its agents live in LDS; PMC traffic 0.40x
# the 18 B per agent-period): its bound is the latency of the per-period work.  Floor: the
# diagnostic build without the table lookups (draws, the partial-sum exchange, prices, the
# asset update) at 6.2 us per period (tools/panel_variants.py, profiles/r02s_panel_variants.jsonl)
C1_NO_LOOKUP_FLOOR_US = 6.2
C3_PANEL_TEMPLATE = "sim_resident_kernel<1024, 4, false, true"
EGM_C1_TEMPLATE = "egm_cycle_kernel<32, 28, false, 2"
C4_TEMPLATE = "hist_pull_kernel<32, 512"
N_TABLE2_CPU_CELL = 6          # (rho 0.6, sigma 0.2, CRRA 1) in stationary.table2_calibrations() order


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


def setup_dist(backend="nccl"):
    """One rank per GPU over RCCL ("nccl").  backend "gloo" is the one-GPU rehearsal of
    the multi-rank bench: every rank on device 0 (LOCAL_RANK modulo the visible devices),
    the rendezvous and the collectives over gloo, configs3's per-period sum through the
    library's two-step sharded period (RCCL refuses two ranks on one device)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def cu_share(world):
    """Fraction of the GPU one rank's resident clusters may hold: 1, or 1 / ranks when the
    gloo rehearsal puts every rank on one device."""
    if world > 1:
        import torch
        import torch.distributed as dist
        if dist.get_backend() == "gloo":
            return 1.0 / max(1, -(-world // max(1, torch.cuda.device_count())))
    return 1.0


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
    on_dev = dist.get_backend() != "gloo"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(obj, world):
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def ge_stats(h, reset, dev=None):
    """Device-resident GE launches (csrc/ge_resident.hip) since the last reset, summed over
    the device's handles: (kernel ms by HIP events, launches, point-matvecs, EGM cycles)."""
    from aiyagari_hark_amd import stationary
    hs = [h] + [hg for (d, _), (hg, _) in stationary._GROUP_CTX.items() if dev is None or d == dev.index]
    tot = [0.0, 0, 0.0, 0.0]
    for hh in hs:
        ms, n, pts, cyc = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        hh.check(hh.lib.aiy_ge_launch_stats(hh.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(pts),
                                            ctypes.byref(cyc), int(reset)), "ge stats")
        tot = [tot[0] + ms.value, tot[1] + n.value, tot[2] + pts.value, tot[3] + cyc.value]
    return tuple(tot)


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

    share = cu_share(world)

    def sweep():
        return solve_table2(cals, n_a=args.grid, device=dev, method="brent", cu_share=share)

    for _ in range(0 if PMC_PASS else args.warmup):
        sweep()
    hist_stats(h, True, dev)
    ge_stats(h, True, dev)
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
    ge_ms, ge_n, ge_pts, ge_cyc = ge_stats(h, True, dev)
    if ge_n > 0:
        # dominant kernel: the device-resident GE search (one launch per sweep): algorithmic
        # bytes = 52 per (state, node) point per matvec of the distribution solves + 32 S
        # (N_a + 1) per calibration and EGM cycle
        kern = "ge_cluster_kernel (device-resident GE search: EGM cycles + lottery + BiCGSTAB + root search)"
        hist_bytes = HIST_BYTES_PER_POINT_KRYLOV * ge_pts + EGM_BYTES_PER_NODE_CYCLE * 7 * (args.grid + 1) * ge_cyc
        # the same launches in SURVEY.md §8d's own units: 28 B per point-iteration of the
        # histogram (no iterate updates counted) + 32 B per (state, node) per EGM cycle
        s8d_bytes = HIST_BYTES_PER_POINT * ge_pts + EGM_BYTES_PER_NODE_CYCLE * 7 * (args.grid + 1) * ge_cyc
        hist_ms, hist_n = ge_ms, ge_n
    else:
        # dominant kernel: the device-resident BiCGSTAB distribution solve (one launch per
        # K_s(r) evaluation); algorithmic bytes 52 per (state, node) point per matvec
        kern = "hist_bicg_kernel (device-resident BiCGSTAB solve of the Young-lottery stationary distribution)"
        hist_bytes = HIST_BYTES_PER_POINT_KRYLOV * point_iters
        s8d_bytes = HIST_BYTES_PER_POINT * point_iters
    if ge_n > 0:
        alg_record("table2", "ge_cluster_kernel<7, 7, ", launches=ge_n, alg_bytes=hist_bytes,
                   note="52 B per point-matvec + 32 B per (state, node) per EGM cycle")
    hist_gbs = hist_bytes / max(1e-12, hist_ms * 1e-3) / 1e9
    s8d_gbs = s8d_bytes / max(1e-12, hist_ms * 1e-3) / 1e9
    per_rank = gather_objects(dict(cells=mine, r=[float(x) for x in res.r], KtoY=[float(x) for x in res.KtoY],
                                   evaluations=res.bisection_steps), world)
    r = [None] * len(cells)
    kty = [None] * len(cells)
    for pr in per_rank:
        for k, rr, ky in zip(pr["cells"], pr["r"], pr["KtoY"]):
            r[k], kty[k] = rr, ky
    out = dict(seconds_per_sweep=el / args.steps, value=len(cells) * args.steps / el, kernel=kern,
               resident=ge_n > 0, egm_cycles_per_sweep=ge_cyc / args.steps if ge_n else None,
               hist_kernel_ms_per_sweep=hist_ms / args.steps, hist_launches_per_sweep=hist_n / args.steps,
               hist_gbs=hist_gbs, hist_bytes_per_launch=hist_bytes / max(1, hist_n), s8d_gbs=s8d_gbs,
               s8d_bytes_per_launch=s8d_bytes / max(1, hist_n),
               hist_avg_launch_ms=hist_ms / max(1, hist_n),
               evaluations_rank0=per_rank[0]["evaluations"], r_percent=[round(100 * x, 5) for x in r],
               saving_rate_percent=[round(100 * 0.08 * x, 4) for x in kty],
               r_note="r_percent rounded to the root search's tolerance (r_tol = 1e-7: 1e-5 percentage points); "
                      "digits below it follow the rebalancing stop points, which follow the wall clock "
                      "(DESIGN.md §4e); with AIY_OPT_GE_REBALANCE = 0 a sweep is bit-reproducible")
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

    if not PMC_PASS:
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
    us_per_period = 1e3 * t_launch_ms / max(1.0, per_launch)
    t_egm_ms = egm_kernel_time(agent)
    egm_bytes = 32 * 28 * 15 * (args.grid + 1)
    egm_gbs = egm_bytes / (t_egm_ms * 1e-3) / 1e9
    alg_record("configs1", C1_PANEL_TEMPLATE, launches=st_n.value, alg_bytes=panel_bytes * st_n.value,
               units=st_per.value * args.agents, unit_name="agent-period", alg_bytes_per_unit=PANEL_BYTES_PER_AGENT,
               note="18 B per agent-period")
    alg_record("configs1", EGM_C1_TEMPLATE, alg_bytes_per_launch=egm_bytes,
               note="32 B per (state, M node, asset node) per cycle; working launches")
    p_traffic, p_info = pmc_traffic(C1_PANEL_TEMPLATE, panel_bytes)
    e_traffic, e_info = pmc_traffic(EGM_C1_TEMPLATE, egm_bytes)
    out = dict(value=world * n_steps / el, unit="GE solves/s", steps=n_steps, seconds=el,
               agent_periods_per_sec=world * n_steps * n_ge * args.act_T * args.agents / el,
               ge_iterations_per_solve=n_ge, egm_cycles_per_ge_iteration=cyc,
               time_share={"panel": stats["panel_s"] / max(1e-9, stats["panel_s"] + stats["egm_s"]),
                           "egm": stats["egm_s"] / max(1e-9, stats["panel_s"] + stats["egm_s"])},
               result={"r": sow["Rnow"] - 1.0, "K_over_Y": K / (sow["Mnow"] - (1 - econ.DeprFac) * K),
                       "note": "the reference's market tolerance 0.01 stops this 1M-agent economy after 5 GE "
                               "iterations; at tolerance 1e-4 the same fixed point gives r = 4.092 % "
                               "(profiles/r02a_ks_tolerance_probe.jsonl, DESIGN.md §7)"},
               roofline={"kernel": C1_PANEL_TEMPLATE + ">", "bound": "latency", "unit": "us/period",
                         "achieved": us_per_period, "peak": C1_NO_LOOKUP_FLOOR_US,
                         "frac": C1_NO_LOOKUP_FLOOR_US / max(1e-9, us_per_period),
                         "bound_note": "agents resident in LDS (PMC traffic well below the 18 B per agent-period): "
                                       "bound by the per-period latency chain, not HBM; peak = the no-lookup "
                                       "diagnostic floor (every step of a period but the table lookups, "
                                       "profiles/r02s_panel_variants.jsonl); frac = floor / achieved",
                         "traffic": p_traffic, **p_info, "algorithmic_bytes_per_launch": panel_bytes,
                         "avg_launch_ms": t_launch_ms, "us_per_period": us_per_period,
                         "launch": f"one history: {per_launch:.0f} periods x {args.agents} agents",
                         "launches_timed": st_n.value,
                         "hbm_units": {"achieved": panel_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": panel_gbs / HBM_PEAK_GBS,
                                       "note": "18 B per agent-period (SURVEY.md §8d) / kernel time"}},
               roofline_egm={"kernel": EGM_C1_TEMPLATE + ">", "bound": "hbm", "achieved": egm_gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": egm_gbs / HBM_PEAK_GBS, "traffic": e_traffic, **e_info,
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
def c3_policy(dev, n_a, n_agents=N_AGENTS):
    """The household every configs[3] rank simulates: the configs[1] economy's converged
    policy at the reference's initial saving rule (intercept 0, slope 1; [HARK] solve_agent
    to 1e-6 from the terminal guess) -- deterministic, identical on every rank.  Returns
    (econ, agent) with agent.solution[0] set."""
    econ, agent = make_economy(seed=0, n_agents=n_agents, n_a=n_a, act_T=ACT_T, device=dev)
    reset_rule(econ, agent)
    agent.solve()
    return econ, agent


def c3_panel(dev, econ, agent, n_total, T, world=1, rank=0):
    """The configs[3] panel of this rank: contiguous agent range, labour states split
    evenly by global index (parallel.initial_labor_states), a_0 = KSS, Philox keyed by
    the global agent index.  Returns (panel, reset)."""
    import torch
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.panel import DevicePanel
    from aiyagari_hark_amd.parallel import initial_labor_states, shard_range
    off, nl = shard_range(n_total, world, rank)
    sol = agent.solution[0]
    lab_level = torch.as_tensor(sm.labor_levels(agent.TauchenAux[0])).to(dev)
    lab_cdf = torch.as_tensor(sm.choice_cdf_table(agent.TauchenAux[1])).to(dev)
    hist = np.resize(np.asarray(econ.MrkvNow_hist, dtype=np.int32), T + 64)
    p = DevicePanel(nl, device=dev, agent_offset=off, n_total=n_total, act_T=T + 64, engine="grid")
    p.bind_model(sol.m_tab, sol.c_tab, sol.M_grid, lab_level, lab_cdf, torch.as_tensor(hist).to(dev),
                 econ.market_constants())
    lab0 = initial_labor_states(n_total, 7, off, nl)

    def reset():
        p.reset(econ.KSS, lab0, econ.sow_init["Mnow"], econ.sow_init["Aprev"], 0, econ.sow_init["Rnow"],
                econ.sow_init["Wnow"])

    reset()
    return p, reset


C3_SEED = 11


def configs3_leg(args, world, rank, dev):
    import torch.distributed as dist
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.parallel import bind_rccl, torch_allreduce, unbind_rccl
    h = _lib.handle(dev.index)
    n_total = args.c3_agents
    T = args.c3_periods
    econ, agent = c3_policy(dev, args.grid)
    # sharded: the library's own RCCL all-reduce (nccl backend) or, in the one-GPU gloo
    # rehearsal, the two-step period with the caller's all-reduce
    gloo = world > 1 and dist.get_backend() == "gloo"
    allreduce = torch_allreduce() if gloo else None
    comm = None
    if world > 1 and not gloo:
        # torch's own RCCL communicator when it exposes one (one communicator per device),
        # else the library's
        comm = bind_rccl(h)[2]
    try:
        p, reset = c3_panel(dev, econ, agent, n_total, T, world, rank)
        if not PMC_PASS:
            p.run(0, 64, shock_mode="philox", seed=C3_SEED, ge_iter=0, allreduce=allreduce)   # warm-up
            reset()
        h.check(h.lib.aiy_panel_launch_stats(h.h, None, None, None, 1), "stats reset")
        barrier(world)
        t0 = time.perf_counter()
        p.run(0, T, shock_mode="philox", seed=C3_SEED, ge_iter=0, allreduce=allreduce)
        barrier(world)
        el = max_over_ranks(time.perf_counter() - t0, world, dev)
        st_ms, st_n, st_per = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        h.check(h.lib.aiy_panel_launch_stats(h.h, ctypes.byref(st_ms), ctypes.byref(st_n), ctypes.byref(st_per), 1),
                "stats")
        K_hist = p.hist_A[:T].cpu().numpy()
        nl = p.n_local
    finally:
        if world > 1 and not gloo:
            unbind_rccl(h)
    aps = n_total * T / el
    # dominant kernel: single rank -> the persistent panel streaming agents from HBM (HIP
    # events around the launch); sharded -> per-period kernel + all-reduce + price kernel,
    # timed on the wall clock of the whole period
    if world == 1 and st_n.value > 0:
        kern_ms = st_ms.value / st_n.value
        kern = "sim_resident_kernel (HBM-streaming form)"
    else:
        kern_ms = 1e3 * el
        kern = ("sim_period_kernel + " + ("gloo all-reduce (two-step period)" if gloo else "ncclAllReduce") +
                " + period_price_kernel (wall clock of the periods)")
    bytes_launch = PANEL_BYTES_PER_AGENT * nl * T
    gbs = bytes_launch / max(1e-12, kern_ms * 1e-3) / 1e9
    traffic, t_info = None, {"traffic_note": "sharded: per-period kernels + all-reduce, not profiled"}
    if world == 1:
        alg_record("configs3", C3_PANEL_TEMPLATE, launches=st_n.value, alg_bytes=bytes_launch * max(1, st_n.value),
                   units=nl * T * max(1, st_n.value), unit_name="agent-period", alg_bytes_per_unit=PANEL_BYTES_PER_AGENT,
                   note="18 B per agent-period")
        traffic, t_info = pmc_traffic(C3_PANEL_TEMPLATE, bytes_launch)
    out = dict(value=aps, unit="agent-periods/s", agents=n_total, periods=T, seconds=el, agents_per_rank=nl,
               us_per_period=1e6 * el / T, K_final=float(K_hist[T - 1]), K_first=[float(x) for x in K_hist[:5]],
               roofline={"kernel": kern, "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS,
                         "traffic": traffic, **t_info,
                         "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": kern_ms},
               communicator=comm,
               workload=f"BASELINE configs[3]: {n_total} agents x {T} periods, agents sharded over {world} rank(s), "
                        "Philox by global agent index, per-period all-reduce of the asset sum when sharded "
                        f"({'gloo two-step rehearsal' if gloo else 'RCCL'})")
    log(f"[bench] configs3: {el:.3f} s for {T} periods ({aps:.3e} agent-periods/s, {1e6 * el / T:.0f} us/period)")
    return out


# ------------------------------------------------------------------------------------
# configs[4]: stress -- 25-state Rouwenhorst, 50 000-point grid, Young histogram
# ------------------------------------------------------------------------------------
STRESS_N_A = 50_000


def stress_calibrations():
    from aiyagari_hark_amd.stationary import Calibration
    return [Calibration(LaborAR=0.9, LaborSD=0.4, CRRA=c, LaborStatesNo=25, income="rouwenhorst")
            for c in (1.0, 3.0, 5.0)]


def configs4_leg(args, world, rank, dev):
    """BASELINE configs[4]: rho 0.9, sigma 0.4, CRRA in {1, 3, 5}, 25-state Rouwenhorst
    (E3), N_a = 50 000, each solved to GE in r with the bench's Table II options; the
    three cells split round-robin over the ranks.  Dominant kernel: the 25-state
    BiCGSTAB distribution solve (hist_pull_kernel: 85 workgroups per calibration at three
    cells, the Krylov vectors in HBM).  roofline.frac counts 52 B per point-matvec (the
    units VERDICT r5 set this leg's target in); s8d_units the 28 B of SURVEY.md §8d."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.parallel import split_calibrations
    from aiyagari_hark_amd.stationary import solve_table2
    cells = stress_calibrations()
    mine = split_calibrations(list(range(len(cells))), world, rank)
    cals = [cells[k] for k in mine]
    h = _lib.handle(dev.index)
    n_a = args.stress_grid

    share = cu_share(world)

    def solve():
        return solve_table2(cals, n_a=n_a, device=dev, method="brent", cu_share=share) if cals else None

    if not PMC_PASS:
        solve()   # warm-up
    hist_stats(h, True, dev)
    barrier(world)
    t0 = time.perf_counter()
    res = solve()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    hist_ms, hist_n = hist_stats(h, True, dev)
    # the host-driven loop (S > 8): the pull-form distribution solve is the dominant kernel
    kern = "hist_pull_kernel<32, 512> (pull-form BiCGSTAB distribution solve, Krylov vectors in HBM)"
    pts = sum(int(np.sum(it)) for it in res.hist_iters) * 25 * n_a if res is not None else 0
    hist_bytes = HIST_BYTES_PER_POINT_KRYLOV * pts
    gbs = hist_bytes / max(1e-12, hist_ms * 1e-3) / 1e9
    alg_record("configs4", C4_TEMPLATE, launches=hist_n, alg_bytes=hist_bytes,
               note="52 B per point-matvec of the pull-form BiCGSTAB solves")
    traffic, t_info = pmc_traffic(C4_TEMPLATE, hist_bytes / max(1, hist_n))
    per_rank = gather_objects(dict(cells=mine, r=[] if res is None else [float(x) for x in res.r],
                                   status=[] if res is None else [int(x) for x in res.status]), world)
    r = [None] * len(cells)
    st = [None] * len(cells)
    for pr in per_rank:
        for k, rr, ss in zip(pr["cells"], pr["r"], pr["status"]):
            r[k], st[k] = rr, ss
    out = dict(value=len(cells) / el, unit="GE solves/s", seconds=el, calibrations=len(cells), n_a=n_a, S=25,
               r_percent=[round(100 * x, 5) for x in r], status=st,
               roofline={"kernel": kern,
                         "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS,
                         "traffic": traffic, **t_info,
                         "algorithmic_bytes_per_launch": hist_bytes / max(1, hist_n),
                         "avg_launch_ms": hist_ms / max(1, hist_n), "launches": hist_n,
                         "kernel_time_share": hist_ms * 1e-3 / max(1e-12, el),
                         "bytes_per_point_matvec": HIST_BYTES_PER_POINT_KRYLOV,
                         "s8d_units": {"achieved": gbs * HIST_BYTES_PER_POINT / HIST_BYTES_PER_POINT_KRYLOV,
                                       "frac": gbs * HIST_BYTES_PER_POINT / HIST_BYTES_PER_POINT_KRYLOV / HBM_PEAK_GBS,
                                       "note": "28 B per state x node point per matvec (SURVEY.md §8d)"}},
               workload="BASELINE configs[4]: rho 0.9, sigma 0.4, CRRA {1,3,5}, 25-state Rouwenhorst, N_a = "
                        f"{n_a}, stationary GE in r (Brent, the Table II options), Young histogram by BiCGSTAB")
    log(f"[bench] configs4: {el:.3f} s for {len(cells)} stress cells ({out['value']:.2f} GE solves/s); "
        f"hist {hist_ms:.1f} ms in {hist_n} launches, {gbs:.0f} GB/s algorithmic")
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


PMC_PASS = False   # --pmc-pass: timed work only, [bench-alg] records for tools/pmc_traffic.py


def alg_record(leg, template, **kw):
    """One [bench-alg] line (stderr) for the PMC passes: the kernel template this leg expects
    the library to launch and its algorithmic bytes over the leg's launches."""
    if PMC_PASS:
        log("[bench-alg] " + json.dumps(dict(leg=leg, template=template, **kw)))


def pmc_traffic(template, alg_bytes_per_launch):
    """HBM traffic per launch of `template` from profiles/pmc_traffic.json (rocprofv3
    FETCH_SIZE x2 + WRITE_SIZE passes of bench.py --pmc-pass, tools/pmc_traffic.py): the
    pass's HBM bytes per algorithmic byte of the same launches x this run's algorithmic bytes
    per launch.  Returns (bytes or None, details): None when no pass profiled this exact
    template, or when the library's sources changed since the pass (source digest)."""
    from aiyagari_hark_amd import build
    try:
        doc = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return None, {"traffic_note": "profiles/pmc_traffic.json missing"}
    e = doc.get(template)
    if e is None:
        return None, {"traffic_note": f"no PMC pass of {template}"}
    cur = build.source_digest()
    if e.get("source_digest") != cur:
        return None, {"traffic_note": (f"stale: the PMC pass profiled sources {e.get('source_digest')} (head "
                                       f"{e.get('git_head')}), the library is built from {cur}")}
    info = {"traffic_hbm_per_alg": e["hbm_per_alg"], "traffic_basis": e["basis"],
            "traffic_pass": {"git_head": e["git_head"], "source_digest": e["source_digest"],
                             "kernels": e["kernels"], "dispatches": e["dispatches"],
                             "hbm_bytes_per_launch_profiled": e["hbm_bytes_per_launch"]}}
    if "hbm_bytes_per_unit" in e:
        info["traffic_per_unit"] = {"unit": e.get("unit_name"), "hbm_bytes": e["hbm_bytes_per_unit"],
                                    "algorithmic_bytes": e.get("alg_bytes_per_unit")}
    return e["hbm_per_alg"] * alg_bytes_per_launch, info


# ------------------------------------------------------------------------------------
# CPU baseline: the oracle on this host (bounded sample of the headline workload)
# ------------------------------------------------------------------------------------
def _cpu_ge_solve(args_tuple):
    """One complete oracle GE solve (oracle/stationary.py ge_bisect: bisection of
    [-delta/2, 1/beta - 1) to 1e-7, every evaluation a cold EGM to 1e-8 and a cold Young
    histogram to 1e-12 from the uniform mass) of one Table II calibration."""
    rho, sig, mu, n_a = args_tuple
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import stationary as ST
    aGrid = ST.make_stationary_grid(0.001, 50.0, n_a, 2)
    lab, P = ST.income_process(7, rho, sig, "tauchen")
    t = time.perf_counter()
    g = ST.ge_bisect(dict(DiscFac=0.96, CRRA=mu, CapShare=0.36, DeprFac=0.08), aGrid, lab, P, r_tol=1e-7, fast=True)
    return time.perf_counter() - t, g["r"], g["iters"]


def _cpu_ks_iteration(agents=350, act_T=ACT_T):
    """One GE iteration of the reference's own algorithm, restated by the oracle
    (oracle/hark_ks.py KSModel: [HARK] solve_agent of the KS-form household on the
    notebook's grids, then Market.make_history over act_T periods of `agents` agents with
    the global-RNG labour draws, Aiyagari_Support.py:1217-1415, 1839-1894) for the
    notebook's calibration (rho 0.3, sigma 0.2, CRRA 1; Aiyagari-HARK.ipynb:292-328)."""
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import hark_ks as H
    cal = dict(LaborAR=0.3, LaborSD=0.2, CRRA=1.0)
    m = H.KSModel(dict(cal), dict(cal, AgentCount=agents))
    t = time.perf_counter()
    mt, ct, cycles, _ = m.solve_agent()
    t1 = time.perf_counter()
    m.make_history(mt, ct, H.numpy_global_u_source(0, agents), ge_iter=0, act_T=act_T)
    t2 = time.perf_counter()
    return t2 - t, t1 - t, t2 - t1, cycles


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


CPU_CELL = (0.6, 0.2, 1.0)   # the BASELINE configs[0] calibration (Aiyagari_Support.py:752-755)


def cpu_baseline(n_a, r_gpu, budget_workers=16, ks_ge_iterations=None):
    """The oracle on this host's cores, timed on complete units of work:
      value     -- one complete oracle GE solve (ge_bisect, 20 cold K_s(r) evaluations)
                   of the configs[0] calibration at the bench's grid, one core
                   (OMP_NUM_THREADS=1);
      all_cores -- the same solve in `workers` processes at once (the GPU box's CPU share
                   per GPU: 16; gpurun caps worker pools there), GE solves/s = workers /
                   wall;
      ks_reference -- one GE iteration of the reference's own Krusell-Smith algorithm
                   (oracle KSModel, 350 agents x 11 000 periods, the notebook's run), one
                   core, beside the GPU's table2_reference leg.
    kind "port": the oracle is a NumPy restatement (HARK is absent)."""
    import multiprocessing as mp
    model, n_cpu, usable = host_info()
    t_one, r_one, steps = _cpu_ge_solve(CPU_CELL + (n_a,))
    workers = max(1, min(budget_workers, usable))
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_cpu_ge_solve, [CPU_CELL + (n_a,)] * workers)
    all_wall = time.perf_counter() - t0
    t_it, t_egm, t_hist, cyc = _cpu_ks_iteration()
    ks = {"value": 1.0 / t_it, "unit": "GE iterations/s", "cores": 1, "kind": "port",
          "sample": (f"oracle/hark_ks.py KSModel, notebook calibration (rho 0.3, sigma 0.2, CRRA 1), 32-pt grid x 15 "
                     f"M nodes x 28 states, 350 agents x {ACT_T} periods: one GE iteration = solve_agent "
                     f"({cyc} cycles, {t_egm:.2f} s) + make_history ({t_hist:.2f} s) = {t_it:.2f} s")}
    if ks_ge_iterations:
        ks["ge_solves_per_s"] = 1.0 / (t_it * float(np.mean(ks_ge_iterations)))
        ks["ge_solves_note"] = (f"x the mean GE iteration count of the GPU table2_reference leg "
                                f"({float(np.mean(ks_ge_iterations)):.1f})")
    return {"value": 1.0 / t_one, "unit": "GE solves/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/stationary.py ge_bisect (vectorised NumPy, OMP_NUM_THREADS=1) of the Table II cell "
                       f"rho={CPU_CELL[0]} sigma={CPU_CELL[1]} CRRA={CPU_CELL[2]} at N_a={n_a}: {steps} cold K_s(r) "
                       f"evaluations, {t_one:.1f} s; r = {100 * r_one:.6f} % (GPU sweep: {100 * r_gpu:.6f} %)"),
            "host": {"cpu_model": model, "nproc": n_cpu, "usable_cores": usable,
                     "threads": os.environ.get("OMP_NUM_THREADS", "unset")},
            "all_cores": {"value": workers / all_wall, "unit": "GE solves/s", "cores": workers, "kind": "port",
                          "sample": (f"{workers} processes, each one complete oracle GE solve of the same cell at "
                                     f"once: {all_wall:.1f} s wall (per solve {min(x[0] for x in res):.1f}-"
                                     f"{max(x[0] for x in res):.1f} s); {workers} = the GPU box's CPU share per GPU "
                                     f"(nproc {n_cpu})")},
            # the whole node: the measured per-process rate x nproc, an extrapolation (the box
            # limits a command to its per-GPU CPU share, so 256 processes are not run here)
            "all_cores_node_estimate": {"value": (workers / all_wall) * n_cpu / workers, "unit": "GE solves/s",
                                        "cores": n_cpu, "kind": "port", "measured": False,
                                        "sample": (f"all_cores' {workers}-process rate scaled to nproc = {n_cpu} "
                                                   "(linear in processes: one solve per process, no shared state)")},
            "ks_reference": ks}


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
    ap.add_argument("--stress-grid", type=int, default=STRESS_N_A)
    ap.add_argument("--legs", default="table2,configs1,configs3,configs4,table2_reference")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: one-GPU rehearsal of the multi-rank run (every rank on device 0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-pass", action="store_true",
                    help="profiling pass (tools/prof_bench.sh): timed work only, [bench-alg] records on stderr")
    ap.add_argument("--hist-pull", type=int, default=None,
                    help="AIY_OPT_HIST_PULL for the Table II / stress distribution solves (default: the library's)")
    ap.add_argument("--ge-rebalance", type=int, default=None,
                    help="AIY_OPT_GE_REBALANCE for the resident searches (default: the library's)")
    ap.add_argument("--ge-anderson", type=int, default=None,
                    help="AIY_OPT_GE_ANDERSON: EGM cycles between Anderson mixes in the resident search (0: off)")
    ap.add_argument("--hist-cluster", type=int, default=None,
                    help="AIY_OPT_HIST_CLUSTER: workgroups per calibration cluster cap (default the library's)")
    ap.add_argument("--ge-loose-hist", type=int, default=None,
                    help="AIY_OPT_GE_LOOSE_HIST (loose-bracketing histogram tolerance 10^-v; default the library's)")
    args = ap.parse_args()
    global PMC_PASS
    PMC_PASS = args.pmc_pass
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)

    import torch
    world, rank, local = setup_dist(args.dist_backend)
    if args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: reporting n_gpus={world}")
    dev = torch.device("cuda", local)
    from aiyagari_hark_amd import build
    if rank == 0:
        build.build(verbose=False)
    barrier(world)
    legs = set(args.legs.split(","))
    if (args.hist_pull is not None or args.ge_rebalance is not None or args.ge_loose_hist is not None or
            args.hist_cluster is not None or args.ge_anderson is not None):
        from aiyagari_hark_amd import _lib
        opts = {}
        if args.hist_pull is not None:
            opts[_lib.AIY_OPT_HIST_PULL] = args.hist_pull
        if args.ge_rebalance is not None:
            opts[_lib.AIY_OPT_GE_REBALANCE] = args.ge_rebalance
        if args.ge_loose_hist is not None:
            opts[_lib.AIY_OPT_GE_LOOSE_HIST] = args.ge_loose_hist
        if args.hist_cluster is not None:
            opts[_lib.AIY_OPT_HIST_CLUSTER] = args.hist_cluster
        if args.ge_anderson is not None:
            opts[_lib.AIY_OPT_GE_ANDERSON] = args.ge_anderson
        _lib.handle(dev.index).set_options(opts)
    t2 = table2_leg(args, world, rank, dev)
    sweep_bytes = t2["hist_bytes_per_launch"] * t2["hist_launches_per_sweep"]
    t2_traffic, t2_info = (pmc_traffic("ge_cluster_kernel<7, 7, ", t2["hist_bytes_per_launch"]) if t2["resident"] else
                           (None, {"traffic_note": "host-driven loop: not profiled"}))
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
                   "parallelism": f"calibrations split round-robin over {world} rank(s), no data-path collective; "
                                  + ("per GPU one device-resident launch, a cluster of workgroups per calibration "
                                     "running its whole root search" if t2["resident"] else
                                     "per GPU 3 independent root searches (own handle, stream, host thread)")},
        # achieved / frac in SURVEY.md §8d's own units (28 B per histogram point per matvec, 32 B
        # per (state, node) per EGM cycle); the same kernel time with the 24 B of
        # BiCGSTAB iterate updates per point-matvec counted too is the secondary krylov_units
        "roofline": {"kernel": t2["kernel"], "bound": "hbm",
                     "achieved": t2["s8d_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": t2["s8d_gbs"] / HBM_PEAK_GBS,
                     "traffic": t2_traffic, **t2_info,
                     "algorithmic_bytes_per_launch": t2["s8d_bytes_per_launch"],
                     "traffic_per_s8d_byte": (t2_traffic / t2["s8d_bytes_per_launch"]
                                              if t2_traffic and t2["s8d_bytes_per_launch"] else None),
                     "avg_launch_ms": t2["hist_avg_launch_ms"],
                     "launch": ("one launch of the device-resident search (a sweep of the rank's calibrations "
                                "runs as a few rebalancing launches, every K_s(r) evaluation of every root search "
                                "in one of them): 28 B per state x node point per matvec of the distribution "
                                "solves (lottery push + mix, SURVEY.md §8d) + 32 B per state x node per EGM "
                                "cycle; traffic: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch of a profiled "
                                "sweep, scaled to this run's launches" if t2["resident"] else
                                "one K_s(r) evaluation of the rank's calibrations: every matvec of the solve "
                                "(28 B per state x node point per matvec, SURVEY.md §8d)"),
                     "kernel_time_share": t2["hist_kernel_ms_per_sweep"] / (1e3 * t2["seconds_per_sweep"]),
                     "krylov_units": {"achieved": t2["hist_gbs"], "frac": t2["hist_gbs"] / HBM_PEAK_GBS,
                                      "algorithmic_bytes_per_launch": t2["hist_bytes_per_launch"],
                                      "note": "52 B per state x node point per matvec (28 B lottery push + mix, 24 B "
                                              "BiCGSTAB iterate updates) + 32 B per state x node per EGM cycle"},
                     # concurrent launches (independent groups) overlap: the device-level rate is the
                     # algorithmic bytes of a whole sweep over the sweep's wall time
                     "device_aggregate": {"achieved": sweep_bytes / t2["seconds_per_sweep"] / 1e9,
                                          "frac": sweep_bytes / t2["seconds_per_sweep"] / 1e9 / HBM_PEAK_GBS,
                                          "note": "algorithmic bytes of all launches of a sweep / sweep wall time"}},
        "table2": {k: t2[k] for k in ("seconds_per_sweep", "evaluations_rank0", "hist_launches_per_sweep",
                                      "hist_kernel_ms_per_sweep", "resident", "egm_cycles_per_sweep", "r_percent",
                                      "saving_rate_percent", "r_note")},
        "cpu_baseline": None,
    }
    if args.dist_backend == "gloo" and world > 1:
        line["rehearsal"] = f"{world} ranks on one GPU (gloo rendezvous and collectives)"
    if "configs1" in legs:
        line["configs1"] = configs1_leg(args, world, rank, dev)[0]
    if "configs3" in legs:
        line["configs3"] = configs3_leg(args, world, rank, dev)
    if "configs4" in legs:
        line["configs4"] = configs4_leg(args, world, rank, dev)
    if "table2_reference" in legs:
        line["table2_reference"] = table2_reference_leg(world, rank, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ks_iters = line.get("table2_reference", {}).get("ge_iterations_rank0")
        line["cpu_baseline"] = cpu_baseline(args.grid, t2["r_percent"][N_TABLE2_CPU_CELL] / 100.0,
                                            ks_ge_iterations=ks_iters)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
