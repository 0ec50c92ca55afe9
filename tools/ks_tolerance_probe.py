#!/usr/bin/env python3
"""Why configs[1]'s KS-form GE reports r = 5.19 %.

Runs the reference's fixed point (Market.solve: damped log-linear saving-rule regression,
AS:1896-1964) for the configs[1] calibration on device at several market tolerances,
grid sizes and populations, and prints one JSON line per run with every GE iteration's
(intercept, slope, r_T) and the saving rule's implied consistency gap at the simulated
steady state: the belief A(M*) against the realised K*.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(n_a, agents, tol, max_loops, act_T=11000, t_discard=1000, seed=0):
    from aiyagari_hark_amd.model import AiyagariEconomy, AiyagariType
    econ = AiyagariEconomy(act_T=act_T, T_discard=t_discard, LaborAR=0.6, LaborSD=0.2, CRRA=1.0,
                           intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0], tolerance=tol)
    econ.verbose = False
    econ.max_loops = max_loops
    agent = AiyagariType(device=torch.device("cuda:0"), shock_mode="philox", shock_seed=seed, LaborAR=0.6,
                         LaborSD=0.2, CRRA=1.0, aCount=n_a, AgentCount=agents)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    t0 = time.perf_counter()
    econ.solve()
    el = time.perf_counter() - t0
    hA = np.asarray(econ.history["Aprev"])
    hM = np.asarray(econ.history["Mnow"])
    Kbar = float(np.mean(hA[t_discard:]))
    Mbar = float(np.mean(hM[t_discard:]))
    belief = [float(np.exp(i + s * np.log(Mbar))) for i, s in zip(econ.intercept_prev, econ.slope_prev)]
    r_mean = 0.36 * Kbar ** (0.36 - 1.0) - 0.08
    return dict(n_a=n_a, agents=agents, tol=tol, ge_iters=len(econ.ge_log), seconds=el,
                r_T=econ.sow_state["Rnow"] - 1.0, r_mean=r_mean, K_mean=Kbar, M_mean=Mbar, belief_A_at_M=belief,
                K_sd=float(np.std(hA[t_discard:])),
                log=[dict(i=g["iter"], icpt=g["intercept"], slope=g["slope"], d=g["distance"], r=g["Rnow"] - 1.0)
                     for g in econ.ge_log])


def main():
    torch.cuda.set_device(0)
    runs = [(10000, 1_000_006, 0.01, 1000), (10000, 1_000_006, 1e-4, 60), (32, 1_000_006, 0.01, 1000),
            (32, 1_000_006, 1e-4, 60), (10000, 7000, 0.01, 1000), (32, 350, 0.01, 1000)]
    for n_a, agents, tol, ml in runs:
        print(json.dumps(run(n_a, agents, tol, ml)), flush=True)


if __name__ == "__main__":
    main()
