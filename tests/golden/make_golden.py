"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference (Dostenlinus/Aiyagari-HARK) ships no tests, fixtures or golden vectors,
and its library (econ-ark 0.12) cannot be imported here, so the
fixtures are produced by the oracle restatement in oracle/ and pinned to the
reference only through the closed forms checked in tests/test_oracle.py.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import hark_ks as H  # noqa: E402
from oracle import stationary as ST  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

CAL = {  # (LaborAR, LaborSD, CRRA, AgentCount): BASELINE config 1, the notebook run, the checkpoint run
    "cfg1": (0.6, 0.2, 1.0, 350),
    "nb": (0.3, 0.2, 1.0, 350),
    "ckpt": (0.9, 0.4, 5.0, 700),
}


def model_for(tag):
    ar, sd, crra, n = CAL[tag]
    e = dict(LaborAR=ar, LaborSD=sd, CRRA=crra)
    a = dict(LaborAR=ar, LaborSD=sd, CRRA=crra, AgentCount=n)
    return H.KSModel(e, a)


def egm_fixture(tag, afunc=None):
    m = model_for(tag)
    if afunc is not None:
        m.AFunc = [H.AggregateSavingRule(*afunc[0]), H.AggregateSavingRule(*afunc[1])]
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, m.a["LaborStatesNo"], m.e)
    mt, ct, cycles, dist = H.egm_solve(m.a["DiscFac"], m.a["CRRA"], m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates,
                                       m.MrkvIndArray)
    return dict(aGrid=m.aGrid, Mgrid=m.Mgrid, P=m.MrkvIndArray, LSStates=m.LSStates, Rk=Rk, Wk=Wk, Mk=Mk,
                m=mt, c=ct, cycles=cycles, dist=dist, DiscFac=m.a["DiscFac"], CRRA=m.a["CRRA"],
                KSS=m.ss["KSS"], MSS=m.ss["MSS"], RSS=m.ss["RSS"], WSS=m.ss["WSS"],
                tauchen_y=m.agent_tauchen[0], tauchen_P=m.agent_tauchen[1], cdf=m.cdf_table,
                MrkvArray=m.MrkvArray, Mrkv_hist=m.Mrkv_hist[:2000])


def panel_fixture(tag, T=50, seed=12345):
    fx = egm_fixture(tag)
    m = model_for(tag)
    N = m.a["AgentCount"]
    emp, lab = H.sim_birth_labor(N, 7, 0.0, seed=0)
    U = np.random.RandomState(seed).random_sample((T, N))
    a = np.full(N, m.ss["KSS"])
    sow = dict(Mnow=m.ss["MSS"], Mrkv=0, Rnow=m.ss["RSS"], Wnow=m.ss["WSS"])
    A_hist, M_hist, a_tr, l_tr = [], [], [], []
    for t in range(T):
        a, lab, _, _ = H.sim_one_period(a, lab, emp, U[t], sow["Rnow"], sow["Wnow"], sow["Mnow"], sow["Mrkv"],
                                        m.LSStates, m.cdf_table, fx["m"], fx["c"], m.Mgrid)
        Mnow, Aprev, Mrkv, Rnow, Wnow, _ = H.calc_R_and_W([a], [emp.astype(float)], m.Mrkv_hist[t], m.e)
        sow = dict(Mnow=Mnow, Mrkv=Mrkv, Rnow=Rnow, Wnow=Wnow)
        A_hist.append(Aprev)
        M_hist.append(Mnow)
        a_tr.append(a.copy())
        l_tr.append(lab.copy())
    return dict(u_seed=seed, T=T, lab0=H.sim_birth_labor(N, 7, 0.0, seed=0)[1], a_final=a, lab_final=lab,
                hist_A=np.array(A_hist), hist_M=np.array(M_hist), a_trace=np.array(a_tr)[::10],
                lab_trace=np.array(l_tr)[::10], R_final=sow["Rnow"])


def stationary_fixture():
    aGrid = ST.make_stationary_grid(0.001, 50.0, 64, 2)
    lab, P = ST.income_process(7, 0.6, 0.2, "tauchen")
    cal = dict(DiscFac=0.96, CRRA=1.0, CapShare=0.36, DeprFac=0.08)
    r = 0.04
    K, info = ST.capital_supply(r, cal, aGrid, lab, P, egm_tol=1e-8, hist_tol=1e-12)
    yR, PR = ST.rouwenhorst(5, 0.9, 0.4)
    return dict(aGrid=aGrid, lab=lab, P=P, r=r, K=K, m=info["m"], c=info["c"], mass=info["mass"],
                cycles=info["cycles"], hist_iters=info["hist_iters"], rouw_y=yR, rouw_P=PR)


def main():
    np.savez_compressed(os.path.join(OUT, "egm_cfg1.npz"), **egm_fixture("cfg1"))
    np.savez_compressed(os.path.join(OUT, "egm_cfg1_afunc2.npz"),
                        **egm_fixture("cfg1", afunc=((0.35, 0.8), (0.36, 0.8))))
    np.savez_compressed(os.path.join(OUT, "egm_ckpt.npz"), **egm_fixture("ckpt"))
    np.savez_compressed(os.path.join(OUT, "panel_cfg1.npz"), **panel_fixture("cfg1"))
    np.savez_compressed(os.path.join(OUT, "stationary.npz"), **stationary_fixture())
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
