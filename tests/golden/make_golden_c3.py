"""Full-size golden fixture for BASELINE configs[3] (the 1e8-agent panel), from the oracle.

The bench's configs3 leg (bench.py configs3_leg) simulates 99 999 998 agents with the
converged configs[1] household (KS form, N_a = 10 000, 28 states x 15 M nodes, the
reference's initial saving rule intercept 0 / slope 1, [HARK] solve_agent to 1e-6 from
the terminal guess), a_0 = KSS, labour states split evenly by global agent index,
employment 1 (Urate = 0), Philox4x32-10 uniforms keyed by (GE iteration 0 << 20 | t,
global agent index) with seed 11, and prices from the per-period mean of assets
(Aiyagari_Support.py:1839-1894).  This script restates the same T periods with the
oracle (oracle/hark_ks.py: egm_solve, sim_one_period, calc_R_and_W; oracle/philox.py),
in chunks of agents, and records for every period:

  hist_A[t] (= K_t, the mean of end-of-period assets), hist_M, hist_R, hist_W,
  lab_counts[t][l] (exact: the labour draws of all 1e8 agents),
  and after the last period a[i], lab[i] at every SAMPLE_STRIDE-th agent.

Output: tests/golden/fullsize_c3.json (a few kB).  About 10 minutes on one core.

    python tests/golden/make_golden_c3.py [--periods 5]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.dirname(os.path.abspath(__file__))

from oracle import hark_ks as H  # noqa: E402
from oracle import philox  # noqa: E402

N_TOTAL = 99_999_998
N_A = 10_000
SEED = 11
GE_ITER = 0
CHUNK = 4_000_000
SAMPLE_STRIDE = 999_983


def policy():
    m = H.KSModel(dict(intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0]), dict(aCount=N_A, AgentCount=N_TOTAL))
    mt, ct, cycles, dist = m.solve_agent()
    return m, mt, ct, cycles, dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--periods", type=int, default=5)
    ap.add_argument("--agents", type=int, default=N_TOTAL)
    ap.add_argument("--out", default=os.path.join(OUT, "fullsize_c3.json"))
    args = ap.parse_args()
    N, T = args.agents, args.periods
    t0 = time.time()
    m, mt, ct, cycles, dist = policy()
    print(f"policy: {cycles} cycles, dist {dist:.3e} ({time.time() - t0:.0f} s)", flush=True)
    per = N // 7
    a = np.full(N, m.ss["KSS"])
    lab = (np.arange(N) // per).astype(np.int64)       # parallel.initial_labor_states restated
    emp = np.ones(CHUNK, dtype=bool)
    sow = dict(Mnow=m.ss["MSS"], Mrkv=0, Rnow=m.ss["RSS"], Wnow=m.ss["WSS"])
    hist = dict(A=[], M=[], R=[], W=[], lab_counts=[])
    for t in range(T):
        sums = []
        counts = np.zeros(7, dtype=np.int64)
        for c0 in range(0, N, CHUNK):
            c1 = min(N, c0 + CHUNK)
            u = philox.uniform((GE_ITER << 20) | t, np.arange(c0, c1, dtype=np.uint64), SEED)
            an, ln, _, _ = H.sim_one_period(a[c0:c1], lab[c0:c1], emp[:c1 - c0], u, sow["Rnow"], sow["Wnow"],
                                            sow["Mnow"], sow["Mrkv"], m.LSStates, m.cdf_table, mt, ct, m.Mgrid)
            a[c0:c1] = an
            lab[c0:c1] = ln
            sums.append(math.fsum(an))
            counts += np.bincount(ln, minlength=7)
        K = math.fsum(sums) / N                           # np.mean to ~1 ulp (exact sum, one rounding)
        # calc_R_and_W (AS:1839-1894) with the mean already formed
        Mnow, Aprev, Mrkv, Rnow, Wnow, _ = H.calc_R_and_W([np.array([K])], [np.ones(1)], m.Mrkv_hist[t], m.e)
        sow = dict(Mnow=Mnow, Mrkv=Mrkv, Rnow=Rnow, Wnow=Wnow)
        for k, v in (("A", Aprev), ("M", Mnow), ("R", Rnow), ("W", Wnow)):
            hist[k].append(float(v))
        hist["lab_counts"].append([int(x) for x in counts])
        print(f"t={t}: K={K!r} ({time.time() - t0:.0f} s)", flush=True)
    idx = np.arange(0, N, SAMPLE_STRIDE)
    out = dict(generator="tests/golden/make_golden_c3.py", agents=N, periods=T, n_a=N_A, seed=SEED, ge_iter=GE_ITER,
               egm_cycles=int(cycles), egm_dist=float(dist),
               policy_sha256=hashlib.sha256(np.ascontiguousarray(ct).tobytes()).hexdigest(),
               policy_c_sum=math.fsum(ct[np.isfinite(ct)].ravel()),
               hist_A=hist["A"], hist_M=hist["M"], hist_R=hist["R"], hist_W=hist["W"], lab_counts=hist["lab_counts"],
               sample_stride=SAMPLE_STRIDE, sample_idx=[int(i) for i in idx], sample_a=[float(x) for x in a[idx]],
               sample_lab=[int(x) for x in lab[idx]], a_sum_final=math.fsum(a), a_sq_sum_final=math.fsum(a * a),
               seconds=time.time() - t0)
    json.dump(out, open(args.out, "w"), indent=1)
    print("wrote", args.out, flush=True)


if __name__ == "__main__":
    main()
