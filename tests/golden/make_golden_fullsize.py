"""Full-size golden fixtures for the benchmarked configurations, from the CPU oracle.

The reference ships no fixtures and HARK 0.12 is absent, so the only
way to pin the bench's configurations at the sizes their numbers are quoted on is the
oracle restatement itself, run here at those sizes (minutes to an hour of CPU):

  table2  BASELINE configs[2]: the 24 Table II cells (rho x sigma x CRRA, the order of
          aiyagari_hark_amd.stationary.table2_calibrations), N_a = 10 000, 7-state
          Tauchen; oracle/stationary.py ge_bisect (cold EGM to 1e-8, cold Young
          histogram to 1e-12 from the uniform mass, bisection of [-delta/2, 1/beta - 1)
          to 1e-7) -> the final bracket, r, K/Y; then K_s at that r.
  stress  BASELINE configs[4]: rho 0.9, sigma 0.4, CRRA in {1, 3, 5}, 25-state
          Rouwenhorst, N_a = 50 000; same search (the EGM expectation as one BLAS
          product, egm_matmul: same sums in another order).
  c3      BASELINE configs[3]: the per-period aggregate history of 99 999 998 agents
          driven by the converged configs[1] household (N_a = 10 000 KS form at the
          initial saving rule), Philox uniforms by global agent index -- see
          make_c3_history (a separate entry: `python make_golden_fullsize.py c3`).

Results are JSON (float repr round-trips exactly): tests/golden/fullsize_<which>.json.
Each finished cell is appended to tests/golden/fullsize_<which>.jsonl as it completes,
so a long run can be resumed (cells already in the .jsonl are skipped).

    python tests/golden/make_golden_fullsize.py table2 stress [--workers 6]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.dirname(os.path.abspath(__file__))

TABLE2_RHO = (0.0, 0.3, 0.6, 0.9)
TABLE2_SIGMA = (0.2, 0.4)
TABLE2_CRRA = (1.0, 3.0, 5.0)
CAL0 = dict(DiscFac=0.96, CapShare=0.36, DeprFac=0.08)
N_A_TABLE2 = 10_000
N_A_STRESS = 50_000


def cells(which):
    if which == "table2":   # the order of stationary.table2_calibrations()
        return [dict(which=which, k=k, rho=r, sigma=s, crra=c, S=7, income="tauchen", n_a=N_A_TABLE2)
                for k, (s, r, c) in enumerate((s, r, c) for s in TABLE2_SIGMA for r in TABLE2_RHO
                                              for c in TABLE2_CRRA)]
    if which == "stress":
        return [dict(which=which, k=k, rho=0.9, sigma=0.4, crra=c, S=25, income="rouwenhorst", n_a=N_A_STRESS)
                for k, c in enumerate(TABLE2_CRRA)]
    raise ValueError(which)


def solve_cell(job):
    import numpy as np
    from oracle import stationary as ST
    t0 = time.time()
    aGrid = ST.make_stationary_grid(0.001, 50.0, job["n_a"], 2)
    lab, P = ST.income_process(job["S"], job["rho"], job["sigma"], job["income"])
    cal = dict(CAL0, CRRA=job["crra"])
    kw = dict(egm_tol=1e-8, hist_tol=1e-12, fast=True, egm_matmul=job["S"] > 8)
    g = ST.ge_bisect(cal, aGrid, lab, P, r_tol=1e-7, **kw)
    Ks, info = ST.capital_supply(g["r"], cal, aGrid, lab, P, **kw)
    _, Kd = ST.prices(g["r"], cal["CapShare"], cal["DeprFac"])
    out = dict(job, r=g["r"], lo=g["lo"], hi=g["hi"], K=g["K"], KtoY=g["KtoY"], saving_rate=g["saving_rate"],
               steps=g["iters"], Ks_at_r=Ks, Kd_at_r=Kd, egm_cycles_at_r=int(info["cycles"]),
               hist_iters_at_r=int(info["hist_iters"]), mass_total_at_r=float(np.sum(info["mass"])),
               seconds=time.time() - t0)
    return out


def run(which_list, workers):
    import multiprocessing as mp
    jobs = []
    for which in which_list:
        path = os.path.join(OUT, f"fullsize_{which}.jsonl")
        done = set()
        if os.path.exists(path):
            for line in open(path):
                done.add(json.loads(line)["k"])
        jobs += [j for j in cells(which) if j["k"] not in done]
    # longest first: the stress cells, then the Table II cells nearest 1/beta - 1
    jobs.sort(key=lambda j: (j["which"] != "stress", j["rho"] == 0.9, j["sigma"]))
    print(f"{len(jobs)} cells to solve on {workers} workers", flush=True)
    with mp.get_context("spawn").Pool(workers) as pool:
        for res in pool.imap_unordered(solve_cell, jobs):
            with open(os.path.join(OUT, f"fullsize_{res['which']}.jsonl"), "a") as f:
                f.write(json.dumps(res) + "\n")
            print(f"{res['which']} {res['k']}: r = {100 * res['r']:.6f} % ({res['seconds']:.0f} s)", flush=True)
    for which in which_list:
        rows = [json.loads(l) for l in open(os.path.join(OUT, f"fullsize_{which}.jsonl"))]
        rows.sort(key=lambda d: d["k"])
        json.dump(dict(which=which, generator="tests/golden/make_golden_fullsize.py", cells=rows),
                  open(os.path.join(OUT, f"fullsize_{which}.json"), "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=["table2", "stress"])
    ap.add_argument("--workers", type=int, default=6)
    args = ap.parse_args()
    ge = [w for w in args.which if w in ("table2", "stress")]
    if ge:
        run(ge, args.workers)
    if "c3" in args.which:
        make_c3_history()


def make_c3_history():
    raise SystemExit("c3: see make_golden_c3.py")


if __name__ == "__main__":
    main()
