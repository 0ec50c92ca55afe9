"""Profile driver: configs[1]-sized EGM solve + panel periods (for rocprofv3)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from aiyagari_hark_amd import setup_math as sm
from aiyagari_hark_amd.egm import EgmBatch, egm_solve, egm_step
from aiyagari_hark_amd.panel import DevicePanel
dev = torch.device("cuda:0")
n_a = int(os.environ.get("NA", 10000)); N = int(os.environ.get("NAG", 1000006)); T = int(os.environ.get("T", 300))
ss = sm.steady_state(1.0, 0.96, 0.08, 0.36, 1.0)
aG = sm.make_grid_exp_mult(0.001, 50.0, n_a, 2)
Mg = ss["MSS"] * sm.MGRID_BASE
agg, E = sm.employment_chain(8, 8, 2.5, 1.5, 0, 0, 0.75, 1.25)
y, P7 = sm.labor_tauchen(7, 0.6, 0.2)
P = sm.kron_states(P7, E)
R, W, M = sm.next_prices([0.35, 0.36], [0.8, 0.8], Mg, 28, 0, 0, 1, 1, 1, 0.36, 0.08)
lv = sm.labor_levels(y)
lab = np.array([lv[s // 4] for s in range(28)])
b = EgmBatch.from_numpy(aG, Mg, P, R, W, M, lab, 0.96, 1.0, device=dev)
torch.cuda.synchronize(); t = time.perf_counter()
m, c, cyc, d = egm_solve(b)
torch.cuda.synchronize(); print("egm solve", time.perf_counter() - t, "s cycles", cyc, flush=True)
p = DevicePanel(N, device=dev, act_T=T)
hist = torch.as_tensor(sm.markov_history(agg, T).astype(np.int32)).to(dev)
p.bind_model(m[0], c[0], b.M_grid[0], torch.as_tensor(lv).to(dev), torch.as_tensor(sm.choice_cdf_table(P7)).to(dev),
             hist, dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
p.reset(ss["KSS"], np.repeat(np.arange(7), N // 7), ss["MSS"], ss["KSS"], 0, ss["RSS"], ss["WSS"])
torch.cuda.synchronize(); t = time.perf_counter()
p.run(0, T, shock_mode="philox", seed=1)
torch.cuda.synchronize(); dt = time.perf_counter() - t
print("panel", T, "periods", dt, "s ->", dt / T * 1e6, "us/period", p.sow_host(), flush=True)
