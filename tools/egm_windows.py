"""Span of the node window each 64-query tile of the EGM phase 1 needs at configs[1]
(N_a = 10 000): percentiles of lb(q_last) - lb(q_first) + 1 over all (k, s', row, tile),
from oracle EGM cycles (CPU; sizes the 128-node window of csrc/egm.hip)."""
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from aiyagari_hark_amd import setup_math as sm
from oracle import hark_ks as H
ss = sm.steady_state(1.0, 0.96, 0.08, 0.36, 1.0)
aG = sm.make_grid_exp_mult(0.001, 50.0, 10000, 2)
Mg = ss["MSS"] * sm.MGRID_BASE
agg, E = sm.employment_chain(8, 8, 2.5, 1.5, 0, 0, 0.75, 1.25)
y, P7 = sm.labor_tauchen(7, 0.6, 0.2)
R, W, M = sm.next_prices([0.35, 0.36], [0.8, 0.8], Mg, 28, 0, 0, 1, 1, 1, 0.36, 0.08)
lv = sm.labor_levels(y)
P = sm.kron_states(P7, E)
ncyc = int(sys.argv[1]) if len(sys.argv) > 1 else 20
m = c = None
t = time.time()
for it in range(ncyc):
    m, c = H.egm_step(m, c, 0.96, 1.0, aG, Mg, R, W, M, lv, P)
print("cycles", ncyc, time.time() - t, "s")
np.savez('/tmp/egm_state.npz', m=m, c=c, aG=aG, Mg=Mg, R=R, W=W, M=M, lv=lv, P=P)
S, nM, n1 = m.shape
n = n1 - 1
lab = np.array([lv[s // 4] for s in range(S)])
spans = []; wins = []
for k in range(nM):
    for sp in range(S):
        j = np.searchsorted(Mg, M[k, sp]); j = min(max(j, 1), nM - 1)
        q = R[k, sp] * aG + W[k, sp] * lab[sp]
        for jj in (j - 1, j):
            x = m[sp, jj, :n]
            lb = np.searchsorted(x, q)
            for t0 in range(0, aG.size, 64):
                seg = lb[t0:t0 + 64]
                spans.append(seg[-1] - seg[0] + 1)
            # index window
            base = (x[1:2].view(np.int64) >> 44)[0]
            keys = (q.view(np.int64) >> 44) - base
            kx = (x.view(np.int64) >> 44) - base
            Hb = np.searchsorted(kx, np.arange(4096))  # first node with key>=b
            kk = np.clip(keys, 0, 4094)
            wins.append(Hb[kk + 1] - Hb[kk])
spans = np.array(spans); wins = np.concatenate(wins)
print("tile span percentiles", np.percentile(spans, [50, 90, 99, 99.9, 100]))
print("index window hist", np.bincount(np.minimum(wins, 10)) / wins.size)
