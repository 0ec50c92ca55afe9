"""Wealth-distribution statistics on device (aiy_wealth_stats) vs
the oracle restatement of HARK 0.12 get_lorenz_shares / get_percentiles
(oracle/hark_utils.py).  Tolerance 1e-12 relative: the device sums are tree-ordered,
NumPy's cumsum sequential."""
import numpy as np
import pytest
import torch

from oracle import hark_utils as HU

pytestmark = pytest.mark.gpu
PCT = np.linspace(0.01, 0.999, 15)      # the notebook's pctiles (Aiyagari-HARK.py:311)
RTOL = 1e-12


def close(a, b, rtol=RTOL):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    both_nan = np.isnan(a) & np.isnan(b)
    err = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    assert np.all(both_nan | (err <= rtol)), (a, b)


# Percentiles interpolate the sorted data over cum_dist, whose spacing is ~1/n: a rounding
# difference of the cumulative weights (HARK's default weights are ones/n, accumulated by
# a sequential cumsum; the device uses (k + 1)/n, or a tree-ordered scan of the weights)
# is amplified by the data spacing in the tail.  Against the same cum_dist (unit
# weights given to the oracle as ones) the device is within 1e-12; against HARK's
# rounded cumsum within 1e-8.
PCTL_RTOL_CUMSUM = 1e-8


@pytest.mark.parametrize("n,weighted", [(100003, False), (100003, True), (2, False), (7, True), (1000006, False)])
def test_lorenz_and_percentiles_match_oracle(gpu, n, weighted):
    from aiyagari_hark_amd import stats
    rng = np.random.RandomState(n)
    x = rng.lognormal(0.5, 1.2, n)
    w = rng.uniform(0.5, 1.5, n) if weighted else None
    d = torch.as_tensor(x).to(gpu)
    dw = None if w is None else torch.as_tensor(w).to(gpu)
    lor = stats.get_lorenz_shares(d, weights=dw, percentiles=PCT)
    pct = stats.get_percentiles(d, weights=dw, percentiles=PCT)
    close(lor, HU.get_lorenz_shares(x, weights=w, percentiles=PCT), RTOL if w is None else 1e-10)
    close(pct, HU.get_percentiles(x, weights=w, percentiles=PCT), PCTL_RTOL_CUMSUM)
    if w is None:
        close(pct, HU.get_percentiles(x, weights=np.ones(n), percentiles=PCT))


def test_ties_and_default_percentile(gpu):
    from aiyagari_hark_amd import stats
    x = np.repeat([0.001, 0.5, 2.0, 7.0], 2500)        # heavy ties, as at the borrowing constraint
    close(stats.get_lorenz_shares(x, device=gpu), HU.get_lorenz_shares(x))
    close(stats.get_percentiles(x, percentiles=PCT, device=gpu), HU.get_percentiles(x, np.ones(x.size), percentiles=PCT))


def test_panel_wealth_lorenz(gpu):
    """The notebook's use: Lorenz points of the simulated panel's assets, read on device."""
    from aiyagari_hark_amd import stats
    from oracle import hark_ks as H
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    from aiyagari_hark_amd.panel import DevicePanel
    m = H.KSModel()
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, 7, m.e)
    lab = np.array([m.LSStates[s // 4] for s in range(28)])
    b = EgmBatch.from_numpy(m.aGrid, m.Mgrid, m.MrkvIndArray, Rk, Wk, Mk, lab, 0.96, 1.0, device=gpu)
    mt, ct, _, _ = egm_solve(b)
    N, T = 70000, 200
    emp, lab0 = H.sim_birth_labor(N, 7, 0.0, seed=0)
    p = DevicePanel(N, device=gpu, act_T=T)
    p.bind_model(mt[0], ct[0], b.M_grid[0], torch.as_tensor(m.LSStates).to(gpu), torch.as_tensor(m.cdf_table).to(gpu),
                 torch.as_tensor(m.Mrkv_hist[:T].astype(np.int32)).to(gpu),
                 dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
    p.reset(m.ss["KSS"], lab0, m.ss["MSS"], m.ss["KSS"], 0, m.ss["RSS"], m.ss["WSS"])
    p.run(0, T, shock_mode="philox", seed=3)
    torch.cuda.synchronize()
    a = p.a.cpu().numpy()
    close(stats.get_lorenz_shares(p.a, percentiles=PCT), HU.get_lorenz_shares(a, percentiles=PCT))
