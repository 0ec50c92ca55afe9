"""ORACLE (test infrastructure only -- imported by tests/, never by the product path).

NumPy/SciPy restatement of the two HARK 0.12 ``HARK.utilities`` routines the reference
notebook applies to the simulated wealth (Aiyagari-HARK.py:298-316):
``get_lorenz_shares(sim_wealth, percentiles=pctiles)`` and ``get_percentiles``.
HARK is not installed here: the restatement follows HARK 0.12's
published algorithm (argsort, cumulative weights over their sum, cumulative weighted
data over its sum, linear interpolation); parity with HARK itself is unpinned beyond
the closed-form checks in tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import interp1d


def get_lorenz_shares(data, weights=None, percentiles=None, presorted=False):
    if percentiles is None:
        percentiles = [0.5]
    elif not isinstance(percentiles, (list, np.ndarray)) or min(percentiles) <= 0 or max(percentiles) >= 1:
        raise ValueError("Percentiles should be a list or numpy array of floats between 0 and 1")
    data = np.asarray(data, dtype=np.float64)
    if weights is None:
        weights = np.ones(data.size)
    if presorted:
        temp, w = data, np.asarray(weights, dtype=np.float64)
    else:
        order = np.argsort(data)
        temp, w = data[order], np.asarray(weights, dtype=np.float64)[order]
    cum_dist = np.cumsum(w) / np.sum(w)
    temp2 = temp * w
    cum_data = np.cumsum(temp2) / sum(temp2)
    return np.interp(percentiles, cum_dist, cum_data)


def get_percentiles(data, weights=None, percentiles=None, presorted=False):
    if percentiles is None:
        percentiles = [0.5]
    elif not isinstance(percentiles, (list, np.ndarray)) or min(percentiles) <= 0 or max(percentiles) >= 1:
        raise ValueError("Percentiles should be a list or numpy array of floats between 0 and 1")
    data = np.asarray(data, dtype=np.float64)
    if weights is None:
        weights = np.ones(data.size) / float(data.size)
    if presorted:
        ds, ws = data, np.asarray(weights, dtype=np.float64)
    else:
        order = np.argsort(data)
        ds, ws = data[order], np.asarray(weights, dtype=np.float64)[order]
    cum_dist = np.cumsum(ws) / np.sum(ws)
    inv_cdf = interp1d(cum_dist, ds, bounds_error=False, assume_sorted=True)
    return inv_cdf(percentiles)
