"""Wealth-distribution statistics of the simulated panel on device.

The reference notebook compares the simulated wealth distribution with the SCF through
HARK's ``get_lorenz_shares`` and imports ``get_percentiles`` alongside it
(Aiyagari-HARK.py:298-316)::

    sim_Lorenz_points = get_lorenz_shares(sim_wealth, percentiles=pctiles)

These are HARK 0.12's two functions (``HARK.utilities``) with the same signature,
defaults and argument checks, computed by libaiyagari's ``aiy_wealth_stats``
(rocPRIM radix sort + scans + one interpolation kernel, ``csrc/stats.hip``) on a
device array -- e.g. ``agent.panel.a``, the 1e6-1e8 agents' assets, which then never
leave HBM.  Host arrays are copied to the device first.  Results equal HARK's to
rounding (tree-ordered sums instead of NumPy's sequential cumsum).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_MAX_PCT = 256


def _check_percentiles(percentiles):
    if percentiles is None:
        return np.array([0.5])
    if not isinstance(percentiles, (list, np.ndarray)) or min(percentiles) <= 0 or max(percentiles) >= 1:
        raise ValueError("Percentiles should be a list or numpy array of floats between 0 and 1")
    p = np.ascontiguousarray(percentiles, dtype=np.float64).ravel()
    if p.size > _MAX_PCT:
        raise ValueError(f"at most {_MAX_PCT} percentiles per call")
    return p


def _device_vector(x, device):
    if isinstance(x, torch.Tensor):
        t = x.detach()
        if t.device.type != "cuda":
            t = t.to(device if device is not None else "cuda")
    else:
        t = torch.as_tensor(np.asarray(x, dtype=np.float64).ravel()).to(device if device is not None else "cuda")
    return t.to(torch.float64).reshape(-1).contiguous()


def _stats(data, weights, percentiles, device):
    p = _check_percentiles(percentiles)
    d = _device_vector(data, device)
    w = None if weights is None else _device_vector(weights, d.device)
    if w is not None and w.numel() != d.numel():
        raise ValueError("weights must have the same size as data")
    n = d.numel()
    if n < 1:
        raise ValueError("data is empty")
    h = _lib.handle(d.device.index)
    lor = np.empty(p.size)
    pct = np.empty(p.size)
    dp = ctypes.POINTER(ctypes.c_double)
    h.check(h.lib.aiy_wealth_stats(h.h, _lib.ptr(d), None if w is None else _lib.ptr(w), n,
                                   p.ctypes.data_as(dp), p.size, lor.ctypes.data_as(dp), pct.ctypes.data_as(dp),
                                   _lib.stream_ptr()), "aiy_wealth_stats")
    return lor, pct


def get_lorenz_shares(data, weights=None, percentiles=None, presorted=False, device=None):
    """[HARK 0.12] utilities.get_lorenz_shares: cumulative share of total wealth held by
    the bottom p of the population, np.interp(p, cumsum(w)/sum(w), cumsum(a w)/sum(a w))
    over the wealth-sorted data.  ``presorted`` is accepted for signature parity (the
    device sort is run either way and gives the same order)."""
    return _stats(data, weights, percentiles, device)[0]


def get_percentiles(data, weights=None, percentiles=None, presorted=False, device=None):
    """[HARK 0.12] utilities.get_percentiles: the weighted inverse CDF,
    interp1d(cumsum(w)/sum(w), sorted data, bounds_error=False)(p) (NaN outside the
    support of the CDF)."""
    return _stats(data, weights, percentiles, device)[1]
