"""Interop views of device policy tables.

``DeviceSolution`` plays ``AiyagariType.solution[0]`` (a ConsumerSolution of 28
``LinearInterpOnInterp1D`` consumption functions, Aiyagari_Support.py:1509-1519):
``cFunc[k](m, M)`` evaluates on device through ``aiy_policy_eval`` and
``cFunc[k].xInterpolators[j]`` exposes ``x_list`` / ``y_list`` host copies of one
M-slice, which is what the notebook's plots read (Aiyagari-HARK.py:271-275).
"""
from __future__ import annotations

import numpy as np

from .egm import policy_eval


class DeviceLinearInterp:
    """One M-slice of one state's consumption table (HARK LinearInterp view)."""

    def __init__(self, sol, state, k):
        self._sol, self._s, self._k = sol, state, k

    @property
    def x_list(self):
        return self._sol.m_host()[self._s, self._k].copy()

    @property
    def y_list(self):
        return self._sol.c_host()[self._s, self._k].copy()

    def __call__(self, x):
        sol = self._sol
        xa = np.asarray(x, dtype=np.float64)
        n_M = sol.m_tab.shape[1]
        Mg = sol.M_grid
        if n_M == 1:
            out = policy_eval(sol.m_tab, sol.c_tab, Mg, self._s, xa.ravel())
        else:
            # evaluating exactly on the k-th M node reproduces the slice (alpha = 0 or 1)
            Mk = float(sol.M_grid_host()[self._k])
            out = policy_eval(sol.m_tab, sol.c_tab, Mg, self._s, xa.ravel(), np.full(xa.size, Mk))
        return out.cpu().numpy().reshape(xa.shape)


class DeviceCFunc:
    """cFunc[state] (HARK LinearInterpOnInterp1D view)."""

    def __init__(self, sol, state):
        self._sol, self._s = sol, state

    @property
    def xInterpolators(self):
        return [DeviceLinearInterp(self._sol, self._s, k) for k in range(self._sol.m_tab.shape[1])]

    @property
    def y_list(self):
        return self._sol.M_grid_host()

    def __call__(self, m, M=None):
        ma = np.asarray(m, dtype=np.float64)
        Ma = None if M is None else np.broadcast_to(np.asarray(M, dtype=np.float64), ma.shape).ravel()
        out = policy_eval(self._sol.m_tab, self._sol.c_tab, self._sol.M_grid, self._s, ma.ravel(), Ma)
        return out.cpu().numpy().reshape(ma.shape)


class DeviceVPFunc:
    """vPfunc[state] = cFunc ** -CRRA (MargValueFuncCRRA, AS:1514)."""

    def __init__(self, cfunc, crra):
        self.cFunc, self.CRRA = cfunc, crra

    def __call__(self, m, M=None):
        return self.cFunc(m, M) ** -self.CRRA


class DeviceSolution:
    def __init__(self, m_tab, c_tab, M_grid, CRRA):
        self.m_tab, self.c_tab, self.M_grid, self.CRRA = m_tab, c_tab, M_grid, CRRA
        self._m = self._c = self._Mg = None
        S = m_tab.shape[0]
        self.cFunc = [DeviceCFunc(self, s) for s in range(S)]
        self.vPfunc = [DeviceVPFunc(f, CRRA) for f in self.cFunc]

    def m_host(self):
        if self._m is None:
            self._m = self.m_tab.cpu().numpy()
        return self._m

    def c_host(self):
        if self._c is None:
            self._c = self.c_tab.cpu().numpy()
        return self._c

    def M_grid_host(self):
        if self._Mg is None:
            self._Mg = self.M_grid.cpu().numpy()
        return self._Mg
