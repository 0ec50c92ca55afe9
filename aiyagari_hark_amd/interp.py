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

    # ---- serialization ------------------------------------------
    def save(self, path, AFunc=None, **meta):
        """Write the policy tables ([S][n_M][n_a + 1] endogenous m and c, the M grid,
        CRRA) and, optionally, the aggregate saving rules (AS:1973-2005 ``intercept`` /
        ``slope`` per aggregate state) and scalar metadata to an ``.npz`` file.  Plain
        arrays only, so ``load`` never unpickles."""
        arrays = dict(m=self.m_host(), c=self.c_host(), M_grid=self.M_grid_host(),
                      CRRA=np.float64(self.CRRA), format_version=np.int64(SOLUTION_FORMAT))
        if AFunc is not None:
            arrays["afunc"] = np.array([[f.intercept, f.slope] for f in AFunc], dtype=np.float64)
        for k, v in meta.items():
            arrays["meta_" + k] = np.asarray(v)
        np.savez(path, **arrays)

    @classmethod
    def load(cls, path, device, with_meta=False):
        """Inverse of ``save``: returns ``(solution, afunc)`` (plus the metadata dict when
        ``with_meta``) with the tables resident on ``device``; ``afunc`` is a
        [n_states][2] (intercept, slope) array or None."""
        import torch

        with np.load(path, allow_pickle=False) as z:
            if int(z["format_version"]) != SOLUTION_FORMAT:
                raise ValueError(f"{path}: solution format {int(z['format_version'])}, expected {SOLUTION_FORMAT}")
            m, c, Mg = z["m"], z["c"], z["M_grid"]
            if m.ndim != 3 or m.shape != c.shape or Mg.shape != (m.shape[1],):
                raise ValueError(f"{path}: inconsistent table shapes m{m.shape} c{c.shape} M_grid{Mg.shape}")
            afunc = z["afunc"].copy() if "afunc" in z.files else None
            crra = float(z["CRRA"])
            meta = {k[5:]: z[k].item() for k in z.files if k.startswith("meta_")}
        to = dict(dtype=torch.float64, device=device)
        sol = cls(torch.as_tensor(m, **to).contiguous(), torch.as_tensor(c, **to).contiguous(),
                  torch.as_tensor(Mg, **to).contiguous(), crra)
        return (sol, afunc, meta) if with_meta else (sol, afunc)


SOLUTION_FORMAT = 1
