"""Device EGM through the libaiyagari C ABI.

``EgmBatch`` holds the per-calibration inputs of ``solve_Aiyagari``
(Aiyagari_Support.py:1423-1434) as device tensors, with precompute_arrays
(Aiyagari_Support.py:906-1037) reduced to its unique [n_M, S] content.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

F64 = torch.float64


def _dev(x, device) -> torch.Tensor:
    return torch.from_numpy(np.array(x, dtype=np.float64, order="C", copy=True)).to(device)


@dataclass
class EgmBatch:
    a_grid: torch.Tensor   # [n_cal, n_a]
    M_grid: torch.Tensor   # [n_cal, n_M]
    P: torch.Tensor        # [n_cal, S, S]
    R_next: torch.Tensor   # [n_cal, n_M, S]
    W_next: torch.Tensor   # [n_cal, n_M, S]
    M_next: torch.Tensor   # [n_cal, n_M, S]
    lab: torch.Tensor      # [n_cal, S]
    beta: torch.Tensor     # [n_cal]
    crra: torch.Tensor     # [n_cal]

    @property
    def dims(self):
        n_cal, n_a = self.a_grid.shape
        return n_cal, self.P.shape[1], self.M_grid.shape[1], n_a

    @property
    def device(self):
        return self.a_grid.device

    @classmethod
    def from_numpy(cls, a_grid, M_grid, P, R_next, W_next, M_next, lab, beta, crra, device=None):
        """Arrays may be per-calibration (leading n_cal axis) or single (broadcast)."""
        device = torch.device(device or "cuda")
        a_grid = np.atleast_2d(a_grid)
        M_grid = np.atleast_2d(M_grid)
        P = P if np.ndim(P) == 3 else np.asarray(P)[None]
        R_next = R_next if np.ndim(R_next) == 3 else np.asarray(R_next)[None]
        W_next = W_next if np.ndim(W_next) == 3 else np.asarray(W_next)[None]
        M_next = M_next if np.ndim(M_next) == 3 else np.asarray(M_next)[None]
        lab = np.atleast_2d(lab)
        n_cal = max(a.shape[0] for a in (a_grid, M_grid, P, R_next, W_next, M_next, lab))
        bc = lambda x: np.broadcast_to(x, (n_cal,) + x.shape[1:])  # noqa: E731
        beta = np.broadcast_to(np.atleast_1d(np.asarray(beta, dtype=np.float64)), (n_cal,))
        crra = np.broadcast_to(np.atleast_1d(np.asarray(crra, dtype=np.float64)), (n_cal,))
        return cls(*(_dev(bc(x), device) for x in (a_grid, M_grid, P, R_next, W_next, M_next, lab)),
                   _dev(beta, device), _dev(crra, device))

    def _abi(self):
        n_cal, S, n_M, n_a = self.dims
        if S > _lib.AIY_MAX_STATES:
            raise ValueError(f"S={S} exceeds {_lib.AIY_MAX_STATES}")
        d = _lib.EgmDims(n_cal, S, n_M, n_a)
        i = _lib.EgmInputs(*(_lib.ptr(t) for t in (self.a_grid, self.M_grid, self.P, self.R_next, self.W_next,
                                                   self.M_next, self.lab, self.beta, self.crra)))
        return d, i

    def table_shape(self):
        n_cal, S, n_M, n_a = self.dims
        return (n_cal, S, n_M, n_a + 1)


def egm_step(batch: EgmBatch, m_next=None, c_next=None, out=None, stream=None):
    """One solve_Aiyagari step for every calibration (terminal guess when m_next is None)."""
    h = _lib.handle(batch.device.index)
    d, i = batch._abi()
    shp = batch.table_shape()
    if out is None:
        out = (torch.empty(shp, dtype=F64, device=batch.device), torch.empty(shp, dtype=F64, device=batch.device))
    for t in (m_next, c_next):
        if t is not None and tuple(t.shape) != shp:
            raise ValueError(f"next-period table shape {tuple(t.shape)} != {shp}")
    h.check(h.lib.aiy_egm_step(h.h, ctypes.byref(d), ctypes.byref(i), _lib.ptr(m_next), _lib.ptr(c_next),
                               _lib.ptr(out[0]), _lib.ptr(out[1]), _lib.stream_ptr(stream)), "aiy_egm_step")
    return out


def egm_solve(batch: EgmBatch, tol=1e-6, max_cycles=5000, chunk=32, work=None, out=None, stream=None, init=None):
    """[HARK] solve_agent (infinite horizon, cold start) on device for every calibration.
    ``init=(m, c)`` warm-starts from those tables instead of the terminal guess
    (aiy_egm_solve_from; the stationary GE search only -- the KS form keeps HARK's cold
    start).

    Returns (m, c, cycles[n_cal], dist[n_cal])."""
    h = _lib.handle(batch.device.index)
    d, i = batch._abi()
    shp = batch.table_shape()
    dev = batch.device
    if work is None:
        work = (torch.empty((2,) + shp, dtype=F64, device=dev), torch.empty((2,) + shp, dtype=F64, device=dev))
    if out is None:
        out = (torch.empty(shp, dtype=F64, device=dev), torch.empty(shp, dtype=F64, device=dev))
    n_cal = shp[0]
    cycles = (ctypes.c_int32 * n_cal)()
    dist = (ctypes.c_double * n_cal)()
    if init is None:
        h.check(h.lib.aiy_egm_solve(h.h, ctypes.byref(d), ctypes.byref(i), float(tol), int(max_cycles), int(chunk),
                                    _lib.ptr(work[0]), _lib.ptr(work[1]), _lib.ptr(out[0]), _lib.ptr(out[1]),
                                    cycles, dist, _lib.stream_ptr(stream)), "aiy_egm_solve")
    else:
        m0, c0 = (t.contiguous() for t in init)
        if tuple(m0.shape) != shp or tuple(c0.shape) != shp:
            raise ValueError(f"initial table shape {tuple(m0.shape)} != {shp}")
        h.check(h.lib.aiy_egm_solve_from(h.h, ctypes.byref(d), ctypes.byref(i), float(tol), int(max_cycles),
                                         int(chunk), _lib.ptr(m0), _lib.ptr(c0), _lib.ptr(work[0]), _lib.ptr(work[1]),
                                         _lib.ptr(out[0]), _lib.ptr(out[1]), cycles, dist, _lib.stream_ptr(stream)),
                "aiy_egm_solve_from")
    return out[0], out[1], np.array(cycles[:], dtype=np.int64), np.array(dist[:], dtype=np.float64)


def policy_eval(m_tab, c_tab, M_grid, state, m, M=None, stream=None):
    """cFunc[state](m, M) on device (HARK LinearInterpOnInterp1D semantics).

    m_tab/c_tab: [S, n_M, n_a+1] device tensors; state/m/M: array-likes of equal length."""
    S, n_M, n1 = m_tab.shape
    dev = m_tab.device
    st = torch.as_tensor(np.asarray(state, dtype=np.int32).ravel()).to(dev)
    mq = torch.from_numpy(np.array(m, dtype=np.float64).ravel()).to(dev)
    n = mq.numel()
    if st.numel() == 1 and n > 1:
        st = st.expand(n).contiguous()
    Mq = None
    if n_M > 1:
        Mq = torch.from_numpy(np.array(M, dtype=np.float64).ravel()).to(dev)
        if Mq.numel() == 1 and n > 1:
            Mq = Mq.expand(n).contiguous()
    out = torch.empty(n, dtype=F64, device=dev)
    h = _lib.handle(dev.index)
    h.check(h.lib.aiy_policy_eval(h.h, S, n_M, n1 - 1, _lib.ptr(m_tab), _lib.ptr(c_tab),
                                  _lib.ptr(M_grid) if n_M > 1 else None, _lib.ptr(st), _lib.ptr(mq),
                                  _lib.ptr(Mq), n, _lib.ptr(out), _lib.stream_ptr(stream)), "aiy_policy_eval")
    return out
