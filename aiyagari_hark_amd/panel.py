"""Device panel through the libaiyagari C ABI.

A ``DevicePanel`` owns the agents of one rank (assets, labour states), the device
market state ("sow_state") and the per-period history buffers.  ``run`` enqueues
whole blocks of periods; the host never touches per-agent data inside a history.

Shock sources (``u`` of get_shocks, Aiyagari_Support.py:1253-1254):
  * ``"numpy"``  -- uniforms drawn on the host from NumPy's *global* RandomState in
    exactly the order the reference's ``np.random.choice`` calls consume them
    (agent-major per period, periods in order); seeding ``np.random.seed(k)``
    before a solve makes the GPU history reproduce the reference's.
  * ``"philox"`` -- counter-based Philox4x32-10 on device (key = seed, counter =
    (GE iteration << 20 | t, global agent index)); independent of sharding.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

F64 = torch.float64


class DevicePanel:
    def __init__(self, n_local: int, device=None, agent_offset: int = 0, n_total: int | None = None,
                 act_T: int = 11000):
        self.device = torch.device(device or "cuda")
        self.n_local = int(n_local)
        self.agent_offset = int(agent_offset)
        self.n_total = int(n_total if n_total is not None else n_local)
        self.a = torch.empty(self.n_local, dtype=F64, device=self.device)
        self.lab = torch.empty(self.n_local, dtype=torch.uint8, device=self.device)
        self.sow = torch.zeros(_lib.AIY_SOW_DOUBLES, dtype=F64, device=self.device)
        self.act_T = int(act_T)
        self.hist_A = torch.zeros(self.act_T, dtype=F64, device=self.device)
        self.hist_M = torch.zeros(self.act_T, dtype=F64, device=self.device)
        self._model = None

    def reset(self, a0, lab0, Mnow, Aprev, Mrkv, Rnow, Wnow):
        """sim_birth + Market.reset sow_init (Aiyagari_Support.py:1621-1628)."""
        a0 = np.broadcast_to(np.asarray(a0, dtype=np.float64), (self.n_local,))
        self.a.copy_(torch.from_numpy(np.ascontiguousarray(a0)))
        self.lab.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(lab0, dtype=np.uint8))))
        sow = np.zeros(_lib.AIY_SOW_DOUBLES)
        sow[:6] = [Mnow, Aprev, Mrkv, Rnow, Wnow, 0.0]
        self.sow.copy_(torch.from_numpy(sow))
        self.hist_A.zero_()
        self.hist_M.zero_()

    def bind_model(self, m_pol, c_pol, M_grid, lab_level, lab_cdf, mrkv_hist, market: dict):
        S, n_M, n1 = m_pol.shape
        n_lab = int(lab_level.numel())
        keep = dict(m_pol=m_pol.contiguous(), c_pol=c_pol.contiguous(), M_grid=M_grid.contiguous(),
                    lab_level=lab_level.contiguous(), lab_cdf=lab_cdf.contiguous(),
                    mrkv_hist=mrkv_hist.to(torch.int32).contiguous())
        # interleaved (m, c) pairs + fine log-bucket search index (built on device once per history)
        h = _lib.handle(self.device.index)
        ipr = h.lib.aiy_panel_index_ints_per_row()
        keep["pol_pairs"] = torch.empty((S, n_M, n1, 2), dtype=F64, device=self.device)
        keep["pol_index"] = torch.empty((S * n_M, ipr), dtype=torch.int32, device=self.device)
        h.check(h.lib.aiy_panel_prepare(h.h, S * n_M, n1, _lib.ptr(keep["m_pol"]), _lib.ptr(keep["c_pol"]),
                                        _lib.ptr(keep["pol_pairs"]), _lib.ptr(keep["pol_index"]), _lib.stream_ptr()),
                "aiy_panel_prepare")
        pm = _lib.PanelModel(S, n_M, n1 - 1, n_lab, *(_lib.ptr(keep[k]) for k in
                                                       ("pol_pairs", "pol_index", "M_grid", "lab_level", "lab_cdf",
                                                        "mrkv_hist")))
        mk = _lib.Market(market["CapShare"], market["DeprFac"], (ctypes.c_double * 2)(*market["prod"]),
                         (ctypes.c_double * 2)(*market["agg_L"]))
        self._model = (pm, mk, keep)

    def run(self, t0: int, n_periods: int, shock_mode="philox", seed=0, ge_iter=0, u_host_source=None,
            chunk=1000, stream=None):
        """Simulate periods [t0, t0 + n_periods).  For shock_mode='numpy', u_host_source(n)
        must return the next n x n_local uniforms (host)."""
        if self._model is None:
            raise RuntimeError("bind_model() first")
        pm, mk, _ = self._model
        h = _lib.handle(self.device.index)
        sp = _lib.stream_ptr(stream)
        if shock_mode == "philox":
            h.check(h.lib.aiy_sim_periods(h.h, ctypes.byref(pm), ctypes.byref(mk), self.n_local, self.agent_offset,
                                          self.n_total, _lib.ptr(self.a), _lib.ptr(self.lab), None, 0,
                                          int(seed) & ((1 << 64) - 1), int(ge_iter), int(t0), int(n_periods),
                                          _lib.ptr(self.sow), _lib.ptr(self.hist_A), _lib.ptr(self.hist_M), sp),
                    "aiy_sim_periods")
            return
        if shock_mode != "numpy":
            raise ValueError(shock_mode)
        t = t0
        end = t0 + n_periods
        while t < end:
            n = min(chunk, end - t)
            u = np.ascontiguousarray(u_host_source(n), dtype=np.float64)
            if u.shape != (n, self.n_local):
                raise ValueError(f"u block shape {u.shape} != {(n, self.n_local)}")
            ud = torch.from_numpy(u).to(self.device, non_blocking=False)
            h.check(h.lib.aiy_sim_periods(h.h, ctypes.byref(pm), ctypes.byref(mk), self.n_local, self.agent_offset,
                                          self.n_total, _lib.ptr(self.a), _lib.ptr(self.lab), _lib.ptr(ud),
                                          self.n_local, 0, int(ge_iter), int(t), int(n), _lib.ptr(self.sow),
                                          _lib.ptr(self.hist_A), _lib.ptr(self.hist_M), sp), "aiy_sim_periods")
            torch.cuda.current_stream(self.device).synchronize() if stream is None else stream.synchronize()
            del ud
            t += n

    def sow_host(self):
        s = self.sow.cpu().numpy()
        return dict(Mnow=float(s[0]), Aprev=float(s[1]), Mrkv=int(s[2]), Rnow=float(s[3]), Wnow=float(s[4]),
                    Urate=float(s[5]))
