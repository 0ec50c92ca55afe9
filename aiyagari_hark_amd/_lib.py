"""ctypes binding of libaiyagari.so (the C ABI declared in include/aiyagari.h).

The library is the only compute path: if it is missing or fails to load, every
device entry point raises -- there is no CPU fallback in the product.

torch is imported first on purpose: PyTorch-ROCm ships its own ``libamdhip64.so``
(SONAME ``libamdhip64.so.7``); loading it before the library makes the dynamic
linker bind libaiyagari to the same HIP runtime instance that owns the tensors whose
``data_ptr()`` we pass in.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

import torch  # noqa: F401  (see module docstring: HIP runtime ordering)

HERE = os.path.dirname(os.path.abspath(__file__))
# AIYAGARI_LIB points at an alternative build of the same library (tuning experiments).
LIB_PATH = os.environ.get("AIYAGARI_LIB") or os.path.join(HERE, "lib", "libaiyagari.so")

AIY_OK = 0
ERRORS = {-1: "AIY_ERR_ARG", -2: "AIY_ERR_HIP", -3: "AIY_ERR_STATE", -4: "AIY_ERR_UNSUPPORTED",
          -5: "AIY_ERR_COMM"}
AIY_MAX_STATES = 64
AIY_SOW_DOUBLES = 8
AIY_OPT_USE_GRAPHS = 1
AIY_OPT_RESIDENT = 2
AIY_OPT_RESIDENT_SHAPE = 3
AIY_OPT_HIST_FUSED = 4
AIY_OPT_RESIDENT_STREAM = 5
AIY_OPT_HIST_RESIDENT = 6
AIY_OPT_HIST_CLUSTER = 7
AIY_OPT_HIST_ACCEL = 8
AIY_OPT_HIST_KRYLOV = 9
AIY_OPT_GE_RESIDENT = 10
AIY_OPT_CU_LIMIT = 11
AIY_OPT_GE_REBALANCE = 12
AIY_OPT_GE_EXTRAP_PERIOD = 13
AIY_OPT_GE_LOGSEC = 14
AIY_OPT_HIST_PULL = 15
AIY_OPT_GE_LOOSE_HIST = 17
AIY_OPT_RESIDENT_SHAPE_STREAM = 18
AIY_OPT_GE_ANDERSON = 23

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_uint8_p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p


class EgmDims(ctypes.Structure):
    _fields_ = [("n_cal", ctypes.c_int32), ("S", ctypes.c_int32), ("n_M", ctypes.c_int32), ("n_a", ctypes.c_int32)]


class EgmInputs(ctypes.Structure):
    _fields_ = [(n, vp) for n in ("a_grid", "M_grid", "P", "R_next", "W_next", "M_next", "lab", "beta", "crra")]


class Market(ctypes.Structure):
    _fields_ = [("cap_share", ctypes.c_double), ("depr_fac", ctypes.c_double),
                ("prod", ctypes.c_double * 2), ("agg_L", ctypes.c_double * 2)]


class PanelModel(ctypes.Structure):
    _fields_ = [("S", ctypes.c_int32), ("n_M", ctypes.c_int32), ("n_a", ctypes.c_int32), ("n_lab", ctypes.c_int32),
                ("tables", vp), ("M_grid", vp), ("lab_level", vp), ("lab_cdf", vp), ("mrkv_hist", vp),
                ("act_T", ctypes.c_int32), ("unemployed", ctypes.c_int32)]


class PanelBatch(ctypes.Structure):
    _fields_ = [("n_cal", ctypes.c_int32), ("S", ctypes.c_int32), ("n_M", ctypes.c_int32), ("n_a", ctypes.c_int32),
                ("n_lab", ctypes.c_int32), ("tables", vp), ("M_grid", vp), ("lab_level", vp), ("lab_cdf", vp),
                ("mrkv_hist", vp), ("unemployed", ctypes.c_int32)]


class StationaryModel(ctypes.Structure):
    _fields_ = [("n_cal", ctypes.c_int32), ("S", ctypes.c_int32), ("n_a", ctypes.c_int32)] + \
               [(n, vp) for n in ("a_grid", "P", "lab", "beta", "crra", "alpha", "delta", "disc")]


class GeOptions(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int32), ("r_tol", ctypes.c_double), ("egm_tol", ctypes.c_double),
                ("hist_tol", ctypes.c_double), ("max_steps", ctypes.c_int32), ("max_egm_cycles", ctypes.c_int32),
                ("max_hist_iter", ctypes.c_int32), ("warm_hist", ctypes.c_int32), ("warm_egm", ctypes.c_int32),
                ("accel", ctypes.c_int32), ("r_lo", vp), ("r_hi", vp), ("secant_start", ctypes.c_int32),
                ("loose_bracket", ctypes.c_int32), ("egm_extrapolate", ctypes.c_int32), ("status_out", vp)]


# name -> (restype, argtypes)
SIGNATURES = {
    "aiy_version": (ctypes.c_int32, []),
    "aiy_create": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(vp)]),
    "aiy_destroy": (ctypes.c_int32, [vp]),
    "aiy_last_error": (ctypes.c_char_p, [vp]),
    "aiy_egm_step": (ctypes.c_int32, [vp, ctypes.POINTER(EgmDims), ctypes.POINTER(EgmInputs), vp, vp, vp, vp, vp]),
    "aiy_egm_solve": (ctypes.c_int32, [vp, ctypes.POINTER(EgmDims), ctypes.POINTER(EgmInputs), ctypes.c_double,
                                       ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, c_int32_p, c_double_p, vp]),
    "aiy_egm_solve_from": (ctypes.c_int32, [vp, ctypes.POINTER(EgmDims), ctypes.POINTER(EgmInputs), ctypes.c_double,
                                            ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp, c_int32_p,
                                            c_double_p, vp]),
    "aiy_egm_kernel_time": (ctypes.c_int32, [vp, ctypes.POINTER(EgmDims), ctypes.POINTER(EgmInputs), vp, vp, vp, vp,
                                             ctypes.c_int32, ctypes.POINTER(ctypes.c_float), vp]),
    "aiy_policy_eval": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp,
                                         ctypes.c_int64, vp, vp]),
    "aiy_sim_periods": (ctypes.c_int32, [vp, ctypes.POINTER(PanelModel), ctypes.POINTER(Market), ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, vp, vp, vp, ctypes.c_int64, vp,
                                         ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32,
                                         ctypes.c_int32, vp, vp, vp, vp]),
    "aiy_sim_period_local": (ctypes.c_int32, [vp, ctypes.POINTER(PanelModel), ctypes.c_int64, ctypes.c_int64, vp, vp,
                                              vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32, vp, vp]),
    "aiy_sim_period_prices": (ctypes.c_int32, [vp, ctypes.POINTER(PanelModel), ctypes.POINTER(Market),
                                               ctypes.c_int64, ctypes.c_int32, vp, vp, vp, vp]),
    "aiy_get_shocks": (ctypes.c_int32, [vp, ctypes.c_int32, vp, ctypes.c_int64, ctypes.c_int64, vp, vp,
                                        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32, vp]),
    "aiy_get_states": (ctypes.c_int32, [vp, vp, ctypes.c_int64, ctypes.c_double, ctypes.c_double, vp, vp, vp, vp,
                                        vp]),
    "aiy_get_controls": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, c_double_p,
                                          ctypes.c_int32, ctypes.c_double, ctypes.c_int64, vp, vp, vp, vp, vp]),
    "aiy_get_poststates": (ctypes.c_int32, [vp, ctypes.c_int64, vp, vp, vp, vp]),
    "aiy_sum": (ctypes.c_int32, [vp, vp, ctypes.c_int64, vp, vp]),
    "aiy_sim_kernel_time": (ctypes.c_int32, [vp, ctypes.POINTER(PanelModel), ctypes.POINTER(Market), ctypes.c_int64,
                                             vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_float), vp]),
    "aiy_panel_launch_stats": (ctypes.c_int32, [vp, c_double_p, ctypes.POINTER(ctypes.c_int64),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]),
    "aiy_sim_block_max_agents": (ctypes.c_int32, []),
    "aiy_sim_block_periods": (ctypes.c_int32, [vp, ctypes.POINTER(PanelBatch), vp, ctypes.c_int64, vp, vp, vp,
                                               vp, vp, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               vp, vp, vp, vp]),
    "aiy_set_option": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int64]),
    "aiy_get_option": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]),
    "aiy_index_ints_per_row": (ctypes.c_int32, []),
    "aiy_panel_table_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "aiy_panel_build": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp]),
    "aiy_build_index": (ctypes.c_int32, [vp, ctypes.c_int64, ctypes.c_int32, vp, vp, vp]),
    "aiy_comm_unique_id": (ctypes.c_int32, [vp]),
    "aiy_comm_init": (ctypes.c_int32, [vp, vp, ctypes.c_int32, ctypes.c_int32]),
    "aiy_comm_bind": (ctypes.c_int32, [vp, vp]),
    "aiy_comm_destroy": (ctypes.c_int32, [vp]),
    "aiy_allreduce_sum": (ctypes.c_int32, [vp, vp, ctypes.c_int64, vp]),
    "aiy_hist_lottery": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp]),
    "aiy_hist_solve": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp,
                                        ctypes.c_double, ctypes.c_int32, ctypes.c_int32, vp, vp, c_double_p,
                                        c_int32_p, vp]),
    "aiy_hist_launch_stats": (ctypes.c_int32, [vp, c_double_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]),
    "aiy_ge_resident_plan": (ctypes.c_int32, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_int32_p]),
    "aiy_ge_last_profile": (ctypes.c_int32, [vp, c_double_p, ctypes.c_int32]),
    "aiy_ge_last_eval_log": (ctypes.c_int32, [vp, c_double_p, ctypes.c_int32]),
    "aiy_ge_last_rounds": (ctypes.c_int32, [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "aiy_ge_launch_stats": (ctypes.c_int32, [vp, c_double_p, ctypes.POINTER(ctypes.c_int64), c_double_p, c_double_p,
                                             ctypes.c_int32]),
    "aiy_ge_stationary_work_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "aiy_ge_stationary": (ctypes.c_int32, [vp, ctypes.POINTER(StationaryModel), ctypes.POINTER(GeOptions), vp,
                                           c_double_p, c_double_p, c_double_p, c_int32_p, c_int32_p, c_int32_p, vp]),
    "aiy_wealth_stats": (ctypes.c_int32, [vp, vp, vp, ctypes.c_int64, c_double_p, ctypes.c_int32, c_double_p,
                                          c_double_p, vp]),
}

_lib = None
_lock = threading.Lock()


class AiyagariLibError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes CDLL with argtypes installed."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise AiyagariLibError(
                f"{p} is missing: build it with `python -m aiyagari_hark_amd.build` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols():
    return sorted(SIGNATURES)


class Handle:
    """RAII wrapper of aiy_handle (one per process and device)."""

    def __init__(self, device: int | None = 0):
        self.lib = load()
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        h = vp()
        rc = self.lib.aiy_create(int(device), ctypes.byref(h))
        if rc != AIY_OK:
            raise AiyagariLibError(f"aiy_create(device={device}) failed: {ERRORS.get(rc, rc)}")
        self.h = h

    def check(self, rc: int, what: str):
        if rc != AIY_OK:
            msg = self.lib.aiy_last_error(self.h)
            raise AiyagariLibError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")

    def get_option(self, option: int) -> int:
        v = ctypes.c_int64()
        self.check(self.lib.aiy_get_option(self.h, int(option), ctypes.byref(v)), "aiy_get_option")
        return int(v.value)

    def set_options(self, values: dict) -> dict:
        """Set several options; returns their previous values (pass them back to restore)."""
        prev = {k: self.get_option(k) for k in values}
        for k, v in values.items():
            self.check(self.lib.aiy_set_option(self.h, int(k), int(v)), "aiy_set_option")
        return prev

    def close(self):
        if getattr(self, "h", None):
            self.lib.aiy_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_handles: dict[int, Handle] = {}


def close_all():
    """Destroy every handle while the HIP runtime is still up (registered with atexit:
    a handle freed from a module destructor after the runtime's own teardown crashes
    the process on exit, e.g. under rocprofv3)."""
    while _handles:
        _, h = _handles.popitem()
        h.close()


atexit.register(close_all)


def handle(device: int | None = None) -> Handle:
    if device is None:
        device = torch.cuda.current_device()
    h = _handles.get(device)
    if h is None:
        h = Handle(device)
        _handles[device] = h
    return h


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise AiyagariLibError("libaiyagari takes device tensors only")
    if not t.is_contiguous():
        raise AiyagariLibError("tensor must be contiguous")
    return t.data_ptr()


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
