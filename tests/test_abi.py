"""CPU tests of the C-ABI boundary: the library builds/loads, exports every entry point
include/aiyagari.h declares, the ctypes layer binds all of them, and host-side argument
validation rejects bad calls before any device work (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "aiyagari.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(aiy_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from aiyagari_hark_amd import build, _lib
    build.build(verbose=False)
    return _lib.load()


def test_header_lists_expected_entry_points():
    fns = header_functions()
    for must in ("aiy_create", "aiy_destroy", "aiy_egm_step", "aiy_egm_solve", "aiy_sim_periods",
                 "aiy_hist_lottery", "aiy_hist_solve", "aiy_comm_init", "aiy_allreduce_sum", "aiy_policy_eval",
                 "aiy_wealth_stats", "aiy_sim_period_local", "aiy_sim_period_prices", "aiy_get_shocks",
                 "aiy_get_states", "aiy_get_controls", "aiy_get_poststates", "aiy_sum", "aiy_ge_stationary"):
        assert must in fns


def test_library_exports_every_header_symbol(lib):
    import subprocess
    from aiyagari_hark_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (aiy_\w+)", out))
    assert set(header_functions()) <= exported
    assert set(_lib.exported_symbols()) == set(header_functions())
    for name in header_functions():
        assert getattr(lib, name) is not None


def test_library_targets_gfx950():
    from aiyagari_hark_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_struct_layouts(lib):
    from aiyagari_hark_amd import _lib
    assert ctypes.sizeof(_lib.EgmDims) == 16
    assert ctypes.sizeof(_lib.EgmInputs) == 9 * 8
    assert ctypes.sizeof(_lib.Market) == 6 * 8
    assert ctypes.sizeof(_lib.PanelModel) == 16 + 5 * 8 + 8   # + act_T, unemployed
    assert ctypes.sizeof(_lib.PanelBatch) == 24 + 5 * 8 + 8   # + unemployed (padded)


def test_argument_validation_without_gpu(lib):
    from aiyagari_hark_amd import _lib
    assert lib.aiy_version() == 210
    # null handle -> AIY_ERR_ARG, nothing launched
    d = _lib.EgmDims(1, 28, 15, 32)
    i = _lib.EgmInputs()
    assert lib.aiy_egm_step(None, ctypes.byref(d), ctypes.byref(i), None, None, None, None, None) == -1
    assert lib.aiy_wealth_stats(None, None, None, 10, None, 1, None, None, None) == -1
    assert lib.aiy_create(0, None) == -1
    assert lib.aiy_comm_unique_id(None) == -1
    assert lib.aiy_destroy(None) == 0
    assert lib.aiy_get_shocks(None, 7, None, 10, 0, None, None, 0, 0, 0, None) == -1
    assert lib.aiy_get_poststates(None, 10, None, None, None, None) == -1
    assert lib.aiy_sum(None, None, 10, None, None) == -1
    assert lib.aiy_last_error(None) == b"null handle"


def test_product_refuses_cpu_tensors():
    import torch
    from aiyagari_hark_amd import _lib
    with pytest.raises(_lib.AiyagariLibError):
        _lib.ptr(torch.zeros(3, dtype=torch.float64))


def test_missing_library_fails_loudly(tmp_path):
    from aiyagari_hark_amd import _lib
    saved = _lib._lib
    _lib._lib = None
    try:
        with pytest.raises(_lib.AiyagariLibError):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved


def test_panel_table_bytes_host_only(lib):
    """aiy_panel_table_bytes is pure host arithmetic: sizes grow with the grid, and
    unsupported shapes are refused with -1 before any device work."""
    small = lib.aiy_panel_table_bytes(7, 15, 32, 0)
    big = lib.aiy_panel_table_bytes(7, 15, 10000, 0)
    assert lib.aiy_panel_table_bytes(7, 15, 32, 1) > small     # + the unemployed cells
    assert 0 < small < big
    assert small % 256 == 0 and big % 256 == 0
    assert lib.aiy_panel_table_bytes(7, 15, 1, 0) == -1
    assert lib.aiy_panel_table_bytes(0, 15, 32, 0) == -1
    assert lib.aiy_panel_table_bytes(17, 15, 32, 0) == -1


def test_option_constants_match_header():
    """Every AIY_OPT_* the header defines has the same value in the Python binding
    (aiyagari_hark_amd._lib), so aiy_set_option calls from Python mean what the C side reads."""
    import re
    from aiyagari_hark_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "aiyagari.h")).read()
    opts = dict((k, int(v)) for k, v in re.findall(r"#define (AIY_OPT_[A-Z0-9_]+) (\d+)", hdr))
    assert "AIY_OPT_GE_REBALANCE" in opts and "AIY_OPT_GE_EXTRAP_PERIOD" in opts
    for k, v in opts.items():
        assert getattr(_lib, k) == v, k


def test_firm_prices_use_libm_pow():
    """The Python GE loops price r through libm's pow, the function csrc/ge.hip calls
    (std::pow): numpy's vectorised power differs from it in the last bit on AVX-512 hosts,
    and one ulp of w moves a BiCGSTAB path."""
    import math

    import numpy as np

    from aiyagari_hark_amd.stationary import firm_prices
    rng = np.random.default_rng(5)
    r = np.concatenate([[float.fromhex("0x1.2a359f8a72972p-5")], rng.uniform(-0.04, 0.04, 500)])
    alpha = np.full_like(r, 0.36)
    w, kd = firm_prices(r, alpha, 0.08)
    for i in range(len(r)):
        k = math.pow(0.36 / (r[i] + 0.08), 1.0 / (1.0 - 0.36))
        assert kd[i] == k and w[i] == (1.0 - 0.36) * math.pow(k, 0.36)
    ws, ks = firm_prices(0.03, 0.36, 0.08)
    assert isinstance(ws, float) and ks == math.pow(0.36 / 0.11, 1.0 / 0.64)
