"""Solution save/load: policy tables and AFunc round-trip through
``.npz`` bit-exactly, the file holds plain arrays only, and malformed files are refused.
CPU only: the tables live in CPU tensors here, no kernel is called."""
import numpy as np
import pytest
import torch

from aiyagari_hark_amd.interp import DeviceSolution
from aiyagari_hark_amd.model import AggregateSavingRule


def _solution(S=28, n_M=15, n_a=33, seed=0):
    rng = np.random.default_rng(seed)
    m = np.cumsum(rng.random((S, n_M, n_a)), axis=2)
    c = m * rng.random((S, n_M, n_a))
    Mg = np.linspace(0.685, 20.56, n_M)
    return DeviceSolution(torch.from_numpy(m), torch.from_numpy(c), torch.from_numpy(Mg), 1.0)


def test_round_trip_bit_exact(tmp_path):
    sol = _solution()
    afunc = [AggregateSavingRule(0.1, 0.9), AggregateSavingRule(-0.05, 1.02)]
    path = tmp_path / "sol.npz"
    sol.save(path, AFunc=afunc)
    back, af = DeviceSolution.load(path, torch.device("cpu"))
    assert torch.equal(back.m_tab, sol.m_tab) and torch.equal(back.c_tab, sol.c_tab)
    assert torch.equal(back.M_grid, sol.M_grid) and back.CRRA == sol.CRRA
    np.testing.assert_array_equal(af, [[0.1, 0.9], [-0.05, 1.02]])
    assert len(back.cFunc) == 28 and len(back.cFunc[3].xInterpolators) == 15
    np.testing.assert_array_equal(back.cFunc[3].xInterpolators[7].x_list, sol.m_host()[3, 7])


def test_without_afunc_and_plain_arrays(tmp_path):
    path = tmp_path / "sol.npz"
    _solution(S=7, n_M=1, n_a=10001).save(path)
    with np.load(path, allow_pickle=False) as z:
        assert "afunc" not in z.files
        assert all(z[k].dtype != object for k in z.files)
    _, af = DeviceSolution.load(path, torch.device("cpu"))
    assert af is None


def test_refuses_inconsistent_file(tmp_path):
    path = tmp_path / "bad.npz"
    np.savez(path, m=np.zeros((2, 3, 4)), c=np.zeros((2, 3, 5)), M_grid=np.zeros(3), CRRA=np.float64(1),
             format_version=np.int64(1))
    with pytest.raises(ValueError, match="inconsistent"):
        DeviceSolution.load(path, torch.device("cpu"))
    np.savez(path, m=np.zeros((2, 3, 4)), c=np.zeros((2, 3, 4)), M_grid=np.zeros(3), CRRA=np.float64(1),
             format_version=np.int64(99))
    with pytest.raises(ValueError, match="format"):
        DeviceSolution.load(path, torch.device("cpu"))
