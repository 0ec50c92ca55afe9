"""CPU checks of the full-size oracle fixtures the -m gpu parity tests pin the benchmarked
configurations with (tests/golden/fullsize_*.json, made by make_golden_fullsize.py and
make_golden_c3.py): internal consistency against closed forms of the model, so a fixture
that was cut short or mis-assembled fails here, not on the GPU box."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ALPHA, DELTA, BETA = 0.36, 0.08, 0.96


def _load(name):
    path = os.path.join(GOLD, f"fullsize_{name}.json")
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: run tests/golden/make_golden_fullsize.py / make_golden_c3.py")
    return json.load(open(path))


def _kd(r):
    return (ALPHA / (r + DELTA)) ** (1.0 / (1.0 - ALPHA))


@pytest.mark.parametrize("which,n,n_a,S", [("table2", 24, 10_000, 7), ("stress", 3, 50_000, 25)])
def test_ge_fixture_consistent(which, n, n_a, S):
    fx = _load(which)
    cells = fx["cells"]
    assert [c["k"] for c in cells] == list(range(n))
    for c in cells:
        assert c["n_a"] == n_a and c["S"] == S
        # ge_bisect's final bracket, r its midpoint, inside the theoretical bracket
        assert 0 < c["hi"] - c["lo"] <= 1e-7
        assert c["r"] == pytest.approx(0.5 * (c["lo"] + c["hi"]), abs=1e-15)
        assert -DELTA / 2 < c["r"] < 1 / BETA - 1
        # K = K_d(r), K/Y = K^(1 - alpha), saving rate = delta K/Y (Table II identity)
        assert c["K"] == pytest.approx(_kd(c["r"]), rel=1e-14)
        assert c["KtoY"] == pytest.approx(c["K"] ** (1 - ALPHA), rel=1e-14)
        assert c["saving_rate"] == pytest.approx(DELTA * c["KtoY"], rel=1e-14)
        # at the root K_s = K_d to the bracket's resolution (dK_s/dr is large near 1/beta - 1)
        assert abs(c["Ks_at_r"] - c["Kd_at_r"]) / c["Kd_at_r"] < 1e-3
        assert c["mass_total_at_r"] == pytest.approx(1.0, abs=1e-9)
        assert c["steps"] >= 19 and c["egm_cycles_at_r"] > 10 and c["hist_iters_at_r"] > 10


def test_table2_fixture_orders():
    """Aiyagari (1994) Table II's comparative statics hold in the oracle's roots: r falls
    with CRRA, with rho and with sigma (more precautionary saving), and every r lies below
    the complete-markets 1/beta - 1."""
    cells = _load("table2")["cells"]
    r = {(c["sigma"], c["rho"], c["crra"]): c["r"] for c in cells}
    for s in (0.2, 0.4):
        for rho in (0.0, 0.3, 0.6, 0.9):
            assert r[(s, rho, 1.0)] > r[(s, rho, 3.0)] > r[(s, rho, 5.0)]
        for mu in (1.0, 3.0, 5.0):
            assert r[(s, 0.0, mu)] > r[(s, 0.3, mu)] > r[(s, 0.6, mu)] > r[(s, 0.9, mu)]
    for rho in (0.0, 0.3, 0.6, 0.9):
        for mu in (1.0, 3.0, 5.0):
            assert r[(0.2, rho, mu)] > r[(0.4, rho, mu)]


def test_c3_fixture_consistent():
    fx = _load("c3")
    N, T = fx["agents"], fx["periods"]
    assert N == 99_999_998 and T >= 3 and fx["n_a"] == 10_000
    assert len(fx["hist_A"]) == len(fx["hist_M"]) == len(fx["lab_counts"]) == T
    for t in range(T):
        assert sum(fx["lab_counts"][t]) == N
        K = fx["hist_A"][t]
        # calc_R_and_W (AS:1839-1894) with L = 1, Prod = 1
        R = 1 + ALPHA * K ** (ALPHA - 1) - DELTA
        W = (1 - ALPHA) * K ** ALPHA
        assert fx["hist_R"][t] == pytest.approx(R, rel=1e-14)
        assert fx["hist_W"][t] == pytest.approx(W, rel=1e-14)
        assert fx["hist_M"][t] == pytest.approx(R * K + W, rel=1e-14)
    assert fx["a_sum_final"] / N == pytest.approx(fx["hist_A"][-1], rel=1e-12)
    assert len(fx["sample_idx"]) == len(fx["sample_a"]) == len(fx["sample_lab"])
    assert all(0 <= l < 7 for l in fx["sample_lab"])
    # from the even birth split the Tauchen chain (symmetric about its middle state) moves
    # mass toward the middle; the counts stay mirror-symmetric up to sampling noise
    for cnt in fx["lab_counts"]:
        assert all(abs(cnt[l] - cnt[6 - l]) < 10 * np.sqrt(cnt[l]) + 1 for l in range(3))
    mid = [c[3] for c in fx["lab_counts"]]
    assert all(b > a for a, b in zip(mid, mid[1:]))
