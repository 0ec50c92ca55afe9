"""Per-wave timeline of one EGM cycle launch at configs[1] size from the AIY_EGM_DIAG=8
build (lib/variants/libaiyagari_stamps.so, built by
`python -m aiyagari_hark_amd.build --variant stamps AIY_EGM_DIAG=8`): phase durations
in shader clocks and the dispatch / occupancy profile in wall time (100 MHz stamps).
Run on the GPU box."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("AIYAGARI_LIB", os.path.join(ROOT, "aiyagari_hark_amd", "lib", "variants",
                                                   "libaiyagari_stamps.so"))


def main():
    import torch
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    dev = torch.device("cuda:0")
    n_a = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    ss = sm.steady_state(1.0, 0.96, 0.08, 0.36, 1.0)
    aG = sm.make_grid_exp_mult(0.001, 50.0, n_a, 2)
    Mg = ss["MSS"] * sm.MGRID_BASE
    agg, E = sm.employment_chain(8, 8, 2.5, 1.5, 0, 0, 0.75, 1.25)
    y, P7 = sm.labor_tauchen(7, 0.6, 0.2)
    R, W, M = sm.next_prices([0.35, 0.36], [0.8, 0.8], Mg, 28, 0, 0, 1, 1, 1, 0.36, 0.08)
    lv = sm.labor_levels(y)
    b = EgmBatch.from_numpy(aG, Mg, sm.kron_states(P7, E), R, W, M, [lv[s // 4] for s in range(28)], 0.96, 1.0,
                            device=dev)
    mt, ct, _, _ = egm_solve(b)
    m0, c0 = mt.contiguous(), ct.contiguous()
    mo, co = torch.empty_like(m0), torch.empty_like(c0)
    d, i = b._abi()
    h = _lib.handle(0)
    ms = ctypes.c_float()
    h.check(h.lib.aiy_egm_kernel_time(h.h, ctypes.byref(d), ctypes.byref(i), _lib.ptr(m0), _lib.ptr(c0), _lib.ptr(mo),
                                      _lib.ptr(co), 3, ctypes.byref(ms), torch.cuda.current_stream().cuda_stream), "t")
    n_tiles = (n_a + 63) // 64
    n_waves = n_tiles * Mg.size * 4
    buf = (ctypes.c_ulonglong * (n_waves * 6))()
    fn = h.lib.aiy_egm_diag_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    assert fn(buf, n_waves * 6) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n_waves, 6).astype(np.int64)
    t0 = st[:, 0] - st[:, 0].min()                       # 10 ns ticks
    clk = st[:, 1:] - st[:, 1:2]                          # shader clocks since the wave's start
    ph = np.diff(st[:, 1:], axis=1)                       # prologue, phase 1, barrier, phase 2
    life = clk[:, -1]
    # clock rate from the longest-lived waves: realtime span vs clock span is not per wave;
    # report cycles and the wall-time spread of starts
    out = dict(kernel_us_avg=ms.value * 1e3 / 3, waves=n_waves,
               start_spread_us=float(t0.max()) / 100.0,
               start_pct_us={p: float(np.percentile(t0, p)) / 100.0 for p in (10, 50, 90, 99)},
               life_cycles_pct={p: float(np.percentile(life, p)) for p in (10, 50, 90, 99)},
               phase_cycles_median=dict(zip(["prologue", "phase1", "sync", "phase2"],
                                            [float(np.median(ph[:, k])) for k in range(4)])),
               phase_cycles_p90=dict(zip(["prologue", "phase1", "sync", "phase2"],
                                         [float(np.percentile(ph[:, k], 90)) for k in range(4)])))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
