"""EGM cycle-kernel timing at configs[1] size (N_a = 10 000, 28 x 15 rows) for the library
builds listed in $AIY_VARIANTS (name=path.so, comma separated) plus the in-tree build; one
child process per library; prints one JSON line each (run on the GPU box)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    if lib != "-":
        os.environ["AIYAGARI_LIB"] = lib
    sys.path.insert(0, ROOT)
    import time
    import torch
    from aiyagari_hark_amd import setup_math as sm
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    dev = torch.device("cuda:0")
    ss = sm.steady_state(1.0, 0.96, 0.08, 0.36, 1.0)
    aG = sm.make_grid_exp_mult(0.001, 50.0, 10000, 2)
    Mg = ss["MSS"] * sm.MGRID_BASE
    agg, E = sm.employment_chain(8, 8, 2.5, 1.5, 0, 0, 0.75, 1.25)
    y, P7 = sm.labor_tauchen(7, 0.6, 0.2)
    R, W, M = sm.next_prices([0.35, 0.36], [0.8, 0.8], Mg, 28, 0, 0, 1, 1, 1, 0.36, 0.08)
    lv = sm.labor_levels(y)
    lab = [lv[s // 4] for s in range(28)]
    b = EgmBatch.from_numpy(aG, Mg, sm.kron_states(P7, E), R, W, M, lab, 0.96, 1.0, device=dev)
    egm_solve(b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    _, _, cyc, _ = egm_solve(b)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    import ctypes
    from aiyagari_hark_amd import _lib
    mt, ct, _, _ = egm_solve(b)
    m0, c0 = mt.contiguous(), ct.contiguous()
    mo, co = torch.empty_like(m0), torch.empty_like(c0)
    d, i = b._abi()
    h = _lib.handle(0)
    ms = ctypes.c_float()
    n = 50
    h.check(h.lib.aiy_egm_kernel_time(h.h, ctypes.byref(d), ctypes.byref(i), _lib.ptr(m0), _lib.ptr(c0), _lib.ptr(mo),
                                      _lib.ptr(co), n, ctypes.byref(ms), torch.cuda.current_stream().cuda_stream), "t")
    print(json.dumps(dict(lib=os.path.basename(lib), cycles=int(cyc[0]), solve_s=dt,
                          us_per_cycle=1e6 * dt / int(cyc[0]), kernel_us=1e3 * ms.value / n)), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    libs = ["-"] + [v.split("=", 1)[1] for v in os.environ.get("AIY_VARIANTS", "").split(",") if v]
    for lib in libs:
        rc = subprocess.run([sys.executable, __file__, "--child", lib], timeout=300).returncode
        if rc:
            sys.exit(rc)
