"""Panel-kernel tuning sweep (run on the GPU box): per-period time of the persistent
panel at configs[1] size (N_a = 10 000, 1 000 006 agents) for every library build
listed in $AIY_VARIANTS (name=path.so, comma separated; default: the in-tree build)
and every (resident, agents-per-lane, order) option.  Each variant runs in its own
child process (the library is loaded once per process).  Prints one JSON line per
measurement."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, opts):
    sys.path.insert(0, ROOT)
    if lib:
        os.environ["AIYAGARI_LIB"] = lib
    import ctypes
    import numpy as np
    import torch
    from aiyagari_hark_amd import _lib, setup_math as sm
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    from aiyagari_hark_amd.panel import DevicePanel
    dev = torch.device("cuda:0")
    n_a = int(os.environ.get("NA", 10000))
    N = int(os.environ.get("NAG", 1000006))
    T = int(os.environ.get("T", 400))
    ss = sm.steady_state(1.0, 0.96, 0.08, 0.36, 1.0)
    aG = sm.make_grid_exp_mult(0.001, 50.0, n_a, 2)
    Mg = ss["MSS"] * sm.MGRID_BASE
    agg, E = sm.employment_chain(8, 8, 2.5, 1.5, 0, 0, 0.75, 1.25)
    y, P7 = sm.labor_tauchen(7, 0.6, 0.2)
    P = sm.kron_states(P7, E)
    R, W, M = sm.next_prices([0.35, 0.36], [0.8, 0.8], Mg, 28, 0, 0, 1, 1, 1, 0.36, 0.08)
    lv = sm.labor_levels(y)
    lab = np.array([lv[s // 4] for s in range(28)])
    b = EgmBatch.from_numpy(aG, Mg, P, R, W, M, lab, 0.96, 1.0, device=dev)
    m, c, cyc, d = egm_solve(b)
    h = _lib.handle(0)
    out = []
    bench_panel = None
    if os.environ.get("BENCH_REGIME"):
        # the bench's own economy after one GE solve (act_T = 2000): its converged policy
        # and end-of-history population
        sys.path.insert(0, ROOT)
        import bench
        econ, agent = bench.make_economy(seed=0, n_agents=N, n_a=n_a, act_T=2000, device=dev, t_discard=500)
        econ.solve()
        bench_panel = agent.panel
    fuse = int(os.environ.get("FUSE", "1"))
    if hasattr(_lib, "AIY_OPT_RESIDENT_FUSE") and hasattr(h.lib, "aiy_get_option"):
        h.set_options({_lib.AIY_OPT_RESIDENT_FUSE: fuse})
    if hasattr(_lib, "AIY_OPT_RESIDENT_SHAPE_STREAM") and hasattr(h.lib, "aiy_get_option"):
        h.set_options({_lib.AIY_OPT_RESIDENT_SHAPE_STREAM: -1})   # the shape under test for both forms
    if hasattr(_lib, "AIY_OPT_RESIDENT_ENGINE") and hasattr(h.lib, "aiy_get_option"):
        h.set_options({_lib.AIY_OPT_RESIDENT_ENGINE: int(os.environ.get("ENGINE", "1"))})
    for (res, agents, order, presort, Tt) in opts:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT, res), "opt")
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT_SHAPE, order), "opt")
        if bench_panel is not None:
            p = bench_panel
            a0, l0, s0 = p.a.clone(), p.lab.clone(), p.sow.clone()
            pm, mk = p._model[:2]
            ms = ctypes.c_float()
            h.check(h.lib.aiy_sim_kernel_time(h.h, ctypes.byref(pm), ctypes.byref(mk), N, _lib.ptr(a0), _lib.ptr(l0),
                                              99, 7, _lib.ptr(s0), Tt, ctypes.byref(ms),
                                              torch.cuda.current_stream().cuda_stream), "time")
            out.append(dict(lib=os.path.basename(lib or "default"), regime="bench", resident=res, agents=agents,
                            order=order, T=Tt, us_per_period=1e3 * ms.value / Tt, K=float(a0.mean())))
            print(json.dumps(out[-1]), flush=True)
            continue
        p = DevicePanel(N, device=dev, act_T=T)
        hist = torch.as_tensor(sm.markov_history(agg, T).astype(np.int32)).to(dev)
        p.bind_model(m[0], c[0], b.M_grid[0], torch.as_tensor(lv).to(dev),
                     torch.as_tensor(sm.choice_cdf_table(P7)).to(dev), hist,
                     dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
        p.reset(ss["KSS"], np.repeat(np.arange(7), N // 7 + 1)[:N], ss["MSS"], ss["KSS"], 0, ss["RSS"], ss["WSS"])
        # burn in to the ergodic wealth distribution, then time T periods
        p.run(0, T, shock_mode="philox", seed=1)
        torch.cuda.synchronize()
        if presort:   # global wealth order (Philox keyed by position: timing experiment only)
            # PRESORT_KEY=la: by (labour state, assets); default: by assets
            pk = os.environ.get("PRESORT_KEY", "")
            k = p.a + 1e4 * p.lab.double() if pk in ("la", "local") else p.a
            if pk == "local":   # within each workgroup's slice of the streaming form (256 slices)
                ch = (N + 255) // 256
                ch += ch & 1
                k = k + 1e6 * (torch.arange(N, device=dev) // ch).double()
            key, perm = torch.sort(k)
            key = p.a[perm]
            p.a.copy_(key)
            p.lab.copy_(p.lab[perm])
            torch.cuda.synchronize()
        pm, mk = p._model[:2]
        ms = ctypes.c_float()
        h.check(h.lib.aiy_sim_kernel_time(h.h, ctypes.byref(pm), ctypes.byref(mk), N, _lib.ptr(p.a), _lib.ptr(p.lab),
                                          3, 1, _lib.ptr(p.sow), Tt, ctypes.byref(ms),
                                          torch.cuda.current_stream().cuda_stream), "time")
        out.append(dict(lib=os.path.basename(lib or "default"), fuse=fuse, engine=os.environ.get("ENGINE", "1"), resident=res, agents=agents, order=order,
                        presort=presort, T=Tt,
                        us_per_period=1e3 * ms.value / Tt, K=float(p.a.mean())))
        print(json.dumps(out[-1]), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        lib = sys.argv[2] if sys.argv[2] != "-" else None
        opts = json.loads(sys.argv[3])
        child(lib, opts)
        return
    variants = os.environ.get("AIY_VARIANTS", "")
    libs = [("default", None)] + [tuple(v.split("=", 1)) for v in variants.split(",") if v]
    # (resident, unused, resident shape, presort, periods)
    opts_all = [(1, 0, 0, 0, 400), (1, 0, 1, 0, 400), (0, 0, 0, 0, 400), (1, 0, 0, 0, 50), (1, 0, 0, 1, 50)]
    opts_var = [(1, 0, 0, 0, 400)]
    if os.environ.get("OPTS"):
        opts_all = opts_var = [tuple(o) for o in json.loads(os.environ["OPTS"])]
    for name, lib in libs:
        opts = opts_all if (lib is None or os.environ.get("OPTS")) else opts_var
        rc = subprocess.run([sys.executable, __file__, "--child", lib or "-", json.dumps(opts)], timeout=300).returncode
        if rc != 0:
            print(json.dumps(dict(lib=name, error=rc)), flush=True)
            sys.exit(rc)


if __name__ == "__main__":
    main()
