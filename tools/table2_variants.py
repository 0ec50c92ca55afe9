"""Table II sweep (native search, Brent) through each library build named in argv (paths;
'-' = the in-tree build), one child process per library, best of 3 sweeps; JSON lines."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import time
    import torch
    from aiyagari_hark_amd.stationary import solve_table2
    dev = torch.device("cuda:0")
    solve_table2(device=dev, method="brent")
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = solve_table2(device=dev, method="brent")
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    print(json.dumps(dict(lib=os.environ.get("AIYAGARI_LIB", "in-tree"), seconds=best, ge_solves_per_s=24 / best,
                          egm_cycles_sum=int(res.egm_cycles[0][0]), hist_matvecs_sum=int(res.hist_iters[0][0]))),
          flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    for lib in sys.argv[1:] or ["-"]:
        env = dict(os.environ)
        if lib != "-":
            env["AIYAGARI_LIB"] = lib
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, check=True)


if __name__ == "__main__":
    main()
