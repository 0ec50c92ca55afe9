"""Table II sweep with the calibrations split into independent searches (solve_table2
groups=k: own handle, stream and host thread per group) on one MI355X, for the full
24-cell sweep and for each rank's 3-cell subset of an 8-GPU run; best of 3; JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd.parallel import split_calibrations
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    cells = table2_calibrations()
    ref = solve_table2(cells, device=dev, method="brent")
    for groups in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]:
        best, res = None, None
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            res = solve_table2(cells, device=dev, method="brent", groups=groups)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        print(json.dumps(dict(cells=24, groups=groups, seconds=best, ge_solves_per_s=24 / best,
                              max_abs_dr=float(np.max(np.abs(res.r - ref.r))))), flush=True)
    for groups in (1, 3):
        times = []
        for rank in range(8):
            mine = [cells[k] for k in split_calibrations(list(range(24)), 8, rank)]
            best = None
            for _ in range(2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                solve_table2(mine, device=dev, method="brent", groups=groups)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            times.append(best)
        print(json.dumps(dict(ranks=8, groups_per_rank=groups, rank_seconds=[round(x, 4) for x in times],
                              predicted_ge_solves_per_s=24 / max(times))), flush=True)


if __name__ == "__main__":
    main()
