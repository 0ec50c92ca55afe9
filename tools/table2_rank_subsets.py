"""Predict the multi-GPU Table II sweep on one MI355X: time the sweep of each rank's
calibration subset (parallel.split_calibrations, as bench.py deals them) for N ranks, one
subset at a time; the N-GPU sweep takes as long as its slowest rank.  Optional second
argument: AIY_OPT_HIST_CLUSTER (max workgroups per calibration cluster).  JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.parallel import split_calibrations
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    n_ranks = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 4, 8]
    cluster = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    h = _lib.handle(0)
    h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_HIST_CLUSTER, cluster), "opt")
    cells = table2_calibrations()
    solve_table2(cells[:3], n_a=10000, device=dev, method="brent")   # warm-up
    for n in n_ranks:
        times = []
        for rank in range(n):
            mine = [cells[k] for k in split_calibrations(list(range(len(cells))), n, rank)]
            best = None
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                solve_table2(mine, n_a=10000, device=dev, method="brent")
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            times.append(best)
        print(json.dumps(dict(ranks=n, cluster_cap=cluster, rank_seconds=[round(t, 4) for t in times],
                              sweep_seconds=max(times), predicted_ge_solves_per_s=len(cells) / max(times))),
              flush=True)


if __name__ == "__main__":
    main()
