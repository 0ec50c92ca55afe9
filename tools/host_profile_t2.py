#!/usr/bin/env python3
"""Host-side cost of one Table II sweep (the bench's step): cProfile of solve_table2 after
warm-up sweeps, top functions by cumulative and own time (the device time is inside the
library's synchronising calls)."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    cals = table2_calibrations()
    for _ in range(3):
        solve_table2(cals, n_a=10000, device=dev, method="brent")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        solve_table2(cals, n_a=10000, device=dev, method="brent")
    torch.cuda.synchronize()
    print(f"plain: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms per sweep", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        solve_table2(cals, n_a=10000, device=dev, method="brent")
    torch.cuda.synchronize()
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(25)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
