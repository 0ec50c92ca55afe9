"""Diagnostic run of the preconditioned resident distribution solve (diag build with
-DAIY_DIAG_PC: restart / iteration / build prints of cluster 0, workgroup 0)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from aiyagari_hark_amd.stationary import solve_table2, table2_calibrations
    dev = torch.device("cuda:0")
    cals = [table2_calibrations()[0]]
    n_a = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    res = solve_table2(cals, n_a=n_a, device=dev, method="bisect", accel=-1, warm_egm=True, groups=1, resident=True,
                       max_steps=2)
    torch.cuda.synchronize()
    print("r", res.r, "status", res.status, "its", res.hist_iters, flush=True)


if __name__ == "__main__":
    main()
