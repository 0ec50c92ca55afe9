"""Native Table II sweep with and without the EGM iterate extrapolation (aiy_ge_options.egm_extrapolate):
wall time, K_s evaluations and the summed EGM cycles / histogram matvecs over all calibrations."""
import sys, time, json
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import torch
from aiyagari_hark_amd.stationary import solve_table2
dev = torch.device("cuda:0")
solve_table2(n_a=1000, device=dev, max_steps=3, method="brent")
for ex in (False, True, False, True):
    torch.cuda.synchronize(); t = time.perf_counter()
    res = solve_table2(device=dev, method="brent", extrapolate=ex)
    torch.cuda.synchronize()
    print(json.dumps(dict(extrapolate=ex, seconds=time.perf_counter() - t, steps=res.bisection_steps,
                          egm_cycles_sum=int(res.egm_cycles[0][0]), hist_matvecs_sum=int(res.hist_iters[0][0]))), flush=True)
