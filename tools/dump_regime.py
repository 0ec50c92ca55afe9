"""Dump the bench regime for host-side table analysis (run on the GPU box): the converged
policy of one bench GE solve (act_T = 2000) and a subsample of its end-of-history panel.
Writes gpurun_out/regime.npz (m_tab [S][n_M][n_a + 1], M_grid, lab_level, a, lab, sow)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    dev = torch.device("cuda:0")
    econ, agent = bench.make_economy(seed=0, n_agents=1000006, n_a=10000, act_T=2000, device=dev, t_discard=500)
    bench.run_step(econ, agent, bench.Probe())
    torch.cuda.synchronize()
    p = agent.panel
    keep = p._model[2]
    sol = agent.solution[0]
    step = int(os.environ.get("SUB", 4))
    out = os.path.join(ROOT, "gpurun_out", "regime.npz")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez(out, m_tab=sol.m_tab.cpu().numpy(), M_grid=keep["M_grid"].cpu().numpy(),
             lab_level=keep["lab_level"].cpu().numpy(), a=p.a[::step].cpu().numpy(), lab=p.lab[::step].cpu().numpy(),
             sow=p.sow.cpu().numpy())
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main()
