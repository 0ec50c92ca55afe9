"""Where the configs[3] panel's table lookups land (design study for the streaming form).

Runs the configs[3] household (bench.c3_policy / c3_panel) for T periods at N agents, then,
for the agents of the last period, reads the merged policy table the kernel uses
(panel_common.h layout: rec [cells][Z + 1][4] double2 | z [cells][Z] | idx) and reports per
active cell: how many agents, the spread of their record positions (quantiles of lower_bound
in z), the distinct records / 128-B record lines / index lines they touch, and how the
index buckets of the occupied window fill.  Prints one JSON line.
    python tools/lookup_locality.py [N] [T]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def align(b):
    return (b + 255) // 256 * 256


def main():
    import torch
    import bench
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_002
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda:0")
    econ, agent = bench.c3_policy(dev, bench.N_A)
    p, reset = bench.c3_panel(dev, econ, agent, N, T)
    p.run(0, T, shock_mode="philox", seed=bench.C3_SEED, ge_iter=0)
    torch.cuda.synchronize()
    pm, mk, keep, pb = p._model
    tab = keep["tables"].cpu().numpy().reshape(-1)
    Mg = keep["M_grid"].cpu().numpy()
    lvl = keep["lab_level"].cpu().numpy()
    sow = p.sow.cpu().numpy()
    Mnow, Mrkv, Rnow, Wnow = float(sow[0]), int(sow[2]), float(sow[3]), float(sow[4])
    n_lab = lvl.size
    n_M = Mg.size
    n_a = int(pm.n_a) if hasattr(pm, "n_a") else bench.N_A
    Z = 2 * n_a
    n_J = n_M - 1 if n_M > 1 else 1
    n_cells = 2 * n_lab * n_J
    lg = 4
    while lg < 13 and (1 << lg) < n_a:
        lg += 1
    shift = 52 - lg
    buckets = 12 << lg
    z_off = align(n_cells * 4 * (Z + 1) * 16)
    z = tab[z_off:z_off + n_cells * Z * 8].view(np.float64).reshape(n_cells, Z)
    j = int(np.clip(np.searchsorted(Mg, Mnow, side="left"), 1, n_M - 1))
    jc = j - 1
    a = p.a.cpu().numpy()
    lab = p.lab.cpu().numpy().astype(np.int64)
    m = Rnow * a + Wnow * lvl[lab]
    out = dict(R=Rnow, W=Wnow, M=Mnow, N=N, T=T, n_a=n_a, Z=Z, n_M=n_M, jc=jc, Mrkv=Mrkv, buckets_per_octave=1 << lg, cells=[])
    tot_rec_lines = tot_idx_lines = 0
    for l in range(n_lab):
        sel = lab == l
        if not sel.any():
            continue
        cell = (2 * l + Mrkv) * n_J + jc
        zz = z[cell]
        mm = m[sel]
        pos = np.searchsorted(zz, mm, side="left")
        q = np.quantile(pos, [0.0, 0.001, 0.01, 0.5, 0.99, 0.999, 1.0]).astype(int).tolist()
        uniq = np.unique(pos)
        rec_lines = np.unique(pos // 2)            # 64-B records, 128-B lines
        keys = (mm.view(np.int64) >> shift)
        kq = np.quantile(keys, [0.001, 0.999]).astype(np.int64)
        nodes_k = (zz[2:].view(np.int64) >> shift)
        in_win = (nodes_k >= kq[0]) & (nodes_k <= kq[1])
        win_buckets = int(kq[1] - kq[0] + 1)
        idx_lines = np.unique(keys // 16)          # 8-B entries, 128-B lines
        tot_rec_lines += rec_lines.size
        tot_idx_lines += idx_lines.size
        pmin = int(pos.min())
        within = {str(K): float(np.mean(pos < pmin + K)) for K in (1, 2, 4, 16, 64, 256, 1024, 4096)}
        out["cells"].append(dict(l=l, agents=int(sel.sum()), pos_q=q, frac_within_K_of_min=within,
                                 m_min=float(mm.min()), W_lvl=float(Wnow * lvl[l]), z_at_min=float(zz[pmin]), distinct_records=int(uniq.size),
                                 record_lines=int(rec_lines.size), index_lines=int(idx_lines.size),
                                 window_buckets_999=win_buckets, window_nodes_999=int(in_win.sum()),
                                 octaves_999=win_buckets / (1 << lg)))
    out["record_lines_total"] = tot_rec_lines
    out["index_lines_total"] = tot_idx_lines
    out["footprint_MB"] = 128 * (tot_rec_lines + tot_idx_lines) / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
