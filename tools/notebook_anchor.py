#!/usr/bin/env python3
"""Seed distribution of the notebook configuration (tests/test_gpu_anchor.py) with the
z-score of every statistic the reference notebook recorded; one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.test_gpu_anchor import NOTEBOOK, seed_distribution  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    dist = seed_distribution(torch.device("cuda:0"), n)
    out = {}
    for k, want in NOTEBOOK.items():
        mu, sd = float(np.mean(dist[k])), float(np.std(dist[k], ddof=1))
        out[k] = dict(notebook=want, seed_mean=mu, seed_sd=sd, z=(want - mu) / sd, seed_min=float(dist[k].min()),
                      seed_max=float(dist[k].max()))
    print(json.dumps(dict(seeds=n, config="rho=0.3 sigma=0.2 CRRA=1, 350 agents, act_T=11000, Philox", stats=out)))


if __name__ == "__main__":
    main()
