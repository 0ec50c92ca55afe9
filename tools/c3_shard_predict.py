#!/usr/bin/env python3
"""Per-rank prediction of the 8-GPU configs[3] period, on ONE GPU.

At 8 ranks each rank simulates 12.5M of the 99 999 998 agents (parallel.shard_range splits
on agent pairs) and every period is: the resident panel kernel on the shard (one launch,
the shard's sum of a left in sow[6]) -> ncclAllReduce of that double -> the price kernel
(csrc/panel.hip, aiy_sim_periods with a communicator bound).  Here one rank holds a
12.5M-agent shard bound to torch's own one-rank RCCL communicator (parallel.bind_rccl), so
every step of the sharded period runs; only the all-reduce's wire time is missing (one
double per period over xGMI).  Printed beside it: the same shard on the single-rank path
(one persistent launch for all periods).

    python tools/c3_shard_predict.py [--agents 12499998] [--periods 1000]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=12_499_998)   # a shard of 99 999 998 over 8, a multiple of 7
    ap.add_argument("--periods", type=int, default=1000)
    ap.add_argument("--grid", type=int, default=10_000)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    from aiyagari_hark_amd import _lib, build
    from aiyagari_hark_amd.parallel import bind_rccl, unbind_rccl
    build.build(verbose=False)
    h = _lib.handle(0)
    econ, agent = bench.c3_policy(dev, args.grid)
    T, N = args.periods, args.agents
    out = {"agents_per_rank": N, "periods": T}
    for mode in ("single_rank", "sharded_rccl"):
        comm = None
        if mode == "sharded_rccl":
            comm = bind_rccl(h)[2]
        try:
            p, reset = bench.c3_panel(dev, econ, agent, N, T)
            p.run(0, 16, shock_mode="philox", seed=bench.C3_SEED, ge_iter=0)   # warm-up
            reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.run(0, T, shock_mode="philox", seed=bench.C3_SEED, ge_iter=0)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            K = p.hist_A[:T].cpu().numpy()
        finally:
            if comm is not None:
                unbind_rccl(h)
        out[mode] = {"seconds": el, "us_per_period": 1e6 * el / T, "agent_periods_per_s": N * T / el,
                     "communicator": comm, "K_first": [float(x) for x in K[:3]], "K_last": float(K[T - 1])}
        print(json.dumps({mode: out[mode]}), flush=True)
    out["same_history"] = out["single_rank"]["K_last"] == out["sharded_rccl"]["K_last"]
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
