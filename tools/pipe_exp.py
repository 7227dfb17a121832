#!/usr/bin/env python3
"""Experiment: the config-3 window-path solve split into P concurrent pipelines (contiguous
date blocks, each with its own plans, workspace, HIP stream and host thread) on one GPU.
Prints wall ms per step for each P given on the command line -- experiment tooling."""
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import engine  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def build(pan, rows, tlen, dev, n):
    D = len(tlen)
    rows_d, tlen_d = pan.rows_to_device(rows, tlen)
    gplan = engine.GroupPlan(rows, tlen, dev)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)),
                                   b=np.ones(1), lb=np.zeros(n), ub=np.ones(n), device=dev)
    qb.batch = D
    qb.P = None
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=dev)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    mu = pan.window_means(rows_d, tlen_d)
    lr = engine.LowRank(pan, rows_d, tlen_d, mu=mu, w_scale=1.0 / (tlen_d.to(torch.float64) - 1.0))
    ws = engine.Workspace(qb, dense=False)
    return dict(rows_d=rows_d, tlen_d=tlen_d, gplan=gplan, qb=qb, mu=mu, lr=lr, ws=ws,
                stream=torch.cuda.Stream(device=dev))


def main():
    Ps = [int(a) for a in sys.argv[1:]] or [1, 2]
    n, T, D = 1000, 252, 4749
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + D], T)
    pan = engine.Panel(R, device=dev)
    settings = engine.Settings()
    for P in Ps:
        cuts = np.linspace(0, D, P + 1).astype(int)
        pipes = [build(pan, rows[a:b], tlen[a:b], dev, n) for a, b in zip(cuts[:-1], cuts[1:])]

        def run(p, out, i):
            torch.cuda.set_device(dev)
            with torch.cuda.stream(p["stream"]):
                pan.window_means(p["rows_d"], p["tlen_d"], out=p["mu"])
                p["lr"].refresh()
                out[i] = engine.solve_lowrank(p["qb"], p["lr"], settings, p["ws"], groups=p["gplan"])

        def step():
            out = [None] * P
            th = [threading.Thread(target=run, args=(p, out, i)) for i, p in enumerate(pipes)]
            for t_ in th:
                t_.start()
            for t_ in th:
                t_.join()
            return out

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            out = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        st = np.concatenate([o.status.cpu().numpy() for o in out])
        print(f"P={P}: {dt * 1e3:.1f} ms/step  {D / dt:.0f} QPs/s  status {np.unique(st, return_counts=True)}",
              flush=True)


if __name__ == "__main__":
    main()
