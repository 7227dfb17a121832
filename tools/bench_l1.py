#!/usr/bin/env python3
"""Throughput of the l1 row on the config-3 workload (n = 1000, T = 252, 4749 daily dates,
long-only min-variance) with a transaction cost c * sum|x - x0| (--cost, default 1e-5) around a fixed x0
(or a turnover budget with --budget TAU): the signed split on the window path over the
panel [R, -R] (2n = 2000 variables per date).  Prints one JSON line; the split setup
(P x0 through one panel GEMM, the split panel) is inside the timed step."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.l1split import L1Split, merge_batch, split_batch  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def stage_ms(events):
    out = {}
    for name, e0, e1 in events:
        out[name] = round(out.get(name, 0.0) + e0.elapsed_time(e1), 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--budget", type=float, default=None)
    ap.add_argument("--cost", type=float, default=1e-5)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--both", type=str, default=None, metavar="TAU,L",
                    help="turnover budget TAU and leverage budget L together, long-short box "
                         "[-0.05, 0.1]: the per-asset-block IPM (porqua_amd/ipm_l1.py)")
    ap.add_argument("--chunk", type=int, default=4749)
    ap.add_argument("--ipm", action="store_true", help="--both: the per-asset-block IPM instead of the segment "
                    "split on the ADMM engine (porqua_amd/l1seg.py)")
    ap.add_argument("--no-gcap", action="store_true", help="per-date capacitances (per-date rho) instead of "
                    "the group capacitance")
    args = ap.parse_args()
    if args.both:
        return both(args)
    n, T, D = 1000, 252, 4749
    dev = torch.device("cuda", 0)
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + D], T)
    pan = engine.Panel(R, device=dev)
    rows_d, tlen_d = pan.rows_to_device(rows, tlen)
    gplan = engine.GroupPlan(rows, tlen, dev)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.ones(n), device=dev)
    qb.batch, qb.P = D, None
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=dev)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    mu = pan.window_means(rows_d, tlen_d)
    lr = engine.LowRank(pan, rows_d, tlen_d, mu=mu, w_scale=1.0 / (tlen_d.to(torch.float64) - 1.0))
    x0 = np.random.default_rng(1).dirichlet(np.ones(n))
    term = L1Split("budget", x0, args.budget) if args.budget else L1Split("cost", x0, args.cost)
    split_panel = engine.Panel(torch.cat([pan.R, -pan.R], 1).contiguous(), None, device=dev)
    from porqua_amd.l1split import split_settings
    ov = dict(kv.split("=", 1) for kv in args.set)
    settings = split_settings(engine.Settings.from_params(ov), ov, term.kind)

    ev = []

    def step():
        ev.clear()
        qb2, lr2, const = split_batch(qb, lr, term, split_panel, np.ones((1, n)), np.ones(1), None, None,
                                      np.zeros(n), np.ones(n))
        res = engine.solve_lowrank(qb2, lr2, settings, groups=gplan, events=ev, gcap=not args.no_gcap)
        return res, merge_batch(res.x, term)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, x = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    st = res.status.cpu().numpy()
    xh = x.cpu().numpy()
    print(json.dumps({"workload": "config3 + " + (f"turnover budget {args.budget}" if args.budget else
                                                  f"transaction cost {args.cost}") + " (l1 split, window path, 2n = 2000)",
                      "qps": D / dt, "ms_per_step": dt * 1e3, "status_counts": {str(k): int(v) for k, v in
                                                                                zip(*np.unique(st, return_counts=True))},
                      "mean_iters": float(res.iters.float().mean().item()),
                      "max_budget_violation": float(np.abs(xh.sum(1) - 1).max()),
                      "mean_turnover": float(np.abs(xh - x0[None, :]).sum(1).mean()),
                      "max_iters": int(res.iters.max().item()), "refactors": res.refactors,
                      "admm_launches": res.admm_launches, "capacitance": res.capacitance,
                      "polish_rounds_mean": float(res.out[:, _lib.PQ_OUT_ROUNDS].mean().item()),
                      "stage_ms": stage_ms(ev), "settings_overrides": args.set}))


def both(args):
    """Turnover budget + leverage together on the config-3 windows (n = 1000, T = 252, 4749
    daily dates, min-variance P = 2 Sigma): the segment split (porqua_amd/l1seg.py: 3n = 3000
    variables, budget + turnover + leverage rows, window path over [R, R, R]; its setup -- P lb
    through one panel GEMM -- inside the step), or with --ipm l1_ipm_batched over chunks of
    dates (the window rows sqrt(2 / (T - 1)) Xc formed inside the step)."""
    from porqua_amd.ipm_l1 import L1Terms, l1_ipm_batched
    tau, lev = (float(v) for v in args.both.split(","))
    if not args.ipm:
        return both_segments(args, tau, lev)
    n, T, D = 1000, 252, 4749
    dev = torch.device("cuda", 0)
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + D], T)
    pan = engine.Panel(R, device=dev)
    rows_d, tlen_d = pan.rows_to_device(rows, tlen)
    x0 = np.random.default_rng(1).dirichlet(np.ones(n))
    terms = L1Terms(x0=x0, to_budget=tau, lev_budget=lev)
    lb, ub = np.full(n, -0.05), np.full(n, 0.1)

    def step():
        out = []
        for s in range(0, D, args.chunk):
            e = min(D, s + args.chunk)
            r = rows_d[s:e].to(torch.int64)
            mu = pan.window_means(rows_d[s:e], tlen_d[s:e])
            UW = ((pan.R[r][:, :, :n] - mu[:, None, :n]) * (2.0 / (T - 1)) ** 0.5).contiguous()
            q = torch.zeros((e - s, n), dtype=torch.float64, device=dev)
            out.append(l1_ipm_batched(UW, None, q, terms, A=np.ones((1, n)), b=np.ones(1), lb=lb, ub=ub))
            del UW
        return out

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    st = torch.cat([o.status for o in out]).cpu().numpy()
    it = torch.cat([o.iters for o in out]).cpu().numpy()
    xh = torch.cat([o.x for o in out]).cpu().numpy()
    print(json.dumps({"workload": f"config3 + turnover budget {tau} + leverage {lev} together, box [-0.05, 0.1] "
                                  "(per-asset-block IPM, window form, coupling k = T + 3)",
                      "qps": D / dt, "ms_per_step": dt * 1e3, "chunk": args.chunk,
                      "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                      "mean_iters": float(it.mean()), "max_iters": int(it.max()),
                      "max_budget_violation": float(np.abs(xh.sum(1) - 1).max()),
                      "max_turnover": float(np.abs(xh - x0[None, :]).sum(1).max()),
                      "max_leverage": float(np.abs(xh).sum(1).max())}))


def both_segments(args, tau, lev):
    from porqua_amd import l1seg
    from porqua_amd.l1split import split_settings
    n, T, D = 1000, 252, 4749
    dev = torch.device("cuda", 0)
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + D], T)
    pan = engine.Panel(R, device=dev)
    rows_d, tlen_d = pan.rows_to_device(rows, tlen)
    gplan = engine.GroupPlan(rows, tlen, dev)
    x0 = np.random.default_rng(1).dirichlet(np.ones(n))
    lb, ub = np.full(n, -0.05), np.full(n, 0.1)
    sd = l1seg.segment_data(x0, lb, ub, to_budget=tau, lev_budget=lev)
    qb = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), lb=lb, ub=ub, device=dev)
    qb.batch, qb.P = D, None
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=dev)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    mu = pan.window_means(rows_d, tlen_d)
    lr = engine.LowRank(pan, rows_d, tlen_d, mu=mu, w_scale=1.0 / (tlen_d.to(torch.float64) - 1.0))
    seg_panel = engine.Panel(torch.cat([pan.R] * 3, 1).contiguous(), None, device=dev)
    ov = dict(kv.split("=", 1) for kv in args.set)
    settings = split_settings(engine.Settings.from_params(ov), ov, "budget")
    ev = []

    def step():
        ev.clear()
        qb3, lr3, const = l1seg.segment_batch(qb, lr, sd, seg_panel, np.ones((1, n)), np.ones(1), None, None)
        res = engine.solve_lowrank(qb3, lr3, settings, groups=gplan, events=ev)
        return res, l1seg.merge_batch(res.x, n, sd["lb"])

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, x = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    st = res.status.cpu().numpy()
    xh = x.cpu().numpy()
    print(json.dumps({"workload": f"config3 + turnover budget {tau} + leverage {lev} together, box [-0.05, 0.1] "
                                  "(segment split on the ADMM engine, window path, 3n = 3000)",
                      "qps": D / dt, "ms_per_step": dt * 1e3,
                      "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                      "mean_iters": float(res.iters.float().mean().item()), "max_iters": int(res.iters.max().item()),
                      "capacitance": res.capacitance, "refactors": res.refactors,
                      "polish_rounds_mean": float(res.out[:, _lib.PQ_OUT_ROUNDS].mean().item()),
                      "max_budget_violation": float(np.abs(xh.sum(1) - 1).max()),
                      "max_turnover": float(np.abs(xh - x0[None, :]).sum(1).max()),
                      "max_leverage": float(np.abs(xh).sum(1).max()),
                      "min_weight": float(xh.min()), "max_weight": float(xh.max()),
                      "stage_ms": stage_ms(ev), "settings_overrides": args.set}))


if __name__ == "__main__":
    main()
