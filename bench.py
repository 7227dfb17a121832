#!/usr/bin/env python3
"""Benchmark of the PorQua backtest hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the 1000-asset configuration the metric is quoted on):
synthetic factor-model panel, n = 1000 assets, 252-day window, daily rebalancing ->
4749 rebalance dates per GPU, long-only min-variance (P = 2 * Pearson covariance, q = 0,
budget 1'x = 1, box 0 <= x <= 1).  One *step* = the whole backtest hot path over all dates
of this rank, inputs (return panel + window row lists) already resident in HBM:
K1 window means + FP64-MFMA SYRK -> K2 KKT formation + Cholesky + inverse -> K3 ADMM
(+ adaptive-rho refactorisations) -> K4 polish -> weights gathered to rank 0's host.

Multi-GPU (torchrun, one rank per GPU, RCCL): dates are independent, so each rank solves
its own contiguous block of 4749 dates of a longer panel (weak scaling); the only
collective is the all-gather of the weight panels.

Prints ONE JSON line on rank 0 (contract in the task statement), with a `roofline` object
for the dominant kernel (K3 ADMM, `k_admm_gcap` on the group-capacitance window path; HBM
roofline; algorithmic bytes per date-iteration = (2 x 8 U n union-row passes + 8 k(k+1)/2
for the group's M_U^-1) / dates per group + 12 x 8 n of per-date ADMM state, timed with HIP
events on the launch stream), the measured HBM fraction from the committed
rocprofv3 PMC summary of the same code (``frac_hbm_measured``: PMC bytes per date-iteration
x date-iterations / kernel time / peak), and a `cpu_baseline` object (the reference
per-date path restated in numpy, oracle/cpu_baseline.py, on a bounded sample of dates).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from porqua_amd import engine  # noqa: E402
from porqua_amd.workloads import (MinVarianceBacktest, ReplicationBacktest, SweepBacktest,  # noqa: E402
                                  TrackingBacktest)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 matrix spec


CPU_PATH_TEXT = {   # the reference's per-QP arithmetic the cpu_baseline leg restates
    "config1": "P = 2 X'X, q = -2 X'y (LeastSquares) + isPD/nearestPD of P",
    "config2": "P = 2 X'X, q = -2 X'y (LeastSquares) + isPD/nearestPD of P",
    "config3": "np.cov + isPD/nearestPD, P = 2 Sigma, + isPD/nearestPD of P",
    "config4": "P = 2 X'X, q = -2 X'y (LeastSquares, 20 sector caps) + isPD/nearestPD of P",
    "config5": "np.cov + isPD/nearestPD, P = 2 lam Sigma, q = -geometric mean, + isPD/nearestPD of P",
}
WORKLOAD_TEXT = {
    "config1": "config1: SPTR index replication, LS tracking (P=2 X'X, q=-2 X'y), budget + box [0,1], n=494 "
               "usa-shaped panel on the real SPTR calendar, the reference notebook's MONTHLY rebalancing "
               "(every 21st date from the first full window: 217 dates)",
    "config2": "config2: SPTR index replication, LS tracking (P=2 X'X, q=-2 X'y), budget + box [0,1], n=494 "
               "usa-shaped panel on the real SPTR calendar, every daily rebalance date (4544)",
    "config3": "config3: long-only min-variance (P=2*Pearson cov, budget + box [0,1]), daily rebalance",
    "config4": "config4: tracking-error LS (P=2 X'X, q=-2 X'y), budget + box [0,1] + 20 sector caps <= 0.15, "
               "daily rebalance",
    "config5": "config5: mean-variance sweep (P=2 lam Sigma, q=-mu geometric), budget + box [0,1], n=5000, "
               "64 monthly dates x 64 risk aversions log-spaced in [0.1, 100]",
}


def dropin_config2(wl, T, reb=None, runs=1):
    """Configs 1 / 2 through the reference API (rank 0, N = 1, outside the timed region):
    Backtest.run(bs) with LeastSquares(solver_name='mi355x') on the same panel and dates (or the
    rebalance dates ``reb``), from the host DataFrames to the Portfolio objects (upload,
    staging, download included); the median of ``runs`` runs after one warm-up run."""
    import pandas as pd
    from porqua_amd.backtest import Backtest, BacktestService
    from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_bm_series,
                                     bibfn_box_constraints, bibfn_budget_constraint, bibfn_return_series,
                                     bibfn_selection_data)
    from porqua_amd.optimization import LeastSquares
    idx = pd.DatetimeIndex(wl.dates_rank)
    X = pd.DataFrame(wl.R_rank, index=idx, columns=[f"u{i:03d}" for i in range(wl.n)])
    y = pd.DataFrame({"SPTR": wl.y_rank}, index=idx)
    if reb is None:
        reb = [str(d.date()) for d in idx[wl.ends_local]]

    def run():
        svc = BacktestService(
            data={"return_series": X, "bm_series": y},
            selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
            optimization_item_builders={
                "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=T),
                "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=T, align=True),
                "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
                "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints, box_type="LongOnly")},
            optimization=LeastSquares(solver_name="mi355x"), rebdates=reb, quiet=True)
        bt = Backtest()
        bt.run(svc)
        torch.cuda.synchronize()
        return bt
    run()
    ts = []
    for _ in range(runs):
        t = time.perf_counter()
        bt = run()
        ts.append(time.perf_counter() - t)
    t = float(np.median(ts))
    return {"api": "porqua_amd.backtest.Backtest.run(bs), LeastSquares(solver_name='mi355x')",
            "qps": len(reb) / t, "s": t, "runs_s": [round(r, 5) for r in ts], "dates": len(reb),
            "solved": bt.stats["solved"], "path": bt.stats["path"],
            "note": "host DataFrames in, Portfolio objects out: panel upload, window staging, device solve and "
                    "weight download included"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks; without a launcher (no WORLD_SIZE in the environment) bench.py starts "
                         "them itself, one child process per GPU, before anything touches the GPU")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["config1", "config2", "config3", "config4", "config5"], default="config3",
                    help="config3: n=1000 long-only min-variance (the metric's configuration); config1: the SPTR "
                         "replication at the notebook's monthly rebalancing (every 21st date, 217 QPs; "
                         "BASELINE configs[0..1]); config2: SPTR "
                         "replication, n=494 LS tracking on the usa-shaped panel, all 4544 daily dates (BASELINE "
                         "configs[1]; strong scaling: the fixed date set split over the ranks); config4: n=3000 "
                         "tracking LS with 20 sector caps (configs[3], 'dates sharded'); config5: n=5000 "
                         "mean-variance, 64 dates x 64 risk aversions (configs[4]; strong scaling, sharded by "
                         "date with every lambda of a date on one rank)")
    ap.add_argument("--n", type=int, default=None, help="assets (config3: 1000, config4: 3000, config5: 5000)")
    ap.add_argument("--window", type=int, default=252)
    ap.add_argument("--dates", type=int, default=None,
                    help="rebalance dates per rank (--strong: in total); config3: 4749, config4: 9749; "
                         "config5: 64 dates in total")
    ap.add_argument("--path", choices=["auto", "dense", "lowrank"], default="auto",
                    help="dense K^-1 (K2 n^3 + K3 n^2 stream) or Woodbury low-rank (T + mg < n)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the end-to-end Backtest.run line")
    ap.add_argument("--no-group", action="store_true",
                    help="low-rank ADMM one workgroup per date instead of per group of sliding windows")
    ap.add_argument("--no-slide", action="store_true",
                    help="K1 as one full T-deep SYRK per date instead of anchor SYRK + rank-2 slides")
    ap.add_argument("--with-cov", action="store_true",
                    help="low-rank path: also materialise every date's n x n covariance with K1 "
                         "(nothing on that path reads it)")
    ap.add_argument("--no-graph", action="store_true",
                    help="config3: host-driven solve (a host check after the ADMM and after every polish "
                         "round) instead of the sync-free solve whose stages replay as HIP graphs")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --dates rebalance dates in total, split over the ranks "
                         "(default: weak scaling, --dates per rank)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="override an engine.Settings field (experiments)")
    return ap.parse_args()


def profile_order(tag: str):
    """Sort key of a profile tag ``rNNx``: round NN, then the run letter in the order the
    rounds used them (a..z first, then A..Z)."""
    import re
    m = re.match(r"r(\d+)([a-zA-Z]*)", tag)
    if not m:
        return (-1, 0, "")
    rnd, let = int(m.group(1)), m.group(2)
    return (rnd, 1 if let[:1].isupper() else 0, let)


def select_pmc_summary(kern: str, it_bytes: float, iters_per_step: int, root: str = ROOT):
    """The PMC summary (tools/pmc_summary.py output under profiles/) that describes this
    run's code: the one ``profiles/EVIDENCE.json`` names if it matches, otherwise the newest
    by profile order, among those whose kernel ``kern`` has the same algorithmic bytes per
    date-iteration AND the same date-iterations per step.  Returns (path, summary) or None."""
    import glob

    def matches(pm):
        k = pm.get("kernels", {}).get(kern)
        return (k is not None and "hbm_bytes_per_admm_iteration" in k
                and int(round(k["algorithmic_bytes_per_admm_iteration"])) == int(it_bytes)
                and int(pm.get("admm_iterations_per_step", -1)) == int(iters_per_step))

    pdir = os.path.join(root, "profiles")
    cands = []
    man = os.path.join(pdir, "EVIDENCE.json")
    if os.path.exists(man):
        try:
            cands.append(os.path.join(pdir, json.load(open(man))["pmc_summary"]))
        except (OSError, ValueError, KeyError):
            pass
    cands += sorted(glob.glob(os.path.join(pdir, "*_pmc_summary.json")),
                    key=lambda f: profile_order(os.path.basename(f)), reverse=True)
    for f in cands:
        try:
            pm = json.load(open(f))
        except (OSError, ValueError):
            continue
        if matches(pm):
            return f, pm
    return None


def launch_plan(gpus: int, env: dict):
    """Environments of the rank processes ``bench.py --gpus N`` starts itself when no
    launcher did (no WORLD_SIZE): ranks 0..N-1 on 127.0.0.1, one per GPU (LOCAL_RANK = RANK).
    None when this process is already a rank (torchrun, or one of our children) or N <= 1."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    port = env.get("MASTER_PORT")
    if not port:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = str(s.getsockname()[1])
    return [dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port) for r in range(gpus)]


def run_ranks(envs, argv, script=None) -> int:
    """Start one child per rank (this process never touches the GPU) and wait for all; if a
    rank fails, the others are terminated (by their own PIDs) so none blocks in a collective."""
    import subprocess
    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e) for e in envs]
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = rc or r
                for o in procs:
                    o.terminate()
                for o in procs:
                    try:
                        o.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        o.kill()
                        o.wait()
                procs = []
                break
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    plan = launch_plan(args.gpus, os.environ)
    if plan is not None:
        sys.exit(run_ranks(plan, sys.argv[1:]))
    wname = args.workload
    cfg4 = wname == "config4"
    if wname in ("config1", "config2", "config5"):
        args.strong = True                 # a fixed problem set split over the ranks
    if args.n is None:
        args.n = {"config1": 494, "config2": 494, "config4": 3000, "config5": 5000}.get(wname, 1000)
    if args.dates is None:
        args.dates = {"config4": 9749, "config5": 64}.get(wname, 4749)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PQ_BENCH_SHARE_DEVICE"):   # rehearsal: every rank on cuda:0 (1-GPU box)
        local = 0
    # CPU baseline first, in a child process, before this process touches the GPU (its
    # process pool forks; bench.py itself never forks after HIP initialisation)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import subprocess
        # bounded samples: the per-QP reference cost grows with n^3 (nearestPD's SVD + eigvals:
        # ~0.3 s at n = 494, ~2 s at 1000, ~40 s at 3000, minutes at 5000 on one core), so the
        # n >= 3000 legs time one QP per worker and one serial QP
        cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--workload", wname, "--n", str(args.n),
               "--window", str(args.window), "--dates", str(args.dates), "--budget", str(args.cpu_budget)]
        cmd += {"config1": ["--serial-dates", "8", "--pool-rounds", "8"],
                "config2": ["--serial-dates", "8", "--pool-rounds", "8"],
                "config4": ["--serial-dates", "1", "--pool-rounds", "1"],
                "config5": ["--serial-dates", "1", "--pool-rounds", "1"]}.get(wname, [])
        # progress lines pass through on stderr (the n = 5000 legs run for minutes)
        r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, text=True, timeout=1500)
        if r.returncode == 0 and r.stdout.strip():
            cpu = json.loads(r.stdout.strip().splitlines()[-1])
        else:
            print("cpu baseline failed: rc", r.returncode, file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PQ_BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    n, T = args.n, args.window
    ov = dict(kv.split("=", 1) for kv in args.set)
    if cfg4:
        settings = engine.Settings.from_params(dict({"rho0_rel": 0.1, "rho0_qrel": 0.0}, **ov))
        wl = TrackingBacktest(n=n, T=T, D=args.dates, rank=rank, world=world, device=dev, settings=settings,
                              strong=args.strong)
    elif wname in ("config1", "config2"):
        g = np.load(os.path.join(ROOT, "tests", "golden", "sptr.npz"), allow_pickle=False)
        settings = engine.Settings.from_params(dict({"rho0_rel": 0.2, "rho0_qrel": 0.0}, **ov))
        wl = ReplicationBacktest(g["days"], g["returns"], T=T, rank=rank, world=world, device=dev,
                                 settings=settings, n=n, stride=21 if wname == "config1" else 1)
    elif wname == "config5":
        from porqua_amd.sweep import SWEEP_SETTINGS
        settings = engine.Settings.from_params(dict(SWEEP_SETTINGS, **ov))
        wl = SweepBacktest(n=n, T=T, dates=args.dates, rank=rank, world=world, device=dev, settings=settings)
    else:
        settings = engine.Settings.from_params(dict(kv.split("=", 1) for kv in args.set))
        wl = MinVarianceBacktest(n=n, T=T, D=args.dates, rank=rank, world=world, device=dev, settings=settings,
                                 path=args.path, group=not args.no_group, slide=not args.no_slide,
                                 with_cov=args.with_cov, strong=args.strong, graph=not args.no_graph)
    if hasattr(wl, "prepare"):   # graph mode: the cache-filling step and the capture, untimed
        wl.prepare()
    gloo = dist is not None and dist.get_backend() != "nccl"
    D = wl.D                                            # dates of this rank
    D_all = wl.global_dates                             # dates of the whole job
    R_rank, y_rank, ends_local, pan = wl.R_rank, wl.y_rank, wl.ends_local, wl.pan
    qb, lr, plan, gplan, ws = wl.qb, wl.lr, wl.plan, wl.gplan, wl.ws
    use_lr, with_cov = wl.use_lr, wl.with_cov
    # weights leave the device on a side stream: step k's all-gather (RCCL) and D2H copy to
    # rank 0's pinned host panel overlap step k + 1's kernels (double-buffered staging)
    nbuf = 2
    Dpad = -(-D_all // world)                           # equal all-gather blocks (strong: last rank padded)
    w_host = [torch.empty((Dpad * world, n), dtype=torch.float64).pin_memory() for _ in range(nbuf)] \
        if rank == 0 else None
    x_stage = [torch.zeros((Dpad if world > 1 else D, n), dtype=torch.float64, device=dev) for _ in range(nbuf)]
    gather_buf = [torch.empty((world * Dpad, n), dtype=torch.float64, device=dev) for _ in range(nbuf)] \
        if world > 1 else None
    side = torch.cuda.Stream(device=dev)
    side_done = [None] * nbuf
    nstep = [0]

    def step(events=None):
        res = wl.step(events)
        k = nstep[0] % nbuf
        nstep[0] += 1
        main = torch.cuda.current_stream()
        if side_done[k] is not None:
            main.wait_event(side_done[k])      # staging buffer k is free again
        x_stage[k][:D].copy_(res.x[:, :n])
        ready = torch.cuda.Event()
        ready.record(main)
        if gloo:   # rehearsal backend (CPU collectives): gather through host memory, synchronously
            ready.synchronize()
            parts = [torch.empty((Dpad, n), dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, x_stage[k].cpu())
            if rank == 0:
                w_host[k].copy_(torch.cat(parts))
            return res
        with torch.cuda.stream(side):
            side.wait_event(ready)
            if world > 1:
                dist.all_gather_into_tensor(gather_buf[k], x_stage[k])
                if rank == 0:
                    w_host[k].copy_(gather_buf[k], non_blocking=True)
            else:
                w_host[k].copy_(x_stage[k], non_blocking=True)
            side_done[k] = torch.cuda.Event()
            side_done[k].record(side)
        return res

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    events = []
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step(events)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        red_dev = torch.device("cpu") if gloo else dev
        t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # ---- accuracy of every solution of the last step (outside the timed region): primal
    # violation and relative stationarity recomputed from the panel rows with torch -------
    cert = wl.certificate(res)
    if dist:
        cv = torch.tensor([cert["max_violation"], cert["max_rel_stationarity"],
                           cert["max_rel_complementarity"]], dtype=torch.float64, device=red_dev)
        dist.all_reduce(cv, op=dist.ReduceOp.MAX)
        cert["max_violation"], cert["max_rel_stationarity"], cert["max_rel_complementarity"] = cv.tolist()
        st_all = torch.bincount((res.status.long() + 8).clamp(0, 15), minlength=16).to(red_dev)
        dist.all_reduce(st_all)
        cert["status_counts"] = {str(i - 8): int(v) for i, v in enumerate(st_all.tolist()) if v}
    # ---- per-kernel timing (HIP events on the launch stream) ------------------------------
    tk = {}
    cnt = {}
    for name, a, b in events:
        tk[name] = tk.get(name, 0.0) + a.elapsed_time(b) * 1e-3
        cnt[name] = cnt.get(name, 0) + 1
    iters = res.iters.to(torch.int64)
    total_iters = int(iters.sum().item()) * args.steps   # identical work every step
    status = res.status.cpu().numpy()
    out_rec = res.out.cpu().numpy()
    from porqua_amd import _lib
    nfree = out_rec[:, _lib.PQ_OUT_NFREE]
    prounds = out_rec[:, _lib.PQ_OUT_ROUNDS]
    # ---- roofline of the ADMM kernel: algorithmic bytes per date-iteration ---------------
    k_lr = T + qb.mg
    grouped = use_lr and engine.grouped_applicable(qb, lr, gplan, ws)
    l2_bytes = None
    if grouped and res.capacitance == "group":
        # k_admm_gcap, per group-iteration: the union rows twice (pass 1 X_U V, pass 2 X_U' Ut;
        # 2.1 MB per group, too big to stay on-chip between the passes), the lower triangle of
        # the group's M_U^-1, and per date the ADMM state read + written (x, Px, z, y, rhs: 10
        # n-vectors) plus q and mu read -- amortised per date-iteration over the mean group
        kern = "k_admm_gcap"
        gp_used = getattr(ws, "gcap_groups", None) or gplan   # the plan the ADMM ran (32-date groups)
        u_mean = float(gp_used.ucnt.double().mean().item())
        g_mean = float(gp_used.sizes.mean())
        k_u = u_mean + qb.mg
        it_bytes = (2 * 8.0 * u_mean * n + 8.0 * k_u * (k_u + 1) / 2) / g_mean + 12 * 8.0 * n
        admm_bytes = it_bytes * total_iters
    elif grouped and getattr(ws, "sweep_admm", None) is not None:
        # risk-aversion sweep (admm_sweep.hip, k_sw_pass + k_sw_mid), per problem-iteration: the
        # ADMM state read + written (x, Px, z, y: 8 n-vectors), the lower-triangle M_b^-1, the
        # problem's rows of the chunk partials of W (written + read), and per group of G
        # problems the window (T n) and q once
        sp = ws.sweep_admm
        kern = "k_sw_pass"
        g_mean = D / sp.ngroups
        nch = (n + 255) // 256
        it_bytes = (8.0 * 8 * n + 8.0 * k_lr * (k_lr + 1) / 2 + 2 * 8.0 * 256 * nch
                    + 8.0 * (T * n + n) / g_mean)
        admm_bytes = it_bytes * total_iters
    elif grouped:
        # HBM level: the date's lower-triangle M^-1 (the only per-date O(k^2) stream; 4749 x
        # 512 KB is far beyond the caches) + the ADMM state read and written (x, z, y, Px);
        # the window passes read the group's union rows, which sit in the XCD's L2
        kern = "k_admm_grp"
        it_bytes = 8.0 * k_lr * (k_lr + 1) / 2 + 8.0 * 8 * n
        u_mean = float(gplan.ucnt.double().mean().item())
        l2_bytes = 2 * 8.0 * u_mean * n / float(gplan.sizes.mean())
        admm_bytes = it_bytes * total_iters
    elif use_lr:
        kern = "k_admm"
        it_bytes = 8.0 * (2 * T * n + k_lr * (k_lr + 1) / 2)
        admm_bytes = it_bytes * total_iters + 8.0 * 8 * n * D * cnt.get("admm", 1)
    else:
        kern = "k_admm"
        it_bytes = 8.0 * n * (n + 1) / 2
        admm_bytes = it_bytes * total_iters + 8.0 * 8 * n * D * cnt.get("admm", 1)
    admm_gbs = admm_bytes / tk["admm"] / 1e9
    ld = qb.ld
    nb = ld // 64
    tiles = nb * (nb + 1) // 2
    if plan is None:
        syrk_flops = D * tiles * 64 * 64 * 2.0 * T * args.steps
    else:   # anchors: full T-deep SYRK; slid dates: one 4-deep (2 s padded) MFMA update
        syrk_flops = (plan.ngroups * T + (D - plan.ngroups) * 4) * tiles * 64 * 64 * 2.0 * args.steps
    cov_t = tk.get("moments+cov") if with_cov else None
    cov_write_gbs = D * ld * ld * 8.0 * args.steps / cov_t / 1e9 if cov_t else None
    kld = ((T + 1 + 63) // 64) * 64
    band = use_lr and res.capacitance == "band"
    # potrf + trtri + lauum (k^3), plus the per-date capacitance SYRK (2 k^2 n) unless the
    # band Gram (one row-band SYRK per panel, stage "gram") supplies it
    factor_flops_per = (kld ** 3 + (0.0 if band else 2.0 * kld * kld * n)) if use_lr else ld ** 3
    # the row-band SYRK of the panel (stage "gram", k_band_gram): x_r . x_{r-j} for the band's
    # W offsets of each of its rows -- 2 n W flop per row (the group path's band is as wide as
    # the widest slide-group union)
    bshape = getattr(ws, "band_shape", None) if use_lr else None
    gram_flops = 2.0 * n * bshape[0] * bshape[1] * args.steps if bshape else None
    n_factor = D * args.steps + res.refactors * args.steps
    factor_flops = factor_flops_per * n_factor
    if use_lr and res.capacitance == "group":   # one M_U (k = U + mg) per slide group
        gp_used = getattr(ws, "gcap_groups", None) or gplan
        k_u = float(gp_used.ucnt.double().mean().item()) + qb.mg
        factor_flops = k_u ** 3 * gp_used.ngroups * args.steps

    # polish (K4) algorithmic flops per step: per problem and active-set round the P_FF Gram
    # of the free columns over the window (|F|^2 T) and its Cholesky (|F|^3 / 3), plus the
    # two exact P x window passes (2 x 2 T n)
    polish_flops = float(((prounds * (nfree ** 2 * T + nfree ** 3 / 3.0)).sum() + 4.0 * T * n * D) * args.steps)

    traffic, traffic_src, mfma_busy, mfma_src = None, None, None, None
    pm_sel = select_pmc_summary(kern, it_bytes, total_iters // args.steps)
    if pm_sel is not None:
        f, pm = pm_sel
        traffic, traffic_src = pm["kernels"][kern]["hbm_bytes_per_admm_iteration"], os.path.relpath(f, ROOT)
        if "mfma_busy_fraction" in pm:
            mfma_busy = {kk: pm["mfma_busy_fraction"][kk] for kk in
                         ("k_band_gram", "k_factor", "k_gcap_prep", "k_admm_grp", "k_admm_gcap", "k_sw_pass",
                          "k_sw_mid", "k_polish_w",
                          "k_pg_form", "k_pg_form_grp", "k_pg_solve", "k_pg_passA", "k_pg_passB")
                         if kk in pm["mfma_busy_fraction"]}
            mfma_src = traffic_src
    # measured HBM fraction: the PMC bytes of the same kernel (same code: algorithmic bytes and
    # date-iterations per step both match) over this run's HIP-event time of the stage
    frac_hbm_measured = (traffic * (total_iters // args.steps) / (tk["admm"] / args.steps) / 1e9 / HBM_PEAK_GBS
                         if traffic is not None else None)

    qps = D_all * args.steps / dt
    out = {
        "metric": "QPs solved/sec (rebalance dates) at N=1000 assets, 1-8 GPU; x vs host CPU",
        "value": qps,
        "unit": "QPs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic usa-shaped panel (494 assets loading on the real SPTR returns, seed 20240101; "
                 "usa_returns absent) on the real SPTR calendar" if wname in ("config1", "config2") else
                 "synthetic (factor-model panel, seed 20240314; usa_returns absent)"),
        "config": {"workload": WORKLOAD_TEXT[wname], "n_assets": n, "window": T,
                   "dates_per_gpu": D, "global_batch": D_all,
                   "parallelism": (f"dates-sharded x{world} (every lambda of a date on its rank)"
                                   if wname == "config5" else f"dates-sharded x{world}")},
        "roofline": {"bound": "hbm", "kernel": kern + (" + k_sw_mid (K3, risk-aversion sweep)" if kern == "k_sw_pass"
                                                       else " (K3, grouped low-rank)" if grouped else " (K3)"),
                     "achieved": admm_gbs,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": admm_gbs / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "traffic_unit": "HBM bytes per date-iteration (PMC: 2*FETCH_SIZE + WRITE_SIZE, "
                                     "gfx950 correction; committed rocprofv3 pass)",
                     "traffic_source": traffic_src,
                     "frac_hbm_measured": frac_hbm_measured,
                     "frac_hbm_measured_note": "traffic x date-iterations per step / this run's kernel time / "
                                               "peak: the HBM bytes the kernel really moves (frac counts the "
                                               "algorithmic bytes, most union rows of which are served by "
                                               "L2 / MALL)",
                     "algorithmic_bytes_per_iteration": int(it_bytes),
                     "algorithmic_bytes_note": ("per date-iteration: (union rows 2 x 8Un + lower-triangle M_U^-1 "
                                                "8k(k+1)/2, k = U + mg) / dates per group + ADMM state 12 x 8n"
                                                if kern == "k_admm_gcap" else
                                                "per problem-iteration: ADMM state 8 x 8n + lower-triangle M_b^-1 "
                                                "8k(k+1)/2 + W chunk partials 2 x 8 x 256 x ceil(n/256) + (window "
                                                "8Tn + q 8n) / problems per group" if kern == "k_sw_pass" else
                                                "per date-iteration: lower-triangle M^-1 8k(k+1)/2 (k = T + mg) "
                                                "+ ADMM state 8 x 8n" if grouped else
                                                "per date-iteration: window rows 2 x 8Tn + M^-1 8k(k+1)/2"
                                                if use_lr else "per date-iteration: lower-triangle K^-1 8n(n+1)/2"),
                     "l2_window_bytes_per_iteration": None if l2_bytes is None else int(l2_bytes),
                     "l2_window_gbs": None if l2_bytes is None else l2_bytes * total_iters / tk["admm"] / 1e9,
                     "path": ("lowrank grouped, group capacitance (one M_U^-1 per slide group + per-date "
                              "Woodbury correction; MFMA passes over the union rows)" if kern == "k_admm_gcap" else
                              "lowrank, risk-aversion sweep (the date's problems as MFMA columns of fused "
                              "chunk passes over its window; per-problem M_b^-1)" if kern == "k_sw_pass" else
                              "lowrank grouped (Woodbury; MFMA passes over the union of sliding windows)"
                              if grouped else "lowrank (Woodbury: window rows + M^-1)" if use_lr
                              else "dense K^-1 (lower)"),
                     "admm_iterations_per_step": total_iters // args.steps},
        "stages_s_per_step": {k: v / args.steps for k, v in tk.items()},
        "stage_rates": {
            "cov_syrk_tflops": syrk_flops / cov_t / 1e12 if cov_t else None,
            "cov_write_gbs": cov_write_gbs,
            "cov_mode": ("not materialised: P = 2 Xc'Xc/(T-1) stays in window form; moments = "
                         "window means + diag(Xc'Xc)") if not with_cov else
                        "full SYRK per date" if plan is None else
                        f"sliding: {plan.ngroups} anchor SYRKs + rank-2 updates",
            "factor_tflops": factor_flops / tk.get("factor", float("nan")) / 1e12,
            "polish_tflops": polish_flops / tk["polish"] / 1e12 if tk.get("polish") else None,
            "polish_flops_note": "sum over problems of rounds x (|F|^2 T + |F|^3/3) + 4 T n (two P x window passes)",
            "gram_tflops": gram_flops / tk["gram"] / 1e12 if gram_flops and tk.get("gram") else None,
            "gram_flops_note": ("2 n W flop per panel row of the band (rows x W: %d x %d)" % tuple(bshape))
            if bshape else None,
            "capacitance": res.capacitance or None,
            "fp64_peak_tflops": FP64_PEAK_TFLOPS,
            "mfma_busy_fraction_pmc": mfma_busy,
            "mfma_busy_source": (mfma_src + " (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs))")
            if mfma_src else None,
        },
        "solver": {"status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
                   "mean_iters": float(iters.float().mean().item()),
                   "max_iters": int(iters.max().item()),
                   "refactors_per_step": res.refactors, "admm_launches_per_step": res.admm_launches,
                   "polish_nfree_mean": float(nfree.mean()), "polish_nfree_max": int(nfree.max()),
                   "polish_rounds_mean": float(prounds.mean()), "polish_rounds_max": int(prounds.max()),
                   "settings_overrides": args.set,
                   "certificate": dict(cert, note="all solutions of the last timed step; P x recomputed "
                                                   "from the panel rows (torch), not by the engine")},
        "cpu_baseline": None,
    }
    if cpu is not None:
        legs = {"serial": cpu["serial"], "pool": cpu["pool"]}
        best = max(legs, key=lambda k: legs[k]["qps"])
        b = legs[best]
        cores = b["workers"] if best == "pool" else b["blas_threads"]
        out["cpu_baseline"] = {
            "value": b["qps"], "unit": "QPs/s", "cores": cores, "kind": "port",
            "sample": (f"better of (a) serial, {cpu['serial']['dates']} dates with {cpu['serial']['blas_threads']} "
                       f"BLAS threads: {cpu['serial']['qps']:.3f} QPs/s and (b) pool of {cpu['pool']['workers']} "
                       f"single-threaded processes, {cpu['pool']['dates']} dates: {cpu['pool']['qps']:.3f} QPs/s "
                       f"(evenly spaced QPs of the same inputs; full per-QP reference path at n={n}: "
                       f"{CPU_PATH_TEXT[wname]} + dense IPM, cvxopt coneqp algorithm, tol 1e-7; "
                       f"qpsolvers unavailable)"),
            "leg": best, "cpu_model": cpu["cpu_model"], "host_cores": cpu["host_cores"],
            "serial": cpu["serial"], "pool": cpu["pool"],
            "solver_only_no_nearestPD": {"serial_qps": cpu.get("serial_solver_only", {}).get("qps"),
                                         "pool_qps": cpu.get("pool_solver_only", {}).get("qps")},
            "speedup": qps / b["qps"]}
    if wname == "config2" and world == 1 and not args.no_dropin:
        out["end_to_end"] = dropin_config2(wl, T)
    if wname == "config1" and world == 1 and not args.no_dropin:
        # the monthly run through the reference API, and the notebook's own 13-date run
        # (example/backtest.ipynb: dates[dates > start][::21]; start 2022-06-01 on this calendar,
        # which ends in 2023, so that the run has the notebook's 13 dates)
        out["end_to_end"] = dropin_config2(wl, T, runs=5)
        d = np.asarray(wl.dates_rank).astype("datetime64[D]")
        nb13 = [str(r) for r in d[d > np.datetime64("2022-06-01")][::21]]
        out["end_to_end_notebook13"] = dict(dropin_config2(wl, T, reb=nb13, runs=9),
                                            rebdates=f"{nb13[0]} .. {nb13[-1]} (every 21st date after 2022-06-01)")
    if wname != "config3":   # the next-row and drop-in legs below are config-3 (n = 1000 min-variance) lines
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    # ---- next row, outside the timed region: Strategy.simulate of
    # the solved weights, one holding period per rebalance date (float, level, turnover) ----
    wx = res.x[:, :n]
    row0 = ends_local.copy()
    nrows = np.full(D, 2, dtype=np.int64)
    nrows[-1] = 1                                       # the last period ends at the panel end
    sim_args = (pan.R, wx, engine.PeriodPlan(row0, nrows, device=dev, panel_rows=pan.D))
    engine.simulate_periods(*sim_args, want_end=True)
    s_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 20
    s_ev[0].record()
    for _ in range(reps):
        engine.simulate_periods(*sim_args, want_end=True)
    s_ev[1].record()
    torch.cuda.synchronize()
    sim_s = s_ev[0].elapsed_time(s_ev[1]) * 1e-3 / reps
    sim_bytes = 8.0 * n * (int((nrows - 1).sum()) + 2 * D) + 16.0 * D   # panel rows + W in + wend out
    out["next_rows"] = {"simulate": {
        "kernel": "k_float_periods (pq_simulate_periods)", "periods": D,
        "us_per_launch": sim_s * 1e6, "algorithmic_bytes": int(sim_bytes),
        "achieved_gbs": sim_bytes / sim_s / 1e9, "frac_hbm": sim_bytes / sim_s / 1e9 / HBM_PEAK_GBS,
        "note": "daily periods: 1 panel row + weights in, floated weights out, per period; "
                "period tables staged once (engine.PeriodPlan)"}}
    # ---- next row, outside the timed region: LAD (the reference's LP,
    # levels + log, budget + long-only box) on the device IPM for the first 256 windows ----
    from porqua_amd import lad as _lad
    nl = min(256, D)
    idx = torch.from_numpy(ends_local[:nl, None] - T + 1 + np.arange(T)[None, :]).to(dev)
    y_d = torch.from_numpy(np.ascontiguousarray(y_rank, dtype=np.float64)).to(dev)
    Xl = torch.log(torch.cumprod(1 + pan.R[idx], 1)).contiguous()
    yl = torch.log(torch.cumprod(1 + y_d[idx], 1)).contiguous()
    lad_pr = _lad.LADProblem(Xl, yl, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
    _lad.lad_ipm_batched(lad_pr)
    torch.cuda.synchronize()
    t_l = time.perf_counter()
    lad_res = _lad.lad_ipm_batched(lad_pr)
    torch.cuda.synchronize()
    lad_s = time.perf_counter() - t_l
    out["next_rows"]["lad"] = {
        "solver": "batched Mehrotra IPM, H^-1 from K2 (pq_factor_batched) applied by k_lad_mv",
        "lps": nl, "lps_per_s": nl / lad_s, "ipm_iterations_max": int(lad_res.iters.max().item()),
        "status_counts": {str(k): int(v) for k, v in
                          zip(*np.unique(lad_res.status.cpu().numpy(), return_counts=True))}}
    # ---- drop-in line, outside the timed region (rank 0, N = 1): the same panel and dates
    # through the reference API -- Backtest.run(bs) with MeanVariance (Pearson covariance,
    # geometric mean: q = -mu, the closest API objective to the step's q = 0), from the host
    # DataFrame to the Portfolio objects (panel upload, staging and result download included) --
    if world == 1 and not args.no_dropin:
        import pandas as pd
        from porqua_amd.backtest import Backtest, BacktestService
        from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                         bibfn_budget_constraint, bibfn_return_series, bibfn_selection_data)
        from porqua_amd.optimization import MeanVariance
        idx = pd.DatetimeIndex(wl.dates_rank)
        Xdf = pd.DataFrame(R_rank, index=idx, columns=[f"a{i}" for i in range(n)])
        reb = [str(d.date()) for d in idx[wl.ends_local]]

        def dropin():
            svc = BacktestService(
                data={"return_series": Xdf},
                selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
                optimization_item_builders={
                    "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=T),
                    "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
                    "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints)},
                optimization=MeanVariance(solver_name="mi355x"), rebdates=reb, quiet=True)
            bt = Backtest()
            bt.run(svc)
            torch.cuda.synchronize()
            return bt
        dropin()
        runs = []
        for _ in range(3):   # the median of three runs (one run's host time varies by a few ms)
            bt = None
            t_d = time.perf_counter()
            bt = dropin()
            runs.append(time.perf_counter() - t_d)
        t_d = float(np.median(runs))
        out["end_to_end"] = {
            "api": "porqua_amd.backtest.Backtest.run(bs), MeanVariance(solver_name='mi355x')",
            "qps": len(reb) / t_d, "s": t_d, "runs_s": [round(r, 5) for r in runs], "dates": len(reb),
            "solved": bt.stats["solved"],
            "path": bt.stats["path"],
            "note": "host DataFrame in, Portfolio objects out: panel upload, window staging, device solve "
                    "and weight download included; q = -mu (geometric) instead of the step's q = 0"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
