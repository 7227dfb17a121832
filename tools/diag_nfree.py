#!/usr/bin/env python3
"""Free-set sizes of the polished answers (out[PQ_OUT_NFREE]) at the config-2, config-4 and
config-5 shapes -- which polish path (grouped LDS buckets <= 128, wide rounds, or the per-date
fallback) they need.  Experiment tool: python tools/diag_nfree.py [2]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.sweep import mean_variance_sweep  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def fallbacks(res, ws):
    """Why the grouped polish handed dates to the per-date kernel: their record at that time."""
    fb = getattr(ws, "pg_fallback", None)
    if fb is None or ws is None:
        return {"fallbacks": res.polish_fallbacks}
    rec = ws.pg_record()[fb.long()].cpu().numpy()
    k, ma, rounds = rec[:, 0], rec[:, 1], rec[:, 4]
    return {"fallbacks": res.polish_fallbacks, "k_eq0": int((k == 0).sum()), "k_gt128": int((k > 128).sum()),
            "ma_max": float(ma.max()), "rounds_hist": {str(int(a)): int(b) for a, b in zip(*np.unique(rounds, return_counts=True))},
            "k_hist": {str(int(a)): int(b) for a, b in zip(*np.unique(np.minimum(k, 999), return_counts=True))}}


def hist(res, tag, ws=None):
    nf = res.out[:, _lib.PQ_OUT_NFREE].cpu().numpy()
    rd = res.out[:, _lib.PQ_OUT_ROUNDS].cpu().numpy()
    edges = [0, 1, 48, 64, 80, 96, 128, 160, 192, 256, 384, 512, 1024, 10 ** 6]
    h, _ = np.histogram(nf, bins=edges)
    print(json.dumps({"tag": tag, "nfree_hist": {f"[{a},{b})": int(c) for a, b, c in zip(edges[:-1], edges[1:], h)},
                      "nfree_max": float(nf.max()), "rounds_mean": float(rd.mean()),
                      "status": {str(k): int(v) for k, v in zip(*np.unique(res.status.cpu().numpy(), return_counts=True))},
                      "polish": fallbacks(res, ws)}),
          flush=True)


def config2(dev):
    """The config-2 engine problem: SPTR replication on the usa-shaped panel, every date,
    least-squares tracking with budget + long-only box (tests/test_configs12_gpu.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_configs12_gpu import usa_data
    X, yb = usa_data()
    d = X.index.values.astype("datetime64[D]")
    rows, tlen = engine.window_rows(d, d[251:], 252)
    n, D = X.shape[1], len(rows)
    pan = engine.Panel(X.to_numpy(), yb.to_numpy()[:, 0], device=dev)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    qb = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n),
                                   device=dev)
    qb.batch = D
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    xty, _ = pan.gram_xy(r_d, t_d)
    qb.q = (-2.0 * xty).contiguous()
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, dev)
    st = engine.Settings.from_params({"rho0_rel": 0.2, "rho0_qrel": 0.0})   # LeastSquares' defaults
    ws = engine.Workspace(qb, dense=False)
    hist(engine.solve_lowrank(qb, lr, st, groups=gp, ws=ws), f"config2 ({D} daily dates)", ws)


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "2":
        config2(dev)
        return
    n, T, ns, cap, D = 3000, 252, 20, 0.15, 600
    dates, R, y, sec = factor_panel(T - 1 + D, n, n_sectors=ns)
    rows, tlen = engine.window_rows(dates, dates[T - 1:], T)
    pan = engine.Panel(R, y, device=dev)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    G = np.stack([(sec == g).astype(float) for g in range(ns)])
    qb = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), G=G, h=np.full(ns, cap),
                                   lb=np.zeros(n), ub=np.ones(n), device=dev)
    qb.batch = D
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    xty, _ = pan.gram_xy(r_d, t_d)
    qb.q = (-2.0 * xty).contiguous()
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, dev)
    st = engine.Settings.from_params({"rho0_rel": 0.1, "rho0_qrel": 0.0})
    ws = engine.Workspace(qb, dense=False)
    hist(engine.solve_lowrank(qb, lr, st, groups=gp, ws=ws), "config4 (600 dates)", ws)
    n, nd, L = 5000, 16, 64
    dates, R, _, _ = factor_panel(T - 1 + 21 * nd, n)
    ends = np.arange(T - 1, T - 1 + 21 * nd, 21)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=dev)
    qb_ws = engine.QPBatch(n, nd * L, 1, device=dev, P=torch.empty(0, dtype=torch.float64, device=dev))
    ws5 = engine.Workspace(qb_ws, dense=False)
    res, _ = mean_variance_sweep(pan, rows, tlen, np.logspace(-1, 2, L), ws=ws5)
    hist(res, "config5 (16 dates x 64)", ws5)
    nf = res.out[:, _lib.PQ_OUT_NFREE].cpu().numpy().reshape(nd, L)
    print(json.dumps({"config5_nfree_by_lambda_index_mean": [round(float(v), 1) for v in nf.mean(0)[::4]]}))


if __name__ == "__main__":
    main()
