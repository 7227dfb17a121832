#!/usr/bin/env python3
"""Engine-level stage timing of the config 1/2 problem family (LS tracking on the usa-shaped
panel, every date): ADMM iterations, polish rounds / fallbacks, stage times.  Experiment tool."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.synthetic import usa_panel  # noqa: E402


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "sptr.npz"))
    dates, R, y = usa_panel(g["days"], g["returns"])
    T = 252
    n = R.shape[1]
    dev = torch.device("cuda", 0)
    reb = dates[T - 1:]
    rows, tlen = engine.window_rows(dates, reb, T)
    pan = engine.Panel(R, y, device=dev)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    B = len(reb)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.ones(n), device=dev)
    qb.batch, qb.P = B, None
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=dev)
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, dev)
    ws = engine.Workspace(qb, dense=False)
    settings = engine.Settings.from_params(dict(kv.split("=", 1) for kv in sys.argv[1:]))
    for it in range(3):
        xty, _ = pan.gram_xy(r_d, t_d)
        qb.q = (-2.0 * xty).contiguous()
        lr.refresh()
        ev = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = engine.solve_lowrank(qb, lr, settings, ws=ws, groups=gp, events=ev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    st = {}
    for name, a, b in ev:
        st[name] = st.get(name, 0.0) + a.elapsed_time(b)
    out = res.out.cpu().numpy()
    status = res.status.cpu().numpy()
    print(json.dumps({"dates": B, "ms": dt * 1e3, "qps": B / dt, "stages_ms": st, "capacitance": res.capacitance,
                      "refactors": res.refactors, "admm_launches": res.admm_launches,
                      "iters_mean": float(res.iters.float().mean()), "iters_max": int(res.iters.max()),
                      "nfree_mean": float(out[:, _lib.PQ_OUT_NFREE].mean()),
                      "nfree_max": int(out[:, _lib.PQ_OUT_NFREE].max()),
                      "rounds_mean": float(out[:, _lib.PQ_OUT_ROUNDS].mean()),
                      "status": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))}}))


if __name__ == "__main__":
    main()
