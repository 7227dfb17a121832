#!/usr/bin/env python3
"""Run the bench workload once and dump every problem whose status is not PQ_SOLVED
(date row, ADMM state after the failed polish, outputs) to gpurun_out/diag_status.npz,
so the failure can be replayed on the CPU with tests/engine_model.py."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import engine  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def main():
    n, T, D = 1000, 252, int(sys.argv[1]) if len(sys.argv) > 1 else 4749
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + D], T)
    pan = engine.Panel(R)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.ones(n))
    qb.batch = D
    qb.P = pan.cov(r_d, t_d, mode=0)
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=qb.P.device)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=qb.P.device)
    ws = engine.Workspace(qb)
    snaps = []
    for rep in range(3):
        res = engine.solve(qb, engine.Settings(), ws)
        snaps.append((ws.x.clone(), ws.status.clone(), ws.iters.clone(), ws.out.clone()))
        print("rep", rep, "status", dict(zip(*np.unique(ws.status.cpu().numpy(), return_counts=True))))
    for rep in (1, 2):
        dx = (snaps[rep][0] != snaps[0][0]).any(dim=1)
        di = snaps[rep][2] != snaps[0][2]
        print("rep", rep, "vs 0: x differs in", int(dx.sum()), "problems; iters differ in", int(di.sum()),
              "first", torch.nonzero(dx).flatten()[:10].tolist())
    # determinism of the stages on their own
    ws2 = engine.Workspace(qb)
    lib = engine._lib.load()
    import ctypes
    s = engine.Settings().to_c()
    outs = []
    for rep in range(2):
        pb = qb.c_struct(); st2 = ws2.c_struct()
        lib.pq_init_state(ctypes.byref(pb), ctypes.byref(st2), None, 0, ctypes.byref(s), engine._stream())
        lib.pq_factor_batched(ctypes.byref(pb), ctypes.byref(st2), None, 0, ctypes.byref(s), 1, engine._stream())
        Kc = torch.tril(ws2.K[:64]).clone()
        lib.pq_admm_batched(ctypes.byref(pb), ctypes.byref(st2), None, 0, ctypes.byref(s), 4000, engine._stream())
        outs.append((Kc, ws2.x.clone(), ws2.z.clone(), ws2.y.clone()))
    print("factor deterministic:", bool(torch.equal(outs[0][0], outs[1][0])),
          "admm x/z/y deterministic:", bool(torch.equal(outs[0][1], outs[1][1])),
          bool(torch.equal(outs[0][2], outs[1][2])), bool(torch.equal(outs[0][3], outs[1][3])))
    st = res.status.cpu().numpy()
    bad = np.flatnonzero(st != 1)
    print("status counts", dict(zip(*np.unique(st, return_counts=True))), "bad", bad.tolist())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "diag_status.npz"), bad=bad, status=st[bad],
             ends=(T - 1 + bad), x=ws.x[bad].cpu().numpy(), z=ws.z[bad].cpu().numpy(),
             y=ws.y[bad].cpu().numpy(), rho=ws.rho[bad].cpu().numpy(), iters=ws.iters[bad].cpu().numpy(),
             out=ws.out[bad].cpu().numpy(), mg_pad=ws.mg_pad)


if __name__ == "__main__":
    main()
