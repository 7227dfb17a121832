#!/usr/bin/env python3
"""Round-by-round trace of the dates the grouped polish hands back on the drop-in's problem
(config-3 panel, q = -mu geometric: nearly linear objectives with few free assets) --
experiment tooling.  Finds the hand-offs with one full solve, then replays the pipeline's
rounds from the same loose ADMM point and prints, per round and watched date, the free-set
size, the variables at a bound other than 0, the largest weights and the budget multiplier."""
import ctypes
import dataclasses
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.workloads import MinVarianceBacktest  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = MinVarianceBacktest(D=4749, device=dev)
    n, ld = wl.n, wl.qb.ld
    wl.qb.q[:, :n] = -wl.pan.window_geomeans_grouped(wl.gplan, wl.tlen_d)[:, :n]
    st = wl.settings
    ws = engine.Workspace(wl.qb, dense=False)
    engine.solve_lowrank(wl.qb, wl.lr, st, ws=ws, groups=wl.gplan, sync_free=True, sf_rounds=4)
    torch.cuda.synchronize()
    fb = getattr(ws, "pg_fallback", None)
    watch = [] if fb is None else fb.cpu().numpy().tolist()[:3]
    print("handed back:", None if fb is None else fb.cpu().numpy().tolist(), flush=True)
    if not watch:
        return
    ws = engine.Workspace(wl.qb, dense=False)
    s_adm = dataclasses.replace(st, polish=0, eps_abs=st.eps_grouped, eps_rel=st.eps_grouped, min_iter=st.min_iter_grouped)
    engine.solve_lowrank(wl.qb, wl.lr, s_adm, ws=ws, groups=wl.gplan, polish=False)
    lib = _lib.load()
    s = st.to_c()
    pb, stc, lrs = wl.qb.c_struct(), ws.c_struct(), wl.lr.c_struct()
    rec = ws.pg_record()
    g = wl.gplan.polish_plan()
    strm = engine._stream()
    _lib.check(lib.pq_polish_grouped_init(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc), rec.data_ptr(),
                                          ctypes.byref(s), strm), "init")
    scr = torch.empty(g.ngroups * _lib.PQ_PG_PASS_SCRATCH, dtype=torch.float64, device=dev)
    fl_off = (8 + ws.mg_pad) * ld
    for r in range(int(st.polish_rounds)):
        _lib.check(lib.pq_polish_grouped_round(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc),
                                               rec.data_ptr(), ws.ldk, engine._ptr(g.gdates), g.ngroups,
                                               engine._ptr(g.urows), engine._ptr(g.ucnt), engine._ptr(g.uoff),
                                               g.umax, ctypes.byref(s), scr.data_ptr(), None, strm), "round")
        torch.cuda.synchronize()
        R = rec.cpu().numpy()
        W = ws.work.cpu()
        for b in watch:
            xs = W[b, :n].numpy()
            fl = W[b, fl_off:fl_off + (n + 1) // 2].contiguous().view(torch.int32).numpy()[:n]
            top = np.argsort(-xs)[:4]
            print(f"round {r + 1} date {b}: state {int(R[b, 3])} k {int(R[b, 0])} kb {int(R[b, 349])} "
                  f"at ub {np.flatnonzero(fl == 2).tolist()} free {np.flatnonzero(fl == 0).tolist()[:8]} "
                  f"top x {[(int(i), round(float(xs[i]), 6)) for i in top]} lam {R[b, 128]:.6e}", flush=True)


if __name__ == "__main__":
    main()
