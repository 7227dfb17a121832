#!/usr/bin/env python3
"""Round-by-round view of the grouped polish at the config-3 shape (experiment tooling):
how many dates are still pending after each active-set round, and how each round changed a
date's free set (grown / shrunk / both), from the polish record between rounds.

Runs the bench workload's ADMM (the solve's own settings), then drives the pipeline's
rounds one by one through the C ABI (pq_polish_grouped_init / _round), reading the record
after each round."""
import ctypes
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
    wl = MinVarianceBacktest(D=int(sys.argv[1]) if len(sys.argv) > 1 else 4749, device=dev)
    res = wl.step()
    torch.cuda.synchronize()
    out = res.out.cpu().numpy()
    rounds = out[:, _lib.PQ_OUT_ROUNDS].astype(int)
    print("final rounds histogram:", dict(zip(*np.unique(rounds, return_counts=True))))
    print("nfree mean / max:", out[:, _lib.PQ_OUT_NFREE].mean(), out[:, _lib.PQ_OUT_NFREE].max())
    # replay the polish round by round from the same ADMM point: re-run the ADMM stop
    import dataclasses
    st = wl.settings
    ws = engine.Workspace(wl.qb, dense=False)
    s_adm = dataclasses.replace(st, polish=0, eps_abs=st.eps_grouped, eps_rel=st.eps_grouped, min_iter=st.min_iter_grouped)   # the loose stop
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
    prev_k = None
    for r in range(int(st.polish_rounds)):
        _lib.check(lib.pq_polish_grouped_round(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc),
                                               rec.data_ptr(), ws.ldk, engine._ptr(g.gdates), g.ngroups,
                                               engine._ptr(g.urows), engine._ptr(g.ucnt), engine._ptr(g.uoff),
                                               g.umax, ctypes.byref(s), scr.data_ptr(), None, strm), "round")
        R = rec.cpu().numpy()
        state = R[:, _lib.PQ_PG_STATE]
        k = R[:, 0]
        pend = state == _lib.PQ_PG_PENDING
        line = f"round {r + 1}: pending {int(pend.sum())}, done {int((state == _lib.PQ_PG_DONE).sum())}, " \
               f"fallback {int((state == _lib.PQ_PG_FALLBACK).sum())}, k mean {k.mean():.1f}"
        kb = R[:, 349]   # R_KB (pg_record.h): the free-set size this round's setup found
        solved = pend_in if prev_k is not None else np.ones(len(kb), bool)
        edges = [0, 48, 64, 80, 96, 128, 256, 1 << 30]
        hist = np.histogram(kb[solved], bins=edges)[0]
        line += "; solve buckets " + " ".join(f"<={e}:{c}" for e, c in zip(edges[1:], hist))
        line += f", reused P_FF {int((R[solved, 7] != 0).sum())}"
        # P_FF of this round: from the group Gram (R_GFORM = 348: polish group + 1) or a window pass
        formed = solved & (R[:, 7] == 0) & (kb >= 1) & (kb <= 128)
        line += f", formed from the group Gram {int((R[formed, 348] != 0).sum())} of {int(formed.sum())}"
        if prev_k is not None:
            was = prev_pend
            dk = k[was] - prev_k[was]
            line += f"; of the {int(was.sum())} solved this round: k grew {int((dk > 0).sum())}, " \
                    f"shrank {int((dk < 0).sum())}, same {int((dk == 0).sum())}"
        print(line, flush=True)
        prev_k, prev_pend = k.copy(), pend.copy()
        pend_in = pend.copy()
        if not pend.any():
            break


if __name__ == "__main__":
    main()
