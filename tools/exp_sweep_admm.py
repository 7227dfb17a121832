#!/usr/bin/env python3
"""Time the config-5 sweep ADMM kernels in isolation (experiment tooling, not a test).

Builds the config-5 batch (workloads.SweepBacktest: n 5000, 64 dates x 64 risk aversions),
solves it once (capacitance inverses, the ADMM point), then re-runs a fixed number of ADMM
iterations from that point with every problem active:
  * pq_admm_lr_sweep (admm_sweep.hip; PQ_LIB_PATH selects an experiment build);
  * pq_admm_lr_grouped (k_admm_grp, the 16-problem groups) for comparison.
Prints ms per iteration of each.  Usage: python tools/exp_sweep_admm.py [iters]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.workloads import SweepBacktest  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    iters = int(args[0]) if args else 12
    wl = SweepBacktest()
    wl.step()
    torch.cuda.synchronize()
    sw, qb, lr, ws = wl.sweep, wl.qb, wl.lr, wl.ws
    lib = _lib.load()
    strm = engine._stream()
    bd = engine._band_setup(qb, lr, strm, w_min=0)
    M = ws.lr_buffers(256)
    x0, z0, y0 = ws.x.clone(), ws.z.clone(), ws.y.clone()
    s = engine.Settings.from_params({"eps_abs": 1e-12, "eps_rel": 1e-12}).to_c()
    s.max_iter = 100000
    s.min_iter = 10 ** 9   # no stop: every variant runs the same iterations
    pb, lrs = qb.c_struct(), lr.c_struct()

    def reset():
        ws.x.copy_(x0)
        ws.z.copy_(z0)
        ws.y.copy_(y0)
        ws.status.fill_(_lib.PQ_UNSOLVED)
        ws.iters.zero_()

    def run_sweep():
        stc = ws.c_struct()
        scr = sw.sp.buffer(qb, lib)
        return lib.pq_admm_lr_sweep(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc), M["Minv"].data_ptr(),
                                    256, 256 * 256, sw.sp.gdates.data_ptr(), sw.sp.ngroups, ctypes.byref(s), iters,
                                    bd["pc"].data_ptr(), bd["pc"].stride(0), bd["r0"], bd["cc"].data_ptr(), 1,
                                    scr.data_ptr(), scr.numel(), strm)

    def run_grp():
        stc = ws.c_struct()
        g = sw.gp
        return lib.pq_admm_lr_grouped(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc), M["Minv"].data_ptr(),
                                      256, 256 * 256, g.gdates.data_ptr(), g.ngroups, g.urows.data_ptr(),
                                      g.ucnt.data_ptr(), g.uoff.data_ptr(), g.umax, ctypes.byref(s), iters,
                                      bd["pc"].data_ptr(), bd["pc"].stride(0), bd["r0"], bd["cc"].data_ptr(), None,
                                      None, 0, strm)

    runs = (("sweep", run_sweep),) if "--sweep-only" in sys.argv else (("sweep", run_sweep), ("grouped", run_grp))
    for name, fn in runs:
        ts = []
        for rep in range(4):
            reset()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            _lib.check(fn(), name)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        it = ws.iters.float().mean().item()
        print("%-8s %d iterations: %s ms  (%.3f ms / iteration, mean iters %.1f)"
              % (name, iters, " ".join("%.2f" % t for t in ts), min(ts[1:]) / iters, it), flush=True)
        if name == "sweep" and "--prof" in sys.argv:   # PQ_SW_PROF build: the last pass's phase clocks
            scr = sw.sp.buffer(qb, lib)
            nch = (qb.n + 255) // 256
            ng = sw.sp.ngroups
            off = qb.batch * 80 + ng * nch * 64 * 256
            rp = scr[off:off + ng * nch * 64 * 16].view(ng * nch, 64, 16)[:, 0, :].cpu().numpy()
            ph = rp[:, [7, 13, 14, 15]]
            tot = ph.sum(1)
            print("k_sw_pass phase clocks per workgroup (last launch): pass 2 %.0f, updates %.0f, pass 1 %.0f,"
                  " setup %.0f, total %.0f (max %.0f)" % (*ph.mean(0), tot.mean(), tot.max()), flush=True)


if __name__ == "__main__":
    main()
