#!/usr/bin/env python3
"""Per-phase wall-clock split of the polish kernel (library built with EXTRA=-DPQ_PROFILE).

Runs the bench workload (config 3, low-rank path) once and prints the mean ticks of each
polish phase per problem (wall_clock64, 100 MHz) -- experiment tooling, not a test."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import engine  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402

PHASES = ["setup+classify", "free list", "rF/dA", "cholesky", "U+S", "refine", "expand",
          "checks", "final", "form P_FF", "exact Px"]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cfg4 = "--config4" in sys.argv   # n = 3000 tracking LS with 20 sector caps (tools/bench_configs.py)
    lsq = "--lsq494" in sys.argv     # config 2's shape: n = 494 tracking LS, budget + long-only box
    n, T, D = (3000 if cfg4 else (494 if lsq else 1000)), 252, int(args[0]) if args else (2000 if cfg4 else 4749)
    stride = 1   # --stride=S: rebalance every S rows (21: the monthly run of the reference notebook)
    for a in sys.argv:
        if a.startswith("--stride="):
            stride = int(a.split("=")[1])
    dates, R, y, sec = factor_panel(T - 1 + (D - 1) * stride + 1, n, n_sectors=20 if cfg4 else 10)
    rows, tlen = engine.window_rows(dates, dates[T - 1:T - 1 + (D - 1) * stride + 1:stride], T)
    pan = engine.Panel(R, y if (cfg4 or lsq) else None)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    G = np.stack([(sec == g).astype(float) for g in range(20)]) if cfg4 else None
    qb = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), G=G,
                                   h=np.full(20, 0.15) if cfg4 else None, lb=np.zeros(n), ub=np.ones(n))
    qb.batch = D
    mu = pan.window_means(r_d, t_d)
    dev = mu.device
    qb.P = None   # window path: P stays in window form
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=dev)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=dev)
    if cfg4 or lsq:
        xty, _ = pan.gram_xy(r_d, t_d)
        qb.q = (-2.0 * xty).contiguous()
        lr = engine.LowRank(pan, r_d, t_d, mu=None)
    else:
        lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    ws = engine.Workspace(qb, dense=False)
    gp = engine.GroupPlan(rows, tlen, dev) if ("--group" in sys.argv or "--gcap" in sys.argv) else None
    off = (9 + ws.mg_pad) * qb.ld   # PQ_WORK_PROF
    for _ in range(2):
        ev = []
        ws.work[:, off + 16:off + 24].zero_()
        st = (engine.Settings.from_params({"rho0_rel": 0.1 if cfg4 else 0.2, "rho0_qrel": 0.0}) if (cfg4 or lsq)
              else engine.Settings())
        for a in sys.argv:   # --refine=N: proximal refinement steps per polish round
            if a.startswith("--refine="):
                st.refine_iters = int(a.split("=")[1])
        res = engine.solve_lowrank(qb, lr, st, ws, events=ev, groups=gp, gcap="--gcap" in sys.argv)
        torch.cuda.synchronize()
    ad = ws.work[:, off + 16:off + 24].cpu().numpy() * 10e-3   # wall_clock64 ticks (100 MHz) -> us
    its = res.iters.cpu().numpy().astype(float)
    atot = ad.sum(1)
    if gp is not None:
        names = (["pass 1 (MFMA)", "M_U^-1 GEMM", "per-date Woodbury", "pass 2 (MFMA)", "updates/resid/rhs"]
                 if "--gcap" in sys.argv else ["pass 1 (MFMA)", "M^-1 symv", "pass 2 (MFMA)", "updates/resid/rhs"])
        print("grouped admm, chip-wide ms per phase (sum over groups / 256 CUs):")
        for i, p in enumerate(names):
            print("  %-18s %8.2f ms" % (p, ad[:, i].sum() / 256 / 1e3))
        print("  groups %d, mean size %.1f" % (gp.ngroups, gp.sizes.mean()))
    print("admm us per problem: mean %.1f  (%.2f us per iteration)" % (atot.mean(), (atot / its).mean()))
    for i, p in enumerate(["rhs", "v, mu.v", "w = U v", "M^-1 symv", "U'u + tree + corr", "updates+resid"]):
        print("  %-18s %8.2f us/iter (%4.1f %%)" % (p, (ad[:, i] / its).mean(), 100 * ad[:, i].mean() / atot.mean()))
    prof = ws.work[:, off:off + 16].cpu().numpy() * 10e-3   # ticks (10 ns) -> us
    tot = prof[:, :11].sum(1)
    print("polish us per problem: mean %.1f  p50 %.1f  p90 %.1f" % (tot.mean(), np.median(tot), np.percentile(tot, 90)))
    for i, p in enumerate(PHASES):
        print("  %-16s %8.1f us  (%4.1f %%)" % (p, prof[:, i].mean(), 100 * prof[:, i].mean() / tot.mean()))
    if "--gcap" in sys.argv or "--group" in sys.argv:
        rec = ws.pg_record()[:, 8:14].cpu().numpy() * 10e-3
        done = ws.pg_record()[:, 4].cpu().numpy()
        print("grouped polish solve kernel, us per date (sum over rounds), mean over dates:")
        for i, nm in enumerate(["load P_FF", "potrf", "U + S", "residual", "solves", "write back"]):
            print("  %-12s %8.1f us" % (nm, rec[:, i].mean()))
        print("  rounds mean %.2f" % done.mean())
        pp = ws.pg_record()[:, 16:19].cpu().numpy() * 10e-3
        for i, nm in enumerate(["potrf: diag chain (+ deferred MFMA update)", "potrf: panel trsm", "potrf: (unused)"]):
            print("  %-20s %8.1f us" % (nm, pp[:, i].mean()))
        bb = ws.pg_record()[:, 25:32].cpu().numpy()
        nb = max(bb[:, 5].sum(), 1)
        print("  k_pg_big: %d date-rounds, mean k %.1f; us per date-round:" % (bb[:, 5].sum(), bb[:, 6].sum() / nb))
        for i, nm in enumerate(["factor (wg_cholesky)", "U + S", "residual", "solves + update", "expand"]):
            print("    %-22s %8.1f us" % (nm, bb[:, i].sum() * 10e-3 / nb))
        ic = ws.pg_record()[:, 20:25].cpu().numpy()
        print("  inner steps: solve calls %.0f, steps taken %.0f, violators per step %.2f, steps with ma + nv > 8: %.0f,"
              " mean k at the check %.1f" % (ic[:, 0].sum(), ic[:, 1].sum(), ic[:, 2].sum() / max(ic[:, 1].sum(), 1),
                                             ic[:, 3].sum(), ic[:, 4].sum() / max(ic[:, 0].sum(), 1)))
    for name, a, b in ev:
        print("stage", name, "%.1f ms" % a.elapsed_time(b))
    out = res.out.cpu().numpy()
    print("nfree mean %.1f rounds mean %.2f" % (out[:, 5].mean(), out[:, 6].mean()))


if __name__ == "__main__":
    main()
