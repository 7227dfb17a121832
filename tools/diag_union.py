#!/usr/bin/env python3
"""Config 2 (n = 494 tracking LS, 4544 daily dates): sizes of the free sets and of their
unions over the grouped polish's 16-date groups, from the final weights (experiment tooling:
sizes the group Gram of free sets beyond the LDS solve)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd.workloads import ReplicationBacktest  # noqa: E402


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "sptr.npz"), allow_pickle=False)
    wl = ReplicationBacktest(g["days"], g["returns"])
    res = wl.step()
    torch.cuda.synchronize()
    x = res.x[:, :wl.n].cpu().numpy()
    free = (x > 1e-9) & (x < 1 - 1e-9)
    k = free.sum(1)
    print("free set: mean %.1f p10 %d p50 %d p90 %d max %d" % (k.mean(), *np.percentile(k, [10, 50, 90]), k.max()))
    rec = wl.ws.pg_record()
    bb = rec[:, 25:32].cpu().numpy()
    nb = max(bb[:, 5].sum(), 1)
    if bb[:, 5].sum() > 0:   # profile build (PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so)
        print("k_pg_big: %d date-rounds, mean k %.1f; us per date-round:" % (bb[:, 5].sum(), bb[:, 6].sum() / nb))
        for i, nm in enumerate(["factor (wg_cholesky)", "U + S", "residual", "solves + update", "expand"]):
            print("    %-22s %8.1f us" % (nm, bb[:, i].sum() * 10e-3 / nb))
    pp = wl.gplan.polish_plan()
    gd = pp.gdates.cpu().numpy()
    for gsz in (16, 8, 4):
        us = []
        for a in range(len(gd) - 1):
            lo, hi = int(gd[a]), int(gd[a + 1])
            for s in range(lo, hi, gsz):
                us.append(int(free[s:min(hi, s + gsz)].any(0).sum()))
        us = np.array(us)
        print("union over %2d dates: mean %.1f p50 %d p90 %d max %d; <=256: %.2f <=320: %.2f <=384: %.2f"
              % (gsz, us.mean(), np.median(us), np.percentile(us, 90), us.max(), (us <= 256).mean(),
                 (us <= 320).mean(), (us <= 384).mean()))


if __name__ == "__main__":
    main()
