#!/usr/bin/env python3
"""Grouped-polish hand-offs and free-set sizes of the uncentred test problem
(tests/test_polish_grouped_gpu.py, case uncentred_q0: q = 0): PQ_PG_GFORM=0 vs the default.  Diagnostic."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from porqua_amd import _lib, engine  # noqa: E402
from tests.test_polish_grouped_gpu import _problem, _solve  # noqa: E402

dev = torch.device("cuda", 0)
for args in [(600, 150, 40, 1.0), (300, 60, 40, 1.0)]:
    qb, lr, gp = _problem(dev, *args, centred=False)
    qb.q.zero_()
    xa, sa, oa, ya, za, outa, _ = _solve(qb, lr, gp, False, engine.Settings(rho0_rel=0.5))
    xb, sb, ob, yb, zb, outb, rec = _solve(qb, lr, gp, True, engine.Settings(rho0_rel=0.5))
    print(args, "nfree", np.percentile(outa[:, _lib.PQ_OUT_NFREE], [0, 50, 100]), "rec", np.unique(rec, return_counts=True),
          "dx", np.abs(xa - xb).max(), flush=True)
