#!/usr/bin/env python3
"""Diagnostics for the LAD IPM (porqua_amd/lad.py): per-iteration residual trace of the
windows of the n = 300 test that do not converge.  Experiment tooling."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import lad  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402

n, D, width = 300, 320, 252
dates, R, yv, _ = factor_panel(D, n, seed=5)
ends = np.arange(width + 11, width + 35)
Xb = np.stack([np.log(np.cumprod(1 + R[e - width:e], 0)) for e in ends])
yb = np.stack([np.log(np.cumprod(1 + yv[e - width:e])) for e in ends])
dev = torch.device("cuda:0")
pr = lad.LADProblem(torch.from_numpy(Xb).to(dev), torch.from_numpy(yb).to(dev), A=np.ones((1, n)), b=np.ones(1),
                    lb=np.zeros(n), ub=np.full(n, 0.05))
tr = []
res = lad.lad_ipm_batched(pr, trace=tr)
print("status", res.status.tolist())
print("iters", res.iters.tolist())
for t in tr:
    print(t)
