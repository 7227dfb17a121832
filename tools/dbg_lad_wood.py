#!/usr/bin/env python3
"""Debug: LAD IPM on n = 300 windows, Woodbury vs dense normal equations (trace per iteration)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from porqua_amd import lad
from porqua_amd.synthetic import factor_panel
from oracle import lad as olad

dates, R, y, _ = factor_panel(320, 300)
T = 252
ends = np.arange(262, 266)
X = np.stack([olad.levels(R[e - T:e]) for e in ends])
Y = np.stack([olad.levels(y[e - T:e]) for e in ends])
dev = torch.device("cuda")
for wood in (False, True):
    lad.WOODBURY = wood
    pr = lad.LADProblem(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), A=np.ones((1, 300)), b=np.ones(1),
                        lb=np.zeros(300), ub=np.full(300, 0.05))
    tr = []
    res = lad.lad_ipm_batched(pr, trace=tr)
    print("woodbury", wood, "status", res.status.tolist(), "iters", res.iters.tolist())
    for t in tr[:40]:
        print("  it %d mu %.3e rp %.3e rd %.3e gap %.3e" % t)
    print("obj", res.obj.tolist())
