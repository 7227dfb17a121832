#!/usr/bin/env python3
"""Debug helper (experiment tooling): group-capacitance ADMM launch by launch on a small
strided problem -- group rho, statuses and iterations after each launch."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import engine  # noqa: E402
from tests.test_gcap_gpu import _problem  # noqa: E402

dev = torch.device("cuda", 0)
qb, lr, gp = _problem(dev, 300, 60, 30, 0.2, 3)
print("groups", gp.ngroups, gp.sizes, "ucnt", gp.ucnt.cpu().numpy(), "corr_max", gp.corr_max)
for rounds in (1, 2, 3, 4, 6, 10):
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, polish=0)
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, st, ws=ws, groups=gp, gcap=True, max_rounds=rounds)
    torch.cuda.synchronize()
    print("rounds", rounds, "grho", ws._gcap["grho"].cpu().numpy().round(6), "status", res.status.cpu().numpy(),
          "iters", res.iters.cpu().numpy())
ws = engine.Workspace(qb, dense=False)
res = engine.solve_lowrank(qb, lr, engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, polish=0), ws=ws,
                           groups=gp, gcap=False)
torch.cuda.synchronize()
print("per-date: rho", ws.rho.cpu().numpy().round(6), "iters", res.iters.cpu().numpy(), "refactors", res.refactors)
