import sys, numpy as np, torch
sys.path.insert(0, '.')
from porqua_amd import engine, _lib
from porqua_amd.synthetic import factor_panel
dev = torch.device('cuda', 0)
n, T, ns, cap = 3000, 252, 20, 0.15
ends = list(range(260, 266))
dates, R, y, sec = factor_panel(max(ends) + 1, n, n_sectors=ns)
rows, tlen = engine.window_rows(dates, dates[ends], T)
pan = engine.Panel(R, y, device=dev)
r_d, t_d = pan.rows_to_device(rows, tlen)
B = len(ends)
G = np.stack([(sec == g).astype(float) for g in range(ns)]); h = np.full(ns, cap)
for rounds in (8, 30):
  for kc in (256, 1024):
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.zeros(n), ub=np.ones(n), device=dev)
    qb.batch = B; qb.P = None
    xty, _ = pan.gram_xy(r_d, t_d)
    qb.q = (-2.0 * xty).contiguous()
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=dev)
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, dev)
    ws = engine.Workspace(qb, dense=False, kcap=kc)
    res = engine.solve_lowrank(qb, lr, engine.Settings(rho0_rel=0.5, polish_rounds=rounds), ws=ws, groups=gp)
    o = res.out.cpu().numpy()
    print("rounds", rounds, "kcap", kc, "status", res.status.cpu().numpy(), "iters", res.iters.cpu().numpy())
    print("  nfree", o[:, 5], "rounds", o[:, 6], "prim", o[:, 1], "dual", o[:, 2], "obj", o[:, 0])
    x = res.x.cpu().numpy()
    print("  nnz", (x > 1e-9).sum(1), "groups at cap", ((G @ x.T) > cap - 1e-9).sum(0))
