"""Debug helper: factor the low-rank capacitance matrices directly and compare with numpy."""
import sys; sys.path.insert(0, '.')
import ctypes
import numpy as np, torch
from porqua_amd import engine, _lib
from porqua_amd.synthetic import factor_panel
n, T = 600, 120
ends = [200, 333]
dates, R, y, sec = factor_panel(400, n)
rows, tlen = engine.window_rows(dates, dates[ends], T)
pan = engine.Panel(R, y)
r_d, t_d = pan.rows_to_device(rows, tlen)
B = 2
qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, 0.05))
qb.batch = B
qb.P = pan.cov(r_d, t_d, mode=1)
xty, _ = pan.gram_xy(r_d, t_d)
qb.q = (-2.0 * xty).contiguous()
qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=qb.P.device)
lr = engine.LowRank(pan, r_d, t_d)
ws = engine.Workspace(qb)
res = engine.solve_lowrank(qb, lr, engine.Settings(rho0_rel=0.5, max_iter=1), ws, polish=False)
Mb = ws._lr
print('info after solve', Mb['info'].tolist())
k_ld = Mb['M'].shape[-1]
Mfull = torch.tril(Mb['M']); Mfull = Mfull + torch.tril(Mfull, -1).transpose(1, 2)
for rep in range(3):
    q2 = engine.QPBatch.from_dense(Mfull.cpu().numpy(), np.zeros((B, k_ld)))
    w2, info = engine.factor_only(q2, invert=False)
    print('factor_only(full M) info', info.tolist())
    q3 = engine.QPBatch.from_dense(Mfull.cpu().numpy(), np.zeros((B, k_ld)))
    q3.P = Mb['M'].clone()
    w3, info3 = engine.factor_only(q3, invert=False)
    print('factor_only(lower-only M buffer) info', info3.tolist())
for b in range(B):
    Mh = Mfull[b].cpu().numpy()
    L = np.linalg.cholesky(Mh)
    print(b, 'numpy chol ok, min diag L', L.diagonal().min(), 'cond', np.linalg.cond(Mh))
    print('   upper garbage finite?', bool(torch.isfinite(Mb['M'][b]).all()), 'asym diag tiles',
          max(float((Mb['M'][b, i*64:(i+1)*64, i*64:(i+1)*64] - Mb['M'][b, i*64:(i+1)*64, i*64:(i+1)*64].T).abs().max()) for i in range(k_ld // 64)))
