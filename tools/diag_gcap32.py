import sys, numpy as np, torch
sys.path.insert(0, '.')
from porqua_amd import engine, _lib
import porqua_amd.engine as eng
from tests.test_gcap_gpu import _problem
dev = torch.device('cuda', 0)
def run(gcap, gmax, cus, n, T, D, ub, centred, caps):
    eng.GCAP_MAX_DATES = gmax
    qb, lr, gp = _problem(dev, n, T, D, ub, centred=centred, caps=caps, cus=cus)
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, adapt_interval=0, eps_grouped=0.0)
    ws = engine.Workspace(qb, dense=False)
    r = engine.solve_lowrank(qb, lr, st, ws=ws, groups=gp, gcap=gcap, polish=False)
    torch.cuda.synchronize()
    g = ws.gcap_groups
    return r.x.cpu().numpy().copy(), r.iters.cpu().numpy().copy(), (None if g is None else int(g.sizes.max()))
for args in [(600, 120, 300, 0.2, True, 2), (600, 150, 40, 0.2, True, 2), (600, 120, 300, 0.2, True, 0)]:
    for cus in (16, 2):
        xa, ia, _ = run(False, 32, cus, *args)
        xb, ib, gb = run(True, 16, cus, *args)
        xc, ic, gc = run(True, 32, cus, *args)
        print(args, 'cus', cus, 'g16', gb, 'g32', gc, 'pd-vs-16 %.2e' % np.abs(xa-xb).max(), 'pd-vs-32 %.2e' % np.abs(xa-xc).max(),
              '16-vs-32 %.2e' % np.abs(xb-xc).max(), 'it', np.abs(ia-ib).max(), np.abs(ia-ic).max(), 'xmax %.2e' % np.abs(xa).max(), flush=True)
