#!/usr/bin/env python3
"""Oracle optimum of the n = 2000 dense QP of porqua_amd.synthetic.dense_qp (TEST
INFRASTRUCTURE ONLY) -> tests/golden/dense_n2000_oracle.npz, for the per-QP drop-in test
beyond 1024 assets (tests/test_large_dense_gpu.py).  oracle.qp_ipm.solve_qp (cvxopt coneqp
restatement + active-set refinement, KKT-certified).  python tools/capture_dense_large.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.qp_ipm import solve_qp  # noqa: E402
from porqua_amd.synthetic import dense_qp  # noqa: E402

if __name__ == "__main__":
    pr = dense_qp(2000)
    t = time.time()
    o = solve_qp(pr["P"], pr["q"], G=pr["G"], h=pr["h"], A=pr["A"], b=pr["b"], lb=pr["lb"], ub=pr["ub"])
    assert o.found
    print("n=2000", o.obj, int((o.x > 1e-9).sum()), o.extras["kkt_primal"], o.extras["kkt_dual"],
          f"{time.time() - t:.1f}s", flush=True)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "dense_n2000_oracle.npz"), x=o.x, obj=o.obj,
                        y=o.y, z=o.z, z_box=o.z_box, kkt_primal=o.extras["kkt_primal"],
                        kkt_dual=o.extras["kkt_dual"], n=2000)
