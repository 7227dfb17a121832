"""porqua_amd -- MI355X-native engine for PorQua's backtest hot path.

Rolling covariance / Gram estimation plus one constrained QP per rebalance date, all dates
solved together on the GPU by hand-written gfx950 HIP kernels (libporqua_hip.so, C ABI in
include/porqua_hip.h), behind PorQua's own API:

    from porqua_amd.optimization import MeanVariance
    opt = MeanVariance(solver_name='mi355x')      # the new solver name

Modules mirror the reference (covariance, mean_estimation, constraints, optimization,
qp_problems, backtest, builders, ...); ``engine`` is the device layer.
"""
from ._lib import PorquaHipError, load as load_library  # noqa: F401

__version__ = "0.1.0"
ENGINE_SOLVER = "mi355x"
