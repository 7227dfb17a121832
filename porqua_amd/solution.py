"""qpsolvers-compatible solution record returned by the MI355X engine.

PorQua reads ``solution.found`` and ``solution.x`` (src/optimization.py:80-87), compares
``solution.obj`` with ``QuadraticProgram.objective_value(x, with_const=False)``
(test/tests_quadratic_program.py:72,82) and serialises ``primal_residual()``,
``dual_residual()`` and ``duality_gap()`` (src/helper_functions.py:69-80).  The residual
definitions are those of qpsolvers >= 3 as quoted in example/compare_solver.ipynb:212-216.
Values are computed on the device by the polish kernel (K4); this class only holds them.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

STATUS_TEXT = {
    0: "unsolved", 1: "solved", 2: "solved_inaccurate", 3: "max_iter_reached",
    4: "refactor_pending", -3: "primal_infeasible", -4: "dual_infeasible", -5: "non_convex",
}


@dataclass
class Solution:
    x: np.ndarray | None = None
    y: np.ndarray | None = None        # equality multipliers (A x = b)
    z: np.ndarray | None = None        # inequality multipliers (G x <= h), >= 0
    z_box: np.ndarray | None = None    # box multipliers: > 0 at the upper, < 0 at the lower bound
    found: bool = False
    obj: float | None = None
    status: int = 0
    iterations: int = 0
    extras: dict = field(default_factory=dict)
    _prim: float = float("nan")
    _dual: float = float("nan")
    _gap: float = float("nan")

    def primal_residual(self) -> float:
        return self._prim

    def dual_residual(self) -> float:
        return self._dual

    def duality_gap(self) -> float:
        return self._gap

    @property
    def status_text(self) -> str:
        return STATUS_TEXT.get(int(self.status), str(self.status))

    def is_optimal(self, eps_abs: float = 1e-7) -> bool:
        return bool(self.found and max(self._prim, self._dual, self._gap) <= eps_abs)
