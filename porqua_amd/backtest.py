# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/backtest.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Backtest service and rebalance loop (mirror of src/backtest.py:42-270).

``Backtest.run(bs)`` keeps the reference semantics.  When the optimization's solver is the
device engine ('mi355x') and the builders are the standard ones (src/builders.py), the
loop runs in two phases instead of one serial QP per date:

  A (host, once): selection + constraints from the first date (they are date-invariant
    for the standard builders), window row lists for every rebalance date
    (``data[index <= rebdate].tail(width)`` minus weekends, src/builders.py:208-211);
  B (device): the whole panel is uploaded once; K1 builds every date's covariance / Gram,
    K2-K4 solve every date's QP in one batch (chunked to bound HBM use), sharded across
    ranks when torch.distributed is initialised (contiguous date blocks, one all-gather of
    the weight panel -- SURVEY.md §8(e));
  C (host): Portfolio objects in date order, ``append_fun`` called per date.

Dates are independent in the reference; an ``append_fun`` that mutates
state read by later dates is not supported in batched mode (set settings['batched'] = False
to force the serial loop, which still solves each date on the device).
"""
from __future__ import annotations

import gc
import os
import pickle
from typing import Optional

import numpy as np
import pandas as pd

from . import builders as _b
from .constraints import Constraints
from .optimization import EmptyOptimization, Optimization
from .optimization_data import OptimizationData
from .portfolio import Portfolio, Strategy
from .selection import Selection

# page-locked weight panels kept for reuse: (rows, n) -> (tensor, weakref to the numpy view
# handed out last).  Pinning tens of MB costs milliseconds per backtest; a panel is reused
# only once nothing (no Portfolio row view) references the previous backtest's array.
_PINNED: dict = {}


def _pinned_panel(rows: int, n: int):
    import weakref
    import torch
    ent = _PINNED.get((rows, n))
    if ent is not None and ent[1]() is None:
        t = ent[0]
    else:
        t = torch.empty((rows, n), dtype=torch.float64, pin_memory=True)
    W = t.numpy()
    _PINNED[(rows, n)] = (t, weakref.ref(W))
    return t, W


class BacktestData:
    def __init__(self):
        pass


class BacktestService:

    def __init__(self, data, selection_item_builders: dict, optimization_item_builders: dict,
                 optimization: Optional[Optimization] = None, settings: Optional[dict] = None, **kwargs) -> None:
        self.data = data
        self.optimization = EmptyOptimization() if optimization is None else optimization
        self.selection_item_builders = selection_item_builders
        self.optimization_item_builders = optimization_item_builders
        self.settings = settings if settings is not None else {}
        self.settings.update(kwargs)
        self.selection = Selection()
        self.optimization_data = OptimizationData([])

    @property
    def selection(self):
        return self._selection

    @selection.setter
    def selection(self, value):
        if not isinstance(value, Selection):
            raise TypeError("Expected a Selection instance for 'selection'")
        self._selection = value

    @property
    def selection_item_builders(self):
        return self._selection_item_builders

    @selection_item_builders.setter
    def selection_item_builders(self, value):
        if not isinstance(value, dict) or not all(isinstance(v, _b.SelectionItemBuilder) for v in value.values()):
            raise TypeError("Expected a dictionary containing SelectionItemBuilder instances "
                            "for 'selection_item_builders'")
        self._selection_item_builders = value

    @property
    def optimization(self):
        return self._optimization

    @optimization.setter
    def optimization(self, value):
        if not isinstance(value, Optimization):
            raise TypeError("Expected an Optimization instance for 'optimization'")
        self._optimization = value

    @property
    def optimization_item_builders(self):
        return self._optimization_item_builders

    @optimization_item_builders.setter
    def optimization_item_builders(self, value):
        if not isinstance(value, dict) or not all(isinstance(v, _b.OptimizationItemBuilder) for v in value.values()):
            raise TypeError("Expected a dictionary containing OptimizationItemBuilder instances "
                            "for 'optimization_item_builders'")
        self._optimization_item_builders = value

    @property
    def settings(self):
        return self._settings

    @settings.setter
    def settings(self, value):
        if not isinstance(value, dict):
            raise TypeError("Expected a dictionary for 'settings'")
        self._settings = value

    def build_selection(self, rebdate: str) -> None:
        for key, item_builder in self.selection_item_builders.items():
            item_builder.arguments["item_name"] = key
            item_builder(self, rebdate)

    def build_optimization(self, rebdate: str) -> None:
        self.optimization.constraints = Constraints(selection=self.selection.selected)
        for item_builder in self.optimization_item_builders.values():
            item_builder(self, rebdate)

    def prepare_rebalancing(self, rebalancing_date: str) -> None:
        self.build_selection(rebdate=rebalancing_date)
        self.build_optimization(rebdate=rebalancing_date)


# ------------------------------------------------------------------------------------------
# batched staging
# ------------------------------------------------------------------------------------------


def shard_range(total: int, rank: int, world: int):
    """Contiguous block of dates for ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class BatchStage:
    """Device staging of one backtest (or one chunk of it) for objective_batch()."""

    def __init__(self, panel, rows_host, tlen_host, device):
        import torch
        self.panel = panel
        self.device = device
        self.rows_host = np.ascontiguousarray(rows_host, dtype=np.int32)
        self.tlen_host = np.ascontiguousarray(tlen_host, dtype=np.int32)
        self.rows = torch.from_numpy(self.rows_host).to(device)
        self.tlen = torch.from_numpy(self.tlen_host).to(device)
        self.batch = len(self.tlen_host)
        self.n = panel.n
        self.ld = ((panel.n + 63) // 64) * 64
        self._P = None
        self._log_panel = None
        self._slide = None
        self._groups = None
        # set by Backtest before objective_batch: the objective may hand back the factored
        # (window) form of P in .lowrank, and then stores P's lower triangle only
        self.prefer_lowrank = False
        self.lowrank = None

    def slide_plan(self):
        """SlidePlan of the windows (sliding K1), None when no window slides."""
        from . import engine
        if self._slide is None:
            plan = engine.SlidePlan(self.rows_host, self.tlen_host, self.device)
            self._slide = plan if plan.ngroups < self.batch else False
        return self._slide or None

    def group_plan(self):
        from . import engine
        if self._groups is None:
            self._groups = engine.GroupPlan(self.rows_host, self.tlen_host, self.device)
        return self._groups

    def P_buffer(self):
        import torch
        if self._P is None:
            self._P = torch.empty((self.batch, self.ld, self.ld), dtype=torch.float64, device=self.device)
        return self._P

    def identity_P(self):
        import torch
        P = self.P_buffer()
        P.zero_()
        idx = torch.arange(self.n, device=self.device)
        P[:, idx, idx] = 1.0
        return P

    def sub_windows(self, a: int, b: int):
        """Rows [a, b) of every window (for estimators that use a sub-window)."""
        import torch
        T = int(self.tlen_host.max())
        if (a, b) == (0, T):
            return self.rows, self.tlen
        r = self.rows_host[:, a:b].copy()
        t = np.clip(self.tlen_host - a, 0, b - a).astype(np.int32)
        return torch.from_numpy(np.ascontiguousarray(r)).to(self.device), torch.from_numpy(t).to(self.device)

    def log1p_panel(self):
        import torch
        from . import engine
        if self._log_panel is None:
            p = engine.Panel(torch.log1p(self.panel.R), None if self.panel.bm is None else torch.log1p(self.panel.bm),
                             device=self.device)
            self._log_panel = p
        return self._log_panel


class _PanelUpload:
    """The return panel's host -> device copy on a worker thread (torch releases the GIL for
    the copy, so the caller's host work -- window rows, constraints, the group plan -- runs
    meanwhile).  ``result()`` joins and returns the device tensor (or re-raises)."""

    def __init__(self, frame):
        import threading
        from . import engine
        self._out = None
        self._err = None
        self._frame = frame
        # the device is resolved HERE, on the calling thread: torch's current device is per
        # host thread, so a worker would see device 0 instead of the rank's set_device choice
        try:
            self._dev = engine.default_device()
        except BaseException as ex:   # (no device: surfaces in result(), as on the serial path)
            self._dev, self._err = None, ex
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        import torch
        if self._err is not None:
            return
        try:
            R = np.ascontiguousarray(self._frame.to_numpy(dtype=np.float64))
            if self._dev.type == "cuda":
                with torch.cuda.device(self._dev):   # the worker's HIP context on the rank's GPU
                    self._out = torch.from_numpy(R).to(self._dev)
            else:
                self._out = torch.from_numpy(R).to(self._dev)
        except BaseException as ex:   # re-raised in the caller's thread
            self._err = ex

    def result(self):
        self._t.join()
        if self._err is not None:
            raise self._err
        return self._out


def _batchable(bs) -> bool:
    """Batched mode needs builders whose output does not depend on the date beyond the
    return / benchmark windows: the standard ones, or any set the caller declares
    date-invariant with ``settings['static_builders'] = True`` (e.g. a builder that adds the
    same l1 terms every date, the usual way to pass a turnover or leverage constraint)."""
    if not bs.settings.get("batched", True):
        return False
    if bs.settings.get("static_builders"):
        return True
    fns = [b.arguments.get("bibfn") for b in list(bs.selection_item_builders.values()) +
           list(bs.optimization_item_builders.values())]
    return all(f in _b.STANDARD_BIBFNS for f in fns)


class Backtest:

    def __init__(self) -> None:
        self._strategy = Strategy([])
        self._output = {}
        self.stats = {}

    @property
    def strategy(self):
        return self._strategy

    @property
    def output(self):
        return self._output

    def append_output(self, date_key=None, output_key=None, value=None):
        if value is None:
            return True
        if date_key in self.output:
            if output_key in self.output[date_key]:
                raise Warning(f"Output key '{output_key}' for date key '{date_key}' already exists and will be overwritten.")
            self.output[date_key][output_key] = value
        else:
            self.output[date_key] = {output_key: value}
        return True

    def rebalance(self, bs: BacktestService, rebalancing_date: str) -> None:
        bs.prepare_rebalancing(rebalancing_date=rebalancing_date)
        try:
            bs.optimization.set_objective(optimization_data=bs.optimization_data)
            bs.optimization.solve()
        except Exception as error:
            raise RuntimeError(error)

    def run(self, bs: BacktestService) -> None:
        from .qp_problems import ENGINE_SOLVERS
        if bs.optimization.params.get("solver_name") in ENGINE_SOLVERS and _batchable(bs):
            if self._run_batched(bs):
                return None
        return self._run_serial(bs)

    def _after_solve(self, bs, rebalancing_date):
        portfolio = Portfolio(rebalancing_date=rebalancing_date, weights=bs.optimization.results["weights"])
        self.strategy.portfolios.append(portfolio)
        append_fun = bs.settings.get("append_fun")
        if append_fun is not None:
            append_fun(backtest=self, bs=bs, rebalancing_date=rebalancing_date,
                       what=bs.settings.get("append_fun_args"))

    def _run_serial(self, bs) -> None:
        for rebalancing_date in bs.settings["rebdates"]:
            if not bs.settings.get("quiet"):
                print(f"Rebalancing date: {rebalancing_date}")
            self.rebalance(bs=bs, rebalancing_date=rebalancing_date)
            self._after_solve(bs, rebalancing_date)

    def _run_batched(self, bs) -> bool:
        """Two-phase batched run: host staging once (phase A), this rank's contiguous block
        of dates solved on the device (phase B, ``_solve_shard``), the blocks all-gathered
        when torch.distributed is initialised (one collective), then the Portfolio objects
        (phase C).  False: not batchable (the caller runs the serial loop)."""
        import torch
        st = self._stage_batched(bs)
        if st is None:
            return False
        world, rank, dist = 1, 0, None
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            dist = torch.distributed
            world, rank = dist.get_world_size(), dist.get_rank()
        nreb = len(st["rebdates"])
        lo, hi = shard_range(nreb, rank, world)
        ok, W, ST, OBJ, path = self._solve_shard(bs, st, lo, hi)
        # batchability of a chunk depends on its own windows (window lengths, WLS runs): a
        # rank that cannot batch must not return while the others block in the all-gather,
        # so every rank finishes its shard and the verdict is agreed collectively
        if dist is not None:
            ok = agree_all(ok, dist)
        if not ok:
            return False                      # some rank cannot batch: serial path everywhere
        if dist is not None:
            W, ST, OBJ = gather_shards(W, ST, OBJ, nreb, world, dist, None)
        self._finish_batched(bs, st, W, ST, OBJ, path)
        return True

    def _stage_batched(self, bs):
        """Phase A (host, once): selection and constraints of the first date (date-invariant
        builders), window row lists of every rebalance date, benchmark alignment, G/h/A/b and
        the box.  Returns the staging dict, or None when the run cannot batch."""
        from . import engine
        rebdates = list(bs.settings["rebdates"])
        if not rebdates:
            return None
        opt = bs.optimization
        # ---- phase A: static selection / constraints, window row lists ------------------
        bs.prepare_rebalancing(rebalancing_date=rebdates[0])
        cons = opt.constraints
        universe = bs.selection.selected
        from .l1split import term_from_model
        l1term = term_from_model(cons, opt.params, universe)   # src/optimization.py:125-142
        l1both = None
        if l1term == "unsupported":           # turnover and leverage together: device IPM
            from .ipm_l1 import terms_from_model
            l1both = terms_from_model(cons, opt.params, universe)
            if l1both is None:
                return None
            l1term = None
        X = bs.data.get("return_series")
        if X is None:
            raise ValueError("Return series data is missing.")
        width = None
        for bld in bs.optimization_item_builders.values():
            if bld.arguments.get("bibfn") is _b.bibfn_return_series:
                width = bld.arguments.get("width")
        if width is None:
            return None
        # the whole frame when the selection is every column in order (no 8 T n-byte copy)
        Xs = X if list(X.columns) == list(universe) else X[universe]
        # the panel upload (D x n FP64 over PCIe) runs on a worker thread while this thread
        # builds the window and group plans (the copy releases the GIL); _solve_shard joins it
        upload = _PanelUpload(Xs)
        idx = pd.DatetimeIndex(Xs.index)
        dates = idx.values.astype("datetime64[D]")
        rows, tlen = engine.window_rows(dates, np.array(rebdates, dtype="datetime64[D]"), width)
        bm = None
        ys = bs.data.get("bm_series")
        if ys is not None:
            yv = ys.reindex(idx)
            yv = yv.iloc[:, 0] if isinstance(yv, pd.DataFrame) else yv
            bm = yv.to_numpy(dtype=np.float64)
            need = np.unique(rows[tlen > 0].ravel())
            if np.isnan(bm[need]).any():
                bm = None                     # benchmark not aligned with the returns
        GhAb = cons.to_GhAb()
        boxed = cons.box["box_type"] != "NA"
        lb = cons.box["lower"].to_numpy(dtype=np.float64) if boxed else None
        ub = cons.box["upper"].to_numpy(dtype=np.float64) if boxed else None
        return {"rebdates": rebdates, "universe": universe, "Xs": Xs, "bm": bm, "rows": rows, "tlen": tlen,
                "GhAb": GhAb, "lb": lb, "ub": ub, "l1term": l1term, "l1both": l1both, "upload": upload}

    def _solve_shard(self, bs, st, lo: int, hi: int):
        """Phase B (device): dates [lo, hi) of the staged run, chunked to bound HBM use.
        Returns (ok, W [hi - lo, n], status, objective, path)."""
        import torch
        from . import engine
        from .l1split import merge_batch, split_batch, split_settings
        opt = bs.optimization
        rows, tlen, GhAb, lb, ub = st["rows"], st["tlen"], st["GhAb"], st["lb"], st["ub"]
        l1term, l1both = st["l1term"], st["l1both"]
        dev = engine.default_device()
        settings = engine.Settings.from_params(opt.params)
        mg = sum(0 if GhAb[k] is None else np.atleast_2d(GhAb[k]).shape[0] for k in ("A", "G"))
        if l1term is not None:
            mg += 1 if l1term.kind == "budget" else 0
        n = len(st["universe"])
        lad = hasattr(opt, "lad_batch")       # LAD: the LP on the device IPM (porqua_amd/lad.py)
        chunk = int(bs.settings.get("batch_chunk", 0) or _auto_chunk(n))
        # the first chunk's group plan (host numpy) while the panel upload is still in flight
        plan0 = None
        if (not lad and l1both is None and bs.settings.get("lowrank", True)
                and engine.lowrank_shape_ok(n, int(rows.shape[1]), mg)):
            e0 = min(hi, lo + chunk)
            plan0 = (lo, e0, engine.GroupPlan(rows[lo:e0], tlen[lo:e0], dev))
        upload = st.get("upload")
        R = upload.result() if upload is not None else st["Xs"].to_numpy(dtype=np.float64)
        panel = engine.Panel(R, st["bm"], device=dev)
        # windows with missing values (checked on the device copy): the objectives that
        # support them batch with the pairwise-complete covariance (MeanVariance); the others
        # keep the serial path
        if panel.has_nan and not getattr(opt, "batch_handles_nan", False):
            return False, None, None, None, None
        # the weight panel lands in page-locked host memory (one DMA, no pageable bounce; the
        # Portfolio objects keep views of its rows)
        if dev.type == "cuda":
            Wt, W = _pinned_panel(hi - lo, n)
        else:
            Wt, W = None, np.zeros((hi - lo, n))
        ST = np.zeros(hi - lo, dtype=np.int32)
        OBJ = np.zeros(hi - lo)
        split_panel = None
        if l1term is not None:
            if lb is None or ub is None:
                return False, None, None, None, None   # the split needs a box (serial path raises)
            split_panel = engine.Panel(torch.cat([panel.R, -panel.R], 1).contiguous(), None, device=dev)
        # turnover + leverage: the per-asset-block IPM by default; settings['l1_segments'] takes the
        # segment split on the ADMM engine (porqua_amd/l1seg.py) when the box holds 0 and x0 and P
        # has no ridge (checked per chunk).  Measured at the config-3 shape (turnover 0.5, leverage
        # 1.3): the split's ADMM needs ~490 iterations (P is singular along s1 - s2 per asset), 1.4k
        # QPs/s against the IPM's 2.1k (profiles/r05s_bench_l1_both_seg.log), so it is opt-in
        seg_sd, seg_panel, seg_mg = None, None, 0
        if (l1both is not None and lb is not None and ub is not None
                and bs.settings.get("l1_segments", False)):
            from . import l1seg
            seg_sd = l1seg.segment_data(l1both.x0, lb, ub, cost=l1both.cost, to_budget=l1both.to_budget,
                                        lev_budget=l1both.lev_budget)
            if seg_sd is not None:
                seg_mg = mg + (seg_sd["to_budget"] is not None and np.isfinite(seg_sd["to_budget"])) + \
                    bool(np.isfinite(seg_sd["lev_budget"]))
        if lad:
            if l1term is not None or l1both is not None:
                return False, None, None, None, None
            tm = int(tlen.max())
            if tm < n:    # m-space normal equations: (mc + T) x n rows + k_ld^2 factor buffers
                k_ld = (tm + mg + 63) // 64 * 64
                per = 8 * (4 * (tm + mg) * n + 3 * k_ld * k_ld) + 64 * n * 8
            else:         # w-space n x n normal matrix
                per = 8 * (n + 64) ** 2 + 64 * n * tm
            chunk = min(chunk, max(1, (1 << 35) // per))
        path = "lp-ipm" if lad else "dense"
        ok = True
        # the lazy Portfolio objects of a single-rank, single-chunk run without append_fun are
        # built while the device solves (views of W's rows, read only after the solve); phase C
        # keeps those of the solved dates
        self._prebuilt = None
        import torch.distributed as _td
        single = not (_td.is_available() and _td.is_initialized())

        def prebuild():
            if single and bs.settings.get("append_fun") is None:
                keys = list(st["universe"])
                gc_was = gc.isenabled()
                gc.disable()
                try:
                    self._prebuilt = [Portfolio._from_row(d, keys, W[i])
                                      for i, d in enumerate(st["rebdates"][lo:hi])]
                finally:
                    if gc_was:
                        gc.enable()
        for s in range(lo, hi, chunk):
            e = min(hi, s + chunk)
            if lad:
                r = opt.lad_batch(panel, rows[s:e], tlen[s:e], GhAb, lb, ub)
                if r is None:
                    ok = False
                    break
                W[s - lo:e - lo], ST[s - lo:e - lo], OBJ[s - lo:e - lo] = r
                continue
            stage = BatchStage(panel, rows[s:e], tlen[s:e], dev)
            if plan0 is not None and plan0[:2] == (s, e):
                stage._groups = plan0[2]
            # T + mg < n: the Woodbury (window-form) solver; its consumers read P's lower
            # triangle only (engine.lowrank_shape_ok: same test as solve_lowrank's)
            stage.prefer_lowrank = (bs.settings.get("lowrank", True)
                                    and engine.lowrank_shape_ok(n, int(stage.rows_host.shape[1]), mg))
            if seg_sd is not None:   # the segment split's window form: 3n variables, seg_mg rows
                stage.prefer_lowrank = (bs.settings.get("lowrank", True)
                                        and engine.lowrank_shape_ok(3 * n, int(stage.rows_host.shape[1]), seg_mg))
            obj = opt.objective_batch(stage)
            if obj is None:
                ok = False
                break
            Pm, scale, pdiag, q, _const = obj
            if stage.lowrank is not None:
                path = "lowrank"
            qb = engine.QPBatch.from_dense(None, None, n=n, A=GhAb["A"], b=GhAb["b"], G=GhAb["G"], h=GhAb["h"],
                                           lb=lb, ub=ub, device=dev)
            qb.batch = e - s
            qb.P = Pm
            qb.p_scale = scale
            qb.p_diag = pdiag
            qq = torch.zeros((e - s, qb.ld), dtype=torch.float64, device=dev)
            qq[:, :n] = q[:, :n]
            qb.q = qq
            seg_go = (seg_sd is not None and stage.lowrank is not None
                      and (pdiag is None or not bool((pdiag != 0).any())))
            if seg_go:   # turnover + leverage: the segment split (porqua_amd/l1seg.py) on the window path
                from . import l1seg
                from .l1split import split_settings
                if seg_panel is None:
                    seg_panel = engine.Panel(torch.cat([panel.R] * 3, 1).contiguous(), None, device=dev)
                qb3, lr3, const = l1seg.segment_batch(qb, stage.lowrank, seg_sd, seg_panel, GhAb["A"], GhAb["b"],
                                                      GhAb["G"], GhAb["h"])
                kind = "budget" if (seg_sd["to_budget"] is not None or np.isfinite(seg_sd["lev_budget"])) else "cost"
                res = engine.solve_lowrank(qb3, lr3, split_settings(settings, opt.params, kind),
                                           groups=stage.group_plan())
                path = "l1-segments"
                W[s - lo:e - lo] = l1seg.merge_batch(res.x, n, seg_sd["lb"]).cpu().numpy()
                OBJ[s - lo:e - lo] = (res.obj + const).cpu().numpy()
            elif l1both is not None:   # turnover + leverage: the per-asset-block IPM (porqua_amd/ipm_l1.py)
                from .ipm_l1 import l1_ipm_batched, window_rows as l1_rows
                UW, pdv = l1_rows(stage, scale, pdiag, Pm, n)
                res = l1_ipm_batched(UW, pdv, q[:, :n].contiguous(), l1both, A=GhAb["A"], b=GhAb["b"],
                                     G=GhAb["G"], h=GhAb["h"], lb=lb, ub=ub)
                del UW
                path = "l1-ipm"
                W[s - lo:e - lo] = res.x[:, :n].cpu().numpy()
                OBJ[s - lo:e - lo] = res.obj.cpu().numpy()
            elif l1term is not None:   # one turnover term: the signed split (porqua_amd/l1split.py)
                qb2, lr2, const = split_batch(qb, stage.lowrank, l1term, split_panel, GhAb["A"], GhAb["b"],
                                              GhAb["G"], GhAb["h"], lb, ub)
                s_split = split_settings(settings, opt.params, l1term.kind)
                if lr2 is not None:
                    res = engine.solve_lowrank(qb2, lr2, s_split, groups=stage.group_plan())
                else:
                    res = engine.solve(qb2, s_split)
                W[s - lo:e - lo] = merge_batch(res.x, l1term).cpu().numpy()
                OBJ[s - lo:e - lo] = (res.obj + const).cpu().numpy()
            else:
                if stage.lowrank is not None:
                    # the sync-free stages -- one ADMM launch, four polish rounds, one flag read
                    # (dates still pending after them, handed back or needing the wide rounds
                    # take the host-driven path); PQ_SF_CENTRED_ONLY=1: centred windows only
                    sf = stage.lowrank.mu is not None or os.environ.get("PQ_SF_CENTRED_ONLY", "0") != "1"
                    res = engine.solve_lowrank(qb, stage.lowrank, settings, groups=stage.group_plan(),
                                               sync_free=sf, sf_rounds=4 if sf else None,
                                               host_work=prebuild if (sf and s == lo and e == hi) else None)
                else:
                    res = engine.solve(qb, settings)
                if Wt is not None:
                    Wt[s - lo:e - lo].copy_(res.x[:, :n], non_blocking=True)   # ordered before the reads below
                else:
                    W[s - lo:e - lo] = res.x[:, :n].cpu().numpy()
                OBJ[s - lo:e - lo] = res.obj.cpu().numpy()
            ST[s - lo:e - lo] = res.status.cpu().numpy()
        return ok, W, ST, OBJ, path

    def _finish_batched(self, bs, st, W, ST, OBJ, path) -> None:
        """Phase C (host): Portfolio objects in date order, ``append_fun`` per date."""
        opt = bs.optimization
        rebdates, universe = st["rebdates"], st["universe"]
        n = W.shape[1]
        # ---- phase C: portfolios -----------------------------------------------------------
        from . import _lib
        solved = (ST == _lib.PQ_SOLVED) | (ST == _lib.PQ_SOLVED_INACCURATE)
        self.stats = {"dates": len(rebdates), "solved": int(solved.sum()), "status": ST, "objective": OBJ,
                      "path": path}
        if not bs.settings.get("quiet"):
            print(f"Rebalanced {len(rebdates)} dates on the device ({int(solved.sum())} solved)")
        keys = list(universe)
        none = [None] * n
        append_fun = bs.settings.get("append_fun")
        portfolios = self.strategy.portfolios
        # thousands of small objects: a cyclic-GC pass over the process's ~2e5 torch / pandas
        # objects can land in this loop (measured 5 -> 110 ms for 4544 dates); nothing here
        # creates reference cycles, so the collector is paused for it
        gc_was = gc.isenabled()
        gc.disable()
        pre = getattr(self, "_prebuilt", None)
        self._prebuilt = None
        if pre is not None and len(pre) != len(rebdates):
            pre = None
        try:
            for i, d in enumerate(rebdates):
                if pre is not None and append_fun is None and solved[i]:
                    portfolios.append(pre[i])   # built during the solve (_solve_shard)
                    continue
                if append_fun is None and solved[i]:
                    # the weights stay a row of W until read (Portfolio._from_row); the dict is
                    # == pd.Series(w, index=universe).to_dict() (Python floats)
                    portfolios.append(Portfolio._from_row(d, keys, W[i]))
                    continue
                w = W[i].tolist() if solved[i] else none
                opt.results = {"weights": dict(zip(keys, w)), "status": bool(solved[i])}
                self._after_solve(bs, d)
        finally:
            if gc_was:
                gc.enable()
        if rebdates:   # the optimisation's results hold the last date's, as after the serial loop
            last = len(rebdates) - 1
            w = W[last].tolist() if solved[last] else none
            opt.results = {"weights": dict(zip(keys, w)), "status": bool(solved[last])}

    def save(self, filename: str, path: Optional[str] = None) -> None:
        try:
            if path is not None and filename is not None:
                filename = os.path.join(path, filename)
            with open(filename, "wb") as f:
                pickle.dump(self, f, protocol=pickle.HIGHEST_PROTOCOL)
        except Exception as ex:
            print("Error during pickling object:", ex)


def _auto_chunk(n: int) -> int:
    """Dates per device batch: P + K^-1 (2 x 8 ld^2 B) per date within ~96 GiB."""
    ld = ((n + 63) // 64) * 64
    per = 2 * 8 * ld * ld + 64 * ld * 8
    return max(1, int((96 << 30) // per))


def agree_all(ok: bool, dist, device=None) -> bool:
    """True iff ``ok`` holds on every rank (one MIN all-reduce)."""
    import torch
    dev = comm_device(dist, device)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def comm_device(dist, device=None):
    """Device of the collective buffers: the rank's GPU under RCCL ('nccl'), the host under gloo."""
    import torch
    if dist.get_backend() == "nccl":
        return device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_blocks(block, total: int, world: int, dist, device=None) -> np.ndarray:
    """All-gather every rank's contiguous block of ``total`` rows (rank r holds rows
    shard_range(total, r, world); ``block`` is its (rows, m) numpy array or FP64 tensor) with
    one collective: RCCL ``all_gather_into_tensor`` over xGMI, gloo ``all_gather`` on CPU.
    Returns the whole (total, m) panel as numpy on every rank."""
    import torch
    per = -(-total // world)
    dev = comm_device(dist, device if device is not None else
                      (block.device if isinstance(block, torch.Tensor) and block.is_cuda else None))
    blk = block if isinstance(block, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(block))
    k, m = int(blk.shape[0]), int(blk.shape[1])
    buf = torch.zeros((per, m), dtype=torch.float64, device=dev)
    buf[:k] = blk.to(dev, torch.float64)
    if dist.get_backend() == "nccl":
        out = torch.zeros((world * per, m), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(out, buf)
    else:
        parts_t = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(parts_t, buf)
        out = torch.cat(parts_t)
    out = out.cpu().numpy()
    parts = []
    for r in range(world):
        s, e = shard_range(total, r, world)
        parts.append(out[r * per:r * per + (e - s)])
    return np.concatenate(parts)


def gather_shards(W, ST, OBJ, total, world, dist, device):
    """All-gather every rank's contiguous block of weights, status and objective (RCCL over
    xGMI on GPUs, gloo on CPU)."""
    n = W.shape[1]
    blk = np.concatenate([W, ST.astype(np.float64)[:, None], np.asarray(OBJ, dtype=np.float64)[:, None]], 1)
    full = gather_blocks(blk, total, world, dist, device if dist.get_backend() == "nccl" else None)
    return full[:, :n], full[:, n].astype(np.int32), full[:, n + 1]


def append_custom(backtest: Backtest, bs: BacktestService, rebalancing_date: Optional[str] = None,
                  what: Optional[list] = None) -> None:
    """src/backtest.py:245-270."""
    what = ["w_dict", "objective"] if what is None else what
    for key in what:
        if key == "w_dict":
            for k, weights in bs.optimization.results["w_dict"].items():
                if hasattr(weights, "to_dict"):
                    weights = weights.to_dict()
                backtest.append_output(date_key=rebalancing_date, output_key=f"weights_{k}",
                                       value=pd.Series(Portfolio(rebalancing_date, weights).weights))
        elif key in bs.optimization.results:
            backtest.append_output(date_key=rebalancing_date, output_key=key, value=bs.optimization.results[key])
