#!/usr/bin/env python3
"""Summarise a round's rocprofv3 output (tools/profile_round.sh) into profiles/<round>_*.

HBM traffic per kernel follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB
from separate --pmc passes; on gfx950 FETCH_SIZE counts exactly half of a 16 B/lane
coalesced stream, so read bytes = 2 * FETCH_SIZE * 1024 (the ADMM K^-1 stream and the
factor kernel's tile staging are 16 B/lane loads); WRITE_SIZE is exact for 16 B stores.

Usage: python tools/pmc_summary.py r01
"""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(s):
    """Kernel name without template arguments (k_pg_solve<80> -> k_pg_solve)."""
    return s.split("<")[0].strip()


def per_kernel(path, counter, first=None):
    """Counter totals per kernel over every dispatch (and, in ``first``, the value of each
    kernel's first dispatch: the bench's timed step runs before its secondary lines)."""
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or 0))
    for r in rows:
        k = kname(r["Kernel_Name"])
        if first is not None and k not in first:
            first[k] = float(r["Counter_Value"])
        agg[k] += float(r["Counter_Value"])
        calls[k] += 1
    return agg, calls


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{rnd}_kernel_stats.csv"))
    f1, w1 = {}, {}
    fetch, calls = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE", f1)
    write, _ = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE", w1)
    line = [l for l in open(os.path.join(src, "pmc_fetch.log")) if l.startswith('{"metric"')][-1]
    bench_pmc = json.loads(line)
    iters = bench_pmc["roofline"]["admm_iterations_per_step"]
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        k = kname(r["Name"])   # template instances merged (calls summed, time-weighted mean)
        if k in stats:
            c0, c1 = int(stats[k]["Calls"]), int(r["Calls"])
            stats[k] = {"Calls": c0 + c1, "AverageNs": (float(stats[k]["AverageNs"]) * c0 +
                                                         float(r["AverageNs"]) * c1) / (c0 + c1)}
        else:
            stats[k] = r
    out = {"round": rnd, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of "
                                   "`bench.py --steps 1 --warmup 0` (one step = the whole backtest)",
           "admm_iterations_per_step": iters, "kernels": {}}
    for k in sorted(fetch, key=lambda k: -fetch[k]):
        rd = 2.0 * fetch[k] * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        e = {"calls_per_step": calls[k], "read_bytes_per_step": rd, "write_bytes_per_step": wr,
             "hbm_bytes_per_step": rd + wr}
        e["hbm_bytes_first_dispatch"] = 2.0 * f1[k] * 1024.0 + w1.get(k, 0.0) * 1024.0
        if k in stats:
            e["trace_avg_ns"] = float(stats[k]["AverageNs"])
            e["trace_calls"] = int(stats[k]["Calls"])
            # HBM bytes actually moved per launch (the step's first dispatch) over the trace's
            # average launch duration: the kernel's measured HBM rate (approximate for kernels
            # whose dispatches differ within a step, e.g. the polish rounds)
            e["measured_hbm_gbs"] = e["hbm_bytes_first_dispatch"] / e["trace_avg_ns"]
            e["measured_hbm_frac"] = e["measured_hbm_gbs"] / 8000.0
        out["kernels"][k] = e
    kern = bench_pmc["roofline"]["kernel"].split()[0]
    adm = out["kernels"].get(kern)
    if adm:
        # the timed step's own dispatch (later dispatches belong to the bench's end-to-end line)
        adm["hbm_bytes_first_dispatch"] = 2.0 * f1[kern] * 1024.0 + w1.get(kern, 0.0) * 1024.0
        adm["hbm_bytes_per_admm_iteration"] = adm["hbm_bytes_first_dispatch"] / iters
        adm["algorithmic_bytes_per_admm_iteration"] = float(bench_pmc["roofline"]["algorithmic_bytes_per_iteration"])
        if kern == "k_sw_pass":   # the sweep's ADMM: two launches per iteration, all of the step's
            mid = out["kernels"].get("k_sw_mid", {})
            adm["hbm_bytes_per_admm_iteration"] = (adm["hbm_bytes_per_step"] + mid.get("hbm_bytes_per_step", 0.0)) / iters
            adm["hbm_bytes_note"] = "k_sw_pass + k_sw_mid, every dispatch of the step / problem-iterations"
    out["admm_kernel"] = kern
    # optional MFMA pass (SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over every
    # SIMD; GRBM_GUI_ACTIVE counts the dispatch's cycles summed over the 8 XCDs): busy
    # fraction = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs) -- the fraction of the
    # chip's FP64-matrix issue capacity the kernel kept busy (1.0 = 78.6 TF/s of FP64 MFMA)
    mf = os.path.join(src, "pmc_mfma", "run_counter_collection.csv")
    if os.path.exists(mf):
        busy, _ = per_kernel(mf, "SQ_VALU_MFMA_BUSY_CYCLES")
        act, _ = per_kernel(mf, "GRBM_GUI_ACTIVE")
        out["mfma_busy_fraction"] = {k: busy[k] / (act[k] / 8.0 * 256 * 4) for k in busy if act.get(k)}
        out["mfma_source"] = "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE (own pass)"
    with open(os.path.join(dst, f"{rnd}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    full = os.path.join(src, "bench_full.log")
    if os.path.exists(full):
        shutil.copy(full, os.path.join(dst, f"{rnd}_bench.log"))
    print(json.dumps(out["kernels"].get(kern), indent=1))


if __name__ == "__main__":
    main()
