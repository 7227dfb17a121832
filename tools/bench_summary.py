#!/usr/bin/env python3
"""One-line summary of a bench.py log (experiment tooling): label, QPs/s, ms per step, stage
ms, ADMM iterations, polish rounds, certificate.  Usage: bench_summary.py <label> <log>"""
import json
import sys


def main():
    label, path = sys.argv[1], sys.argv[2]
    line = [x for x in open(path) if x.startswith("{")][-1]
    d = json.loads(line)
    st = {k: round(v * 1e3, 3) for k, v in d["stages_s_per_step"].items()}
    so = d["solver"]
    c = so["certificate"]
    print(label, round(d["value"]), round(d["ms_per_step"], 3), st, round(so["mean_iters"], 2),
          round(so["polish_rounds_mean"], 3), c["status_counts"], "%.2e" % c["max_rel_stationarity"],
          "%.1e" % c["max_violation"], flush=True)


if __name__ == "__main__":
    main()
