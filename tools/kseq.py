#!/usr/bin/env python3
"""Per-dispatch kernel timeline of one bench step from a rocprofv3 kernel trace:
python tools/kseq.py <run_kernel_trace.csv> [step index, default 1] [name prefix filter]
[step's first kernel, default k_window_moments_grp; k_window_mean:2 for the risk-aversion sweep,
whose steps launch it twice]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    pref = sys.argv[3] if len(sys.argv) > 3 else "k_"
    first = sys.argv[4] if len(sys.argv) > 4 else "k_window_moments_grp"
    first, _, per = first.partition(":")
    per = int(per or 1)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = []
    for r in rows:
        k = r["Kernel_Name"]
        for pre in ("void pq::", "pq::(anonymous namespace)::", "pq::", ""):   # (-T: truncated names)
            if k.startswith(pre):
                k = k[len(pre):].split("(")[0]
                seq.append((k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                            int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
                break
    starts = [i for i, (k, *_) in enumerate(seq) if k.startswith(first)][::per]
    i0 = starts[step]
    i1 = starts[step + 1] if len(starts) > step + 1 else len(seq)
    tot = collections.defaultdict(float)
    t00 = seq[i0][2]
    for k, d, t0, t1 in seq[i0:i1]:   # start offset from the step's first kernel, duration
        if k.startswith(pref):
            print(f"{k:40s} @{(t0 - t00) / 1e3:9.1f} {d:9.1f} us")
        tot[k.split("<")[0]] += d
    print(f"step span {(seq[i1 - 1][3] - t00) / 1e3:.1f} us")
    print("--- totals per kernel (us)")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{k:40s} {v:9.1f}")


if __name__ == "__main__":
    main()
