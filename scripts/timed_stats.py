#!/usr/bin/env python3
"""Kernel statistics of bench.py's TIMED K1 launches only, from a rocprofv3
--kernel-trace CSV of `bench.py --steps K --warmup W`: bench.py launches the
headline kernel W times (warm-up), then K times inside the timed region,
before any other use of that kernel instantiation, so the timed launches are
dispatches [W, W + K) of the first fm_rows kernel in the trace.  Writes a
CSV row per kernel in the same columns rocprofv3's --stats summary uses.
usage: timed_stats.py <kernel_trace.csv> <warmup> <steps> [out.csv]"""
import csv
import sys


def main():
    trace, W, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    k1 = [r for r in rows if "fm_rows" in r["Kernel_Name"]]
    name = k1[0]["Kernel_Name"]
    same = [r for r in k1 if r["Kernel_Name"] == name]
    timed = same[W:W + K]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    allr = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in same]
    res = [("timed", name, len(d), sum(d), sum(d) / len(d), min(d), max(d)),
           ("all_dispatches", name, len(allr), sum(allr), sum(allr) / len(allr), min(allr),
            max(allr))]
    hdr = ["Selection", "Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"]
    w = csv.writer(open(out, "w") if out else sys.stdout)
    w.writerow(hdr)
    for r in res:
        w.writerow(r)


if __name__ == "__main__":
    main()
