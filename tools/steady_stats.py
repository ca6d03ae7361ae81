"""Steady-state kernel averages from a rocprofv3 kernel trace.

rocprofv3's --stats average counts every dispatch, including the warmup
launches that run while the GPU clock is still ramping.  bench.py times only
the last --steps launches; this prints, per kernel, the average over all
dispatches and over the last K (the timed region), so a profile can be set
against the bench line it came from.

usage: python tools/steady_stats.py <kernel_trace.csv> [K=20] [name-substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    pat = sys.argv[3] if len(sys.argv) > 3 else ""
    durs = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Name")
        if pat and pat not in name:
            continue
        durs[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for name, d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        last = d[-k:]
        print("%-60s calls %4d  avg_all %10.1f us  avg_last%-3d %10.1f us  min %10.1f us  max %10.1f us" % (
            name[:60], len(d), sum(d) / len(d) / 1e3, len(last), sum(last) / len(last) / 1e3,
            min(d) / 1e3, max(d) / 1e3))


if __name__ == "__main__":
    main()
