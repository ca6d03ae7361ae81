"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, average and total time."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        print("  %-64s %6s calls  avg %10.1f us  total %9.2f ms  %5.1f%%" % (
            r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6,
            float(r["Percentage"])))
