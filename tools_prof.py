"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print("%6.2f%% %9.1f us avg %6d calls  %s" % (100 * float(r["TotalDurationNs"]) / tot, float(r["AverageNs"]) / 1e3,
                                                 int(r["Calls"]), r["Name"][:100]))
print("total ms %.2f" % (tot / 1e6))
