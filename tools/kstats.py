"""Per-kernel summary of a rocprofv3 kernel_stats.csv (name, calls, avg us, total ms), sorted by total."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    print("%-100s %5s %8.1f %8.2f" % (r['Name'][:100], r['Calls'], float(r['AverageNs']) / 1000,
                                      float(r['TotalDurationNs']) / 1e6))
