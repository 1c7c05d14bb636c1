"""Summarise a rocprofv3 kernel_stats.csv: name (shortened), calls, total ms, avg us."""
import csv
import sys

for path in sys.argv[1:]:
    print(path)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Name"].split("(")[0].replace("void ", "")
            print("  %-40s %6s %9.2f ms %9.1f us" % (name[:40], row["Calls"], int(row["TotalDurationNs"]) / 1e6,
                                                 float(row["AverageNs"]) / 1e3))
