#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, total ms."""
import csv
import sys
for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("mipx::", "").replace("(anonymous namespace)::", "")[:64]
        print(f"{n:64s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f}us {float(r['TotalDurationNs'])/1e6:8.2f}ms")
