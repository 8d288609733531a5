#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 kernel_stats.csv of N train steps.
    python tools/prof_table.py <kernel_stats.csv> <steps> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
out, tot, calls = [], 0.0, 0.0
for r in rows:
    ms = float(r["TotalDurationNs"]) / 1e6 / steps
    c = int(r["Calls"]) / steps
    tot += ms
    calls += c
    out.append((ms, c, float(r["AverageNs"]) / 1e3, r["Name"][:100]))
out.sort(reverse=True)
for o in out[:top]:
    print("%7.3f ms %6.1f calls %8.1f us  %s" % o)
print("total %.3f ms/step, %.0f dispatches/step" % (tot, calls))
