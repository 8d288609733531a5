"""Per-kernel-family time per train step, two rocprofv3 kernel traces side by side.

    python tools/prof_diff.py A/run_kernel_trace.csv B/run_kernel_trace.csv
"""
import collections
import csv
import sys


def load(p):
    rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    use = steps[2:6]
    agg = collections.defaultdict(lambda: [0.0, 0.0])
    for st in use:
        for r in st:
            n = r["Kernel_Name"].replace("fscnn::", "").replace("void ", "").split("(")[0]
            agg[n][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / len(use)
            agg[n][1] += 1 / len(use)
    return agg


a, b = load(sys.argv[1]), load(sys.argv[2])
keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, [0])[0] - a.get(k, [0])[0]))
print("%-70s %9s %5s %9s %5s %8s" % ("kernel", "A us", "n", "B us", "n", "B-A"))
for k in keys[:40]:
    x, y = a.get(k, [0, 0]), b.get(k, [0, 0])
    print("%-70s %9.1f %5.1f %9.1f %5.1f %8.1f" % (k[:70], x[0], x[1], y[0], y[1], y[0] - x[0]))
print("total kernel us: A %.1f (%d launches)  B %.1f (%d launches)" % (
    sum(v[0] for v in a.values()), round(sum(v[1] for v in a.values())),
    sum(v[0] for v in b.values()), round(sum(v[1] for v in b.values()))))
