#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 kernel trace for ONE training step.

    python tools/trace_layers.py <run_kernel_trace.csv> [filter-substring] [--step K]

Prints, in dispatch order, the kernels of the K-th step (steps are delimited by the sgd kernel),
with duration, grid and VGPRs, so per-layer costs can be read against SURVEY Appendix C.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    step = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 3
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_kernel" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    sel = steps[min(step, len(steps) - 1)]
    tot = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        name = r["Kernel_Name"]
        if filt and filt not in name:
            continue
        short = name.replace("void fscnn::", "").replace("fscnn::", "")[:60]
        print("%8.1f us  grid %7s x %5s x %5s  wg %3sx%-3s vgpr %3s agpr %3s  %s" % (
            d, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"],
            r["Workgroup_Size_Y"], r["VGPR_Count"], r["Accum_VGPR_Count"], short))
    first = int(sel[0]["Start_Timestamp"])
    last = int(sel[-1]["End_Timestamp"])
    print("step %d: %d dispatches, kernel sum %.1f us, span %.1f us" % (
        step, len(sel), tot, (last - first) / 1e3))


if __name__ == "__main__":
    main()
