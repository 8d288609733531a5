#!/usr/bin/env python3
"""Per-dispatch listing of ONE eval forward from a rocprofv3 kernel trace of tools/fwd_run.py
(forwards are delimited by bn_fold, the first launch of every eval forward).

    python tools/trace_fwd.py <run_kernel_trace.csv> [--which -2]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[sys.argv.index("--which") + 1]) if "--which" in sys.argv else -2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fwds, cur = [], []
    for r in rows:
        if "bn_fold" in r["Kernel_Name"] and cur:
            fwds.append(cur)
            cur = []
        cur.append(r)
    fwds.append(cur)
    sel = fwds[which]
    tot = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print("%8.1f us  grid %8s x %5s x %5s  wg %3s vgpr %3s  %s" % (
            d, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"],
            r["VGPR_Count"], r["Kernel_Name"].replace("void fscnn::", "").replace("fscnn::", "")[:64]))
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
    print("%d dispatches, kernel sum %.1f us, span %.1f us" % (len(sel), tot, span))


if __name__ == "__main__":
    main()
