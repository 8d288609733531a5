"""One train step from a rocprofv3 kernel trace, in issue order: kernel, grid, duration, gap.

    python tools/trace_step.py gpurun_out/prof_<tag>/run_kernel_trace.csv [--step K]

Steps are delimited by the SGD launch (sgd_kernel), the last launch of every train step.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    st = steps[k]
    t0 = int(st[0]["Start_Timestamp"])
    prev_end = t0
    tot = 0
    for r in st:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("fscnn::", "").replace("void ", "")
        name = name[:90]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        print("%8.1f %7.1f %6.1f q%s %6d %-90s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3,
                                               r["Queue_Id"], grid // wg, name))
        prev_end = max(prev_end, e)
        tot += e - s
    print("step span %.1f us, kernel sum %.1f us, %d launches, %d steps in trace" % (
        (prev_end - t0) / 1e3, tot / 1e3, len(st), len(steps)))


if __name__ == "__main__":
    main()
