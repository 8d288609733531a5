#!/usr/bin/env python3
"""Per-family kernel time from a rocprofv3 --kernel-trace --stats summary of the bench train step.

    python tools/rocprof_family.py <kernel_stats.csv> <round> [out.json]

Groups kernels into the launch profiler's families (bench.py PROF_KINDS; one launch of a family =
one kernel of these names), counts steps by the fused loss head (one launch per step) and writes
{"families": {family: {"launches_per_step", "avg_us", "ms_per_step"}}, "steps", "round"} —
the kernel-only durations bench.py reports beside its event-timed roofline.
"""
import csv
import json
import re
import sys

FAMILIES = [
    ("gemm_nt", ("gemm_stream_kernel", "gemm_stream_x3_kernel", "gemm_nt_kernel")),
    ("gemm_tn", ("gemm_tn_kernel",)),
    ("dw_fwd", ("dw_fwd_kernel", "dw_fwd_loop_kernel")),
    ("dw_dgrad", ("dw_dgrad_kernel", "dw_dgrad_s2_kernel")),
    ("dw_wgrad", ("dw_wgrad_kernel",)),
    ("bn_bwd_apply", ("bn_bwd_apply_kernel",)),
    ("bn_apply", ("bn_apply_kernel",)),
    ("ce_head", ("ce_head_kernel", "ce_head2_kernel")),
    ("conv0_fwd", ("conv0_fwd_kernel",)),
    ("conv0_wgrad", ("ltd_c0_bwd_kernel", "conv0_wgrad_kernel")),
    ("lowres_block", ("lowres_",)),
]


def family(name):
    short = name.split("<")[0].split("(")[0].replace("void ", "").replace("fscnn::", "")
    if short == "dw_fwd_kernel":
        # dw_fwd_kernel<T, S, FLIP, ...>: FLIP = the stride-1 input gradient (dw_dgrad family)
        m = re.search(r"dw_fwd_kernel<[^,]+, ?\d, ?(true|false)", name)
        return "dw_dgrad" if m and m.group(1) == "true" else "dw_fwd"
    for fam, keys in FAMILIES:
        if any(short.startswith(k) for k in keys):
            return fam
    return None


def main():
    path, rnd = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    steps = sum(int(r["Calls"]) for r in rows if family(r["Name"]) == "ce_head") or 1
    acc = {}
    for r in rows:
        f = family(r["Name"])
        if f is None:
            continue
        a = acc.setdefault(f, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"])
    fams = {f: {"launches_per_step": round(n / steps, 2), "avg_us": round(t / n / 1e3, 2),
                "ms_per_step": round(t / steps / 1e6, 4)} for f, (n, t) in acc.items()}
    out = {"round": rnd, "source": path, "steps": steps, "families": fams}
    js = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
