#!/usr/bin/env python3
"""Summarise tools/pmc_step.sh passes: per kernel family, per-launch HBM bytes (FETCH_SIZE x 2 +
WRITE_SIZE, MI355X_MICROARCH.md §HBM gfx950 correction) for the last train step, and write
profiles-ready JSON (hbm_bytes_per_launch) per family.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> [--json-dir profiles --tag r01 --dtype bf16]
"""
import collections
import csv
import glob
import json
import os
import sys

# bench.py PROF_KINDS names -> alternatives, each a list of kernel-name substrings that must all
# match (gemm_nt is the launcher's family: the tiled kernel and the streaming kernel it picks)
FAMILIES = {
    "conv0_fwd": [["conv0_fwd_kernel"]], "dw_fwd": [["dw_fwd_kernel<", "false>"], ["dw_fwd_loop_kernel<"]],
    "dw_dgrad": [["dw_dgrad_s2_kernel"]], "dw_wgrad": [["dw_wgrad_kernel"]],
    "gemm_nt": [["gemm_nt_kernel"], ["gemm_stream_kernel"]], "gemm_tn": [["gemm_tn_kernel"]],
    "ce_head": [["ce_head_kernel"], ["ce_head2_kernel"]], "conv0_wgrad": [["conv0_wgrad_kernel"], ["ltd_c0_bwd_kernel"]],
}


def load(pdir):
    files = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    return rows


def per_dispatch(rows):
    d = collections.OrderedDict()
    for r in rows:
        key = int(r["Dispatch_Id"])
        e = d.setdefault(key, {"name": r["Kernel_Name"], "c": {}})
        e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def last_step(disp):
    items = list(disp.values())
    idx = [i for i, e in enumerate(items) if "sgd_kernel" in e["name"]]
    if len(idx) >= 2:
        return items[idx[-2] + 1:idx[-1] + 1]
    return items


def main():
    root = sys.argv[1]
    args = sys.argv[2:]
    jdir = args[args.index("--json-dir") + 1] if "--json-dir" in args else None
    tag = args[args.index("--tag") + 1] if "--tag" in args else "r01"
    dtype = args[args.index("--dtype") + 1] if "--dtype" in args else "bf16"
    passes = sorted(glob.glob(os.path.join(root, "p*")))
    merged = None
    for p in passes:
        rows = load(p)
        if not rows:
            continue
        st = last_step(per_dispatch(rows))
        if merged is None:
            merged = [{"name": e["name"], "c": dict(e["c"])} for e in st]
        else:
            for m, e in zip(merged, st):
                if m["name"] == e["name"]:
                    m["c"].update(e["c"])
    if not merged:
        print("no counter data")
        return
    fam = collections.defaultdict(lambda: {"n": 0, "fetch": 0.0, "write": 0.0})
    print("%-58s %10s %10s %8s" % ("kernel (last step, dispatch order)", "read MB", "write MB", "busy%"))
    for e in merged:
        c = e["c"]
        rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024  # FETCH_SIZE in KB, x2 (gfx950)
        wr = c.get("WRITE_SIZE", 0.0) * 1024
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        act = c.get("SQ_ACTIVE_INST_ANY", 0.0)
        name = e["name"].replace("void fscnn::", "").replace("fscnn::", "")
        print("%-58s %10.2f %10.2f %8s" % (name[:58], rd / 1e6, wr / 1e6,
                                           "%.0f" % (100 * act / wc) if wc else "-"))
        for f, alts in FAMILIES.items():
            if any(all(k in e["name"] for k in keys) for keys in alts):
                fam[f]["n"] += 1
                fam[f]["fetch"] += rd
                fam[f]["write"] += wr
    print()
    for f, v in fam.items():
        per = (v["fetch"] + v["write"]) / max(1, v["n"])
        print("%-12s launches %3d  HBM bytes/launch %.3e (read %.3e, write %.3e)" % (
            f, v["n"], per, v["fetch"] / max(1, v["n"]), v["write"] / max(1, v["n"])))
        if jdir:
            with open(os.path.join(jdir, "pmc_%s_%s.json" % (f, dtype)), "w") as fh:
                json.dump({"kernel_family": f, "dtype": dtype, "round": tag,
                           "launches_per_step": v["n"], "hbm_bytes_per_launch": per,
                           "read_bytes_per_launch": v["fetch"] / max(1, v["n"]),
                           "write_bytes_per_launch": v["write"] / max(1, v["n"]),
                           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                                     "FETCH_SIZE x2 (gfx950 correction), last train step of "
                                     "bench.py --steps 2"}, fh, indent=1)


if __name__ == "__main__":
    main()
