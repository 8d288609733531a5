#!/usr/bin/env python3
"""Per-dispatch PMC table of the LAST forward (delimited by bn_fold) or train step (sgd) in the
passes written by tools/pmc_run.sh.  HBM bytes = FETCH_SIZE x 2 (gfx950 correction for 16-B
streaming reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE.

    python tools/pmc_table.py gpurun_out/pmc_<tag> [--delim bn_fold|sgd_kernel]
"""
import collections
import csv
import glob
import os
import sys


def dispatches(pdir):
    d = collections.OrderedDict()
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            e = d.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def last_block(items, delim):
    idx = [i for i, e in enumerate(items) if delim in e["name"]]
    if not idx:
        return items
    if delim == "sgd_kernel":
        return items[idx[-2] + 1:idx[-1] + 1] if len(idx) >= 2 else items
    return items[idx[-1]:]


def main():
    root = sys.argv[1]
    delim = sys.argv[sys.argv.index("--delim") + 1] if "--delim" in sys.argv else "bn_fold"
    merged = None
    for p in sorted(glob.glob(os.path.join(root, "p*/"))):
        blk = last_block(dispatches(p), delim)
        if merged is None:
            merged = [{"name": e["name"], "c": dict(e["c"])} for e in blk]
        else:
            for m, e in zip(merged, blk):
                if m["name"] == e["name"]:
                    m["c"].update(e["c"])
    print("%-50s %9s %9s %6s %6s %6s %6s %8s" % ("kernel", "rd MB", "wr MB", "act%", "wait%",
                                                "istl%", "ldsbc", "valu/wv"))
    for e in merged or []:
        c = e["c"]
        rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024 / 1e6
        wr = c.get("WRITE_SIZE", 0.0) * 1024 / 1e6
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        nw = c.get("SQ_WAVES", 0.0) or 1.0
        name = e["name"].replace("void fscnn::", "").replace("fscnn::", "")
        print("%-50s %9.2f %9.2f %6.0f %6.0f %6.0f %6.0f %8.0f" % (
            name[:50], rd, wr, 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            100 * c.get("SQ_WAIT_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc,
            c.get("SQ_LDS_BANK_CONFLICT", 0) / 1e3, c.get("SQ_INSTS_VALU", 0) / nw))


if __name__ == "__main__":
    main()
