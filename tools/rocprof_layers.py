#!/usr/bin/env python3
"""Per-layer KERNEL-time table: every executor launch labelled with its reference module
(models/fast_scnn.py), algorithmic bytes from SURVEY.md §8(d), and the kernel duration from a
rocprofv3 kernel trace of the same run (no HIP-event latency in the times).

Two steps, the first under rocprofv3 on the GPU box:

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \\
        python3 tools/rocprof_layers.py record OUT/scopes.json [--eval-only]
    python3 tools/rocprof_layers.py table OUT/.../run_kernel_trace.csv OUT/scopes.json table.md

`record` runs (weight-gradient side stream off, so every launch of a phase is on one stream in
issue order) a few warm-up cfg3 bf16 train steps, then ONE profiled train step and ONE profiled
cfg2 fp32 eval forward with the library's launch profiler in "every launch" mode: it lists the
launch scopes (layer tag, kernel family, algorithmic bytes and flops) in issue order.  A
synchronised marker kernel (a 1-element torch bitwise_not, which no step launches) brackets each
phase.
`table` walks the trace's dispatches between the markers in order and gives each scope the next
dispatch whose kernel name belongs to the scope's family (unscoped launches -- weight prep, slab
reductions, SGD -- are skipped), then prints the per-launch and per-family tables.
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM = 8000.0  # GB/s (MI355X_MICROARCH.md)

# launch-profiler family -> kernel names it covers (csrc/*.hip)
FAMILY_RE = {
    "conv0_fwd": r"conv0_fwd_kernel",
    "dw_fwd": r"dw_fwd(_dma)?_kernel<[^,]+, \d, false",
    "dw_dgrad": r"dw_fwd(_dma)?_kernel<[^,]+, \d, true|dw_dgrad_s2_kernel",
    "dw_wgrad": r"dw_wgrad_kernel",
    "gemm_nt": r"gemm_nt_kernel|gemm_stream(_x3)?_kernel",
    "gemm_tn": r"gemm_tn_kernel",
    "bn_apply": r"bn_apply_kernel",
    "bn_bwd": r"bn_bwd_apply_kernel",
    "upsample_bwd": r"axis_bwd_kernel|up_nhwc_bwd_kernel",
    "upsample": r"up_nchw|up_nhwc|up_argmax",
    "cross_entropy": r"ce_head2?_kernel|ce_fwd_kernel|ce_pack_targets",
    "conv0_wgrad": r"conv0_wgrad_kernel|ltd_c0_bwd_kernel",
    "bn_bwd_reduce": r"bn_bwd_reduce_kernel",
    "bn_finalize": r"bn_(stats_fold_fin|stats_fold|finalize|bwd_fold_fin|bwd_fold|bwd_finalize)_kernel",
    "ppm_branches": r"ppm_(fwd|fwd_mma|eval_mma|bwd)_kernel",
    "ir_block": r"ir_block_kernel|ir_train_fwd_kernel",
    "ltd_stem": r"stem_walk_kernel",
    "dsconv": r"dsconv_fwd_kernel|ds2_fwd_kernel",
}
MARK = re.compile(r"bitwise_not")  # torch's bitwise_not kernel (the phase marker: no step uses it)


def record(out, eval_only=False):
    import ctypes
    import numpy as np
    import torch
    os.environ["FSCNN_SIDE_STREAM"] = "0"
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import _lib, arch, portable_init
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN
    lib = _lib.load()
    dev = torch.device("cuda", 0)

    def scopes(fn):
        _lib.check(lib.fscnn_prof_begin(100, 4096), "fscnn_prof_begin")
        fn()
        torch.cuda.synchronize()
        ms, n, b, f = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
        _lib.check(lib.fscnn_prof_end(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b),
                                      ctypes.byref(f)), "fscnn_prof_end")
        res = []
        for i in range(n.value):
            k, t, by, fl, tag = (ctypes.c_int(), ctypes.c_float(), ctypes.c_double(),
                                 ctypes.c_double(), ctypes.c_char_p())
            _lib.check(lib.fscnn_prof_launch(i, ctypes.byref(k), ctypes.byref(t), ctypes.byref(by),
                                             ctypes.byref(fl), ctypes.byref(tag)), "prof_launch")
            res.append({"tag": tag.value.decode(), "family": lib.fscnn_prof_kind_name(k.value).decode(),
                        "bytes": by.value, "flops": fl.value, "event_us": t.value * 1e3})
        return res

    marker = torch.zeros(1, dtype=torch.int32, device=dev)

    def mark():
        torch.cuda.synchronize()
        marker.bitwise_not_()
        torch.cuda.synchronize()

    m = FastSCNN(19)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(19, seed=0).items()})
    m = m.to(dev)
    x = torch.from_numpy(portable_init.input_tensor(1, (8, 3, 1024, 2048))).to(dev)
    phases = []
    if not eval_only:
        m.train()
        xb = x.to(torch.bfloat16)
        t = torch.from_numpy(portable_init.target_tensor(3, (8, 1024, 2048), 19, 0.05)).to(dev)
        opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)

        def step():
            opt.zero_grad(set_to_none=True)
            m.forward_loss(xb, t).backward()
            opt.step()
        for _ in range(3):
            step()
        mark()
        phases.append({"name": "cfg3 train step (bf16, 8 x 3 x 1024 x 2048, fused CE head, "
                               "FusedSGD; weight-gradient side stream off)", "scopes": scopes(step)})
        mark()
    m.eval()
    with torch.no_grad():
        for _ in range(2):
            m(x)
        mark()
        phases.append({"name": "cfg2 eval forward (fp32, 8 x 3 x 1024 x 2048)",
                       "scopes": scopes(lambda: m(x))})
        mark()
    json.dump({"phases": phases}, open(out, "w"))
    print("recorded", [(p["name"][:30], len(p["scopes"])) for p in phases])


def table(trace, scopes_json, out):
    import csv
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    marks = [i for i, n in enumerate(names) if MARK.search(n) and "fscnn" not in n]
    phases = json.load(open(scopes_json))["phases"]
    # every phase is bracketed by its own pair of markers (warm-up runs lie between the pairs)
    spans = [(marks[2 * i] + 1, marks[2 * i + 1]) for i in range(len(marks) // 2)]
    lines = ["# Per-layer kernel time (MI355X, one GPU, rocprofv3 kernel trace)", "",
             "Generated by `tools/rocprof_layers.py`: launch order and algorithmic bytes from the "
             "library's launch profiler, durations from `rocprofv3 --kernel-trace` of the same run "
             "(kernel time only: no HIP-event latency, no launch gaps).  Weight-gradient side "
             "stream off, so no two kernels overlap.", ""]
    for ph, (a, b) in zip(phases, spans):
        lines += ["## " + ph["name"], "",
                  "| # | layer | kernel family | kernel | us | MB | GB/s | HBM frac |",
                  "|---|---|---|---|---:|---:|---:|---:|"]
        fam = {}
        j = a
        tot_us = tot_b = 0.0
        unmatched = 0
        for i, sc in enumerate(ph["scopes"]):
            rx = re.compile(FAMILY_RE.get(sc["family"], "^$"))
            k = j
            while k < b and not rx.search(names[k]):
                k += 1
            if k >= b:
                unmatched += 1
                continue
            j = k + 1
            us = dur[k]
            gbs = sc["bytes"] / (us * 1e-6) / 1e9 if us > 0 else 0.0
            short = re.sub(r"^void |fscnn::|\(.*$", "", names[k])[:48]
            lines.append("| %d | %s | %s | `%s` | %.1f | %.1f | %.0f | %.2f |" % (
                i, sc["tag"], sc["family"], short, us, sc["bytes"] / 1e6, gbs, gbs / HBM))
            f = fam.setdefault(sc["family"], [0, 0.0, 0.0])
            f[0] += 1
            f[1] += us
            f[2] += sc["bytes"]
            tot_us += us
            tot_b += sc["bytes"]
        lines += ["", "Total over %d matched launches: %.3f ms kernel time, %.1f MB algorithmic, "
                  "%.0f GB/s aggregate (%.2f of HBM peak)%s." % (
                      len(ph["scopes"]) - unmatched, tot_us / 1e3, tot_b / 1e6,
                      tot_b / (tot_us * 1e-6) / 1e9 if tot_us else 0,
                      tot_b / (tot_us * 1e-6) / 1e9 / HBM if tot_us else 0,
                      ("; %d scopes without a matching dispatch" % unmatched) if unmatched else ""),
                  "", "| kernel family | launches | ms | GB/s | HBM frac |",
                  "|---|---:|---:|---:|---:|"]
        for k, (n, us, by) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
            g = by / (us * 1e-6) / 1e9 if us else 0
            lines.append("| %s | %d | %.3f | %.0f | %.2f |" % (k, n, us / 1e3, g, g / HBM))
        lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "record":
        record(sys.argv[2], eval_only="--eval-only" in sys.argv)
    else:
        table(sys.argv[2], sys.argv[3], sys.argv[4])
