#!/usr/bin/env python3
"""Where a low-resolution pointwise GEMM launch spends its time: per-wave wall-clock stamps
(common.hpp stamp(), 100 MHz) of the tiled / streaming gemm_nt kernels at the cfg3 bottleneck2/3
shapes (M = 8 x 32 x 64 = 16384 pixels), one launch each after warm-up.

Stamp slots: 0 kernel entry, 1 after the prologue (first K chunk staged / weights in LDS),
2 after the K loop (tiled) / chunk loop (streaming), 3 after the stores (tiled) / BN record
(streaming), 4 before the in-kernel BN finish (tiled) / after it (streaming), 5 after the finish
(tiled).  Printed per launch: the kernel span (first entry -> last stamp), the spread of wave
entry times (dispatch ramp) and the median / max of every phase.

    python tools/stamp_probe.py           # isolated launches at the low-res shapes
    python tools/stamp_probe.py step      # every instrumented launch of one cfg3 train step
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _fscnn_boot  # noqa: E402

_fscnn_boot.load()
from fast_scnn_pytorch_amd import _lib  # noqa: E402

SLOTS = 8
STRIDE = 8192 * 4 * SLOTS
DEV = "cuda"


def analyse(label, st, base=None):
    t = st.view(-1, SLOTS).cpu().double()
    if t.numel() == 0:
        print("%-40s no stamps" % label)
        return
    t = t[t[:, 0] > 0]
    if t.numel() == 0:
        print("%-40s no stamps" % label)
        return
    place = t[:, 7].long()
    t = t[:, :7]
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0  # us
    rel[t == 0] = float("nan")
    last = torch.nan_to_num(rel, nan=-1.0).max(dim=1).values
    span = last.max().item()
    entry = rel[:, 0]
    parts = []
    for a, b in [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (1, 5), (5, 6)]:
        d = rel[:, b] - rel[:, a]
        d = d[~torch.isnan(d)]
        if d.numel():
            parts.append("%d-%d %.1f/%.1f" % (a, b, d.median().item(), d.max().item()))
    at = "" if base is None else "@%7.1f " % ((t0.item() - base) / 100.0)
    print("%-40s %swaves %5d span %6.1f us  entry med %.1f max %.1f | %s"
          % (label, at, t.shape[0], span, entry.median().item(), entry.max().item(),
             "  ".join(parts)), flush=True)
    if os.environ.get("STAMP_PLACE") and t.shape[0] <= 8192:
        # phase 1-2 (the main loop) and the wave's end (last stamp) by placement
        loop = rel[:, 2] - rel[:, 1]
        end = torch.nan_to_num(rel, nan=-1.0).max(dim=1).values
        xcc = (place >> 32) & 15
        hw = place & 0xFFFFFFFF
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 7
        def by(name, key, n):
            row = []
            for k in range(n):
                sel = (key == k) & ~torch.isnan(loop)
                if sel.any():
                    row.append("%d:%.1f/%.1f" % (k, loop[sel].median().item(), end[sel].median().item()))
            print("    %-5s loop/end med: %s" % (name, " ".join(row)))
        by("xcc", xcc, 8)
        by("simd", simd, 4)
        by("se", se, 8)
        by("wave", torch.arange(t.shape[0]) % 4, 4)
        slow = torch.argsort(torch.nan_to_num(loop, nan=0.0), descending=True)[:6]
        print("    slowest waves (block, wave, xcc, se, cu, simd, loop us, entry us):",
              [(int(i) // 4, int(i) % 4, int(xcc[i]), int(se[i]), int(cu[i]), int(simd[i]),
                round(loop[i].item(), 1), round(entry[i].item(), 1)) for i in slow])


def main():
    lib = _lib.load()
    st = _lib.stream_ptr()
    buf = torch.zeros(8192 * 4 * SLOTS, dtype=torch.int64, device=DEV)
    dt = torch.bfloat16
    M = 16384
    shapes = [  # (label, K, N, kind): fwd = statistics form, dgrad = BN-backward form + finish
        ("b2.x expand fwd", 96, 576, "fwd"), ("b3.x expand fwd", 128, 768, "fwd"),
        ("b2.x project fwd", 576, 96, "fwd"), ("b3.x project fwd", 768, 128, "fwd"),
        ("b2.x project dgrad", 96, 576, "dgrad"), ("b3.x project dgrad", 128, 768, "dgrad"),
        ("b2.x expand dgrad", 576, 96, "dgrad"), ("b3.x expand dgrad", 768, 128, "dgrad"),
    ]
    for label, K, N, kind in shapes:
        A = torch.randn(M, K, device=DEV).to(dt)
        B = (torch.randn(N, K, device=DEV) / K ** 0.5).to(dt)
        C = torch.empty(M, N, dtype=dt, device=DEV)
        part = torch.empty((M + 127) // 128 * 3 * N, device=DEV)
        if kind == "fwd":
            def run():
                _lib.call("fscnn_pw_gemm", M, N, K, _lib.ptr(A), K, _lib.ptr(B), K, 0, None, None,
                          None, 0, 0, _lib.ptr(C), N, _lib.ptr(part), _lib.dtype_code(dt), st)
        else:
            z = torch.randn(M, N, device=DEV).to(dt)
            mean, invstd = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
            sc, sh = torch.ones(N, device=DEV), torch.zeros(N, device=DEV)
            ctr = torch.zeros(512, dtype=torch.int32, device=DEV)
            tsum = torch.zeros(32 * 3 * 1024, dtype=torch.float64, device=DEV)
            dg, db, coef = (torch.empty(N, device=DEV), torch.empty(N, device=DEV),
                            torch.empty(2 * N, device=DEV))

            def run():
                _lib.call("fscnn_pw_dgrad_bnbwd", M, N, K, _lib.ptr(A), K, _lib.ptr(B), K, None,
                          N, _lib.ptr(C), N, _lib.ptr(z), N, _lib.ptr(mean), _lib.ptr(invstd),
                          _lib.ptr(sc), _lib.ptr(sh), 2, _lib.ptr(part), _lib.ptr(ctr),
                          _lib.ptr(tsum), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(coef),
                          _lib.dtype_code(dt), None, st)
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.fscnn_debug_stamps(_lib.ptr(buf), 1))
        run()
        torch.cuda.synchronize()
        _lib.check(lib.fscnn_debug_stamps(None, 0))
        analyse("%s K%d N%d (%.1f us/launch)" % (label, K, N, us), buf[:STRIDE])


def step():
    """One cfg3 train step (bench.py's workload) with every instrumented launch stamped."""
    import numpy as np
    from fast_scnn_pytorch_amd import arch, portable_init
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN
    lib = _lib.load()
    m = FastSCNN(19)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(19, seed=0).items()})
    m = m.to(DEV).train()
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x = torch.from_numpy(portable_init.input_tensor(1, (8, 3, 1024, 2048))).to(DEV).to(torch.bfloat16)
    t = torch.from_numpy(portable_init.target_tensor(3, (8, 1024, 2048), 19, 0.05)).to(DEV)

    def one():
        opt.zero_grad(set_to_none=True)
        m.forward_loss(x, t).backward()
        opt.step()
    for _ in range(4):
        one()
    nmax = 160
    buf = torch.zeros(nmax * STRIDE, dtype=torch.int64, device=DEV)
    torch.cuda.synchronize()
    _lib.check(lib.fscnn_debug_stamps(_lib.ptr(buf), nmax))
    one()
    torch.cuda.synchronize()
    n = lib.fscnn_debug_stamp_count()
    tags = [lib.fscnn_debug_stamp_tag(i).decode() for i in range(n)]
    _lib.check(lib.fscnn_debug_stamps(None, 0))
    firsts = []
    for i in range(n):
        v = buf[i * STRIDE:i * STRIDE + 8192 * 4 * SLOTS].view(-1, SLOTS)[:, 0]
        v = v[v > 0]
        if v.numel():
            firsts.append(int(v.min().item()))
    base = float(min(firsts)) if firsts else None
    for i in range(n):
        analyse("%3d %s" % (i, tags[i][:36]), buf[i * STRIDE:(i + 1) * STRIDE], base)


def eval_fwd():
    """One cfg2 fp32 eval forward (bench.py's forward_fp32) with every instrumented launch stamped."""
    import numpy as np
    from fast_scnn_pytorch_amd import arch, portable_init
    from models.fast_scnn import FastSCNN
    lib = _lib.load()
    m = FastSCNN(19)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(19, seed=0).items()})
    m = m.to(DEV).eval()
    x = torch.from_numpy(portable_init.input_tensor(1, (8, 3, 1024, 2048))).to(DEV)
    with torch.no_grad():
        for _ in range(3):
            m(x)
        nmax = 40
        buf = torch.zeros(nmax * STRIDE, dtype=torch.int64, device=DEV)
        torch.cuda.synchronize()
        _lib.check(lib.fscnn_debug_stamps(_lib.ptr(buf), nmax))
        m(x)
        torch.cuda.synchronize()
    n = lib.fscnn_debug_stamp_count()
    tags = [lib.fscnn_debug_stamp_tag(i).decode() for i in range(n)]
    _lib.check(lib.fscnn_debug_stamps(None, 0))
    for i in range(n):
        analyse("%3d %s" % (i, tags[i][:36]), buf[i * STRIDE:(i + 1) * STRIDE])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "step":
        step()
    elif len(sys.argv) > 1 and sys.argv[1] == "eval":
        eval_fwd()
    else:
        main()
