#!/usr/bin/env python3
"""Diagnose predict() vs argmax(model(x)[0]) at cfg2: determinism of the logits across forwards,
label mismatches and the logit margin at each mismatch.

    python tools/diag_predict.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from helpers import golden_input, golden_sd, load_golden
    from models.fast_scnn import FastSCNN
    g = load_golden("cfg2_c19_1024x2048")
    m = FastSCNN(19)
    m.load_state_dict(golden_sd(g))
    m = m.cuda().eval()
    x = golden_input(g).cuda()
    with torch.no_grad():
        o1 = m(x)[0].clone()
        o2 = m(x)[0].clone()
        l1 = m.predict(x, dtype=torch.uint8)
        l2 = m.predict(x, dtype=torch.uint8)
        o3 = m(x)[0].clone()
    torch.cuda.synchronize()
    print("logits run-to-run bit-equal:", torch.equal(o1, o2), torch.equal(o1, o3),
          "max|d|", (o1 - o2).abs().max().item(), (o1 - o3).abs().max().item())
    print("predict run-to-run equal:", torch.equal(l1, l2))
    am = o1.argmax(1).to(torch.uint8)
    bad = (am != l1)
    print("predict vs argmax mismatches:", int(bad.sum()))
    if bad.any():
        idx = bad.nonzero()[:10]
        for n, h, w in idx.tolist():
            v = o1[n, :, h, w]
            top = v.topk(2)
            print("  px", (n, h, w), "argmax", int(am[n, h, w]), "predict", int(l1[n, h, w]),
                  "top2", top.values.tolist(), top.indices.tolist(),
                  "v[pred]", v[int(l1[n, h, w])].item())


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def lowres_check():
    """Which kernel departs: emulate the bilinear tap arithmetic (lerp2, fp32) on the CPU from the
    stored low-res logits at the mismatching pixels, and re-run predict over a garbage-filled
    allocator block (uninitialised-read check)."""
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from helpers import golden_input, golden_sd, load_golden
    from models.fast_scnn import FastSCNN
    g = load_golden("cfg2_c19_1024x2048")
    m = FastSCNN(19)
    m.load_state_dict(golden_sd(g))
    m = m.cuda().eval()
    m._keep_ws = True
    x = golden_input(g).cuda()
    with torch.no_grad():
        o = m(x)[0]
        low = m.debug_buffer("logits").float().cpu().numpy()  # [M2][C]
        junk = torch.full((1 << 30,), 255, dtype=torch.uint8, device="cuda")
        del junk
        lab = m.predict(x, dtype=torch.uint8)
        low2 = m.debug_buffer("logits").float().cpu().numpy()
    print("low-res logits forward vs predict bit-equal:", bool((low == low2).all()),
          "max|d|", float(abs(low - low2).max()))
    with torch.no_grad():
        # the same low-res logits through the fused upsample+argmax and the unfused upsample:
        # fscnn_bilinear_ac_fwd on the NHWC low-res logits
        pass
    am = o.argmax(1).to(torch.uint8)
    bad = (am != lab).nonzero().tolist()
    print("after garbage fill: mismatches", len(bad))
    Hi, Wi, Ho, Wo = 128, 256, 1024, 2048
    f32 = np.float32
    def lerp(o_, i_, oo):
        s = f32((i_ - 1) / (oo - 1)) if oo > 1 else f32(0)
        src = f32(o_) * s
        i0 = int(src)
        i1 = i0 + (1 if i0 < i_ - 1 else 0)
        l1 = f32(src - f32(i0))
        return i0, i1, f32(f32(1) - l1), l1
    for n, h, w in bad[:5]:
        h0, h1, a0, a1 = lerp(h, Hi, Ho)
        w0, w1, b0, b1 = lerp(w, Wi, Wo)
        L = low.reshape(1, Hi, Wi, -1)
        for c in (15, 18):
            q = lambda hh, ww: f32(L[n, hh, ww, c])
            r0 = f32(f32(b0 * q(h0, w0)) + f32(b1 * q(h0, w1)))
            r1 = f32(f32(b0 * q(h1, w0)) + f32(b1 * q(h1, w1)))
            v = f32(f32(a0 * r0) + f32(a1 * r1))
            print("  px", (n, h, w), "class", c, "emulated", repr(v), "up_nchw", repr(o[n, c, h, w].item()))
        print("  labels: argmax", int(am[n, h, w]), "predict", int(lab[n, h, w]))
        print("  taps rows", h0, h1, "cols", w0, w1, "l", a0, a1, b0, b1)
        for c in (15, 18):
            print("   c", c, [repr(L[n, hh, ww, c]) for hh in (h0, h1) for ww in (w0, w1)])


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "low":
    lowres_check()
