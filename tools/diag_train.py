#!/usr/bin/env python3
"""GPU diagnostic: train-mode forward / backward of the HIP FastSCNN vs the oracle.

Prints forward logits error, running-stat errors, stage-level activation / gradient errors (via
the plan's named buffers) and per-parameter gradient errors in backward order, with the oracle's
own fp32-vs-fp64 error beside each so conditioning is visible.  Not a test (no assertions).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _fscnn_boot  # noqa: E402

_fscnn_boot.load()
from fast_scnn_pytorch_amd import arch, portable_init  # noqa: E402
from fast_scnn_pytorch_amd.loss import cross_entropy  # noqa: E402
from models.fast_scnn import FastSCNN  # noqa: E402
from oracle import fast_scnn_ref as ref  # noqa: E402


DROP_SEED = 1234


def oracle(sd, x, t, nc, p, dt):
    s = {k: (v.detach().clone().to(dt).requires_grad_(True)
             if v.is_floating_point() and "running" not in k else
             (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
    outs, stats, acts = ref.forward(s, x.to(dt), nc, training=True,
                                    dropout_seed=DROP_SEED if p > 0 else None, dropout_p=p,
                                    record=True)
    for a in acts.values():
        a.retain_grad()
    loss = ref.cross_entropy(outs[0], t)
    loss.backward()
    return s, outs, stats, acts, loss


def nhwc_rows(t):
    return t.detach().permute(0, 2, 3, 1).reshape(-1, t.shape[1]).double()


def rel(a, b):
    return (a.double().cpu() - b.double().cpu()).abs().max().item() / (b.abs().max().item() + 1e-30)


def main(dtype=torch.float32, p=0.0, shape=(2, 3, 128, 256), nc=19, case=None):
    seed = 1234
    if case:  # a golden train case: its weights, batch, targets and dropout seed
        from helpers import golden_input, golden_sd, golden_target, load_golden
        g = load_golden(case)
        nc, sd, x, t = int(g["num_classes"]), golden_sd(g), golden_input(g), golden_target(g)
        seed, p = int(g["drop_seed"]), 0.1
    else:
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
              arch.portable_state_dict(nc, seed=0, variant="bnrand").items()}
        x = torch.from_numpy(portable_init.input_tensor(1, shape))
        t = torch.from_numpy(portable_init.target_tensor(3, (shape[0],) + shape[2:], nc, 0.05))
    global DROP_SEED
    DROP_SEED = seed
    m = FastSCNN(nc)
    m.load_state_dict(sd)
    m = m.cuda().train()
    m.classifier.conv[0].p = p
    m._dropout_seed = seed
    m._keep_ws = True
    out = m(x.cuda().to(dtype))[0]
    loss = cross_entropy(out, t.cuda())
    loss.backward()
    torch.cuda.synchronize()
    s64, outs, stats, acts, lref = oracle(sd, x, t, nc, p, torch.float64)
    s32, _, _, acts32, _ = oracle(sd, x, t, nc, p, torch.float32)
    o = out.detach().float().cpu()
    print("dtype", dtype, "p", p, "loss hip %.7f oracle %.7f" % (loss.item(), lref.item()))
    print("logits rel %.3e" % rel(o, outs[0]))
    msd = m.state_dict()
    worst = sorted(((msd[k].cpu().double() - v).abs().max().item(), k)
                   for k, v in stats.items() if "running" in k)[::-1]
    print("running-stat worst:", worst[:3])
    print("stage-level (ours vs fp64 | oracle-fp32 vs fp64):")
    pairs = [("c2pw.a", "cls.dsconv2", False), ("c2pw.ga", "cls.dsconv2", True),
             ("f", "ffm", False), ("lbp8.a", "global_feature_extractor.bottleneck3.2", False),
             ("po.a", "ppm", False)]
    for mine, theirs, grad in pairs:
        a = m.debug_buffer(mine).float()
        r = acts[theirs].grad if grad else acts[theirs]
        r32 = acts32[theirs].grad if grad else acts32[theirs]
        print("  %-8s vs %-40s %s rel %.2e | %.2e" % (mine, theirs, "grad" if grad else "act ",
                                                      rel(a, nhwc_rows(r)),
                                                      rel(nhwc_rows(r32), nhwc_rows(r))))
    gl = m.debug_buffer("g_logits").float()
    gr = acts["logits_lowres"].grad
    print("  g_logits rel %.2e | %.2e" % (rel(gl, nhwc_rows(gr)),
                                         rel(nhwc_rows(acts32["logits_lowres"].grad), nhwc_rows(gr))))
    named = dict(m.named_parameters())
    # BN backward of classifier.dsconv2.conv.4 recomputed in fp64 from OUR saved buffers
    a = m.debug_buffer("c2pw.a").double().cpu()
    ga = m.debug_buffer("c2pw.ga").double().cpu()
    z = m.debug_buffer("c2pw.z").double().cpu()
    mu = m.debug_buffer("c2pw.mean").double().cpu()[0]
    ist = m.debug_buffer("c2pw.invstd").double().cpu()[0]
    dyr = ga * (a > 0)
    db = dyr.sum(0)
    dg = (dyr * (z - mu) * ist).sum(0)
    gb = named["classifier.dsconv2.conv.4.bias"].grad.double().cpu()
    gg = named["classifier.dsconv2.conv.4.weight"].grad.double().cpu()
    rb = s64["classifier.dsconv2.conv.4.bias"].grad
    print("dbeta: kernel vs own-buffers-fp64 %.2e ; own-buffers vs oracle %.2e" % (rel(gb, db), rel(db, rb)))
    print("dgamma: kernel vs own-buffers-fp64 %.2e" % rel(gg, dg))
    # mask flips vs oracle
    ra = nhwc_rows(acts["cls.dsconv2"]).cpu()
    flips = ((a > 0) != (ra > 0)).sum().item()
    print("mask flips vs oracle:", flips, "of", a.numel(), " min|a_ref| at flips",
          ra[(a > 0) != (ra > 0)].abs().max().item() if flips else 0)
    print("per-parameter grads (backward order): ours vs fp64 | oracle-fp32 vs fp64 (max-normalised)")
    for k, *_ in list(reversed(arch.param_specs(nc))):
        g = named[k].grad.detach().double().cpu()
        r = s64[k].grad
        print("  %-60s %.2e | %.2e" % (k, rel(g, r), rel(s32[k].grad, r)))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main(torch.float32, case=sys.argv[1])
    else:
        main(torch.float32, 0.0)
