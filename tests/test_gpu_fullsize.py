"""Full-size parity at the literal BASELINE.json configs (cfg1 / cfg2 / cfg3 / cfg5).

Forward (cfg2 is north_star's "logits vs CPU within 1e-3, argmax masks bit-exact"): the HIP fp32
logits at 1 x 3 x 1024 x 2048 against the reference-generated golden
``tests/golden/cfg2_c19_1024x2048.npz`` (tools/gen_golden.py imported the reference FastSCNN and
ran it on the CPU) and against the fp64 oracle.

Argmax contract.  The reference's own fp32 CPU result is not the exact answer: at cfg2 it
disagrees with the fp64 oracle on 20 of 2.1 M pixels (cfg1: 8) whose top-2 margin is below its
own fp32 rounding noise (|ref32 - fp64| <= 3.1e-5 on these weights; measured on the CPU
against the fp64 oracle).  Bit-equality with that noise cannot be required of any other summation order, so the
gate is: (1) every pixel is bit-exact with the reference wherever the fp64 top-2 margin exceeds
1e-4 (3x the reference's own fp32 error), (2) the HIP path departs from the fp64 truth only at
pixels whose fp64 margin is within twice its own measured max |logit error| (itself gated at 1e-4),
and (3) a golden whose every fp64 margin exceeds 1e-4 is held to ``np.array_equal`` and the
golden's sha256 outright (flip counts and the sha256 comparison are printed for the others;
measured on MI355X: cfg2 23 pixels off the fp64 truth vs the reference's own 20, cfg1 10 vs 8,
cfg5 2 vs 0).
"""
import hashlib

import numpy as np
import pytest
import torch

from helpers import golden_input, golden_sd, golden_target, load_golden, portable_sd
from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
MARGIN = 1e-4


def _model(g, nc):
    from models.fast_scnn import FastSCNN
    m = FastSCNN(nc)
    m.load_state_dict(golden_sd(g))
    return m.to(DEV).eval()


def _oracle64(g, nc):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    sd = golden_sd(g)
    with torch.no_grad():
        return ref.forward({k: v.double() if v.is_floating_point() else v for k, v in sd.items()},
                           golden_input(g).double(), nc)[0][0]


def _check_argmax(o, g, o64):
    err = (o.double() - o64.double()).abs().max().item()
    am = o.argmax(1).to(torch.uint8).numpy()
    gold = g["out0.argmax"]
    sha_ok = hashlib.sha256(am.tobytes()).digest() == bytes(g["out0.argmax_sha256"])
    srt = torch.sort(o64, dim=1).values
    margin = (srt[:, -1] - srt[:, -2]).numpy()
    t64 = o64.argmax(1).to(torch.uint8).numpy()
    # (1) bit-exact wherever the decision is numerically determined
    assert int(((am != gold) & (margin > MARGIN)).sum()) == 0
    # (2) departures from the exact answer only where this path's own rounding can reach
    assert int(((am != t64) & (margin > 2 * err)).sum()) == 0
    if margin.min() > MARGIN:  # (3) every decision determined: the whole mask, bit for bit
        assert np.array_equal(am, gold) and sha_ok
    print("argmax: %d flips vs reference, %d vs fp64 (reference: %d), max|d| %.2e, sha256 equal %s"
          % (int((am != gold).sum()), int((am != t64).sum()), int((gold != t64).sum()), err,
             sha_ok))


@pytest.mark.parametrize("case", ["cfg2_c19_1024x2048", "cfg1_c19_768", "cfg5_c2_480x640"])
def test_literal_config_forward_fp32(case):
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = _model(g, nc)
    x = golden_input(g)
    with torch.no_grad():
        o = m(x.to(DEV))[0].float().cpu()
    assert o.shape == (x.shape[0], nc) + tuple(x.shape[2:])
    # sampled logits: within 1e-3 of the reference (north_star), gated at 1e-4
    idx = g["out0.sample_idx"]
    np.testing.assert_allclose(o.numpy().ravel()[idx], g["out0.sample_val"], rtol=0, atol=1e-4)
    o64 = _oracle64(g, nc)
    assert (o.double() - o64).abs().max().item() < 1e-4
    np.testing.assert_allclose(o.mean(dim=(0, 2, 3)).double().numpy(), g["out0.class_mean"],
                               rtol=0, atol=1e-5)
    _check_argmax(o, g, o64)


@pytest.mark.parametrize("case", ["eval_c19_default", "eval_c19_calib", "eval_c2_calib"])
def test_eval_goldens_argmax_bit_exact(case):
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = _model(g, nc)
    with torch.no_grad():
        o = m(golden_input(g).to(DEV))[0].float().cpu()
    _check_argmax(o, g, _oracle64(g, nc))


def test_cfg2_predict_labels_bit_exact_with_logits_argmax():
    """FastSCNN.predict (fused final upsample + argmax) == argmax of the returned logits."""
    g = load_golden("cfg2_c19_1024x2048")
    m = _model(g, 19)
    x = golden_input(g).to(DEV)
    with torch.no_grad():
        lab = m.predict(x, dtype=torch.uint8)
        am = m(x)[0].argmax(1).to(torch.uint8)
    assert torch.equal(lab, am)


def test_cfg3_full_size_bf16_train_step_properties():
    """cfg3 at its literal size (8 x 3 x 1024 x 2048, bf16, 19 classes): finite gradients, the
    fused low-res loss head equals the unfused full-resolution CE, loss decreasing over 3 SGD
    steps on a fixed batch, running statistics finite and updated."""
    from fast_scnn_pytorch_amd import portable_init
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN
    sd = portable_sd(19)
    B, H, W = 8, 1024, 2048
    x = torch.from_numpy(portable_init.input_tensor(1, (B, 3, H, W))).to(DEV).to(torch.bfloat16)
    t = torch.from_numpy(portable_init.target_tensor(3, (B, H, W), 19, 0.05)).to(DEV)

    def fresh():
        m = FastSCNN(19)
        m.load_state_dict(sd)
        m = m.to(DEV).train()
        m._dropout_seed = 21
        return m

    m1 = fresh()
    l1 = m1.forward_loss(x, t)
    l1.backward()
    g1 = torch.cat([p.grad.flatten() for p in m1.parameters()])
    assert torch.isfinite(g1).all() and g1.norm().item() > 0
    m2 = fresh()
    l2 = cross_entropy(m2(x)[0], t)
    l2.backward()
    g2 = torch.cat([p.grad.flatten() for p in m2.parameters()])
    # the unfused path rounds the full-resolution logits to bf16 before the CE
    assert abs(l1.item() - l2.item()) <= 2e-3 * abs(l2.item())
    cos = (g1.double() @ g2.double() / (g1.double().norm() * g2.double().norm())).item()
    assert cos > 0.9, cos
    del m2, g2
    opt = FusedSGD(m1.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    losses = [l1.item()]
    opt.step()
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        loss = m1.forward_loss(x, t)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses
    for k, v in m1.state_dict().items():
        if "running" in k:
            assert torch.isfinite(v).all(), k
    assert int(m1.state_dict()["classifier.dsconv2.conv.4.num_batches_tracked"]) == 4


@pytest.mark.parametrize("half", ["bf16", "fp16"])
def test_bf16_train_step_within_emulated_bf16_budget(half):
    """cfg3's arithmetic (bf16 activations, fp32 master weights / statistics) at golden size,
    and (half="fp16") the reference's own AMP arithmetic, train.py:269's fp16 autocast over fp32
    images, against the same oracle emulating fp16 storage,
    against the fp64 oracle, with the budget bf16 itself implies: the oracle run with every conv
    input, weight and output (and, through autograd, every conv gradient) rounded to bf16
    (``oracle_bf16_train_emulated``).  At random init train-mode BN backward cancels most of dy,
    so that budget is large (emulated-vs-fp64 relative error ~0.9 per tensor, whole-gradient cosine
    ~0.5 — measured with this helper on the CPU); the HIP bf16 gradients are gated against that
    budget (the HIP path also stores every intermediate gradient and BN output in bf16, more
    rounding points than the emulation).  Loss and the classifier gradients (before any BN
    backward) are held tight."""
    from helpers import oracle_bf16_train_emulated
    from fast_scnn_pytorch_amd import arch
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from models.fast_scnn import FastSCNN
    g = load_golden("train_c19")
    nc = 19
    sd = golden_sd(g)
    x, t = golden_input(g), golden_target(g)
    m = FastSCNN(nc)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    m._dropout_seed = int(g["drop_seed"])
    if half == "bf16":
        loss = cross_entropy(m(x.to(DEV).to(torch.bfloat16))[0], t.to(DEV))
    else:
        with torch.autocast("cuda"):
            out = m(x.to(DEV))[0]
            assert out.dtype == torch.float16
            loss = cross_entropy(out, t.to(DEV))
    loss.backward()
    hdt = torch.bfloat16 if half == "bf16" else torch.float16
    l64, g64 = oracle_bf16_train_emulated(sd, x, t, nc, int(g["drop_seed"]), emulate=False)
    lem, gem = oracle_bf16_train_emulated(sd, x, t, nc, int(g["drop_seed"]), emulate=True,
                                          dtype=hdt)
    assert abs(loss.item() - l64) <= 1.5 * abs(lem - l64) + 2e-3 * abs(l64)
    named = dict(m.named_parameters())
    mine, truth, emu, ratios = [], [], [], {}
    for k, *_ in arch.param_specs(nc):
        a = named[k].grad.detach().double().cpu().flatten()
        b, e = g64[k].flatten(), gem[k].flatten()
        mine.append(a); truth.append(b); emu.append(e)
        if k == "global_feature_extractor.ppm.conv1.conv.0.weight":
            # its BN normalises N*1*1 = 2 values: xhat = +-1 and the BN backward
            # dy - mean(dy) - xhat * mean(dy * xhat) is identically 0, so this gradient is zero
            # in exact arithmetic and pure rounding noise in every precision (no ratio to take)
            continue
        floor = 1e-3 * b.abs().max().item() * np.sqrt(b.numel()) + 1e-9
        ratios[k] = (a - b).norm().item() / ((e - b).norm().item() + floor)
    # BatchNorms over few values (the pool-1 / pool-2 PPM branches: N*1*1 = 2 and N*2*2 = 8
    # values; bottleneck3 at 1/32 resolution: 30) amplify whichever bf16 roundings land in front
    # of them, so single tensors there scatter widely around the emulation's error (measured up
    # to 5.7x); the gate is per tensor <= 4x (<= 8x for those), median <= 1.5x, and the
    # whole-vector error / cosine within 2x / 2.5x of the emulation's
    few = lambda k: ".ppm.conv1." in k or ".ppm.conv2." in k or ".bottleneck3." in k  # noqa: E731
    print("%s train step: per-tensor error / emulated error: median %.2f, max %.2f (%s)"
          % (half, np.median(list(ratios.values())), max(ratios.values()),
             max(ratios, key=ratios.get)))
    bad = {k: r for k, r in ratios.items() if r > (8.0 if few(k) else 4.0)}
    assert not bad, (bad, sorted(ratios.items(), key=lambda kv: -kv[1])[:8])
    assert np.median(list(ratios.values())) <= 1.5, sorted(ratios.items(), key=lambda kv: -kv[1])[:8]
    a, b, e = torch.cat(mine), torch.cat(truth), torch.cat(emu)
    cos = lambda u, v: (u @ v / (u.norm() * v.norm())).item()  # noqa: E731
    assert cos(a, b) >= cos(e, b) / 2.5, (cos(a, b), cos(e, b))
    assert (a - b).norm() <= 2.0 * (e - b).norm(), ((a - b).norm(), (e - b).norm())
    for k in ("classifier.conv.1.weight", "classifier.conv.1.bias"):
        u, v = named[k].grad.detach().double().cpu().flatten(), g64[k].flatten()
        assert cos(u, v) > 0.99, k


def test_cfg5_fp16_inference_within_fp16_budget():
    """cfg5 (TuSimple 2-class, 480 x 640, fp16 inference; BASELINE.json configs[4]) with fp16
    images in, fp16 MFMA arithmetic (fp32 accumulation) and fp16 logits out.

    Contract.  SURVEY Appendix B proposed |logit delta| <= 5e-3 / argmax >= 99.9 % from default-
    init measurements; on the calibrated golden weights the reference's OWN fp16 autocast
    arithmetic (oracle_half_emulated) is 6.8e-2 / 98.84 % away from its fp32 result, so the gate
    is that budget: max |delta| vs the fp32 oracle <= 1.5x the emulated fp16 reference's, and
    argmax agreement with the reference's fp32 mask no more than 0.5 % below the emulation's
    (measured: 3.7e-2 / 99.11 %, better than the emulation on both)."""
    from helpers import oracle_half_emulated
    g = load_golden("cfg5_c2_480x640")
    m = _model(g, 2)
    x = golden_input(g)
    with torch.no_grad():
        out = m(x.to(DEV).half())[0]
        lab = m.predict(x.to(DEV).half(), dtype=torch.uint8)
    assert out.dtype == torch.float16
    o = out.float().cpu()
    o64 = _oracle64(g, 2).float()
    oem = oracle_half_emulated(golden_sd(g), x, 2, torch.float16)
    gold = g["out0.argmax"]
    d, d_em = (o - o64).abs().max().item(), (oem - o64).abs().max().item()
    agree = (o.argmax(1).to(torch.uint8).numpy() == gold).mean()
    agree_em = (oem.argmax(1).to(torch.uint8).numpy() == gold).mean()
    print("cfg5 fp16: max|d| %.2e (emulated fp16 reference %.2e), argmax %.5f (emulated %.5f)"
          % (d, d_em, agree, agree_em))
    assert d <= 1.5 * d_em
    assert agree >= agree_em - 0.005
    # labels from the fused upsample + argmax: exactly the argmax of the returned fp16 logits
    assert np.array_equal(lab.cpu().numpy(), o.argmax(1).to(torch.uint8).numpy())
