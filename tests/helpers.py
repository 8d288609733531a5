"""Shared test helpers: fixture loading, portable weights → torch state_dicts."""
import os

import numpy as np
import torch

from fast_scnn_pytorch_amd import arch, portable_init

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def portable_sd(num_classes, aux=False, seed=0, variant="default", dtype=torch.float32):
    sd = arch.portable_state_dict(num_classes, aux, seed, variant)
    out = {}
    for k, v in sd.items():
        t = torch.from_numpy(np.asarray(v))
        out[k] = t.to(dtype) if t.is_floating_point() else t
    return out


def golden_sd(g, dtype=torch.float32):
    """Weights of a golden fixture: portable generator + stored calibrated BN stats."""
    sd = portable_sd(int(g["num_classes"]), bool(g["aux"]), int(g["seed_w"]), str(g["variant"]),
                     dtype)
    for k in list(g.keys()):
        if k.startswith("bn.") and ("running" in k):
            sd[k[3:]] = torch.from_numpy(g[k]).to(dtype)
    return sd


def golden_input(g, dtype=torch.float32):
    shape = tuple(int(s) for s in g["shape"])
    return torch.from_numpy(portable_init.input_tensor(int(g["seed_x"]), shape)).to(dtype)


def golden_target(g):
    shape = tuple(int(s) for s in g["shape"])
    return torch.from_numpy(portable_init.target_tensor(
        int(g["seed_t"]), (shape[0],) + shape[2:], int(g["num_classes"]),
        ignore_frac=float(g["ignore_frac"])))


def oracle_bf16_emulated(sd, x, nc):
    """Oracle forward with bf16 rounding of conv inputs / weights / outputs (autocast-like).

    Its deviation from the fp32 oracle is the error budget bf16 arithmetic itself implies for a
    given weight set; the HIP bf16 path is held to that budget (plus margin)."""
    import torch.nn.functional as F
    from oracle import fast_scnn_ref as ref
    q = lambda v: v.to(torch.bfloat16).float()  # noqa: E731
    oc = F.conv2d
    F.conv2d = lambda a, w, b=None, *r, **k: q(oc(q(a), q(w), b, *r, **k))
    try:
        with torch.no_grad():
            return ref.forward(sd, x, nc)[0][0]
    finally:
        F.conv2d = oc


def oracle_half_emulated(sd, x, nc, dtype=torch.float16):
    """Oracle forward as fp16 (or bf16) autocast runs it (test_specific_images.py:121,
    train.py:269): every conv's input, weights and output, every BatchNorm and interpolate output
    rounded to ``dtype``.  Its distance from the fp32 oracle is the error half precision itself
    implies for a weight set (cfg5 golden weights: fp16 max |d| 6.8e-2, argmax 98.84 %)."""
    import torch.nn.functional as F
    from oracle import fast_scnn_ref as ref
    q = lambda v: v.to(dtype).float()  # noqa: E731
    oc, ob, oi = F.conv2d, F.batch_norm, F.interpolate
    F.conv2d = lambda a, w, b=None, *r, **k: q(oc(q(a), q(w), b, *r, **k))
    F.batch_norm = lambda *a, **k: q(ob(*a, **k))
    F.interpolate = lambda *a, **k: q(oi(*a, **k))
    try:
        with torch.no_grad():
            return ref.forward(sd, q(x), nc)[0][0]
    finally:
        F.conv2d, F.batch_norm, F.interpolate = oc, ob, oi


def oracle_bf16_train_emulated(sd, x, t, nc, drop_seed, emulate=True, dtype=torch.bfloat16,
                               relu_masks=None, record=False, round_out=False,
                               round_blocks=False, round_all=False):
    """One train step (forward, CE(ignore -1), backward) of the oracle: fp64 when ``emulate`` is
    False, else fp32 with every conv input / weight / output rounded to ``dtype`` (bf16: cfg3's
    storage precision; fp16: train.py:269's autocast) — and, because autograd casts gradients
    back through those roundings, every conv input / output gradient rounded to ``dtype`` as
    well.  Returns (loss, {name: fp64 grad}); with ``record`` also the recorded activations.
    ``relu_masks``: evaluate under given ReLU masks (oracle ``_Ctx.relu``).  ``round_out``: the
    module's output, the full-resolution logits, is itself ``dtype`` (a 16-bit model returns
    16-bit logits, models/fast_scnn.py:40 under autocast), so it and its gradient are rounded.
    ``round_blocks``: every LinearBottleneck's output (after the shortcut add,
    models/fast_scnn.py:112-114) and its gradient rounded as well — the one activation a 16-bit
    implementation stores that is not a conv input or output (the residual stream).
    ``round_all``: 16-bit storage of every op output, as torch.autocast runs the reference in
    16 bits (train.py:269): conv, BatchNorm, interpolate and adaptive-pool outputs and the
    LinearBottleneck sums (implies ``round_blocks``), each with its gradient."""
    import torch.nn.functional as F
    from oracle import fast_scnn_ref as ref
    dt = torch.float32 if emulate else torch.float64
    s = {k: (v.detach().clone().to(dt).requires_grad_(True)
             if v.is_floating_point() and "running" not in k else
             (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
    oc, ob = F.conv2d, ref._bottleneck
    obn, oi, op = F.batch_norm, F.interpolate, F.adaptive_avg_pool2d
    if emulate:
        q = lambda v: v.to(dtype).float()  # noqa: E731
        F.conv2d = lambda a, w, b=None, *r, **k: q(oc(q(a), q(w), b, *r, **k))
        if round_blocks or round_all:
            ref._bottleneck = lambda *a, **k: q(ob(*a, **k))
        if round_all:
            F.batch_norm = lambda *a, **k: q(obn(*a, **k))
            F.interpolate = lambda *a, **k: q(oi(*a, **k))
            F.adaptive_avg_pool2d = lambda *a, **k: q(op(*a, **k))
    try:
        outs, _, acts = ref.forward(s, x.to(dt), nc, training=True, dropout_seed=drop_seed,
                                    relu_masks=relu_masks, record=record)
        out = outs[0].to(dtype).float() if (emulate and round_out) else outs[0]
        loss = ref.cross_entropy(out, t)
        loss.backward()
    finally:
        F.conv2d, ref._bottleneck = oc, ob
        F.batch_norm, F.interpolate, F.adaptive_avg_pool2d = obn, oi, op
    grads = {k: v.grad.double() for k, v in s.items() if v.grad is not None}
    if record:
        return loss.item(), grads, acts
    return loss.item(), grads


def argmax_agreement(logits, ref_argmax, ref_logits=None, margin_tol=1e-4):
    """Fraction of equal argmax pixels, and count of disagreements at margin > margin_tol.

    Near class boundaries the upsampled top-2 logits cross continuously, so a few pixels have a
    reference margin below fp32 reordering noise; those are the only mismatches allowed.
    """
    am = logits.argmax(1).to(torch.uint8).cpu().numpy()
    eq = am == ref_argmax
    bad_confident = None
    if ref_logits is not None:
        srt = torch.sort(ref_logits, dim=1).values
        margin = (srt[:, -1] - srt[:, -2]).cpu().numpy()
        bad_confident = int(((~eq) & (margin > margin_tol)).sum())
    return float(eq.mean()), bad_confident


# ReLU sites of the HIP plan (named plan units) -> the oracle's ReLU names (oracle/_Ctx.relu)
def relu_sites(aux=False):
    sites = [("c0", "learning_to_downsample.conv.conv.1"),
             ("l1dw", "learning_to_downsample.dsconv1.conv.1"),
             ("l1pw", "learning_to_downsample.dsconv1.conv.4"),
             ("l2dw", "learning_to_downsample.dsconv2.conv.1"),
             ("l2pw", "learning_to_downsample.dsconv2.conv.4")]
    for i in range(9):
        b = "global_feature_extractor.bottleneck%d.%d.block" % (i // 3 + 1, i % 3)
        sites += [("lbe%d" % i, b + ".0.conv.1"), ("lbd%d" % i, b + ".1.conv.1")]
    sites += [("ppk%d" % i, "global_feature_extractor.ppm.conv%d.conv.1" % (i + 1))
              for i in range(4)]
    sites += [("po", "global_feature_extractor.ppm.out.conv.1"),
              ("fdw", "feature_fusion.dwconv.conv.1"), ("f", "feature_fusion"),
              ("c1dw", "classifier.dsconv1.conv.1"), ("c1pw", "classifier.dsconv1.conv.4"),
              ("c2dw", "classifier.dsconv2.conv.1"), ("c2pw", "classifier.dsconv2.conv.4")]
    if aux:
        sites.append(("aux0", "auxlayer.1"))
    return sites


def hip_relu_masks(m, pre_ref, aux=False):
    """The ReLU masks the HIP forward of model ``m`` (run with ``m._keep_ws = True``) took at every
    ReLU, as NCHW bool tensors keyed by oracle ReLU name.  Pre-activations are recomputed from the
    unit's saved z / scale / shift exactly as the kernels evaluate them (fmaf(z, scale, shift) > 0:
    the fp64 product of two fp32 values is exact, so its one-rounding sum has the fmaf's sign);
    the FFM sum's mask is its stored output f > 0.  ``pre_ref``: the oracle's recorded
    pre-activations (shapes)."""
    out = {}
    for unit, name in relu_sites(aux):
        ref = pre_ref["pre:" + name]
        N, C, H, W = ref.shape
        if unit == "f":
            pre = m.debug_buffer("f").double().cpu()
        else:
            z = m.debug_buffer(unit + ".z").double().cpu()
            pre = z * m.debug_buffer(unit + ".scale").double().cpu() + \
                m.debug_buffer(unit + ".shift").double().cpu()
        if unit.startswith("ppk"):  # bin-major rows (bin = y * k + x, then n)
            mask = (pre > 0).reshape(H, W, N, C).permute(2, 3, 0, 1)
        else:
            mask = (pre > 0).reshape(N, H, W, C).permute(0, 3, 1, 2)
        out[name] = mask.contiguous()
    return out


def relu_flips(masks, pre_ref, tie=1e-5):
    """Sites where the HIP mask differs from the oracle's sign test: (name, count, worst relative
    |pre-activation| at a flip, relative to the channel's max |pre|).  Every flip of a correct
    implementation sits at a near-tie (worst <= tie)."""
    res = []
    for name, mk in masks.items():
        ref = pre_ref["pre:" + name].detach()
        diff = mk != (ref > 0)
        n = int(diff.sum())
        if n:
            scale = ref.abs().amax(dim=(0, 2, 3), keepdim=True).clamp_min(1e-30).expand_as(ref)
            res.append((name, n, float((ref.abs() / scale)[diff].max())))
    return res
