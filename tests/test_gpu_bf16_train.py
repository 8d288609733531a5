"""cfg3's own arithmetic (bf16 training) held to the oracle in a regime where bf16 is informative.

Why a separate regime.  At batch 2 and default init the bf16-emulating oracle is itself far from
fp64 (whole-gradient cosine ~0.45, tests/test_gpu_fullsize.py), so a gate relative to it says
little.  Two things make it so, both measured on the CPU with the oracle alone:
  * ReLU mask flips.  bf16 rounds ~3e4 x more pre-activations across zero than fp32 does, and at
    random init every flipped pixel moves each upstream gradient by O(1/sqrt(pixels)) (the same
    effect the fp32 tests remove with ``reference_grads``).  With the masks pinned, the emulation
    moves from cosine 0.46 to 0.77-0.98.
  * the pool-1 PPM BatchNorm normalises N values per channel: at N = 2 it is ill-conditioned; at
    cfg3's own batch, N = 8, it is not.
At bs 8, BN-randomised weights, 128 x 256 images and the masks pinned, the emulated-bf16 oracle
sits at whole-gradient cosine ~0.978 against fp64 (per-tensor relative error median ~0.22): the
error bf16 storage itself implies is small enough that a kernel bug shows.

Contract (both the unfused ``model(x)`` + CE path and the fused ``forward_loss`` head, so the
fused Dropout / BN-backward epilogue is covered against the oracle, not only against itself):
  * the fp64 oracle and the bf16-emulating oracle (``oracle_bf16_train_emulated``: fp32 with
    bf16 storage of every conv input / weight / output and, through autograd, every conv gradient;
    for ``model(x)`` also of the bf16 full-resolution logits it returns) run under the ReLU masks
    the HIP forward took; the HIP masks may differ from fp64's only where the emulation's own
    masks do (count <= 2x the emulation's flips, worst |pre| <= 2x its worst);
  * the budget per tensor is the emulation's error, taken as the largest over four equally valid
    bf16 realisations (conv-only and every-op rounding; the image as given and moved by one bf16
    ulp) -- the fp32 tests' "largest of three fp32 runs" in bf16;
  * every gradient tensor within 1.5x that budget, median ratio <= 1.0;
  * whole-vector cosine to fp64 >= the worst realisation's - 0.02 (and that one >= 0.95);
  * the loss within 1.5x the largest realisation's loss error.
Reference: /root/reference/train.py:269-275 (the AMP train step), SURVEY Appendix B.
"""
import numpy as np
import pytest
import torch

from helpers import (golden_input, golden_target, hip_relu_masks, oracle_bf16_train_emulated,
                     portable_sd, relu_flips)
from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
SHAPE = (8, 3, 128, 256)
NC = 19
DROP_SEED = 99


def _case():
    g = {"shape": np.array(SHAPE), "num_classes": np.int64(NC), "seed_w": np.int64(0),
         "seed_x": np.int64(5), "seed_t": np.int64(6), "ignore_frac": np.float64(0.05)}
    return portable_sd(NC, variant="bnrand"), golden_input(g), golden_target(g)


def _flip_stats(masks, acts, dtype_pre):
    """(flip count, worst relative |pre| at a flip) of masks against pre-activations acts."""
    fl = relu_flips(masks, acts, tie=1.0)
    return sum(n for _, n, _ in fl), max([w for _, _, w in fl] or [0.0])


@pytest.mark.parametrize("head", ["model_ce", "forward_loss"])
def test_bf16_train_grads_vs_emulated_oracle_tight(head):
    from fast_scnn_pytorch_amd import arch
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from models.fast_scnn import FastSCNN
    sd, x, t = _case()
    m = FastSCNN(NC)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    m._dropout_seed = DROP_SEED
    m._keep_ws = True
    xd, td = x.to(DEV).to(torch.bfloat16), t.to(DEV)
    if head == "model_ce":
        loss = cross_entropy(m(xd)[0], td)
    else:
        loss = m.forward_loss(xd, td)
    loss.backward()
    torch.cuda.synchronize()

    # pre-activations of fp64 and of the emulation (shapes + flip references)
    with torch.no_grad():
        s64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        _, _, acts64 = ref.forward(s64, x.double(), NC, training=True, dropout_seed=DROP_SEED,
                                   record=True)
    masks = hip_relu_masks(m, acts64)
    _, _, acts_em = oracle_bf16_train_emulated(sd, x, t, NC, DROP_SEED, emulate=True,
                                               record=True)
    em_masks = {k[4:]: (v.detach() > 0) for k, v in acts_em.items() if k.startswith("pre:")}
    n_hip, w_hip = _flip_stats(masks, acts64, torch.bfloat16)
    n_em, w_em = _flip_stats(em_masks, acts64, torch.bfloat16)
    print("ReLU flips vs fp64: HIP %d (worst rel |pre| %.2e), emulation %d (worst %.2e)"
          % (n_hip, w_hip, n_em, w_em))
    assert n_hip <= 2 * n_em + 16, (n_hip, n_em)
    assert w_hip <= 2 * w_em + 1e-6, (w_hip, w_em)

    named = dict(m.named_parameters())
    l64, g64, _ = oracle_bf16_train_emulated(sd, x, t, NC, DROP_SEED, emulate=False,
                                             relu_masks=masks, record=True)
    # the bf16 budget: the largest error of four equally valid bf16 realisations of the step
    # (model(x) returns bf16 full-resolution logits and receives their gradient in bf16; the fused
    # head never materialises them): storage rounding at every conv input / weight / output, or
    # at every op output as autocast runs the reference (round_all), each on the image as given
    # and moved by one bf16 ulp.  The error of tensors next to the loss is set by how the forward's
    # rounding errors happen to fall: one ulp of input moves the conv-only emulation's
    # classifier-bias error 3.4x and its loss error 5x (measured on the CPU), so one realisation
    # is not a budget -- as for fp32, where the budget is the largest of three fp32 runs
    # (tests/test_gpu_model.py reference_fp32_spread).
    xb = x.to(torch.bfloat16)
    ens = []
    for xx in (x, torch.nextafter(xb, torch.full_like(xb, float("inf"))).float(),
               torch.nextafter(xb, torch.full_like(xb, -float("inf"))).float()):
        for full in ((False, True) if xx is x else (False,)):
            ens.append(oracle_bf16_train_emulated(sd, xx, t, NC, DROP_SEED, emulate=True,
                                                  relu_masks=masks, round_out=head == "model_ce",
                                                  round_all=full))
    lerr = max(abs(l - l64) for l, _ in ens)
    print("loss: HIP %.6f fp64 %.6f emulated %s" % (loss.item(), l64,
                                                    " ".join("%.6f" % l for l, _ in ens)))
    assert abs(loss.item() - l64) <= 1.5 * lerr + 1e-5 * abs(l64)

    mine, truth, ratios, zeros = [], [], {}, {}
    gscale = max(g64[k].abs().max().item() for k in g64)
    for k, *_ in arch.param_specs(NC):
        a = named[k].grad.detach().double().cpu().flatten()
        b = g64[k].flatten()
        mine.append(a); truth.append(b)
        if b.norm().item() <= 1e-9 * gscale:
            # analytically zero (a conv bias in front of a train-mode BN, the pool-1 PPM conv):
            # rounding noise in every precision; held to the emulation's noise level
            zeros[k] = (a.norm().item(), max(g[k].norm().item() for _, g in ens))
            continue
        budget = max((g[k].flatten() - b).norm().item() for _, g in ens)
        ratios[k] = (a - b).norm().item() / budget
    med = float(np.median(list(ratios.values())))
    worst = max(ratios, key=ratios.get)
    a, b = torch.cat(mine), torch.cat(truth)
    cos = lambda u, v: (u @ v / (u.norm() * v.norm())).item()  # noqa: E731
    c_hip = cos(a, b)
    c_em = min(cos(torch.cat([g[k].flatten() for k, *_ in arch.param_specs(NC)]), b)
               for _, g in ens)
    print("%s bf16 train step vs fp64 (masks pinned): cosine HIP %.5f emulated (worst) %.5f; "
          "per-tensor error / emulated error: median %.3f, max %.3f (%s)"
          % (head, c_hip, c_em, med, ratios[worst], worst))
    top = sorted(ratios.items(), key=lambda kv: -kv[1])[:8]
    assert c_em >= 0.95, c_em  # the regime is informative
    assert c_hip >= c_em - 0.02, (c_hip, c_em)
    bad = {k: r for k, r in ratios.items() if r > 1.5}
    assert not bad, (bad, top)
    assert med <= 1.0, (med, top)
    for k, (na, ne) in zeros.items():
        assert na <= 4.0 * ne + 1e-6 * gscale, (k, na, ne)
