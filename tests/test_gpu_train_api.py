"""The reference's train step as written (train.py:195-201, 265-275) through the HIP FastSCNN:

    with torch.cuda.amp.autocast():
        outputs = model(images); loss = criterion(outputs, targets)
    scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()

with ``torch.optim.SGD`` and ``FusedSGD``; input-layout robustness of the saved input (channels_last
/ permuted / fp16 / expanded batches give the same gradients as the dense fp32 batch); and the
FusedSGD edge cases of torch.optim.SGD's semantics (frozen parameters, interleaved groups).
"""
import numpy as np
import pytest
import torch

from helpers import golden_input, golden_sd, golden_target, load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(g, seed=5):
    from models.fast_scnn import FastSCNN
    m = FastSCNN(int(g["num_classes"]))
    m.load_state_dict(golden_sd(g))
    m = m.to(DEV).train()
    m._dropout_seed = seed
    return m


def _grads(m):
    return torch.cat([p.grad.detach().flatten() for p in m.parameters()]).double()


@pytest.mark.parametrize("amp", ["fp16", "bf16"])
@pytest.mark.parametrize("opt_name", ["torch_sgd", "fused_sgd"])
def test_autocast_gradscaler_step_as_train_py(opt_name, amp):
    """AMP step of train.py:269-275: ``torch.cuda.amp.autocast()`` selects fp16 arithmetic (the
    reference's), ``autocast(dtype=torch.bfloat16)`` bf16; fp32 master weights either way.
    GradScaler scales the loss, unscales the arena-view gradients in place, skips nothing (finite)
    and steps.  bf16: every backward kernel is linear in dy and the scale is a power of two, so
    the unscaled gradients and the stepped parameters are bit-identical to the same autocast step
    run without the scaler.  fp16: the scaled backward keeps small gradients out of fp16's
    subnormal range (GradScaler's purpose), so the two agree to fp16 rounding only."""
    from fast_scnn_pytorch_amd.loss import MixSoftmaxCrossEntropyLoss
    from fast_scnn_pytorch_amd.optim import FusedSGD
    g = load_golden("train_c19")
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    crit = MixSoftmaxCrossEntropyLoss(aux=False, ignore_label=-1)

    def make_opt(m):
        if opt_name == "torch_sgd":
            return torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        return FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)

    dt = torch.float16 if amp == "fp16" else torch.bfloat16
    ac = (lambda: torch.autocast("cuda")) if amp == "fp16" else \
        (lambda: torch.autocast("cuda", dtype=torch.bfloat16))  # noqa: E731
    m_amp = _model(g)
    opt = make_opt(m_amp)
    scaler = torch.amp.GradScaler("cuda")
    for it in range(2):
        opt.zero_grad()
        with ac():
            outputs = m_amp(x)
            assert outputs[0].dtype == dt  # the reference's logits dtype under this autocast
            loss = crit(outputs, t)
        scaler.scale(loss).backward()
        if it == 0:
            g_scaled = _grads(m_amp)
        scaler.step(opt)
        scaler.update()
        if it == 0:
            g_unscaled = _grads(m_amp)
            assert torch.isfinite(g_unscaled).all()
            p_after = [p.detach().clone() for p in m_amp.parameters()]
    # reference: the same autocast step without the scaler
    m_ref = _model(g)
    opt2 = make_opt(m_ref)
    opt2.zero_grad()
    with ac():
        loss2 = crit(m_ref(x), t)
    loss2.backward()
    g_ref = _grads(m_ref)
    opt2.step()
    scale = (g_scaled.norm() / g_unscaled.norm()).item()
    assert scale > 1.0 and abs(np.log2(scale) - round(np.log2(scale))) < 1e-4
    if amp == "bf16":
        assert torch.equal(g_unscaled, g_ref)
        for a, b in zip(p_after, m_ref.parameters()):
            assert torch.equal(a, b.detach())
    else:
        rel = ((g_unscaled - g_ref).norm() / g_ref.norm()).item()
        cos = (g_unscaled @ g_ref / (g_unscaled.norm() * g_ref.norm())).item()
        print("fp16 AMP: scaled vs unscaled backward, relative difference %.3g, cosine %.6f"
              % (rel, cos))
        assert rel < 5e-2 and cos > 0.998


def test_gradscaler_skips_a_step_on_fp16_overflow():
    """fp16 AMP with a loss scale so large that the scaled logits gradient overflows fp16: the
    HIP backward produces non-finite gradients (as the reference's fp16 autograd would),
    GradScaler finds them, skips optimizer.step() (parameters unchanged) and halves its scale;
    the next step at a sane scale is finite and updates the parameters."""
    from fast_scnn_pytorch_amd.loss import MixSoftmaxCrossEntropyLoss
    g = load_golden("train_c19")
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    crit = MixSoftmaxCrossEntropyLoss(aux=False, ignore_label=-1)
    m = _model(g)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 40)
    before = [p.detach().clone() for p in m.parameters()]
    opt.zero_grad()
    with torch.autocast("cuda"):
        loss = crit(m(x), t)
    scaler.scale(loss).backward()
    assert not torch.isfinite(_grads(m)).all()  # the overflow really happened
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() == 2.0 ** 39
    for a, b in zip(before, m.parameters()):
        assert torch.equal(a, b.detach())  # step skipped
    scaler.update(2.0 ** 10)
    opt.zero_grad()
    with torch.autocast("cuda"):
        loss = crit(m(x), t)
    scaler.scale(loss).backward()
    assert torch.isfinite(_grads(m)).all()
    scaler.step(opt)
    scaler.update()
    assert any(not torch.equal(a, b.detach()) for a, b in zip(before, m.parameters()))


@pytest.mark.parametrize("layout", ["channels_last", "permuted", "fp16", "expanded"])
def test_train_input_layouts_give_dense_fp32_gradients(layout):
    """The conv0 weight gradient re-reads the forward input; the autograd function must keep the
    dense NCHW copy it computed on, whatever layout / dtype the caller passed."""
    from fast_scnn_pytorch_amd.loss import cross_entropy
    g = load_golden("train_c2")
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    m0 = _model(g)
    cross_entropy(m0(x)[0], t).backward()
    ref_g = _grads(m0)
    if layout == "channels_last":
        xi = x.to(memory_format=torch.channels_last)
    elif layout == "permuted":
        xi = x.permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
    elif layout == "fp16":  # fp16 images (fp16 arithmetic), channels_last: same as dense fp16
        xi = x.half().to(memory_format=torch.channels_last)
        m0 = _model(g)
        cross_entropy(m0(x.half().contiguous())[0], t).backward()
        ref_g = _grads(m0)
    else:
        xi = x[:1].expand(2, -1, -1, -1)
        m0 = _model(g)
        cross_entropy(m0(xi.contiguous())[0], t).backward()
        ref_g = _grads(m0)
    assert not xi.is_contiguous()
    m = _model(g)
    cross_entropy(m(xi)[0], t).backward()
    assert torch.equal(_grads(m), ref_g)


def _fused_vs_torch(groups_fn, steps=3):
    """Run FusedSGD and torch.optim.SGD on identical FastSCNN parameter arenas with the same
    (real) gradients; parameter groups / frozen parameters from groups_fn(model)."""
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from fast_scnn_pytorch_amd.optim import FusedSGD
    g = load_golden("train_c2")
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    m = _model(g)
    names = [n for n, _ in m.named_parameters()]
    groups, frozen = groups_fn(names)
    prm = dict(m.named_parameters())
    for n in frozen:
        prm[n].requires_grad_(False)
    ref = {n: p.detach().clone() for n, p in prm.items()}
    tparams = {n: ref[n].clone().requires_grad_(n not in frozen) for n in names}
    opt = FusedSGD([{"params": [prm[n] for n in gr["names"]], **gr["hp"]} for gr in groups],
                   lr=0.01, momentum=0.9, weight_decay=1e-4)
    topt = torch.optim.SGD([{"params": [tparams[n] for n in gr["names"]], **gr["hp"]}
                            for gr in groups], lr=0.01, momentum=0.9, weight_decay=1e-4)
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        m.forward_loss(x, t).backward()
        for n in names:
            tparams[n].grad = None if prm[n].grad is None else prm[n].grad.detach().clone()
        opt.step()
        topt.step()
        torch.cuda.synchronize()
        for n in names:
            assert torch.allclose(prm[n].detach(), tparams[n].detach(), rtol=1e-6, atol=1e-7), n
    for n in frozen:
        assert torch.equal(prm[n].detach(), ref[n]), n  # never touched (no weight decay)


def test_fused_sgd_skips_frozen_parameters_inside_the_arena():
    def fn(names):
        mid = [n for n in names if "bottleneck2.1" in n]
        return [{"names": [n for n in names if n not in mid], "hp": {}}], mid
    _fused_vs_torch(fn)


def test_fused_sgd_interleaved_param_groups():
    def fn(names):
        a = [n for i, n in enumerate(names) if i % 3 == 0]
        b = [n for i, n in enumerate(names) if i % 3 != 0]
        return [{"names": a, "hp": {"lr": 0.02, "weight_decay": 0.0}},
                {"names": b, "hp": {"momentum": 0.5}}], []
    _fused_vs_torch(fn)
