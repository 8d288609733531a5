"""Autograd semantics of the drop-in module beyond the training step (SURVEY §8(b) "mode
semantics"): the reference FastSCNN (models/fast_scnn.py:33-46) is an ordinary nn.Module, so

* in eval mode with grad enabled (eval.py:43 calls ``model(image)`` without ``no_grad``) its
  output is differentiable: BatchNorm normalises with the running statistics and the gradient
  flows through that affine map (no batch-mean terms), Dropout is the identity;
* the input image gets a gradient when it requires one, in train and in eval mode.

Both are checked against fp64 autograd of the oracle under the same ReLU masks the HIP forward
took (tests/test_gpu_model.py ``reference_grads``: every differing mask bit a near-tie), with the
gate of the fp32 training tests (3x the reference's own fp32-vs-fp64 spread per tensor)."""
import numpy as np
import pytest
import torch

from helpers import (golden_input, golden_sd, golden_target, hip_relu_masks, load_golden,
                     portable_sd, relu_flips)
from oracle import fast_scnn_ref as ref
from test_gpu_model import _check_grads, make_model

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _oracle(sd, x, t, nc, training, drop_seed=None, dt=torch.float64, relu_masks=None):
    """Loss, parameter gradients and input gradient of the oracle (CE over the upsampled logits)."""
    s = {k: (v.detach().clone().to(dt).requires_grad_(True)
             if v.is_floating_point() and "running" not in k else
             (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
    xr = x.detach().clone().to(dt).requires_grad_(True)
    outs, _, _ = ref.forward(s, xr, nc, training=training, dropout_seed=drop_seed,
                             relu_masks=relu_masks)
    loss = ref.cross_entropy(outs[0], t)
    loss.backward()
    return loss.item(), {k: v.grad for k, v in s.items() if v.grad is not None}, xr.grad


def _reference(m, sd, x, t, nc, training, drop_seed=None):
    with torch.no_grad():
        s64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        _, _, acts = ref.forward(s64, x.double(), nc, training=training, dropout_seed=drop_seed,
                                 record=True)
    masks = hip_relu_masks(m, acts)
    flips = relu_flips(masks, acts)
    assert all(w <= 1e-4 for _, _, w in flips), flips
    l64, g64, dx64 = _oracle(sd, x, t, nc, training, drop_seed, relu_masks=masks)
    # the reference's own fp32 variability (test_gpu_model.reference_fp32_spread): as is,
    # single-threaded, and on the input moved by one ulp
    runs = [_oracle(sd, x, t, nc, training, drop_seed, dt=torch.float32, relu_masks=masks)]
    nth = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        runs.append(_oracle(sd, x, t, nc, training, drop_seed, dt=torch.float32, relu_masks=masks))
    finally:
        torch.set_num_threads(nth)
    xp = torch.nextafter(x.float(), torch.full_like(x.float(), float("inf")))
    runs.append(_oracle(sd, xp, t, nc, training, drop_seed, dt=torch.float32, relu_masks=masks))
    spread = {k: max((r[1][k].double() - g64[k].double()).norm().item() for r in runs) for k in g64}
    dx_spread = max((r[2].double() - dx64.double()).norm().item() for r in runs)
    return l64, g64, spread, dx64, dx_spread


def _check_dx(dx, dx64, spread):
    err = (dx.detach().double().cpu() - dx64).norm().item()
    gate = 3.0 * spread + 1e-5 * dx64.norm().item()
    print("dx: err %.3e gate %.3e (|dx| %.3e)" % (err, gate, dx64.norm().item()))
    assert err <= gate, (err, gate)
    a, b = dx.detach().double().cpu().flatten(), dx64.flatten()
    assert (a @ b / (a.norm() * b.norm())).item() > 0.99999


def test_eval_mode_param_and_input_grads_vs_oracle():
    """model.eval(); loss(model(x)[0]).backward(): every parameter gradient and x.grad against
    fp64 autograd of the eval-mode oracle (running-statistics BatchNorm)."""
    from fast_scnn_pytorch_amd import portable_init
    from fast_scnn_pytorch_amd.loss import cross_entropy
    g = load_golden("eval_c19_calib")
    nc = int(g["num_classes"])
    sd = golden_sd(g)
    m = make_model(sd, nc).eval()
    m._keep_ws = True
    x = golden_input(g)
    t = torch.from_numpy(portable_init.target_tensor(3, (x.shape[0],) + tuple(x.shape[2:]), nc))
    xd = x.to(DEV).requires_grad_(True)
    out = m(xd)[0]
    assert out.requires_grad and out.grad_fn is not None
    with torch.no_grad():  # the differentiable eval forward is the inference forward
        o2 = m(x.to(DEV))[0]
    assert torch.equal(out.detach(), o2)
    loss = cross_entropy(out, t.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    sd_after = m.state_dict()
    for k, v in sd.items():  # eval: no running-stat update, no num_batches_tracked step
        if "running" in k or "num_batches" in k:
            assert torch.equal(sd_after[k].cpu(), v), k
    lref, gref, spread, dx64, dx_spread = _reference(m, sd, x, t, nc, training=False)
    assert abs(loss.item() - lref) < 1e-5 * max(1.0, abs(lref))
    # (no analytically-zero tensor in eval mode: the pool-1 branch's BN is a fixed affine map)
    _check_grads(m, gref, nc, spread)
    w = "global_feature_extractor.ppm.conv1.conv.0.weight"
    a, b = dict(m.named_parameters())[w].grad.double().cpu(), gref[w].double()
    assert (a - b).norm().item() <= 3.0 * spread[w] + 1e-5 * b.norm().item(), w
    _check_dx(xd.grad, dx64, dx_spread)


@pytest.mark.parametrize("fused_loss", [False, True])
def test_train_mode_input_grad_vs_oracle(fused_loss):
    """x.grad of the training step (train_c19, Dropout active), through model(x) + CE and through
    the fused loss head, against fp64 autograd of the oracle; the parameter gradients stay those
    of the step without an input gradient (conv0's fused backward is replaced by the unfused one
    plus the input gradient)."""
    from fast_scnn_pytorch_amd.loss import cross_entropy
    g = load_golden("train_c19")
    nc = int(g["num_classes"])
    sd = golden_sd(g)
    m = make_model(sd, nc).train()
    m._dropout_seed = int(g["drop_seed"])
    m._keep_ws = True
    x, t = golden_input(g), golden_target(g)
    xd = x.to(DEV).requires_grad_(True)
    if fused_loss:
        loss = m.forward_loss(xd, t.to(DEV))
    else:
        loss = cross_entropy(m(xd)[0], t.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    assert xd.grad is not None and xd.grad.shape == x.shape and xd.grad.dtype == x.dtype
    lref, gref, spread, dx64, dx_spread = _reference(m, sd, x, t, nc, training=True,
                                                     drop_seed=int(g["drop_seed"]))
    assert abs(loss.item() - lref) < 1e-5 * max(1.0, abs(lref))
    _check_grads(m, gref, nc, spread)
    _check_dx(xd.grad, dx64, dx_spread)


def test_input_grad_16bit_and_channels_last():
    """bf16 compute (cfg3's arithmetic) with a channels_last fp32 image under autocast: x.grad
    keeps x's dtype and shape and is finite in both modes; in eval mode (no batch-statistics
    amplification of the bf16 storage rounding -- train-mode BN turns it into a ~40 %
    perturbation at default init, tests/test_gpu_model.py) it points where the fp32 gradient
    does."""
    from fast_scnn_pytorch_amd.loss import cross_entropy
    g = load_golden("train_c19")
    nc = int(g["num_classes"])
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    for train in (True, False):
        grads = {}
        for mode in ("fp32", "bf16"):
            m = make_model(golden_sd(g), nc).train(train)
            m._dropout_seed = 5
            xd = x.clone().to(memory_format=torch.channels_last).requires_grad_(True)
            if mode == "bf16":
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = m(xd)[0]
                assert out.dtype == torch.bfloat16
            else:
                out = m(xd)[0]
            cross_entropy(out, t).backward()
            assert xd.grad.dtype == torch.float32 and xd.grad.shape == x.shape
            assert torch.isfinite(xd.grad).all() and xd.grad.abs().sum() > 0
            grads[mode] = xd.grad.double().flatten()
        if not train:
            a, b = grads["fp32"], grads["bf16"]
            cos = (a @ b / (a.norm() * b.norm())).item()
            assert cos > 0.98, "bf16 eval-mode input gradient direction: cosine %.4f" % cos


def test_eval_grad_refuses_inplace_param_change():
    m = make_model(portable_sd(19, variant="bnrand"), 19).eval()
    x = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, (1, 3, 64, 96))
                         .astype(np.float32)).to(DEV)
    out = m(x)[0]
    with torch.no_grad():
        m.classifier.conv[1].bias.add_(1.0)
    with pytest.raises(RuntimeError, match="inplace operation"):
        out.sum().backward()


def test_eval_no_grad_and_frozen_params_stay_on_inference_path():
    """eval() under no_grad, or with every parameter frozen and an input that does not require
    grad, builds no graph (the inference path); freezing the parameters but asking for x.grad
    still differentiates (e.g. input attribution)."""
    m = make_model(portable_sd(19, variant="bnrand"), 19).eval()
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, (2, 3, 64, 96))
                         .astype(np.float32)).to(DEV)
    with torch.no_grad():
        assert m(x)[0].grad_fn is None
    for p in m.parameters():
        p.requires_grad_(False)
    assert m(x)[0].grad_fn is None
    xd = x.clone().requires_grad_(True)
    out = m(xd)[0]
    out.float().square().mean().backward()
    assert xd.grad is not None and torch.isfinite(xd.grad).all() and xd.grad.abs().sum() > 0
    assert all(p.grad is None for p in m.parameters())


def test_grad_arena_fully_written():
    """The gradient arena is not zeroed before the backward: every parameter gradient element must
    be written by it.  A NaN-filled arena gives exactly the gradients of a zero-filled one."""
    from fast_scnn_pytorch_amd.loss import cross_entropy
    g = load_golden("train_c2")
    res = {}
    for mode in ("train", "eval"):
        for fill in (0.0, float("nan")):
            m = make_model(golden_sd(g), 2)
            m.train(mode == "train")
            m._dropout_seed = 3
            m._debug_fill_grads = fill
            x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
            cross_entropy(m(x)[0], t).backward()
            res[(mode, fill == 0.0)] = torch.cat([p.grad.flatten() for p in m.parameters()])
        assert torch.isfinite(res[(mode, False)]).all(), mode
        assert torch.equal(res[(mode, False)], res[(mode, True)]), mode


def test_forward_loss_allows_inplace_ops_on_the_loss():
    """train.py-style gradient accumulation divides the loss in place (``loss /= accum``); the
    reference's loss tensor allows it, so the fused head's must too, with the gradient scaled."""
    sd = portable_sd(19, variant="bnrand")
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1.5, 1.5, (2, 3, 96, 160))
                         .astype(np.float32)).to(DEV)
    t = torch.from_numpy(np.random.default_rng(4).integers(-1, 19, (2, 96, 160))).to(DEV)
    m = make_model(sd, 19).train()
    m._dropout_seed = 7
    l1 = m.forward_loss(x, t)
    l1.backward()
    g1 = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    m.load_state_dict(sd)
    l2 = m.forward_loss(x, t)
    v = l2.item()
    l2 /= 4.0
    l2 += 0.0
    assert abs(l2.item() - v / 4.0) <= 1e-7 * abs(v)
    l2.backward()
    for k, p in m.named_parameters():
        torch.testing.assert_close(p.grad, g1[k] / 4.0, rtol=1e-5, atol=1e-9, msg=k)


def test_eval_backward_refuses_changed_running_stats():
    """The eval-mode backward recomputes the forward from the running statistics; a train-mode
    forward in between changes them, so (as the reference's saved native_batch_norm inputs
    would) the backward raises instead of returning gradients of other BN constants."""
    sd = portable_sd(19, variant="bnrand")
    x = torch.from_numpy(np.random.default_rng(5).uniform(-1.5, 1.5, (2, 3, 64, 96))
                         .astype(np.float32)).to(DEV)
    m = make_model(sd, 19).eval()
    out = m(x)[0]
    m.train()
    with torch.no_grad():
        m(x)
    m.eval()
    with pytest.raises(RuntimeError, match="inplace operation"):
        out.sum().backward()
    # untouched statistics: the same graph shape backpropagates
    out = m(x)[0]
    out.sum().backward()
