"""Whole-network parity of the HIP FastSCNN against the oracle and the reference's golden vectors.

fp32 contract (BASELINE.json north_star): logits within 1e-3 of the reference, argmax equal
wherever the reference's top-2 margin exceeds fp32 reordering noise (1e-4); internally gated at
1e-4.  bf16 contract: |dlogit| small relative to the logit range, argmax
agreement >= 99 %.  Train-mode gradients are checked tensor by tensor.
"""
import numpy as np
import pytest
import torch

from helpers import (argmax_agreement, golden_input, golden_sd, golden_target, load_golden,
                     portable_sd)
from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def make_model(g_or_sd, num_classes, aux=False):
    from models.fast_scnn import FastSCNN
    m = FastSCNN(num_classes, aux=aux)
    sd = golden_sd(g_or_sd) if isinstance(g_or_sd, dict) and "shape" in g_or_sd else g_or_sd
    m.load_state_dict(sd)
    return m.to(DEV)


def oracle_eval(sd, x, nc):
    with torch.no_grad():
        return ref.forward({k: v.double() if v.is_floating_point() else v for k, v in sd.items()},
                           x.double(), nc)[0][0].float()


@pytest.mark.parametrize("case", ["eval_c19_default", "eval_c19_calib", "eval_c2_calib"])
def test_eval_fp32_vs_golden(case):
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = make_model(g, nc).eval()
    x = golden_input(g)
    with torch.no_grad():
        out = m(x.to(DEV))
    assert isinstance(out, tuple) and len(out) == 1
    o = out[0].float().cpu()
    assert o.shape == (x.shape[0], nc) + tuple(x.shape[2:])
    idx = g["out0.sample_idx"]
    np.testing.assert_allclose(o.numpy().ravel()[idx], g["out0.sample_val"], rtol=0, atol=1e-4)
    oref = oracle_eval(golden_sd(g), x, nc)
    err = (o - oref).abs().max().item()
    assert err < 1e-4, err
    frac, bad = argmax_agreement(o, g["out0.argmax"], oref, 1e-4)
    assert bad == 0 and frac > 0.999


@pytest.mark.parametrize("case", ["cfg1_c19_768", "cfg5_c2_480x640"])
def test_eval_fp32_literal_configs(case):
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = make_model(g, nc).eval()
    x = golden_input(g)
    with torch.no_grad():
        o = m(x.to(DEV))[0].float().cpu()
    idx = g["out0.sample_idx"]
    np.testing.assert_allclose(o.numpy().ravel()[idx], g["out0.sample_val"], rtol=0, atol=1e-3)
    am = o.argmax(1).to(torch.uint8).numpy()
    assert (am == g["out0.argmax"]).mean() > 0.9999
    hist = np.bincount(am.ravel(), minlength=nc)
    assert np.abs(hist - g["out0.hist"]).sum() <= max(4, 1e-5 * am.size)


def test_eval_odd_sizes_vs_oracle():
    sd = portable_sd(19, variant="bnrand")
    m = make_model(sd, 19).eval()
    for shape in [(2, 3, 100, 150), (1, 3, 67, 93), (3, 3, 64, 64)]:
        x = torch.from_numpy(np.random.default_rng(0).uniform(-1.7, 1.7, shape).astype(np.float32))
        with torch.no_grad():
            o = m(x.to(DEV))[0].float().cpu()
        oref = oracle_eval(sd, x, 19)
        assert (o - oref).abs().max().item() < 1e-4


def _train_step_parity(case, dtype_ok_tol=1e-4):
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = make_model(g, nc).train()
    m._dropout_seed = int(g["drop_seed"])
    from fast_scnn_pytorch_amd.loss import MixSoftmaxCrossEntropyLoss
    crit = MixSoftmaxCrossEntropyLoss(aux=False, ignore_label=-1)
    x, t = golden_input(g).to(DEV), golden_target(g).to(DEV)
    out = m(x)
    loss = crit(out, t)
    loss.backward()
    torch.cuda.synchronize()
    return g, m, loss


@pytest.mark.parametrize("case", ["train_c19", "train_c2"])
def test_train_fp32_grads_vs_golden(case):
    g, m, loss = _train_step_parity(case)
    assert abs(loss.item() - float(g["loss"])) < 1e-4
    from fast_scnn_pytorch_amd import arch
    named = dict(m.named_parameters())
    for k, *_ in arch.param_specs(int(g["num_classes"])):
        gr = named[k].grad.detach().float().cpu().numpy().ravel()
        idx, rv = g["grad_idx." + k], g["grad_val." + k]
        scale = max(1e-8, float(np.abs(rv).max()))
        np.testing.assert_allclose(gr[idx], rv, rtol=0, atol=2e-3 * scale + 1e-8, err_msg=k)
        gn = float(g["grad_norm." + k])
        assert abs(np.linalg.norm(gr.astype(np.float64)) - gn) <= 2e-3 * gn + 1e-8, k
    sd = m.state_dict()
    for k in g:
        if k.startswith("stats."):
            np.testing.assert_allclose(sd[k[6:]].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5,
                                       err_msg=k)
        if k.endswith("num_batches_tracked"):
            pass
    assert int(sd["learning_to_downsample.conv.conv.1.num_batches_tracked"]) == 1


def test_sgd_step_vs_golden():
    g, m, _ = _train_step_parity("train_c19")
    from fast_scnn_pytorch_amd.optim import FusedSGD
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    # the gradient arena must be shared → one fused launch
    opt.step()
    torch.cuda.synchronize()
    from fast_scnn_pytorch_amd import arch
    named = dict(m.named_parameters())
    for k, *_ in arch.param_specs(19):
        v = named[k].detach().cpu().numpy().ravel()
        idx = g["grad_idx." + k]
        np.testing.assert_allclose(v[idx], g["sgd_val." + k], rtol=0, atol=1e-6, err_msg=k)


def test_grads_are_arena_views():
    _, m, _ = _train_step_parity("train_c2")
    grads = [p.grad for p in m.parameters()]
    st = grads[0].untyped_storage().data_ptr()
    assert all(gg.untyped_storage().data_ptr() == st for gg in grads)


def test_bf16_train_and_eval_close_to_fp32():
    g = load_golden("train_c19")
    m = make_model(g, 19)
    x = golden_input(g).to(DEV)
    m.eval()
    with torch.no_grad():
        o32 = m(x)[0].float()
        o16 = m(x.to(torch.bfloat16))[0].float()
    rng = (o32.max() - o32.min()).item()
    assert (o16 - o32).abs().max().item() < 0.05 * rng
    assert (o16.argmax(1) == o32.argmax(1)).float().mean().item() > 0.98
    # train step in bf16: loss and gradient directions agree with fp32
    from fast_scnn_pytorch_amd.loss import cross_entropy
    t = golden_target(g).to(DEV)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        mm = make_model(g, 19).train()
        mm._dropout_seed = 7
        loss = cross_entropy(mm(x.to(dt))[0], t)
        loss.backward()
        res[dt] = (loss.item(), torch.cat([p.grad.flatten() for p in mm.parameters()]))
    assert abs(res[torch.float32][0] - res[torch.bfloat16][0]) < 0.02 * abs(res[torch.float32][0])
    a, b = res[torch.float32][1], res[torch.bfloat16][1]
    cos = (a @ b / (a.norm() * b.norm())).item()
    assert cos > 0.98, cos


def test_train_bs1_raises_like_reference():
    m = make_model(portable_sd(19), 19).train()
    with pytest.raises(ValueError):
        m(torch.zeros(1, 3, 64, 64, device=DEV))


def test_cpu_input_raises():
    from models.fast_scnn import FastSCNN
    m = FastSCNN(19)
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 3, 64, 64))
