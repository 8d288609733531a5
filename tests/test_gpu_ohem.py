"""OHEM cross entropy (SoftmaxCrossEntropyOHEMLoss, utils/loss.py:127-206 — train.py's
``--loss-type ce`` criterion, train.py:190-191) on the HIP path against the reference's own outputs (tests/golden/ohem.npz, made by
tools/gen_ohem_golden.py) and the oracle restatement.  Tolerance: loss 1e-5 relative, gradient
1e-6 absolute (fp32 exp/log ulps; the kept set is identical on these inputs)."""
import numpy as np
import pytest
import torch

from helpers import load_golden
from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("case", ["default", "kth", "keepall", "c2"])
def test_ohem_matches_reference(case):
    from fast_scnn_pytorch_amd.loss import SoftmaxCrossEntropyOHEMLoss
    g = load_golden("ohem")
    x = torch.from_numpy(g[case + ".logits"]).to(DEV).requires_grad_(True)
    t = torch.from_numpy(g[case + ".target"]).to(DEV)
    crit = SoftmaxCrossEntropyOHEMLoss(ignore_label=-1, thresh=0.7,
                                       min_kept=int(g[case + ".min_kept"]),
                                       use_weight=bool(g[case + ".use_weight"]))
    loss = crit(x, t)
    loss.backward()
    want = float(g[case + ".loss"])
    assert abs(loss.item() - want) <= 1e-5 * abs(want), (loss.item(), want)
    np.testing.assert_allclose(x.grad.cpu().numpy(), g[case + ".grad"], rtol=0, atol=1e-6)


def test_ohem_kth_threshold_selection():
    """The radix select returns exactly the k-th smallest label probability."""
    from fast_scnn_pytorch_amd.loss import ohem_threshold
    g = load_golden("ohem")
    x = torch.from_numpy(g["kth.logits"])
    t = torch.from_numpy(g["kth.target"])
    k = int(g["kth.min_kept"])
    prob, thr = ohem_threshold(x.to(DEV).contiguous(), t.to(DEV), -1, 0.7, k)
    thr = float(thr.item())
    p = prob.cpu().numpy()
    valid = p <= 1.0
    assert thr > 0.7 and thr == np.sort(p[valid])[k - 1]
    _, thr_ref = ref.ohem_target(x, t, -1, 0.7, k)
    assert abs(thr - float(thr_ref)) <= 1e-6


def test_mix_ohem_with_model_outputs():
    from fast_scnn_pytorch_amd.loss import MixSoftmaxCrossEntropyOHEMLoss
    from models.fast_scnn import FastSCNN
    m = FastSCNN(19, aux=True).to(DEV).train()
    x = torch.randn(2, 3, 96, 128, device=DEV)
    t = torch.randint(0, 19, (2, 96, 128), device=DEV)
    crit = MixSoftmaxCrossEntropyOHEMLoss(aux=True, aux_weight=0.4, ignore_index=-1)
    outs = m(x)
    loss = crit(outs, t)
    lref = ref.ohem_cross_entropy(outs[0].detach().cpu(), t.cpu()) + \
        0.4 * ref.ohem_cross_entropy(outs[1].detach().cpu(), t.cpu())
    assert abs(loss.item() - lref.item()) <= 1e-5 * abs(lref.item())
    loss.backward()
    assert torch.isfinite(m.classifier.conv[1].weight.grad).all()


def test_ohem_step_has_no_host_sync():
    """The OHEM criterion's forward + backward enqueue without any synchronising torch call
    (SURVEY.md §7 hard part x: no host sync in the step)."""
    from fast_scnn_pytorch_amd.loss import SoftmaxCrossEntropyOHEMLoss
    g = load_golden("ohem")
    x = torch.from_numpy(g["kth.logits"]).to(DEV).requires_grad_(True)
    t = torch.from_numpy(g["kth.target"]).to(DEV)
    crit = SoftmaxCrossEntropyOHEMLoss(ignore_label=-1, thresh=0.7,
                                       min_kept=int(g["kth.min_kept"]),
                                       use_weight=bool(g["kth.use_weight"]))
    crit(x, t)  # first call moves the class weights to the device (once)
    x.grad = None
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        loss = crit(x, t)
        loss.backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    lref = float(g["kth.loss"])
    assert abs(loss.item() - lref) <= 1e-5 * max(1.0, abs(lref))
