"""Dice / MixDice / Focal+Dice criteria (utils/loss.py:12-100; train.py:183-188) on the HIP path
against the reference's own outputs (tests/golden/dice.npz, tools/gen_dice_golden.py).
Tolerance: loss 2e-6 absolute (fp64 vs fp32 sums), gradient 1e-7 absolute."""
import numpy as np
import pytest
import torch

from helpers import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("case", ["dice_c2", "dice_c1", "focal_c2", "focal_c4", "mix_aux",
                                  "focal_c1"])
def test_dice_losses_match_reference(case):
    from fast_scnn_pytorch_amd.loss import DiceLoss, FocalDiceLoss, MixDiceLoss
    g = load_golden("dice")
    x = torch.from_numpy(g[case + ".logits"]).to(DEV).requires_grad_(True)
    t = torch.from_numpy(g[case + ".target"]).to(DEV)
    x2 = None
    if case.startswith("dice"):
        loss = DiceLoss()(x, t)
    elif case in ("focal_c2", "focal_c1"):
        loss = FocalDiceLoss()(x, t)
    elif case == "focal_c4":
        loss = FocalDiceLoss(alpha=0.25, gamma=1.5)(x, t)
    else:
        x2 = torch.from_numpy(g[case + ".logits2"]).to(DEV).requires_grad_(True)
        loss = MixDiceLoss(aux=True, aux_weight=0.4)((x, x2), t)
    loss.backward()
    assert abs(loss.item() - float(g[case + ".loss"])) <= 2e-6, (loss.item(), float(g[case + ".loss"]))
    np.testing.assert_allclose(x.grad.cpu().numpy(), g[case + ".grad"], rtol=0, atol=1e-7)
    if x2 is not None:
        np.testing.assert_allclose(x2.grad.cpu().numpy(), g[case + ".grad2"], rtol=0, atol=1e-7)
