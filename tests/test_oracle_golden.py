"""Pin the CPU oracle (oracle/fast_scnn_ref.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by importing the reference FastSCNN
(models/fast_scnn.py) in the survey container (tools/gen_golden.py).  If these pass, the oracle is
a faithful restatement and may be used as the checker for the HIP path.
"""
import numpy as np
import pytest
import torch

from helpers import golden_input, golden_sd, golden_target, load_golden
from oracle import fast_scnn_ref as ref
from fast_scnn_pytorch_amd import arch

EVAL_CASES = ["eval_c19_default", "eval_c19_calib", "eval_c2_calib", "eval_c19_bnrand_aux"]


def test_schema_matches_reference():
    g = load_golden("schema")
    for c, aux in ((19, False), (19, True), (2, False)):
        tag = "c%d%s" % (c, "_aux" if aux else "")
        specs = arch.state_dict_specs(c, aux)
        assert list(specs.keys()) == list(g[tag + "_keys"])
        shapes = [",".join(str(s) for s in v[0]) for v in specs.values()]
        assert shapes == list(g[tag + "_shapes"])
        assert [k for k, *_ in arch.param_specs(c, aux)] == list(g[tag + "_params"])
    assert len(arch.state_dict_specs(19)) == 268
    assert len(arch.state_dict_specs(19, True)) == 276
    n = sum(int(np.prod(s)) for _, s, _, _ in arch.param_specs(19))
    assert n == 1138051


@pytest.mark.parametrize("case", EVAL_CASES)
def test_oracle_eval_matches_reference(case):
    g = load_golden(case)
    sd = golden_sd(g)
    x = golden_input(g)
    with torch.no_grad():
        outs, _, acts = ref.forward(sd, x, int(g["num_classes"]), training=False,
                                    aux=bool(g["aux"]), record=True)
    for i, o in enumerate(outs):
        idx = g["out%d.sample_idx" % i]
        np.testing.assert_allclose(o.numpy().ravel()[idx], g["out%d.sample_val" % i],
                                   rtol=0, atol=1e-5)
        am = o.argmax(1).to(torch.uint8).numpy()
        assert (am == g["out%d.argmax" % i]).mean() > 0.9999
    stage = {"ltd": "act.learning_to_downsample",
             "global_feature_extractor.bottleneck3.2": "act.global_feature_extractor.bottleneck3",
             "ppm": "act.global_feature_extractor.ppm", "ffm": "act.feature_fusion"}
    for mine, theirs in stage.items():
        if theirs in g:
            np.testing.assert_allclose(acts[mine].numpy(), g[theirs], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", ["train_c19", "train_c2", "train_c19_aux"])
def test_oracle_train_matches_reference(case):
    g = load_golden(case)
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
          for k, v in golden_sd(g).items()}
    x = golden_input(g)
    t = golden_target(g)
    aux = bool(g["aux"])
    outs, stats, _ = ref.forward(sd, x, int(g["num_classes"]), training=True, aux=aux,
                                 dropout_seed=int(g["drop_seed"]))
    loss = ref.cross_entropy(outs[0], t)
    if aux:
        loss = loss + 0.4 * ref.cross_entropy(outs[1], t)
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    for k, *_ in arch.param_specs(int(g["num_classes"]), aux):
        gr = sd[k].grad.numpy().ravel()
        idx = g["grad_idx." + k]
        ref_vals = g["grad_val." + k]
        scale = max(1e-8, float(np.abs(ref_vals).max()))
        np.testing.assert_allclose(gr[idx], ref_vals, rtol=0, atol=1e-4 * scale + 1e-9, err_msg=k)
        assert abs(np.linalg.norm(gr.astype(np.float64)) - float(g["grad_norm." + k])) <= \
            1e-4 * float(g["grad_norm." + k]) + 1e-9
    for k in g:
        if k.startswith("stats."):
            np.testing.assert_allclose(stats[k[6:]].numpy(), g[k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("nc", [19, 2])
def test_oracle_metric_matches_reference(nc):
    """oracle.seg_counts against the reference's own batch_pix_accuracy /
    batch_intersection_union outputs (tools/gen_metric_golden.py), incl. -1 and 255 labels."""
    g = load_golden("metric_c%d" % nc)
    c = ref.seg_counts(g["pred"], g["label"], nc)
    assert c[0] == int(g["correct"]) and c[1] == int(g["labeled"])
    inter = c[2:2 + nc]
    union = c[2 + nc:2 + 2 * nc] + c[2 + 2 * nc:] - inter
    np.testing.assert_array_equal(inter, g["inter"])
    np.testing.assert_array_equal(union, g["union"])


def test_oracle_label_map_known_answers():
    """_class_to_index (data_loader/cityscapes.py:56-71): the reference's valid_classes list maps
    to train ids 0..18 in order and every other id in [-1, 33] to -1."""
    valid = [7, 8, 11, 12, 13, 17, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 31, 32, 33]
    out = ref.cityscapes_class_to_index(np.arange(-1, 34))
    assert [int(out[v + 1]) for v in valid] == list(range(19))
    assert (np.delete(out, [v + 1 for v in valid]) == -1).all()


@pytest.mark.parametrize("case", ["default", "kth", "keepall", "c2"])
def test_oracle_ohem_matches_reference(case):
    """oracle.ohem_cross_entropy against the reference SoftmaxCrossEntropyOHEMLoss run on CPU
    (tools/gen_ohem_golden.py): loss and d(loss)/d(logits)."""
    g = load_golden("ohem")
    x = torch.from_numpy(g[case + ".logits"]).requires_grad_(True)
    t = torch.from_numpy(g[case + ".target"])
    loss = ref.ohem_cross_entropy(x, t, -1, 0.7, int(g[case + ".min_kept"]),
                                  bool(g[case + ".use_weight"]))
    loss.backward()
    assert abs(loss.item() - float(g[case + ".loss"])) <= 1e-6 * abs(float(g[case + ".loss"]))
    np.testing.assert_allclose(x.grad.numpy(), g[case + ".grad"], rtol=0, atol=1e-7)
    if case == "kth":  # the k-th smallest threshold branch is what this case exercises
        _, thr = ref.ohem_target(x, t, -1, 0.7, int(g[case + ".min_kept"]))
        assert thr > 0.7


@pytest.mark.parametrize("case", ["dice_c2", "dice_c1", "focal_c2", "focal_c4", "mix_aux",
                                  "focal_c1"])
def test_oracle_dice_matches_reference(case):
    """oracle Dice / Focal+Dice against the reference criteria run on CPU
    (tools/gen_dice_golden.py)."""
    g = load_golden("dice")
    x = torch.from_numpy(g[case + ".logits"]).requires_grad_(True)
    t = torch.from_numpy(g[case + ".target"])
    if case.startswith("dice"):
        loss = ref.dice_loss(x, t)
    elif case in ("focal_c2", "focal_c1"):
        loss = ref.focal_dice_loss(x, t)
    elif case == "focal_c4":
        loss = ref.focal_dice_loss(x, t, alpha=0.25, gamma=1.5)
    else:
        x2 = torch.from_numpy(g[case + ".logits2"]).requires_grad_(True)
        loss = ref.dice_loss(x, t) + 0.4 * ref.dice_loss(x2, t)
    loss.backward()
    assert abs(loss.item() - float(g[case + ".loss"])) <= 1e-6
    np.testing.assert_allclose(x.grad.numpy(), g[case + ".grad"], rtol=0, atol=1e-8)
