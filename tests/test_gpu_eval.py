"""Eval path: the final upsample fused with the argmax
(``FastSCNN.predict``, eval.py:43-45 / demo.py:43-48) and the on-GPU SegmentationMetric
counters (utils/metric.py:73-105), both checked bit-exactly: labels against
torch.argmax(model(x)[0], 1) of the same model, counters against the oracle restatement
(itself pinned to the reference's metric by tests/test_oracle_golden.py)."""
import numpy as np
import pytest
import torch

from helpers import load_golden, portable_sd
from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(nc):
    from models.fast_scnn import FastSCNN
    m = FastSCNN(nc)
    m.load_state_dict(portable_sd(nc, variant="bnrand"))
    return m.to(DEV).eval()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nc,shape", [(19, (2, 3, 128, 256)), (19, (1, 3, 67, 93)),
                                      (2, (2, 3, 96, 160))])
def test_predict_equals_argmax_of_forward(dt, nc, shape):
    m = _model(nc)
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1.7, 1.7, shape).astype(np.float32))
    x = x.to(DEV).to(dt)
    with torch.no_grad():
        want = torch.argmax(m(x)[0], 1)
        got = m.predict(x)
        got8 = m.predict(x, dtype=torch.uint8)
    assert got.dtype == torch.int64 and got.shape == want.shape
    assert torch.equal(got, want)
    assert got8.dtype == torch.uint8 and torch.equal(got8.long(), want)


def test_predict_needs_eval_mode():
    m = _model(19).train()
    with pytest.raises(RuntimeError):
        m.predict(torch.zeros(2, 3, 64, 64, device=DEV))


@pytest.mark.parametrize("nc", [19, 2])
def test_seg_metric_matches_reference_golden(nc):
    from fast_scnn_pytorch_amd.metric import SegmentationMetric
    g = load_golden("metric_c%d" % nc)
    met = SegmentationMetric(nc)
    met.update(torch.from_numpy(g["pred"]).to(DEV), torch.from_numpy(g["label"]).to(DEV))
    c = met.counts()
    assert c[0] == int(g["correct"]) and c[1] == int(g["labeled"])
    inter = c[2:2 + nc]
    np.testing.assert_array_equal(inter, g["inter"])
    np.testing.assert_array_equal(c[2 + nc:2 + 2 * nc] + c[2 + 2 * nc:] - inter, g["union"])


def test_seg_metric_accumulates_like_oracle():
    from fast_scnn_pytorch_amd.metric import SegmentationMetric
    rng = np.random.default_rng(7)
    nc = 19
    met = SegmentationMetric(nc)
    total = np.zeros(2 + 3 * nc, dtype=np.int64)
    for shape in [(2, 256, 512), (1, 67, 93), (3, 1, 1)]:
        pred = rng.integers(0, nc, shape)
        label = rng.integers(-1, nc, shape)
        label[rng.random(shape) < 0.02] = 255
        # int64 batch, then the same batch as uint8 predictions
        met.update(torch.from_numpy(pred).to(DEV), torch.from_numpy(label).to(DEV))
        met.update([torch.from_numpy(pred.astype(np.uint8)).to(DEV)], [label])
        total += 2 * ref.seg_counts(pred, label, nc)
    np.testing.assert_array_equal(met.counts(), total)
    pa, miou = met.get()
    pa_ref, miou_ref = ref.seg_scores(total, nc)
    assert pa == pa_ref and miou == miou_ref
