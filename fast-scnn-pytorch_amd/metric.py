"""SegmentationMetric on the HIP path (utils/metric.py:12-105).

Same interface as the reference class: ``update(preds, labels)`` (one array / tensor or a list of
them) and ``get() -> (pixAcc, mIoU)``.  The per-batch counters of batch_pix_accuracy /
batch_intersection_union (utils/metric.py:73-105) are accumulated on the device by one kernel
(exact integer counts); ``get`` applies the reference's formulas (utils/metric.py:42-54).
Predictions may be int64 (torch.argmax) or uint8 (``FastSCNN.predict(x, torch.uint8)``).
"""
import numpy as np
import torch

from . import _lib


class SegmentationMetric:
    def __init__(self, nclass, device=None):
        self.nclass = int(nclass)
        self.device = device
        self.reset()

    def reset(self):
        self._counts = None

    def update(self, preds, labels):
        if isinstance(preds, (list, tuple)):
            for p, l in zip(preds, labels):
                self._update(p, l)
        else:
            self._update(preds, labels)

    def _update(self, pred, label):
        pred = torch.as_tensor(pred)
        label = torch.as_tensor(label)
        dev = pred.device if pred.is_cuda else (label.device if label.is_cuda else
                                                torch.device(self.device or "cuda"))
        if tuple(pred.shape) != tuple(label.shape):
            raise AssertionError("prediction %s and label %s shapes differ"
                                 % (tuple(pred.shape), tuple(label.shape)))
        if pred.dtype not in (torch.int64, torch.uint8):
            pred = pred.to(torch.int64)
        pred = pred.to(dev).contiguous()
        label = label.to(dev, torch.int64).contiguous()
        if self._counts is None:
            self._counts = torch.zeros(2 + 3 * self.nclass, dtype=torch.int64, device=dev)
        _lib.call("fscnn_seg_metric", _lib.ptr(pred), 1 if pred.dtype == torch.uint8 else 0,
                  _lib.ptr(label), pred.numel(), self.nclass, _lib.ptr(self._counts),
                  _lib.stream_ptr(dev))

    def counts(self):
        """[correct, labeled, inter[C], area_pred[C], area_lab[C]] accumulated so far (numpy)."""
        if self._counts is None:
            return np.zeros(2 + 3 * self.nclass, dtype=np.int64)
        return self._counts.cpu().numpy()

    def get(self):
        c = self.counts()
        n = self.nclass
        inter, area_pred, area_lab = c[2:2 + n], c[2 + n:2 + 2 * n], c[2 + 2 * n:]
        union = area_pred + area_lab - inter
        pix_acc = 1.0 * c[0] / (np.spacing(1) + c[1])
        iou = 1.0 * inter / (np.spacing(1) + union)
        return pix_acc, iou.mean()
