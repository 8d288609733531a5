"""Cross-entropy criterion on the HIP path (the consumer of the logits in train.py:270-271).

``SoftmaxCrossEntropyOHEMLoss`` / ``MixSoftmaxCrossEntropyOHEMLoss`` mirror utils/loss.py:127-206
(train.py's ``--loss-type ce`` criterion, train.py:190-191): the label probabilities, the OHEM
threshold (k-th smallest label probability by a radix select when fewer than ``min_kept`` pixels
fall under ``thresh``) and the class-weighted CE over the kept pixels all run on the device with
no host synchronisation, where the reference copies the whole logits tensor to numpy.

``MixSoftmaxCrossEntropyLoss`` mirrors utils/loss.py:103-124 (``nn.CrossEntropyLoss`` with
``ignore_index=-1`` over a tuple of predictions, aux terms weighted by ``aux_weight``).  One
fused kernel computes log-softmax + NLL per pixel with fixed-order partial sums; the backward
recomputes the softmax and writes ``(softmax - onehot) * grad / count`` in one pass.
"""
import ctypes
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib


# Targets outside [0, C) other than ignore_index: nn.CrossEntropyLoss raises (IndexError on the
# CPU, a device assert on CUDA).  The kernels here treat them as ignored, which keeps the step free
# of host synchronisation; FSCNN_CHECK_TARGETS=1 (or CHECK_TARGETS = True) adds the reference's
# failure as one device reduction + host read per loss call (a debugging aid: it syncs).
CHECK_TARGETS = os.environ.get("FSCNN_CHECK_TARGETS", "0") == "1"


def check_targets(target, num_classes, ignore_index):
    """Raise IndexError like aten's nll_loss if a target is neither ignore_index nor in
    [0, num_classes)."""
    bad = (target != ignore_index) & ((target < 0) | (target >= num_classes))
    if bool(bad.any()):
        v = int(target[bad].flatten()[0])
        raise IndexError("Target %d is out of bounds." % v)


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        if not logits.is_cuda:
            raise RuntimeError("fused cross entropy needs ROCm device tensors")
        if logits.dim() != 4 or target.dim() != 3:
            raise RuntimeError("expected logits [N,C,H,W] and target [N,H,W]")
        logits = logits.contiguous()
        target = target.to(torch.int64).contiguous()
        N, C, H, W = logits.shape
        if CHECK_TARGETS:
            check_targets(target, C, ignore_index)
        HW = H * W
        parts = int(_lib.load().fscnn_ce_parts(N, HW))
        part = torch.empty(parts * 2, dtype=torch.float32, device=logits.device)
        out2 = torch.empty(2, dtype=torch.float32, device=logits.device)
        _lib.call("fscnn_ce_fwd", _lib.ptr(logits), _lib.dtype_code(logits.dtype), _lib.ptr(target),
                  N, C, HW, int(ignore_index), _lib.ptr(part), _lib.ptr(out2),
                  _lib.stream_ptr(logits.device))
        ctx.save_for_backward(logits, target, out2)
        ctx.ignore_index = int(ignore_index)
        return out2[0].clone()

    @staticmethod
    def backward(ctx, grad):
        logits, target, out2 = ctx.saved_tensors
        N, C, H, W = logits.shape
        g = grad.to(torch.float32).reshape(1).contiguous()
        dlogits = torch.empty_like(logits)
        _lib.call("fscnn_ce_bwd", _lib.ptr(logits), _lib.dtype_code(logits.dtype), _lib.ptr(target),
                  N, C, H * W, ctx.ignore_index, _lib.ptr(g), _lib.ptr(out2), _lib.ptr(dlogits),
                  _lib.stream_ptr(logits.device))
        return dlogits, None, None


def cross_entropy(logits, target, ignore_index=-1):
    return _CrossEntropyFn.apply(logits, target, ignore_index)


class MixSoftmaxCrossEntropyLoss(nn.Module):
    """utils/loss.py:103-124 on the HIP path."""

    def __init__(self, aux=True, aux_weight=0.2, ignore_label=-1, **kwargs):
        super().__init__()
        self.aux = aux
        self.aux_weight = aux_weight
        self.ignore_index = ignore_label

    def forward(self, *inputs, **kwargs):
        preds, target = tuple(inputs)
        if isinstance(preds, torch.Tensor):
            preds = (preds,)
        loss = cross_entropy(preds[0], target, self.ignore_index)
        if self.aux:
            for p in preds[1:]:
                loss = loss + self.aux_weight * cross_entropy(p, target, self.ignore_index)
        return loss


# utils/loss.py:134-136 (use_weight=True)
OHEM_CLASS_WEIGHT = (0.8373, 0.918, 0.866, 1.0345, 1.0166, 0.9969, 0.9754, 1.0489, 0.8786, 1.0023,
                     0.9539, 0.9843, 1.1116, 0.9037, 1.0865, 1.0955, 1.0865, 1.1529, 1.0507)


def ohem_threshold(logits, target, ignore_index, thresh, min_kept):
    """(prob, threshold) of SoftmaxCrossEntropyOHEMLoss.forward (utils/loss.py:151-170): prob of
    the label per pixel and the float32 threshold a pixel's prob must not exceed to be kept (inf:
    every labelled pixel), both on the device.  The counters and the k-th-smallest radix select
    never leave the device, so the step has no host synchronisation (the reference's
    ``print('Labels: ...')`` on the keep-all branch, which would need one, is not reproduced)."""
    N, C, H, W = logits.shape
    HW = H * W
    dev = logits.device
    st = _lib.stream_ptr(dev)
    prob = torch.empty(N * HW, dtype=torch.float32, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    work = torch.empty(2056, dtype=torch.int32, device=dev)
    thr = torch.empty(1, dtype=torch.float32, device=dev)
    thr32 = float(np.float32(thresh))
    _lib.call("fscnn_ohem_prob", _lib.ptr(logits), _lib.dtype_code(logits.dtype), _lib.ptr(target),
              N, C, HW, int(ignore_index), ctypes.c_float(thr32), _lib.ptr(prob), _lib.ptr(counts),
              st)
    _lib.call("fscnn_ohem_threshold", _lib.ptr(prob), prob.numel(), _lib.ptr(counts),
              int(min_kept), ctypes.c_float(thr32), _lib.ptr(work), _lib.ptr(thr), st)
    return prob, thr


class _OhemCrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, thresh, min_kept, weight):
        if not logits.is_cuda:
            raise RuntimeError("OHEM cross entropy needs ROCm device tensors")
        logits = logits.contiguous()
        target = target.to(device=logits.device, dtype=torch.int64).contiguous()
        N, C, H, W = logits.shape
        if weight is not None and weight.numel() != C:
            raise RuntimeError("weight tensor should be defined either for all %d classes or no "
                               "classes but got weight tensor of shape: [%d]" % (C, weight.numel()))
        if CHECK_TARGETS:
            check_targets(target, C, ignore_index)
        prob, thr = ohem_threshold(logits, target, ignore_index, thresh, min_kept)
        parts = int(_lib.load().fscnn_ce_parts(N, H * W))
        part = torch.empty(parts * 2, dtype=torch.float32, device=logits.device)
        out2 = torch.empty(2, dtype=torch.float32, device=logits.device)
        wp = _lib.ptr(weight) if weight is not None else None
        _lib.call("fscnn_ce_weighted_fwd", _lib.ptr(logits), _lib.dtype_code(logits.dtype),
                  _lib.ptr(target), N, C, H * W, int(ignore_index), wp, _lib.ptr(prob),
                  _lib.ptr(thr), _lib.ptr(part), _lib.ptr(out2),
                  _lib.stream_ptr(logits.device))
        ctx.save_for_backward(logits, target, prob, out2, thr)
        ctx.weight, ctx.ignore_index = weight, int(ignore_index)
        return out2[0].clone()

    @staticmethod
    def backward(ctx, grad):
        logits, target, prob, out2, thr = ctx.saved_tensors
        N, C, H, W = logits.shape
        g = grad.to(torch.float32).reshape(1).contiguous()
        dlogits = torch.empty_like(logits)
        wp = _lib.ptr(ctx.weight) if ctx.weight is not None else None
        _lib.call("fscnn_ce_weighted_bwd", _lib.ptr(logits), _lib.dtype_code(logits.dtype),
                  _lib.ptr(target), N, C, H * W, ctx.ignore_index, wp, _lib.ptr(prob),
                  _lib.ptr(thr), _lib.ptr(g), _lib.ptr(out2), _lib.ptr(dlogits),
                  _lib.stream_ptr(logits.device))
        return dlogits, None, None, None, None, None


class SoftmaxCrossEntropyOHEMLoss(nn.Module):
    """utils/loss.py:127-176 on the HIP path."""

    def __init__(self, ignore_label=-1, thresh=0.7, min_kept=256, use_weight=True, **kwargs):
        super().__init__()
        self.ignore_label = ignore_label
        self.thresh = float(thresh)
        self.min_kept = int(min_kept)
        if use_weight:
            print("w/ class balance")
            self.weight = torch.tensor(OHEM_CLASS_WEIGHT, dtype=torch.float32)
        else:
            print("w/o class balance")
            self.weight = None

    def forward(self, predict, target, weight=None):
        assert not target.requires_grad
        assert predict.dim() == 4
        assert target.dim() == 3
        assert predict.size(0) == target.size(0)
        assert predict.size(2) == target.size(1)
        assert predict.size(3) == target.size(2)
        w = None
        if self.weight is not None:
            if self.weight.device != predict.device:  # once: later steps do no H2D copy
                self.weight = self.weight.to(predict.device)
            w = self.weight
        return _OhemCrossEntropyFn.apply(predict, target, self.ignore_label, self.thresh,
                                         self.min_kept, w)


class MixSoftmaxCrossEntropyOHEMLoss(SoftmaxCrossEntropyOHEMLoss):
    """utils/loss.py:179-206 on the HIP path."""

    def __init__(self, aux=False, aux_weight=0.2, ignore_index=-1, **kwargs):
        super().__init__(ignore_label=ignore_index, **kwargs)
        self.aux = aux
        self.aux_weight = aux_weight

    def forward(self, *inputs, **kwargs):
        preds, target = tuple(inputs)
        if isinstance(preds, torch.Tensor):
            preds = (preds,)
        loss = super().forward(preds[0], target)
        if self.aux:
            for p in preds[1:]:
                loss = loss + self.aux_weight * super().forward(p, target)
        return loss


# ---- Dice / Focal + Dice (utils/loss.py:12-100; train.py:183-188) ----------------------------
class _DiceFocalFn(torch.autograd.Function):
    """dice_weight * (1 - dice) + focal_weight * mean(focal) of one prediction (one kernel for the
    per-pixel terms, fixed-order fp64 sums)."""

    @staticmethod
    def forward(ctx, pred, target, smooth, dice_weight, focal_weight, alpha, gamma):
        if not pred.is_cuda:
            raise RuntimeError("Dice loss needs ROCm device tensors")
        if pred.dim() != 4:
            raise RuntimeError("Dice loss: expected logits [N, C, H, W]")
        pred = pred.contiguous()
        target = target.to(device=pred.device, dtype=torch.int64).contiguous()
        N, C, H, W = pred.shape
        if target.numel() != N * H * W:
            raise RuntimeError("Dice loss: target %s does not match %s"
                               % (tuple(target.shape), tuple(pred.shape)))
        focal = 1 if focal_weight != 0.0 else 0
        parts = int(_lib.load().fscnn_ce_parts(N, H * W))
        part = torch.empty(parts * 4, dtype=torch.float32, device=pred.device)
        stats = torch.empty(4, dtype=torch.float64, device=pred.device)
        _lib.call("fscnn_dice_fwd", _lib.ptr(pred), _lib.dtype_code(pred.dtype), _lib.ptr(target),
                  N, C, H * W, ctypes.c_float(alpha), ctypes.c_float(gamma), focal, _lib.ptr(part),
                  _lib.ptr(stats), _lib.stream_ptr(pred.device))
        dice = (2.0 * stats[0] + smooth) / (stats[1] + stats[2] + smooth)
        loss = dice_weight * (1.0 - dice) + focal_weight * stats[3] / float(N * H * W)
        ctx.save_for_backward(pred, target, stats)
        ctx.args = (float(smooth), float(dice_weight), float(focal_weight), float(alpha),
                    float(gamma), focal)
        return loss.to(torch.float32)

    @staticmethod
    def backward(ctx, grad):
        pred, target, stats = ctx.saved_tensors
        smooth, dw, fw, alpha, gamma, focal = ctx.args
        N, C, H, W = pred.shape
        g = grad.to(torch.float32).reshape(1).contiguous()
        dpred = torch.empty_like(pred)
        _lib.call("fscnn_dice_bwd", _lib.ptr(pred), _lib.dtype_code(pred.dtype), _lib.ptr(target),
                  N, C, H * W, ctypes.c_float(alpha), ctypes.c_float(gamma), focal,
                  _lib.ptr(stats), _lib.ptr(g), ctypes.c_float(smooth), ctypes.c_float(dw),
                  ctypes.c_float(fw), _lib.ptr(dpred), _lib.stream_ptr(pred.device))
        return dpred, None, None, None, None, None, None


class DiceLoss(nn.Module):
    """utils/loss.py:12-39 on the HIP path."""

    def __init__(self, smooth=1e-6, **kwargs):
        super().__init__()
        self.smooth = smooth

    def forward(self, pred, target):
        return _DiceFocalFn.apply(pred, target, self.smooth, 1.0, 0.0, 0.5, 2.0)


class MixDiceLoss(nn.Module):
    """utils/loss.py:42-68 on the HIP path."""

    def __init__(self, aux=True, aux_weight=0.4, smooth=1e-6, **kwargs):
        super().__init__()
        self.aux = aux
        self.aux_weight = aux_weight
        self.dice_loss = DiceLoss(smooth=smooth)

    def forward(self, preds, target):
        if isinstance(preds, tuple):
            loss = self.dice_loss(preds[0], target)
            if self.aux and len(preds) > 1:
                loss = loss + self.aux_weight * self.dice_loss(preds[1], target)
            return loss
        return self.dice_loss(preds, target)


class FocalDiceLoss(nn.Module):
    """utils/loss.py:71-100 on the HIP path (multi-class logits, C > 1)."""

    def __init__(self, alpha=0.5, gamma=2.0, dice_weight=0.5, smooth=1e-6, **kwargs):
        super().__init__()
        self.alpha = alpha
        self.gamma = gamma
        self.dice_weight = dice_weight
        self.smooth = smooth

    def forward(self, pred, target):
        return _DiceFocalFn.apply(pred, target, self.smooth, self.dice_weight,
                                  1.0 - self.dice_weight, self.alpha, self.gamma)
