"""Cross-entropy criterion on the HIP path (the consumer of the logits in train.py:270-271).

``MixSoftmaxCrossEntropyLoss`` mirrors utils/loss.py:103-124 (``nn.CrossEntropyLoss`` with
``ignore_index=-1`` over a tuple of predictions, aux terms weighted by ``aux_weight``).  One
fused kernel computes log-softmax + NLL per pixel with fixed-order partial sums; the backward
recomputes the softmax and writes ``(softmax - onehot) * grad / count`` in one pass.
"""
import torch
import torch.nn as nn

from . import _lib


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
