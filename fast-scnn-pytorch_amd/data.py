"""GPU input path: what the reference's DataLoader does per image on the
CPU, done for a whole batch on the device.

* ``normalize_images``: ``transforms.ToTensor()`` + ``transforms.Normalize(mean, std)``
  (train.py:104-107, eval.py:22-25, demo.py:37-40) of uint8 HWC RGB images -> NCHW fp32/bf16
  network input, bit-identical to torchvision's fp32 result.
* ``CityscapesLabelMap``: ``CitySegmentation._class_to_index`` (data_loader/cityscapes.py:56-71),
  dataset label ids -> train ids (ignored ids -> -1) through a device lookup table.
"""
import ctypes

import torch

from . import _lib

IMAGENET_MEAN = (.485, .456, .406)
IMAGENET_STD = (.229, .224, .225)

# data_loader/cityscapes.py:58-64 (label id v -> _key[v + 1], v in [-1, 33])
CITYSCAPES_KEY = (-1, -1, -1, -1, -1, -1, -1, -1, 0, 1, -1, -1, 2, 3, 4, -1, -1, -1, 5, -1, 6, 7,
                  8, 9, 10, 11, 12, 13, 14, 15, -1, -1, 16, 17, 18)


def normalize_images(images, mean=IMAGENET_MEAN, std=IMAGENET_STD, dtype=torch.float32):
    """uint8 [N, H, W, 3] (or [H, W, 3]) device tensor -> normalised [N, 3, H, W] ``dtype``."""
    if images.dim() == 3:
        images = images.unsqueeze(0)
    if images.dim() != 4 or images.shape[3] != 3 or images.dtype != torch.uint8:
        raise RuntimeError("normalize_images: expected uint8 [N, H, W, 3], got %s %s"
                           % (images.dtype, tuple(images.shape)))
    if not images.is_cuda:
        raise RuntimeError("normalize_images: the HIP path needs a ROCm device tensor")
    if dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("normalize_images: dtype must be float32 or bfloat16")
    images = images.contiguous()
    N, H, W, _ = images.shape
    out = torch.empty((N, 3, H, W), dtype=dtype, device=images.device)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    _lib.call("fscnn_normalize_u8", _lib.ptr(images), N, H, W, ctypes.cast(m, ctypes.c_void_p),
              ctypes.cast(s, ctypes.c_void_p), _lib.ptr(out), _lib.dtype_code(dtype),
              _lib.stream_ptr(images.device))
    return out


class CityscapesLabelMap:
    """``CitySegmentation._class_to_index`` on the device.

    Like the reference (data_loader/cityscapes.py:66-68 ``assert value in self._mapping``), a
    label id outside the table raises ``AssertionError`` (one device reduction + host read per
    call: this is the data-loading path, where the reference inspects every mask on the CPU).
    ``strict=False`` maps such ids to -1 (ignored) without the check."""

    def __init__(self, key=CITYSCAPES_KEY, offset=1, device="cuda", strict=True):
        self.lut = torch.tensor(key, dtype=torch.int64, device=device)
        self.offset = int(offset)
        self.strict = bool(strict)

    def __call__(self, mask):
        if mask.dtype != torch.uint8 or not mask.is_cuda:
            raise RuntimeError("CityscapesLabelMap: expected a uint8 ROCm device tensor")
        mask = mask.contiguous()
        if self.strict and mask.numel():
            hi = int(mask.max())  # uint8 ids are >= 0 > -offset; valid ids are < len - offset
            assert hi < self.lut.numel() - self.offset, \
                "label id %d is not in the Cityscapes mapping" % hi
        out = torch.empty(mask.shape, dtype=torch.int64, device=mask.device)
        _lib.call("fscnn_remap_labels", _lib.ptr(mask), mask.numel(), _lib.ptr(self.lut),
                  self.lut.numel(), self.offset, -1, _lib.ptr(out), _lib.stream_ptr(mask.device))
        return out
