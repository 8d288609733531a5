"""Fused inference LearningToDownsample stem (csrc/stem.hip; models/fast_scnn.py:153-154) through
the C ABI (``fscnn_block_ltd_fwd``) against a plain PyTorch fp32 restatement: conv 3x3 s2 p0 ->
folded BN -> ReLU -> depthwise 3x3 s2 p1 -> folded BN -> ReLU -> 1x1 conv (32 -> 48) -> folded
BN -> ReLU.

fp32: conv0 runs on exact fp32 MFMA, the pointwise on the six-product bf16 split (fp32 products):
only the summation order differs (2e-5 of the output magnitude).  bf16 / fp16: the restatement
rounds the conv0 operands, conv0's output, the depthwise output and the pointwise weights to the
storage type exactly where the HIP path does, so the difference is accumulation order plus the
final rounding.  Shapes: cfg5's 480 x 640 slice, ragged maps (partial 31-column strips and
16-row segments), a
16-bit image, an output row stride larger than 48.  Bit-identity with the three unfused
launches: tests/test_gpu_switches.py::test_stem_fused_bit_identical.
"""
import pytest
import torch
import torch.nn.functional as F

from fast_scnn_pytorch_amd import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


def _stem_ref(x, w0, wd, wp, bn, dt):
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (s0, h0), (sd, hd), (sp, hp) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    a = q(F.relu(F.conv2d(q(x), q(w0), stride=2) * c(s0) + c(h0)))
    d = q(F.relu(F.conv2d(a, wd.reshape(32, 1, 3, 3), stride=2, padding=1, groups=32) * c(sd)
                 + c(hd)))
    return F.relu(F.conv2d(d, q(wp)[:, :, None, None]) * c(sp) + c(hp))


CASES = [  # (N, H, W, x dtype, ldy)
    (2, 120, 160, torch.float32, 48),
    (1, 101, 132, torch.float32, 48),   # H2 = 25, W2 = 33: partial tiles in both axes
    (2, 64, 96, torch.bfloat16, 48),    # 16-bit image (16-B vectors of 8)
    (1, 70, 104, torch.float16, 64),    # row stride > 48
    (1, 270, 520, torch.bfloat16, 48),  # 5 strips (16-bit image vectors at both alignments) x
                                        # 5 row segments, the last partial
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,xdt,ldy", CASES)
def test_ltd_stem_fwd_vs_torch(dt, N, H, W, xdt, ldy):
    x = rnd(N, 3, H, W, seed=1).to(xdt).float()
    w0 = rnd(32, 3, 3, 3, seed=2, scale=0.4)
    wd = rnd(32, 9, seed=3, scale=0.4)
    wp = rnd(48, 32, seed=4, scale=1.0 / 32 ** 0.5)
    bn = [(rnd(c, seed=10 + i) * 0.5 + 1.0, rnd(c, seed=20 + i) * 0.2)
          for i, c in enumerate((32, 32, 48))]
    ref = _stem_ref(x, w0, wd, wp, bn, dt)
    H2, W2 = ref.shape[2:]
    xd = x.to(xdt).to(DEV).contiguous()
    dev = [t.to(DEV).contiguous() for t in (w0, wd)]
    wpd = wp.to(dt).to(DEV).contiguous()
    bnd = [(s.to(DEV), h.to(DEV)) for s, h in bn]
    y = torch.full((N, H2, W2, ldy), float("nan"), dtype=dt, device=DEV)
    _lib.call("fscnn_block_ltd_fwd", _lib.ptr(xd), _lib.dtype_code(xdt), _lib.dtype_code(dt),
              N, H, W, _lib.ptr(dev[0]), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]),
              _lib.ptr(dev[1]), _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(wpd),
              _lib.ptr(bnd[2][0]), _lib.ptr(bnd[2][1]), _lib.ptr(y), ldy, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y[..., :48].float().cpu().permute(0, 3, 1, 2)
    if ldy > 48:  # the padding columns are not written
        assert torch.isnan(y[..., 48:].float()).all()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -7 * scale
    assert err <= tol, (err, tol, scale)
    if dt != torch.float32:  # at most a few elements off by more than one output rounding
        far = ((got - ref).abs() > 2 ** -8 * ref.abs() + 1e-3 * scale).float().mean().item()
        assert far < 1e-3, far


def test_ltd_stem_rejects_unaligned_width():
    x = torch.zeros(1, 3, 34, 66, device=DEV)  # W % 4 != 0 for fp32 16-B vectors
    w = torch.zeros(48 * 32, device=DEV)
    y = torch.zeros(1, 8, 16, 48, device=DEV)
    rc = _lib.load().fscnn_block_ltd_fwd(_lib.ptr(x), 0, 0, 1, 34, 66, *([_lib.ptr(w)] * 9),
                                         _lib.ptr(y), 48, _lib.stream_ptr())
    assert rc != 0
