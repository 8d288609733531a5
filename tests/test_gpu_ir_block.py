"""Fused LinearBottleneck, inference (csrc/ir.hip; models/fast_scnn.py:95-115) through the C ABI
(``fscnn_block_ir_fwd``, stride 1; ``fscnn_block_ir_s2_fwd``, stride 2) against a plain PyTorch fp32 restatement of the same block:
1x1 conv -> folded BN -> ReLU -> depthwise 3x3 (pad 1) -> folded BN -> ReLU -> 1x1 conv ->
folded BN (+ x).

fp32: the six-product bf16 split reproduces fp32 products; only the summation order differs
(tolerance 2e-5 of the output magnitude).  bf16 / fp16: the restatement rounds the block input,
weights, the expand output and the depthwise output to the storage type exactly where the HIP
path stores them, so the remaining difference is accumulation order plus the final rounding.
Shapes: the Fast-SCNN stride-1 blocks (64 -> 384 -> 64, 96 -> 576 -> 96, 96 -> 576 -> 128 without
shortcut, 128 -> 768 -> 128), map sizes that are not multiples of the 8 x 8 tile, and an output
written with a row stride larger than Cout (the PPM concat buffer).
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


def _block_ref(x, we, wd, wp, bn, residual, dt, stride=1):
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (se, he), (sd, hd), (sp, hp) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    e = q(F.relu(F.conv2d(q(x), q(we)[:, :, None, None]) * c(se) + c(he)))
    d = q(F.relu(F.conv2d(e, wd.reshape(-1, 1, 3, 3), stride=stride, padding=1,
                          groups=e.shape[1]) * c(sd) + c(hd)))
    y = F.conv2d(d, q(wp)[:, :, None, None]) * c(sp) + c(hp)
    if residual:
        y = y + q(x)
    return y


CASES = [  # (N, H, W, Cin, Cout, ldy)
    (2, 32, 64, 96, 96, 96),     # bottleneck2.1 / 2.2 at cfg2 scale
    (2, 32, 64, 128, 128, 256),  # bottleneck3.2 writing into the PPM concat (ld 256)
    (3, 15, 20, 96, 128, 128),   # bottleneck3.0 (no shortcut) at cfg5's 15 x 20
    (1, 13, 21, 64, 64, 64),     # bottleneck1.x, ragged tiles
    (2, 9, 7, 128, 128, 128),    # map smaller than a tile in one axis
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,cin,cout,ldy", CASES)
def test_ir_block_fwd_vs_torch(dt, N, H, W, cin, cout, ldy):
    E = 6 * cin
    residual = cin == cout
    x = rnd(N, cin, H, W, seed=1)
    we = rnd(E, cin, seed=2, scale=1.0 / cin ** 0.5)
    wd = rnd(E, 9, seed=3, scale=0.4)
    wp = rnd(cout, E, seed=4, scale=1.0 / E ** 0.5)
    bn = [(rnd(c, seed=5 + 2 * i).abs() + 0.5, rnd(c, seed=6 + 2 * i, scale=0.2))
          for i, c in enumerate((E, E, cout))]
    ref = _block_ref(x, we, wd, wp, bn, residual, dt)
    xd = x.permute(0, 2, 3, 1).contiguous().to(dt).to(DEV)
    y = torch.full((N, H, W, ldy), float("nan"), dtype=dt, device=DEV)
    wed, wpd = we.to(dt).to(DEV), wp.to(dt).to(DEV)
    wdd = wd.to(DEV)
    bnd = [t.to(DEV) for pair in bn for t in pair]
    _lib.call("fscnn_block_ir_fwd", _lib.ptr(xd), cin, _lib.dtype_code(dt), N, H, W, cin, E, cout,
              _lib.ptr(wed), _lib.ptr(wdd), _lib.ptr(wpd), *[_lib.ptr(t) for t in bnd],
              int(residual), _lib.ptr(y), ldy, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    if ldy > cout:  # channels past Cout of each row are not touched
        assert torch.isnan(y[..., cout:].float()).all()
    err = (got - ref).abs().max().item()
    mag = ref.abs().max().item()
    tol = {torch.float32: 2e-5, torch.bfloat16: 1.6e-2, torch.float16: 2.5e-3}[dt]
    print("%s N%d %dx%d %d->%d->%d: max|d| %.3e (|ref| %.3e)" % (dt, N, H, W, cin, E, cout, err, mag))
    assert err <= tol * mag


S2_CASES = [  # (N, H, W, Cin, Cout): input map; output (H-1)//2+1 x (W-1)//2+1
    (2, 32, 64, 64, 64),    # bottleneck1.0 at cfg2 scale / 4
    (2, 16, 32, 64, 96),    # bottleneck2.0
    (1, 30, 40, 64, 96),    # cfg5's bottleneck2.0 input (30 x 40 -> 15 x 20)
    (1, 27, 45, 64, 64),    # odd maps, ragged 4 x 8 output tiles
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,cin,cout", S2_CASES)
def test_ir_block_stride2_vs_torch(dt, N, H, W, cin, cout):
    """The stride-2 form (bottleneck1.0 / 2.0: 4 x 8 output tiles over 9 x 17 input tiles)."""
    E = 6 * cin
    x = rnd(N, cin, H, W, seed=11)
    we = rnd(E, cin, seed=12, scale=1.0 / cin ** 0.5)
    wd = rnd(E, 9, seed=13, scale=0.4)
    wp = rnd(cout, E, seed=14, scale=1.0 / E ** 0.5)
    bn = [(rnd(c, seed=15 + 2 * i).abs() + 0.5, rnd(c, seed=16 + 2 * i, scale=0.2))
          for i, c in enumerate((E, E, cout))]
    ref = _block_ref(x, we, wd, wp, bn, False, dt, stride=2)
    Ho, Wo = ref.shape[2:]
    xd = x.permute(0, 2, 3, 1).contiguous().to(dt).to(DEV)
    y = torch.full((N, Ho, Wo, cout), float("nan"), dtype=dt, device=DEV)
    wed, wpd = we.to(dt).to(DEV), wp.to(dt).to(DEV)
    wdd = wd.to(DEV)
    bnd = [t.to(DEV) for pair in bn for t in pair]
    _lib.call("fscnn_block_ir_s2_fwd", _lib.ptr(xd), cin, _lib.dtype_code(dt), N, H, W, cin, E,
              cout, _lib.ptr(wed), _lib.ptr(wdd), _lib.ptr(wpd), *[_lib.ptr(t) for t in bnd],
              _lib.ptr(y), cout, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs().max().item()
    mag = ref.abs().max().item()
    tol = {torch.float32: 2e-5, torch.bfloat16: 1.6e-2, torch.float16: 2.5e-3}[dt]
    print("s2 %s N%d %dx%d %d->%d->%d: max|d| %.3e (|ref| %.3e)" % (dt, N, H, W, cin, E, cout, err, mag))
    assert err <= tol * mag


def test_ir_block_rejects_unsupported_shapes():
    x = torch.zeros(1, 8, 8, 48, device=DEV)
    y = torch.zeros_like(x)
    z = torch.zeros(1024, device=DEV)
    rc = _lib.load().fscnn_block_ir_fwd(_lib.ptr(x), 48, 0, 1, 8, 8, 48, 288, 48, _lib.ptr(z),
                                         _lib.ptr(z), _lib.ptr(z), *[_lib.ptr(z)] * 6, 1,
                                         _lib.ptr(y), 48, _lib.stream_ptr())
    assert rc == -2  # Cin = 48 is not a multiple of 32
