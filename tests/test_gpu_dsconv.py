"""Fused inference DSConv (csrc/dsconv.hip; models/fast_scnn.py:64-79 _DSConv, the Classifer's
dsconv1 / dsconv2 at :228-231, and the FeatureFusionModule, :200-218) through the C ABI
(``fscnn_block_dsconv_fwd`` / ``_res_fwd``, ``fscnn_block_ffm_fwd``) against a plain
PyTorch fp32 restatement: depthwise 3x3 s1 p1 -> folded BN -> ReLU -> 1x1 conv (128 -> 128) ->
folded BN -> ReLU.

fp32: the depthwise is an fp32 fma chain, the pointwise the six-product bf16 split (fp32
products): only the summation order differs (2e-5 of the output magnitude).  bf16 / fp16: the
restatement rounds the input, the depthwise output and the pointwise weights to the storage type
exactly where the HIP path does, so the difference is accumulation order plus the final
rounding.  Shapes: whole and partial 16-column strips, row segments that do not divide the map,
an output row stride larger than 128.  Bit-identity with the two unfused launches:
tests/test_gpu_switches.py::test_dsconv_fused_bit_identical.
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


def _ref(x, wd, wp, bn, dt):
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (sd, hd), (sp, hp) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    xc = q(x).permute(0, 3, 1, 2)
    d = q(F.relu(F.conv2d(xc, wd.reshape(128, 1, 3, 3), padding=1, groups=128) * c(sd) + c(hd)))
    return F.relu(F.conv2d(d, q(wp)[:, :, None, None]) * c(sp) + c(hp))


CASES = [  # (N, H, W, ldy)
    (2, 24, 48, 128),
    (1, 37, 53, 128),   # partial strip (53 = 3 x 16 + 5), rows not a multiple of the segment
    (1, 9, 16, 136),    # row stride > 128
    (3, 5, 7, 128),     # one partial strip, maps smaller than the window
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,ldy", CASES)
def test_dsconv_fwd_vs_torch(dt, N, H, W, ldy):
    x = rnd(N, H, W, 128, seed=1)
    wd = rnd(128, 9, seed=3, scale=0.4)
    wp = rnd(128, 128, seed=4, scale=1.0 / 128 ** 0.5)
    bn = [(rnd(128, seed=10 + i) * 0.5 + 1.0, rnd(128, seed=20 + i) * 0.2) for i in range(2)]
    ref = _ref(x, wd, wp, bn, dt)
    xd = x.to(dt).to(DEV).contiguous()
    wdd = wd.to(DEV).contiguous()
    wpd = wp.to(dt).to(DEV).contiguous()
    bnd = [(s.to(DEV), h.to(DEV)) for s, h in bn]
    y = torch.full((N, H, W, ldy), float("nan"), dtype=dt, device=DEV)
    _lib.call("fscnn_block_dsconv_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, 128, 128,
              _lib.ptr(wdd), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]), _lib.ptr(wpd),
              _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(y), ldy, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y[..., :128].float().cpu().permute(0, 3, 1, 2)
    if ldy > 128:  # the padding columns are not written
        assert torch.isnan(y[..., 128:].float()).all()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -7 * scale
    assert err <= tol, (err, tol, scale)
    if dt != torch.float32:  # at most a few elements off by more than one output rounding
        far = ((got - ref).abs() > 2 ** -8 * ref.abs() + 1e-3 * scale).float().mean().item()
        assert far < 1e-3, far


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_dsconv_fwd_residual_vs_torch(dt):
    """The FFM form (models/fast_scnn.py:213-218): relu(BN_l(conv_l(relu(BN_d(dw(x))))) + f),
    the residual f read from the output buffer itself (y aliases f, as in the executor)."""
    N, H, W = 2, 19, 37
    x = rnd(N, H, W, 128, seed=5)
    f = rnd(N, H, W, 128, seed=6)
    wd = rnd(128, 9, seed=7, scale=0.4)
    wp = rnd(128, 128, seed=8, scale=1.0 / 128 ** 0.5)
    bn = [(rnd(128, seed=30 + i) * 0.5 + 1.0, rnd(128, seed=40 + i) * 0.2) for i in range(2)]
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (sd, hd), (sp, hp) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    d = q(F.relu(F.conv2d(q(x).permute(0, 3, 1, 2), wd.reshape(128, 1, 3, 3), padding=1,
                          groups=128) * c(sd) + c(hd)))
    ref = F.relu(F.conv2d(d, q(wp)[:, :, None, None]) * c(sp) + c(hp) + q(f).permute(0, 3, 1, 2))
    xd = x.to(dt).to(DEV).contiguous()
    y = f.to(dt).to(DEV).contiguous()
    wdd, wpd = wd.to(DEV).contiguous(), wp.to(dt).to(DEV).contiguous()
    bnd = [(s.to(DEV), h.to(DEV)) for s, h in bn]
    _lib.call("fscnn_block_dsconv_res_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, 128, 128,
              0, 0, _lib.ptr(wdd), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]), _lib.ptr(wpd),
              _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(y), 128, _lib.ptr(y), 128,
              _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -7 * scale
    assert err <= tol, (err, tol, scale)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
@pytest.mark.parametrize("N,Hi,Wi,H,W", [(2, 8, 12, 32, 48), (1, 7, 9, 25, 33), (1, 16, 16, 64, 64)])
def test_dsconv_upsample_residual_vs_torch(dt, N, Hi, Wi, H, W):
    """The whole eval FeatureFusionModule low-res branch (models/fast_scnn.py:207-218):
    relu(BN_l(conv_l(relu(BN_d(dw(up(x)))))) + f) with up = F.interpolate(size (H, W), bilinear,
    align_corners=True) formed in LDS (the unfused path stores it, rounded to the storage type)."""
    x = rnd(N, Hi, Wi, 128, seed=11)
    f = rnd(N, H, W, 128, seed=12)
    wd = rnd(128, 9, seed=13, scale=0.4)
    wp = rnd(128, 128, seed=14, scale=1.0 / 128 ** 0.5)
    bn = [(rnd(128, seed=50 + i) * 0.5 + 1.0, rnd(128, seed=60 + i) * 0.2) for i in range(2)]
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (sd, hd), (sp, hp) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    up = q(F.interpolate(q(x).permute(0, 3, 1, 2), size=(H, W), mode="bilinear",
                         align_corners=True))
    d = q(F.relu(F.conv2d(up, wd.reshape(128, 1, 3, 3), padding=1, groups=128) * c(sd) + c(hd)))
    ref = F.relu(F.conv2d(d, q(wp)[:, :, None, None]) * c(sp) + c(hp) + q(f).permute(0, 3, 1, 2))
    xd = x.to(dt).to(DEV).contiguous()
    y = f.to(dt).to(DEV).contiguous()
    wdd, wpd = wd.to(DEV).contiguous(), wp.to(dt).to(DEV).contiguous()
    bnd = [(s.to(DEV), h.to(DEV)) for s, h in bn]
    _lib.call("fscnn_block_dsconv_res_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, 128, 128,
              Hi, Wi, _lib.ptr(wdd), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]), _lib.ptr(wpd),
              _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(y), 128, _lib.ptr(y), 128,
              _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -7 * scale
    assert err <= tol, (err, tol, scale)



@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,Hi,Wi,H,W,ldh", [(2, 8, 12, 32, 48, 64), (1, 7, 9, 25, 33, 72),
                                             (1, 16, 16, 64, 64, 64)])
def test_ffm_fwd_vs_torch(dt, N, Hi, Wi, H, W, ldh):
    """The whole eval FeatureFusionModule (models/fast_scnn.py:200-218) in one launch
    (``fscnn_block_ffm_fwd``): relu(BN_l(conv_l(relu(BN_d(dw(up(low)))))) + BN_h(conv_h(high)))
    -- the high-res branch is a second GEMM on the same strip, rounded to the storage type where
    the unfused path stores it; partial strips, a high-res row stride above 64."""
    low = rnd(N, Hi, Wi, 128, seed=15)
    high = rnd(N, H, W, ldh, seed=16)
    wd = rnd(128, 9, seed=17, scale=0.4)
    wl = rnd(128, 128, seed=18, scale=1.0 / 128 ** 0.5)
    wh = rnd(128, 64, seed=19, scale=1.0 / 64 ** 0.5)
    bn = [(rnd(128, seed=70 + i) * 0.5 + 1.0, rnd(128, seed=80 + i) * 0.2) for i in range(3)]
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    (sd, hd), (sl, hl), (sh, hh) = bn
    c = lambda t: t[None, :, None, None]  # noqa: E731
    up = q(F.interpolate(q(low).permute(0, 3, 1, 2), size=(H, W), mode="bilinear",
                         align_corners=True))
    d = q(F.relu(F.conv2d(up, wd.reshape(128, 1, 3, 3), padding=1, groups=128) * c(sd) + c(hd)))
    fh = q(F.conv2d(q(high[..., :64]).permute(0, 3, 1, 2), q(wh)[:, :, None, None]) * c(sh) + c(hh))
    ref = F.relu(F.conv2d(d, q(wl)[:, :, None, None]) * c(sl) + c(hl) + fh)
    lowd, highd = low.to(dt).to(DEV).contiguous(), high.to(dt).to(DEV).contiguous()
    wdd = wd.to(DEV).contiguous()
    wld, whd = wl.to(dt).to(DEV).contiguous(), wh.to(dt).to(DEV).contiguous()
    bnd = [(s.to(DEV), h.to(DEV)) for s, h in bn]
    y = torch.full((N, H, W, 128), float("nan"), dtype=dt, device=DEV)
    _lib.call("fscnn_block_ffm_fwd", _lib.ptr(lowd), _lib.dtype_code(dt), N, Hi, Wi, H, W,
              _lib.ptr(highd), ldh, _lib.ptr(wdd), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]),
              _lib.ptr(wld), _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(whd),
              _lib.ptr(bnd[2][0]), _lib.ptr(bnd[2][1]), _lib.ptr(y), 128, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -7 * scale
    assert err <= tol, (err, tol, scale)
    if dt != torch.float32:
        far = ((got - ref).abs() > 2 ** -8 * ref.abs() + 1e-3 * scale).float().mean().item()
        assert far < 1e-3, far


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,ncls,ldl", [(2, 24, 48, 19, 19), (1, 37, 53, 2, 8)])
def test_cls_fwd_vs_torch(dt, N, H, W, ncls, ldl):
    """The whole eval Classifer (models/fast_scnn.py:221-237) through ``fscnn_block_cls_fwd``:
    conv_cls(dsconv2(dsconv1(x))) + bias, dsconv2's output never stored; logits row stride
    above ncls (the padding columns untouched)."""
    x = rnd(N, H, W, 128, seed=21)
    w = [rnd(128, 9, seed=22, scale=0.4), rnd(128, 128, seed=23, scale=128 ** -0.5),
         rnd(128, 9, seed=24, scale=0.4), rnd(128, 128, seed=25, scale=128 ** -0.5)]
    wc = rnd(ncls, 128, seed=26, scale=128 ** -0.5)
    bc = rnd(ncls, seed=27, scale=0.1)
    bn = [(rnd(128, seed=90 + i) * 0.5 + 1.0, rnd(128, seed=95 + i) * 0.2) for i in range(4)]
    q = (lambda t: t) if dt == torch.float32 else (lambda t: t.to(dt).float())  # noqa: E731
    h1 = q(_ref(x, w[0], w[1], bn[0:2], dt)).permute(0, 2, 3, 1)
    h2 = q(_ref(h1, w[2], w[3], bn[2:4], dt))
    ref = F.conv2d(h2, q(wc)[:, :, None, None]) + bc[None, :, None, None]
    xd = x.to(dt).to(DEV).contiguous()
    wd = [w[0].to(DEV), w[1].to(dt).to(DEV), w[2].to(DEV), w[3].to(dt).to(DEV)]
    bnd = [(s_.to(DEV), h_.to(DEV)) for s_, h_ in bn]
    tmp = torch.empty(N, H, W, 128, dtype=dt, device=DEV)
    lg = torch.full((N, H, W, ldl), float("nan"), dtype=dt, device=DEV)
    wcd, bcd = wc.to(dt).to(DEV).contiguous(), bc.to(DEV).contiguous()
    _lib.call("fscnn_block_cls_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W,
              _lib.ptr(wd[0]), _lib.ptr(bnd[0][0]), _lib.ptr(bnd[0][1]), _lib.ptr(wd[1]),
              _lib.ptr(bnd[1][0]), _lib.ptr(bnd[1][1]), _lib.ptr(wd[2]), _lib.ptr(bnd[2][0]),
              _lib.ptr(bnd[2][1]), _lib.ptr(wd[3]), _lib.ptr(bnd[3][0]), _lib.ptr(bnd[3][1]),
              _lib.ptr(wcd), _lib.ptr(bcd), ncls, _lib.ptr(tmp), _lib.ptr(lg), ldl,
              _lib.stream_ptr())
    torch.cuda.synchronize()
    got = lg[..., :ncls].float().cpu().permute(0, 3, 1, 2)
    if ldl > ncls:
        assert torch.isnan(lg[..., ncls:].float()).all()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    tol = 2e-5 * scale if dt == torch.float32 else 2 ** -6 * scale
    assert err <= tol, (err, tol, scale)

def test_dsconv_rejects_other_widths():
    x = torch.zeros(1, 4, 4, 64, device=DEV)
    w = torch.zeros(128 * 128, device=DEV)
    y = torch.zeros(1, 4, 4, 128, device=DEV)
    rc = _lib.load().fscnn_block_dsconv_fwd(_lib.ptr(x), 0, 1, 4, 4, 64, 128,
                                            *([_lib.ptr(w)] * 6), _lib.ptr(y), 128,
                                            _lib.stream_ptr())
    assert rc != 0


def test_ffm_rejects_bad_high_stride():
    """fscnn_block_ffm_fwd needs the high-res rows as whole 16-B vectors (ldhigh >= 64, a multiple
    of 8): anything else is refused (E_UNSUPPORTED), nothing is launched."""
    low = torch.zeros(1, 4, 4, 128, device=DEV)
    high = torch.zeros(1, 16, 16, 64, device=DEV)
    w = torch.zeros(128 * 128, device=DEV)
    y = torch.full((1, 16, 16, 128), 7.0, device=DEV)
    for ldh in (60, 68):
        rc = _lib.load().fscnn_block_ffm_fwd(_lib.ptr(low), 0, 1, 4, 4, 16, 16, _lib.ptr(high), ldh,
                                             *([_lib.ptr(w)] * 9), _lib.ptr(y), 128,
                                             _lib.stream_ptr())
        assert rc != 0
    torch.cuda.synchronize()
    assert (y == 7.0).all()
