"""Parity of the code paths that only run at the literal BASELINE.json sizes.

* The deep-K streaming dgrad (``gemm_stream.hip`` ``gemm_stream_ok``: 16-bit, K = 384 / 512 / 576,
  M >= 131072) runs in a cfg3 step only as bottleneck1.0's expand dgrad (M = 8 x 128 x 256,
  K = 384, N = 64), with that BN's backward partial sums and in-kernel finish (mode 2: the BN of
  LearningToDownsample.dsconv2.pw feeds a ReLU; models/fast_scnn.py:103-104,160 autograd).  It is
  called here through the C ABI in exactly the executor's form (``fscnn_pw_dgrad_bnbwd`` =
  net.cpp ``Exec::pw_bwd`` + ``set_btarget``) and checked against a torch fp32 restatement: the
  stored dX, and dbeta / dgamma / the apply coefficients recomputed in fp64 from the stored dX.
* cfg2 at its literal batch (8 x 3 x 1024 x 2048 fp32, eval): every image's logits against its
  own batch-1 forward (the bs = 8 launches use other grids: the streaming GEMMs' chunking and
  8x the fused-block tiles), image 0 (the cfg2 golden input) against the golden + fp64 argmax
  contract of tests/test_gpu_fullsize.py, image 7 against the fp64 oracle.
"""
import numpy as np
import pytest
import torch

from fast_scnn_pytorch_amd import _lib, portable_init
from helpers import golden_input, golden_sd, load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rnd(shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * (hi - lo) + lo)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K,mode,res,deep", [
    (262144, 64, 384, 2, True, True),    # bottleneck1.0 expand dgrad at cfg3 (+ FFM's gx)
    (262144, 64, 384, 0, False, True),   # no-ReLU BN target
    (200003, 64, 384, 2, False, True),   # ragged M (partial last chunk)
    (131072, 96, 576, 2, True, True),    # ks = 18
    (131075, 64, 384, 0, True, True),    # ragged, no-ReLU target, residual
    (131072, 64, 512, 2, True, False),   # ks = 16 at N = 64 would spill: the tiled kernel
    (65536, 64, 384, 2, True, False),    # below the deep-K threshold: the tiled kernel
])
def test_pw_dgrad_bnbwd_executor_form(dt, M, N, K, mode, res, deep):
    """dX = D . W^T (+R) stored in 16 bits, and the BN-backward sums of the stored dX."""
    torch.manual_seed(0)
    D = _rnd((M, K), 1).to(dt).to(DEV)
    W = (_rnd((N, K), 2) / K ** 0.5).to(dt).to(DEV)          # transposed weight [N][K]
    R = _rnd((M, N), 3).to(dt).to(DEV) if res else None
    z = (_rnd((M, N), 4) * 2.0 + 0.7).to(dt).to(DEV)          # BN input, mean away from 0
    zf = z.float()
    mean = zf.mean(0)
    invstd = 1.0 / torch.sqrt(zf.var(0, unbiased=False) + 1e-5)
    scale = (_rnd((N,), 5, 0.5, 1.5)).to(DEV) * invstd
    shift = _rnd((N,), 6, -0.5, 0.5).to(DEV) - mean * scale
    dX = torch.empty(M, N, dtype=dt, device=DEV)
    part = torch.full((((M + 127) // 128) * 2 * N,), float("nan"), device=DEV)
    counters = torch.zeros(512, dtype=torch.int32, device=DEV)
    tsum = torch.zeros(32 * 3 * 1024, dtype=torch.float64, device=DEV)
    dgamma, dbeta = torch.empty(N, device=DEV), torch.empty(N, device=DEV)
    coef = torch.empty(2 * N, device=DEV)
    path = _lib.c_int(-1)
    _lib.call("fscnn_pw_dgrad_bnbwd", M, N, K, _lib.ptr(D), K, _lib.ptr(W), K, _lib.ptr(R), N,
              _lib.ptr(dX), N, _lib.ptr(z), N, _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(scale),
              _lib.ptr(shift), mode, _lib.ptr(part), _lib.ptr(counters), _lib.ptr(tsum),
              _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(coef), _lib.dtype_code(dt),
              _lib.ctypes.byref(path), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert path.value == (1 if deep else 0), "expected the %s kernel" % ("deep-K streaming" if deep else "tiled")
    # (1) dX: fp32 accumulation rounded once to the storage type
    ref = D.float() @ W.float().t()
    if res:
        ref += R.float()
    ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    err = (dX.float() - ref).abs()
    bound = ulp * ref.abs() + 1e-5 * ref.abs().max()
    assert bool((err <= bound).all()), "dX: max err %.3e" % err.max().item()
    # (2) BN backward of the STORED dX (fp64 over the same fp32 terms the kernel forms)
    g = dX.double()
    if mode == 2:
        mask = (z.double() * scale.double() + shift.double()) > 0   # = fmaf(z, scale, shift) > 0
    else:
        mask = torch.ones_like(g, dtype=torch.bool)
    gm = torch.where(mask, g, torch.zeros_like(g))
    xhat = ((zf - mean) * invstd).double()
    s1 = gm.sum(0)
    s2 = (gm * xhat).sum(0)
    a1 = gm.abs().sum(0)
    a2 = (gm * xhat).abs().sum(0)
    assert bool(((dbeta.double() - s1).abs() <= 2e-6 * a1 + 1e-6).all()), \
        "dbeta: max err %.3e" % (dbeta.double() - s1).abs().max().item()
    assert bool(((dgamma.double() - s2).abs() <= 2e-6 * a2 + 1e-6).all()), \
        "dgamma: max err %.3e" % (dgamma.double() - s2).abs().max().item()
    torch.testing.assert_close(coef[:N].double(), (dbeta.double() / M), rtol=1e-6, atol=0)
    torch.testing.assert_close(coef[N:].double(), (dgamma.double() / M), rtol=1e-6, atol=0)
    # the in-kernel finish leaves its counters zero for the next producer
    assert int(counters.abs().sum().item()) == 0


def test_cfg2_literal_batch8_matches_batch1():
    """cfg2 as BASELINE.json states it: bs = 8, fp32, eval; image 0 is the cfg2 golden input.

    The batch-8 forward is not bit-identical to batch 1 by design: the fused inference
    bottleneck (ir.hip) runs only when a block's map gives >= 128 tiles, so bottleneck3 is one
    launch at bs = 8 (256 tiles) and three at bs = 1 (32 tiles); both evaluate every product as
    six bf16 MFMAs of exact fp32 splits, but in a different k order (measured: max |d| 1.0e-5 on
    the logits, no image bit-identical).  Gate: image 0 of the batch meets the golden + fp64
    contract (1e-4, argmax bit-exact off near-ties); image 7 is within 1e-4 of the fp64 oracle;
    every image is within 1e-4 of its own batch-1 forward and its argmax differs only where the
    batch-1 top-2 margin is < 1e-4."""
    from models.fast_scnn import FastSCNN
    from oracle import fast_scnn_ref as ref
    from test_gpu_fullsize import _check_argmax, _oracle64
    g = load_golden("cfg2_c19_1024x2048")
    m = FastSCNN(19)
    sd = golden_sd(g)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x0 = golden_input(g)
    assert tuple(x0.shape) == (1, 3, 1024, 2048)
    xs = [x0] + [torch.from_numpy(portable_init.input_tensor(100 + i, (1, 3, 1024, 2048)))
                 for i in range(7)]
    x8 = torch.cat(xs).to(DEV)
    with torch.no_grad():
        o8 = m(x8)[0]
        worst, exact = 0.0, 0
        for i in range(8):
            o1 = m(x8[i:i + 1])[0]
            d = (o8[i:i + 1] - o1).abs().max().item()
            worst = max(worst, d)
            exact += int(torch.equal(o8[i:i + 1], o1))
            srt = torch.sort(o1, dim=1).values
            margin = srt[:, -1] - srt[:, -2]
            flips = (o8[i:i + 1].argmax(1) != o1.argmax(1)) & (margin > 1e-4)
            assert int(flips.sum()) == 0, "image %d: %d confident argmax flips" % (i, int(flips.sum()))
        o0 = o8[0:1].float().cpu()
        o7 = o8[7:8].float().cpu()
    print("cfg2 bs=8 vs bs=1: %d of 8 images bit-identical, max |d| %.2e" % (exact, worst))
    assert worst <= 1e-4
    np.testing.assert_allclose(o0.numpy().ravel()[g["out0.sample_idx"]], g["out0.sample_val"],
                               rtol=0, atol=1e-4)
    _check_argmax(o0, g, _oracle64(g, 19))
    with torch.no_grad():
        o64 = ref.forward({k: v.double() if v.is_floating_point() else v for k, v in sd.items()},
                          xs[7].double(), 19)[0][0]
    d7 = (o7.double() - o64).abs().max().item()
    print("cfg2 bs=8 image 7 vs fp64 oracle: max |d| %.2e" % d7)
    assert d7 < 1e-4


def _low_res(n):
    """Spatial size of the 1/8-resolution logits (conv0 k3 s2 p0, then two stride-2 3x3 p1)."""
    n = (n - 3) // 2 + 1
    n = (n - 1) // 2 + 1
    return (n - 1) // 2 + 1


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nc,N,H,W,ign", [
    (19, 2, 256, 512, -1),    # one column chunk, int8 targets (4-row ring)
    (19, 2, 64, 2112, -1),    # Wl = 264: two column chunks (carry), W > 2048: int64 targets
    (2, 2, 128, 256, -1),     # the TuSimple class count
    (19, 2, 64, 260, -1),     # W % 8 != 0: int64 targets staged per row; odd low-res width
    (19, 2, 128, 256, 255),   # another ignore_index (the int8 pack's validity test)
])
def test_fused_ce_head_16bit_vs_fp64(dt, nc, N, H, W, ign):
    """The 16-bit fused loss head (head.hip ce_head2_kernel: row-factored accumulation, target
    one-hots in LDS) against autograd in fp64 on the SAME low-res logits the forward stored:
    bilinear align_corners upsample (models/fast_scnn.py:51) + nn.CrossEntropyLoss(ignore_index=-1)
    (utils/loss.py:103-124).  Loss to 1e-5; dlogits to one 16-bit rounding of the fp32 sum."""
    import torch.nn.functional as F
    from models.fast_scnn import FastSCNN
    torch.manual_seed(7)
    m = FastSCNN(nc).to(DEV).train()
    m._dropout_seed = 3
    m._keep_ws = True
    x = _rnd((N, 3, H, W), 11).to(DEV).to(dt)
    t = (_rnd((N, H, W), 12, 0, nc).floor().long()).clamp_(0, nc - 1)
    drop = _rnd((N, H, W), 13, 0, 1) < 0.05
    t[drop] = ign
    t[:, 5:9, :] = ign          # whole ignored rows
    t = t.to(DEV)
    loss = m.forward_loss(x, t, ignore_index=ign)
    loss.backward()
    torch.cuda.synchronize()
    Hl, Wl = _low_res(H), _low_res(W)
    L = m.debug_buffer("logits").double().view(N, Hl, Wl, nc).permute(0, 3, 1, 2).clone()
    G = m.debug_buffer("g_logits").double().view(N, Hl, Wl, nc).permute(0, 3, 1, 2)
    L.requires_grad_(True)
    up = F.interpolate(L, (H, W), mode="bilinear", align_corners=True)
    lref = F.cross_entropy(up, t, ignore_index=ign)
    lref.backward()
    gref = L.grad
    assert abs(loss.item() - lref.item()) <= 1e-5 * abs(lref.item()), (loss.item(), lref.item())
    ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    err = (G - gref).abs()
    # f16 stores |g| < 2^-14 as subnormals (spacing 2^-24): unscaled CE gradients at this pixel
    # count are ~3e-5, so one f16 rounding is up to half that spacing (GradScaler lifts them)
    sub = 2.0 ** -24 if dt == torch.float16 else 0.0
    bound = ulp * gref.abs() + 2e-5 * gref.abs().max() + sub
    assert bool((err <= bound).all()), "dlogits: max err %.3e (max |g| %.3e)" % (
        err.max().item(), gref.abs().max().item())
