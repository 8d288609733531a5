"""Per-kernel parity of the HIP library (through the C ABI) against plain PyTorch fp32 CPU ops.

fp32 tolerances are relative to the magnitude of the reference (exact-f32 MFMA / FMA paths differ
from oneDNN only by summation order); bf16 tolerances reflect 8-bit mantissa storage.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from fast_scnn_pytorch_amd import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


def close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-12
    assert err <= tol * ref, "max err %.3e vs tol %.3e (ref max %.3e)" % (err, tol * ref, ref)


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2}
S = _lib.stream_ptr


def sync():
    torch.cuda.synchronize()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 67, 131), (1, 128, 256), (3, 33, 300)])
def test_conv0_fwd(dt, shape):
    N, H, W = shape
    x = rnd(N, 3, H, W, seed=1)
    w = rnd(32, 3, 3, 3, seed=2, scale=0.3)
    sc, sh = rnd(32, seed=3).abs() + 0.5, rnd(32, seed=4)
    ref = F.relu(F.conv2d(x.to(dt).float(), w, stride=2) * sc[None, :, None, None]
                 + sh[None, :, None, None])
    Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    y = torch.empty(N, Ho, Wo, 32, dtype=dt, device=DEV)
    xd = x.to(dt).to(DEV)
    wd, scd, shd = w.to(DEV), sc.to(DEV), sh.to(DEV)
    _lib.call("fscnn_conv0_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, _lib.ptr(wd),
              _lib.ptr(scd), _lib.ptr(shd), 1, _lib.ptr(y), _lib.dtype_code(dt), S())
    sync()
    close(nchw(y), ref, TOL[dt])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 67, 131), (1, 128, 256), (3, 33, 1100), (2, 9, 8)])
def test_conv0_wgrad(dt, shape):
    """MFMA wgrad of the first conv (K = pixels, tiles of 256, tails and multi-segment rows)."""
    N, H, W = shape
    Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    x = rnd(N, 3, H, W, seed=11).to(dt)
    gz = rnd(N, 32, Ho, Wo, seed=12).to(dt)
    xq = x.float().clone()
    wq = torch.zeros(32, 3, 3, 3, requires_grad=True)
    F.conv2d(xq, wq, stride=2).backward(gz.float())
    xd, gzd = x.to(DEV).contiguous(), nhwc(gz).to(DEV)
    slab = torch.empty(_lib.load().fscnn_conv0_wgrad_slab_floats(N, H, W), device=DEV)
    dw = torch.empty(32, 3, 3, 3, device=DEV)
    _lib.call("fscnn_conv0_wgrad", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, _lib.ptr(gzd),
              _lib.dtype_code(dt), _lib.ptr(slab), _lib.ptr(dw), S())
    sync()
    # operands are exactly representable in dt; only the fp32 summation order differs
    close(dw, wq.grad, 1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,C,s", [(2, 17, 23, 32, 1), (2, 17, 23, 48, 2), (1, 64, 128, 384, 2),
                                       (2, 32, 64, 576, 1), (1, 31, 63, 768, 1), (2, 16, 32, 128, 1)])
def test_dw3x3_fwd_bwd(dt, N, H, W, C, s):
    x = rnd(N, C, H, W, seed=5)
    w = rnd(C, 1, 3, 3, seed=6, scale=0.5)
    sc, sh = rnd(C, seed=7).abs() + 0.5, rnd(C, seed=8)
    xq = x.to(dt).float().clone().requires_grad_(True)
    wq = w.clone().requires_grad_(True)
    z = F.conv2d(xq, wq, stride=s, padding=1, groups=C)
    ref = F.relu(z * sc[None, :, None, None] + sh[None, :, None, None])
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    xd = nhwc(x.to(dt)).to(DEV)
    y = torch.empty(N, Ho, Wo, C, dtype=dt, device=DEV)
    wd = w.to(DEV).contiguous()
    scd, shd = sc.to(DEV), sh.to(DEV)
    _lib.call("fscnn_dw3x3_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H, W, C, s, _lib.ptr(wd),
              _lib.ptr(scd), _lib.ptr(shd), 1, _lib.ptr(y), S())
    sync()
    close(nchw(y), ref.detach(), TOL[dt])
    # backward of the raw conv
    gy = rnd(N, C, Ho, Wo, seed=9).to(dt)
    z.backward(gy.float())
    dx = torch.empty(N, H, W, C, dtype=dt, device=DEV)
    gyd = nhwc(gy).to(DEV)
    _lib.call("fscnn_dw3x3_dgrad", _lib.ptr(gyd), _lib.dtype_code(dt), N, H, W, C, s, _lib.ptr(wd),
              _lib.ptr(dx), S())
    nsl = _lib.load().fscnn_dw3x3_wgrad_slab_floats(N, H, W, C, s, _lib.dtype_code(dt))
    slab = torch.empty(nsl, dtype=torch.float32, device=DEV)
    dw = torch.empty(C, 1, 3, 3, dtype=torch.float32, device=DEV)
    _lib.call("fscnn_dw3x3_wgrad", _lib.ptr(xd), _lib.ptr(gyd), _lib.dtype_code(dt), N, H, W, C, s,
              _lib.ptr(slab), _lib.ptr(dw), S())
    sync()
    close(nchw(dx), xq.grad, TOL[dt])
    close(dw, wq.grad, 1e-4 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1000, 48, 32), (4096, 384, 64), (777, 64, 384), (300, 96, 576),
                                   (513, 128, 768), (129, 19, 128), (40, 32, 128), (2048, 128, 256),
                                   (999, 2, 128), (3000, 128, 48), (5000, 576, 96), (2500, 768, 128),
                                   (70001, 128, 128),
                                   # the bottleneck2/3 projects / expand dgrads at cfg3 (M = 16 K)
                                   (16384, 128, 768), (16383, 96, 576), (65536, 64, 384)])
def test_pw_gemm(dt, M, N, K):
    A = rnd(M, K, seed=10)
    B = rnd(N, K, seed=11, scale=1 / math.sqrt(K))
    R = rnd(M, N, seed=12)
    sc, sh = rnd(N, seed=13).abs() + 0.5, rnd(N, seed=14)
    Aq, Bq, Rq = A.to(dt).float(), B.to(dt).float(), R.to(dt).float()
    ref = F.relu((Aq @ Bq.t()) * sc + sh + Rq)
    ldc = (N + 7) // 8 * 8
    C = torch.zeros(M, ldc, dtype=dt, device=DEV)
    Rd = torch.zeros(M, ldc, dtype=dt, device=DEV)
    Rd[:, :N] = R.to(dt).to(DEV)
    Ad, Bd = A.to(dt).to(DEV), B.to(dt).to(DEV)
    scd, shd = sc.to(DEV), sh.to(DEV)
    _lib.call("fscnn_pw_gemm", M, N, K, _lib.ptr(Ad), K, _lib.ptr(Bd), K, 0, _lib.ptr(scd),
              _lib.ptr(shd), _lib.ptr(Rd), ldc, 1, _lib.ptr(C), ldc, None,
              _lib.dtype_code(dt), S())
    sync()
    close(C[:, :N], ref, TOL[dt] * (10 if dt == torch.float32 else 1))
    # dgrad form: dA[M][K] = G[M][N] . B[N][K]  (b_trans reads B as [Kred=N][Nout=K])
    G = rnd(M, N, seed=15)
    Gq = G.to(dt).float()
    ref2 = Gq @ Bq
    ldg = (N + 7) // 8 * 8
    Gd = torch.zeros(M, ldg, dtype=dt, device=DEV)
    Gd[:, :N] = G.to(dt).to(DEV)
    dA = torch.empty(M, K, dtype=dt, device=DEV)
    _lib.call("fscnn_pw_gemm", M, K, N, _lib.ptr(Gd), ldg, _lib.ptr(Bd), K, 1, None, None, None, 0,
              0, _lib.ptr(dA), K, None, _lib.dtype_code(dt), S())
    sync()
    close(dA, ref2, TOL[dt] * (10 if dt == torch.float32 else 1))
    # wgrad: dW[N][K] = G^T . A
    ref3 = Gq.t() @ Aq
    nsl = _lib.load().fscnn_pw_wgrad_slab_floats(M, N, K)
    slab = torch.empty(nsl, dtype=torch.float32, device=DEV)
    dW = torch.empty(N, K, dtype=torch.float32, device=DEV)
    _lib.call("fscnn_pw_wgrad", M, N, K, _lib.ptr(Gd), ldg, _lib.ptr(Ad), K, _lib.ptr(slab),
              _lib.ptr(dW), _lib.dtype_code(dt), S())
    sync()
    close(dW, ref3, 1e-4 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(4099, 128, 128), (300, 128, 64)])
def test_pw_gemm_residual_in_place(dt, M, N, K):
    # FFM eval form (models/fast_scnn.py:217-218): C = relu(A.W^T * sc + sh + C), C read and
    # overwritten in place by the same launch
    A = rnd(M, K, seed=20)
    B = rnd(N, K, seed=21, scale=1 / math.sqrt(K))
    R = rnd(M, N, seed=22)
    sc, sh = rnd(N, seed=23).abs() + 0.5, rnd(N, seed=24)
    Aq, Bq, Rq = A.to(dt).float(), B.to(dt).float(), R.to(dt).float()
    ref = F.relu((Aq @ Bq.t()) * sc + sh + Rq)
    C = R.to(dt).to(DEV).contiguous()
    Ad, Bd = A.to(dt).to(DEV), B.to(dt).to(DEV)
    scd, shd = sc.to(DEV), sh.to(DEV)  # held: raw pointers do not keep tensors alive
    _lib.call("fscnn_pw_gemm", M, N, K, _lib.ptr(Ad), K, _lib.ptr(Bd), K, 0, _lib.ptr(scd),
              _lib.ptr(shd), _lib.ptr(C), N, 1, _lib.ptr(C), N, None,
              _lib.dtype_code(dt), S())
    sync()
    close(C, ref, TOL[dt] * (10 if dt == torch.float32 else 1))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(3001, 96, 64), (20001, 48, 32), (70000, 64, 64),
                                   (16384, 128, 768), (16385, 96, 384)])
def test_gemm_bn_statistics(dt, M, N, K):
    """Tiled (M < 4096: one record per 128-row tile) and streaming (one shifted-sum record per
    workgroup) statistics forms; the call reports how many records it writes."""
    A = rnd(M, K, seed=20) + 3.0  # large mean: catches E[x^2]-E[x]^2 cancellation
    B = rnd(N, K, seed=21, scale=0.2)
    z = A.to(dt).float() @ B.to(dt).float().t()
    slots = (M + 127) // 128
    parts = _lib.load().fscnn_pw_gemm_stats_parts(M, N, K, K, N, _lib.dtype_code(dt))
    assert 1 <= parts <= slots
    part = torch.full((slots * 3 * N,), float("nan"), dtype=torch.float32, device=DEV)
    C = torch.empty(M, N, dtype=dt, device=DEV)
    Ad, Bd = A.to(dt).to(DEV), B.to(dt).to(DEV)
    _lib.call("fscnn_pw_gemm", M, N, K, _lib.ptr(Ad), K, _lib.ptr(Bd),
              K, 0, None, None, None, 0, 0, _lib.ptr(C), N, _lib.ptr(part), _lib.dtype_code(dt), S())
    sync()
    close(C.float(), z, TOL[dt] * (10 if dt == torch.float32 else 1))
    assert torch.isfinite(part[:parts * 3 * N]).all()  # every reported record written
    gamma, beta = (rnd(N, seed=22).abs() + 0.5).to(DEV), rnd(N, seed=23).to(DEV)
    rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    mean, invstd, scale, shift = (torch.empty(N, device=DEV) for _ in range(4))
    _lib.call("fscnn_bn_finalize", _lib.ptr(part), parts, N, _lib.ptr(gamma),
              _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nbt), _lib.c_float(0.1),
              _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(scale), _lib.ptr(shift), S())
    sync()
    tol = 1e-5 if dt == torch.float32 else 2e-3
    close(mean, z.mean(0), tol)
    close(invstd, 1 / torch.sqrt(z.var(0, unbiased=False) + 1e-5), tol * 10)
    close(rm, 0.1 * z.mean(0), tol)
    close(rv, 0.9 + 0.1 * z.var(0, unbiased=True), tol)
    assert int(nbt.item()) == 1


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Hi,Wi,Ho,Wo,C", [(4, 8, 32, 64, 32), (1, 1, 15, 20, 32),
                                           (32, 64, 128, 256, 128), (16, 32, 128, 256, 24),
                                           (15, 20, 60, 80, 8), (6, 6, 32, 64, 32),
                                           (5, 7, 33, 63, 19), (16, 32, 1023, 2046, 19)])
def test_bilinear_ac(dt, Hi, Wi, Ho, Wo, C):
    N = 2
    x = rnd(N, C, Hi, Wi, seed=30)
    xq = x.to(dt).float().clone().requires_grad_(True)
    ref = F.interpolate(xq, (Ho, Wo), mode="bilinear", align_corners=True)
    xd = nhwc(x.to(dt)).to(DEV)
    nhwc_ok = C % 8 == 0  # the NHWC form needs whole 16-B channel vectors
    y = torch.empty(N, Ho, Wo, C, dtype=dt, device=DEV)
    if nhwc_ok:
        _lib.call("fscnn_bilinear_ac_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, Hi, Wi, C, Ho,
                  Wo, _lib.ptr(y), 0, _lib.dtype_code(dt), S())
    y2 = torch.empty(N, C, Ho, Wo, dtype=torch.float32, device=DEV)
    _lib.call("fscnn_bilinear_ac_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, Hi, Wi, C, Ho, Wo,
              _lib.ptr(y2), 1, _lib.DT_F32, S())
    sync()
    if nhwc_ok:
        close(nchw(y), ref.detach(), TOL[dt])
    close(y2, ref.detach(), 1e-5)  # fp32 out: only FMA-contraction / order differences
    y3 = torch.empty(N, C, Ho, Wo, dtype=torch.bfloat16, device=DEV)
    _lib.call("fscnn_bilinear_ac_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, Hi, Wi, C, Ho, Wo,
              _lib.ptr(y3), 1, _lib.DT_BF16, S())
    sync()
    close(y3.float(), ref.detach(), TOL[torch.bfloat16])
    if not nhwc_ok:
        return
    g = rnd(N, C, Ho, Wo, seed=31).to(dt)
    ref.backward(g.float())
    tmp = torch.empty(N * Ho * Wi * C, dtype=torch.float32, device=DEV)
    dx = torch.empty(N, Hi, Wi, C, dtype=dt, device=DEV)
    gd = nhwc(g).to(DEV)
    _lib.call("fscnn_bilinear_ac_bwd", _lib.ptr(gd), _lib.dtype_code(dt), N, Hi, Wi, C,
              Ho, Wo, _lib.ptr(tmp), _lib.ptr(dx), S())
    sync()
    close(nchw(dx), xq.grad, TOL[dt] * 5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,W", [(32, 64), (15, 20), (4, 8), (24, 24), (2, 3)])
def test_pyramid_pool(dt, H, W):
    N, C = 2, 128
    x = rnd(N, C, H, W, seed=40)
    xq = x.to(dt).float().clone().requires_grad_(True)
    refs = [F.adaptive_avg_pool2d(xq, k) for k in (1, 2, 3, 6)]
    pooled = torch.empty(50, N, C, dtype=dt, device=DEV)
    xd = nhwc(x.to(dt)).to(DEV)
    _lib.call("fscnn_pyramid_pool_fwd", _lib.ptr(xd), _lib.dtype_code(dt), N, H,
              W, C, C, _lib.ptr(pooled), S())
    sync()
    base = 0
    gs = []
    for i, k in enumerate((1, 2, 3, 6)):
        got = pooled[base:base + k * k].float().cpu().reshape(k, k, N, C).permute(2, 3, 0, 1)
        close(got, refs[i].detach(), TOL[dt])
        g = rnd(N, C, k, k, seed=41 + i).to(dt).float()
        gs.append(g)
        base += k * k
    sum((r * g).sum() for r, g in zip(refs, gs)).backward()
    gp = torch.cat([g.permute(2, 3, 0, 1).reshape(-1, N, C) for g in gs]).to(dt).to(DEV)
    dx = torch.zeros(N, H, W, C, dtype=dt, device=DEV)
    _lib.call("fscnn_pyramid_pool_bwd", _lib.ptr(gp), _lib.dtype_code(dt), N, H, W, C, _lib.ptr(dx),
              C, 1, S())
    sync()
    close(nchw(dx), xq.grad, TOL[dt] * 5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_cross_entropy(dt):
    from fast_scnn_pytorch_amd.loss import cross_entropy
    N, C, H, W = 2, 19, 33, 65
    x = rnd(N, C, H, W, seed=50, scale=4)
    t = torch.randint(0, C, (N, H, W), generator=torch.Generator().manual_seed(51))
    t[:, ::7, ::5] = -1
    xq = x.to(dt).float().clone().requires_grad_(True)
    ref = F.cross_entropy(xq, t, ignore_index=-1)
    ref.backward()
    xd = x.detach().to(dt).to(DEV).requires_grad_(True)
    loss = cross_entropy(xd, t.to(DEV), -1)
    loss.backward()
    sync()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item()))
    close(xd.grad, xq.grad, 1e-5 if dt == torch.float32 else 1e-2)


def test_sgd():
    n = 10007
    p, g = rnd(n, seed=60), rnd(n, seed=61)
    pd, gd, buf = p.to(DEV), g.to(DEV), torch.empty(n, device=DEV)
    lr, m, wd = 0.01, 0.9, 1e-4
    _lib.call("fscnn_sgd", _lib.ptr(pd), _lib.ptr(gd), _lib.ptr(buf), n, _lib.c_float(lr),
              _lib.c_float(m), _lib.c_float(0.0), _lib.c_float(wd), 0, 1, _lib.c_float(1.0), S())
    d = g + wd * p
    p1 = p - lr * d
    close(pd, p1, 1e-6)
    _lib.call("fscnn_sgd", _lib.ptr(pd), _lib.ptr(gd), _lib.ptr(buf), n, _lib.c_float(lr),
              _lib.c_float(m), _lib.c_float(0.0), _lib.c_float(wd), 0, 0, _lib.c_float(1.0), S())
    sync()
    d2 = g + wd * p1
    b2 = m * d + d2
    close(pd, p1 - lr * b2, 1e-6)
    close(buf, b2, 1e-6)
