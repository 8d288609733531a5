#!/usr/bin/env python3
"""fscnn_block_ffm_fwd against its unfused form (fscnn_pw_gemm for the high-res branch, then
fscnn_block_dsconv_res_fwd with it as the residual): bitwise comparison per dtype.

    python tools/ffm_bitcheck.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import _fscnn_boot

_fscnn_boot.load()
from fast_scnn_pytorch_amd import _lib

DEV = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


for dt in (torch.float32, torch.bfloat16, torch.float16):
    for (N, Hi, Wi, H, W) in [(1, 15, 20, 60, 80), (2, 8, 16, 32, 64)]:
        M = N * H * W
        dc = _lib.dtype_code(dt)
        low = rnd(N, Hi, Wi, 128, seed=1).to(dt).to(DEV)
        high = rnd(N, H, W, 64, seed=2).to(dt).to(DEV)
        wd = rnd(128, 9, seed=3, scale=0.4).to(DEV)
        wl = rnd(128, 128, seed=4, scale=128 ** -0.5).to(dt).to(DEV)
        wh = rnd(128, 64, seed=5, scale=64 ** -0.5).to(dt).to(DEV)
        bn = [((rnd(128, seed=10 + i) * 0.5 + 1.0).to(DEV), (rnd(128, seed=20 + i) * 0.2).to(DEV))
              for i in range(3)]
        f = torch.empty(N, H, W, 128, dtype=dt, device=DEV)
        _lib.call("fscnn_pw_gemm", M, 128, 64, _lib.ptr(high), 64, _lib.ptr(wh), 64, 0,
                  _lib.ptr(bn[2][0]), _lib.ptr(bn[2][1]), None, 0, 0, _lib.ptr(f), 128, None, dc,
                  _lib.stream_ptr())
        fh = f.clone()
        _lib.call("fscnn_block_dsconv_res_fwd", _lib.ptr(low), dc, N, H, W, 128, 128, Hi, Wi,
                  _lib.ptr(wd), _lib.ptr(bn[0][0]), _lib.ptr(bn[0][1]), _lib.ptr(wl),
                  _lib.ptr(bn[1][0]), _lib.ptr(bn[1][1]), _lib.ptr(f), 128, _lib.ptr(f), 128,
                  _lib.stream_ptr())
        y = torch.empty_like(f)
        _lib.call("fscnn_block_ffm_fwd", _lib.ptr(low), dc, N, Hi, Wi, H, W, _lib.ptr(high), 64,
                  _lib.ptr(wd), _lib.ptr(bn[0][0]), _lib.ptr(bn[0][1]), _lib.ptr(wl),
                  _lib.ptr(bn[1][0]), _lib.ptr(bn[1][1]), _lib.ptr(wh), _lib.ptr(bn[2][0]),
                  _lib.ptr(bn[2][1]), _lib.ptr(y), 128, _lib.stream_ptr())
        torch.cuda.synchronize()
        ne = (f.view(torch.int16 if dt != torch.float32 else torch.int32) !=
              y.view(torch.int16 if dt != torch.float32 else torch.int32))
        print(dt, (N, Hi, Wi, H, W), "differing elements", int(ne.sum()), "of", ne.numel(),
              "max |d|", float((f.float() - y.float()).abs().max()))
        if ne.any():
            idx = ne.nonzero()[:5].tolist()
            for (n, h, w, c) in idx:
                print("  at", (n, h, w, c), float(f[n, h, w, c]), float(y[n, h, w, c]),
                      "fhigh", float(fh[n, h, w, c]))
