#!/usr/bin/env python3
"""Time the pointwise GEMMs of the low-resolution bottlenecks (fscnn_pw_gemm / fscnn_pw_wgrad)
one shape at a time, with and without the fused BN statistics, for rocprofv3.

    python tools/lowres_gemm_bench.py [--dtype bf16] [--m 16384] [--reps 50]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import _fscnn_boot

_fscnn_boot.load()
from fast_scnn_pytorch_amd import _lib

# (label, K, N): the bottleneck2/3 expand / project forwards and their dgrads
SHAPES = [("b2 expand", 64, 384), ("b2.0 project", 384, 96), ("b3 expand", 96, 576),
          ("b3.0 project", 576, 128), ("b2.x project", 576, 96), ("b3.x project", 768, 128),
          ("b3 project dgrad", 128, 576)]


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def copy_floor(nbytes_read, nbytes_write, reps):
    """A plain device copy moving the same bytes (read + write): the per-launch floor of a
    bandwidth-bound kernel of that size on this box."""
    n = max(nbytes_read, nbytes_write) // 2
    src = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    dst = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    return timed(lambda: dst.copy_(src), reps)


def dw_shapes(a, dt, lib, st):
    """Depthwise 3x3 forward (eval form: folded BN + ReLU) at the low-resolution shapes."""
    E = 4 if dt == torch.float32 else 2
    for (N, H, W, C, s) in [(8, 32, 64, 576, 1), (8, 32, 64, 768, 1), (8, 64, 128, 384, 2),
                            (8, 128, 256, 128, 1)]:
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        x = torch.randn(N, H, W, C, device="cuda").to(dt)
        y = torch.empty(N, Ho, Wo, C, device="cuda", dtype=dt)
        w = torch.randn(C, 9, device="cuda")
        sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        us = timed(lambda: _lib.call("fscnn_dw3x3_fwd", _lib.ptr(x), _lib.dtype_code(dt), N, H, W,
                                     C, s, _lib.ptr(w), _lib.ptr(sc), _lib.ptr(sh), 1, _lib.ptr(y),
                                     st), a.reps)
        mb = E * (N * H * W * C + N * Ho * Wo * C) / 1e6
        fl = copy_floor(E * N * H * W * C, E * N * Ho * Wo * C, a.reps)
        print("dw3x3 s%d %dx%dx%dx%d     : %6.1f us  %6.1f MB  %5.0f GB/s   (copy of equal bytes %5.1f us)"
              % (s, N, H, W, C, us, mb, mb / us * 1e3, fl), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    dev = torch.device("cuda", 0)
    E = 4 if dt == torch.float32 else 2
    st = _lib.stream_ptr()
    lib = _lib.load()
    for label, K, N in SHAPES:
        A = torch.randn(a.m, K, device=dev).to(dt)
        B = (torch.randn(N, K, device=dev) / K ** 0.5).to(dt)
        C = torch.empty(a.m, N, dtype=dt, device=dev)
        sc = torch.ones(N, device=dev)
        sh = torch.zeros(N, device=dev)
        part = torch.empty((a.m + 127) // 128 * 3 * N, device=dev)
        slab = torch.empty(int(lib.fscnn_pw_wgrad_slab_floats(a.m, N, K)), device=dev)
        dW = torch.empty(N, K, device=dev)
        for stats in (False, True):
            args = [a.m, N, K, _lib.ptr(A), K, _lib.ptr(B), K, 0, _lib.ptr(sc), _lib.ptr(sh), None,
                    0, 0, _lib.ptr(C), N, _lib.ptr(part) if stats else None,
                    _lib.dtype_code(dt), st]
            for _ in range(3):
                _lib.call("fscnn_pw_gemm", *args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                _lib.call("fscnn_pw_gemm", *args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.reps * 1e3
            mb = E * (a.m * K + a.m * N + N * K) / 1e6
            fl = copy_floor(E * (a.m * K + N * K), E * a.m * N, a.reps) if not stats else 0.0
            print("%-18s M%d K%d N%d stats=%d: %6.1f us  %6.1f MB  %5.0f GB/s   (copy floor %5.1f us)"
                  % (label, a.m, K, N, stats, us, mb, mb / us * 1e3, fl), flush=True)
        # weight gradient dW[N][K] = D^T X with D = C (M x N), X = A (M x K)
        wargs = [a.m, N, K, _lib.ptr(C), N, _lib.ptr(A), K, _lib.ptr(slab), _lib.ptr(dW),
                 _lib.dtype_code(dt), st]
        for _ in range(3):
            _lib.call("fscnn_pw_wgrad", *wargs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            _lib.call("fscnn_pw_wgrad", *wargs)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        mb = E * (a.m * K + a.m * N) / 1e6
        print("%-18s M%d K%d N%d wgrad  : %6.1f us  %6.1f MB  %5.0f GB/s"
              % (label, a.m, K, N, us, mb, mb / us * 1e3), flush=True)


if __name__ == "__main__":
    main()
    a = argparse.Namespace(reps=50)
    dw_shapes(a, torch.bfloat16, _lib.load(), _lib.stream_ptr())
