#!/usr/bin/env python3
"""Time the fused inference bottleneck (fscnn_block_ir_fwd) on one block shape, for rocprofv3.

    python tools/ir_bench.py [--dtype fp32|bf16|fp16] [--n 8 --h 32 --w 64 --cin 128 --cout 128]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import _fscnn_boot

_fscnn_boot.load()
from fast_scnn_pytorch_amd import _lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--w", type=int, default=64)
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.dtype]
    dev = torch.device("cuda", 0)
    E = 6 * a.cin
    g = torch.Generator().manual_seed(0)
    r = lambda *s: (torch.rand(*s, generator=g) * 2 - 1)  # noqa: E731
    x = r(a.n, a.h, a.w, a.cin).to(dt).to(dev)
    y = torch.empty(a.n, a.h, a.w, a.cout, dtype=dt, device=dev)
    we = (r(E, a.cin) / a.cin ** 0.5).to(dt).to(dev)
    wp = (r(a.cout, E) / E ** 0.5).to(dt).to(dev)
    wd = (r(E, 9) * 0.4).to(dev)
    bn = [t.to(dev) for c in (E, E, a.cout) for t in (r(c).abs() + 0.5, r(c) * 0.2)]
    args = [_lib.ptr(x), a.cin, _lib.dtype_code(dt), a.n, a.h, a.w, a.cin, E, a.cout,
            _lib.ptr(we), _lib.ptr(wd), _lib.ptr(wp)] + [_lib.ptr(t) for t in bn] + \
        [int(a.cin == a.cout), _lib.ptr(y), a.cout, _lib.stream_ptr()]
    for _ in range(3):
        _lib.call("fscnn_block_ir_fwd", *args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        _lib.call("fscnn_block_ir_fwd", *args)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / a.reps * 1e6
    fl = 2.0 * a.n * a.h * a.w * E * (a.cin + a.cout)
    print("ir_block %s N%d %dx%d %d->%d->%d: %.1f us/launch (%.1f TFLOP/s on the 1x1s)"
          % (a.dtype, a.n, a.h, a.w, a.cin, E, a.cout, us, fl / us / 1e6))


if __name__ == "__main__":
    main()
