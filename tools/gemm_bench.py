"""Microbenchmark of the pointwise GEMM C ABI (fscnn_pw_gemm) on the network's 1x1 shapes,
with and without the BN-statistics epilogue.  Prints us / GB/s per shape (HIP events, median of
20 launches).

    python tools/gemm_bench.py [--dtype bf16|f32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # (name, M, N, K)
    ("b1.0 expand", 262144, 384, 64),
    ("b1.1 expand", 65536, 384, 64),
    ("b2.0 expand", 65536, 384, 64),
    ("b3.0 expand", 16384, 576, 96),
    ("ltd1 pw", 1048576, 48, 32),
    ("ltd2 pw", 262144, 64, 48),
    ("cls pw", 262144, 128, 128),
    ("ffm high", 262144, 128, 64),
    ("b1.0 proj dgrad", 65536, 384, 64),
    ("b1 project", 65536, 64, 384),
    ("b2.1 project", 16384, 96, 576),
    ("b3.0 project", 16384, 128, 576),
    ("b2.1 exp dgrad", 16384, 96, 576),
    ("b1.0 exp dgrad", 262144, 64, 384),
    ("ppm out", 16384, 128, 256),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import _lib
    lib = _lib.load()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    code = _lib.dtype_code(dt)
    E = 2 if dt == torch.bfloat16 else 4
    dev = torch.device("cuda", 0)
    for name, M, N, K in SHAPES:
        A = torch.randn(M, K, device=dev).to(dt)
        B = (torch.randn(N, K, device=dev) * 0.1).to(dt)
        C = torch.empty(M, N, device=dev, dtype=dt)
        part = torch.empty(((M + 127) // 128) * 3 * N, device=dev)
        for stats in (False, True):
            def run():
                _lib.call("fscnn_pw_gemm", M, N, K, _lib.ptr(A), K, _lib.ptr(B), K, 0, None, None,
                          None, 0, 0, _lib.ptr(C), N, _lib.ptr(part) if stats else None, code,
                          _lib.stream_ptr())
            for _ in range(3):
                run()
            ts = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = sorted(ts)[len(ts) // 2]
            by = E * (M * K + M * N + N * K)
            parts = lib.fscnn_pw_gemm_stats_parts(M, N, K, K, N, code) if stats else 0
            print("%-18s M=%8d N=%4d K=%4d stats=%d parts=%5d  %7.1f us  %6.0f GB/s"
                  % (name, M, N, K, stats, parts, us, by / (us * 1e-6) / 1e9), flush=True)


if __name__ == "__main__":
    main()
