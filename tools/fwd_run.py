#!/usr/bin/env python3
"""Eval forward only (cfg2 fp32 8x3x1024x2048, or cfg5 fp16 32x3x480x640) for rocprofv3 runs.

    python tools/fwd_run.py [--cfg 2|5] [--reps K]

Prints the wall ms per batch.  Dispatches of one batch are delimited by the bn_fold kernel
(first launch of every eval forward), so tools/trace_layers.py-style per-layer reading works
with --delim bn_fold.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import _fscnn_boot

_fscnn_boot.load()
from fast_scnn_pytorch_amd import arch, portable_init
from models.fast_scnn import FastSCNN


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bf16", action="store_true", help="bf16 input (bf16 compute)")
    a = ap.parse_args()
    if a.cfg == 5:
        C, shape, dt = 2, (32, 3, 480, 640), torch.float16
    else:
        C, shape, dt = 19, (8, 3, 1024, 2048), torch.float32
    if a.bf16:
        dt = torch.bfloat16
    dev = torch.device("cuda", 0)
    m = FastSCNN(C)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(C, seed=0, variant="bnrand").items()})
    m = m.to(dev).eval()
    x = torch.from_numpy(portable_init.input_tensor(1, shape)).to(dev).to(dt)
    with torch.no_grad():
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            m(x)
        torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / a.reps
    print("cfg%d forward: %.3f ms/batch, %.1f img/s" % (a.cfg, ms, shape[0] * 1e3 / ms))


if __name__ == "__main__":
    main()
