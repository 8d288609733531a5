#!/usr/bin/env python3
"""Host-side cost of one bench train step: time to ENQUEUE K steps (no sync inside) vs the
wall time until the GPU finishes them.  enqueue ~ wall  =>  the host is the bottleneck."""
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
from fast_scnn_pytorch_amd.optim import FusedSGD
from models.fast_scnn import FastSCNN


def main():
    dev = torch.device("cuda", 0)
    m = FastSCNN(19)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(19, seed=0).items()})
    m = m.to(dev).train()
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x = torch.from_numpy(portable_init.input_tensor(1, (8, 3, 1024, 2048))).to(dev).bfloat16()
    t = torch.from_numpy(portable_init.target_tensor(3, (8, 1024, 2048), 19, 0.05)).to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = m.forward_loss(x, t)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    K = 10
    parts = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0}
    t0 = time.perf_counter()
    for _ in range(K):
        a = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = m.forward_loss(x, t)
        b = time.perf_counter()
        loss.backward()
        c = time.perf_counter()
        opt.step()
        d = time.perf_counter()
        parts["fwd"] += b - a
        parts["bwd"] += c - b
        parts["opt"] += d - c
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("enqueue ms/step %.3f  wall ms/step %.3f  (fwd %.3f bwd %.3f opt %.3f host ms/step)" % (
        1e3 * (t1 - t0) / K, 1e3 * (t2 - t0) / K, 1e3 * parts["fwd"] / K, 1e3 * parts["bwd"] / K,
        1e3 * parts["opt"] / K))


if __name__ == "__main__":
    main()
