#!/usr/bin/env python3
"""Eval forward time of one configuration (A/B helper): cfg2 fp32 8x3x1024x2048 (default) or
cfg5 fp16 32x3x480x640 with --cfg5.  Prints ms per batch (mean and median of --reps timed
forwards after 3 warm-ups)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _fscnn_boot  # noqa: E402

_fscnn_boot.load()
from fast_scnn_pytorch_amd import arch, portable_init  # noqa: E402
from models.fast_scnn import FastSCNN  # noqa: E402


def main():
    cfg5 = "--cfg5" in sys.argv
    reps = 30
    nc, shape = (2, (32, 3, 480, 640)) if cfg5 else (19, (8, 3, 1024, 2048))
    m = FastSCNN(nc)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(nc, seed=0).items()})
    m = m.to("cuda").eval()
    x = torch.from_numpy(portable_init.input_tensor(1, shape)).to("cuda")
    if cfg5:
        x = x.half()
    ts = []
    with torch.no_grad():
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        for _ in range(reps):
            t0 = time.perf_counter()
            m(x)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    print("%s ms per batch: mean %.3f median %.3f" % ("cfg5" if cfg5 else "cfg2", ts.mean(), np.median(ts)))


if __name__ == "__main__":
    main()
