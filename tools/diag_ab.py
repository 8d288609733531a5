#!/usr/bin/env python3
"""A/B diagnostic: one fp32 train step on a golden case with the plan's buffers kept; saves every
unit's BN statistics (mean / invstd), pre-BN z and every gradient to an npz, so two runs under
different executor switches can be compared tensor by tensor.

    python tools/diag_ab.py OUT.npz [case]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(out, case="train_c2"):
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from helpers import golden_input, golden_sd, golden_target, load_golden
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from models.fast_scnn import FastSCNN
    g = load_golden(case)
    nc = int(g["num_classes"])
    m = FastSCNN(nc)
    m.load_state_dict(golden_sd(g))
    m = m.cuda().train()
    m._dropout_seed = int(g["drop_seed"])
    m._keep_ws = True
    loss = cross_entropy(m(golden_input(g).cuda())[0], golden_target(g).cuda())
    loss.backward()
    torch.cuda.synchronize()
    res = {"loss": np.float64(loss.item())}
    units = ["c0", "l1dw", "l1pw", "l2dw", "l2pw"] + ["lb%s%d" % (k, i) for i in range(9)
                                                       for k in "edp"] + ["po", "fdw", "flow",
                                                                           "fhigh", "c1dw", "c1pw",
                                                                           "c2dw", "c2pw"]
    units += ["ppk%d" % i for i in range(4)]
    res["f"] = m.debug_buffer("f").float().cpu().numpy()
    for u in units:
        for f in ("mean", "invstd", "z", "scale", "shift"):
            try:
                res[u + "." + f] = m.debug_buffer(u + "." + f).float().cpu().numpy()
            except Exception:
                pass
    for k, p in m.named_parameters():
        res["grad." + k] = p.grad.cpu().numpy()
    np.savez(out, **res)
    print("saved", out, len(res))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
