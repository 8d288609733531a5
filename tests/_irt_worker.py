"""Worker for tests/test_gpu_switches.py::test_ir_train_recompute_*: one bf16 train step (fresh
process: the executor reads FSCNN_IR_TRAIN once) on a 2 x 3 x 512 x 1024 image, saving the
bottleneck1 blocks' depthwise pre-BN outputs (forward), their expand outputs (as the backward
holds them: recomputed when the forward did not store them), the loss and the gradients.

    FSCNN_IR_TRAIN=0|1 python tests/_irt_worker.py OUT.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import arch, portable_init
    from models.fast_scnn import FastSCNN

    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          arch.portable_state_dict(19, seed=0, variant="bnrand").items()}
    m = FastSCNN(19)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    shape = (2, 3, 512, 1024)
    x = torch.from_numpy(portable_init.input_tensor(3, shape)).to(dev).to(torch.bfloat16)
    t = torch.from_numpy(portable_init.target_tensor(4, (2,) + shape[2:], 19, 0.05)).to(dev)
    m._keep_ws = True
    m._dropout_seed = 5
    res = {}
    loss = m.forward_loss(x, t)
    torch.cuda.synchronize()
    for i in range(3):
        res["lbd%d.z" % i] = m.debug_buffer("lbd%d.z" % i).view(torch.int16).cpu().numpy()
        res["lbd%d.mean" % i] = m.debug_buffer("lbd%d.mean" % i).cpu().numpy()
    loss.backward()
    torch.cuda.synchronize()
    for i in range(3):
        res["lbe%d.z" % i] = m.debug_buffer("lbe%d.z" % i).view(torch.int16).cpu().numpy()
    res["loss"] = np.float32(loss.item())
    res["grad"] = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu().numpy()
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
