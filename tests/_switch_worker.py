"""Worker for tests/test_gpu_switches.py (run in a fresh process: the executor reads its FSCNN_*
switches once per process).  Three fp32 train steps with Dropout(0.1) active and dropout seeds
5, 9, 5 — alternating the unfused ``model(x)`` + CE path and the fused ``forward_loss`` head —
then saves every step's loss and flat gradient arena, and the step-3 running statistics.
With ``bf16`` the image is bf16 (the bf16 train plan, cfg3's arithmetic); ``bf16shift`` adds 4.0 to
a 2 x 3 x 512 x 1024 image, which moves conv0's output (hence its BN mean) well away from 0;
``bf16drop`` runs a bf16 2 x 3 x 256 x 512 image (M = 4096 low-res pixels: the classifier conv's
dgrad takes the streaming kernel with the Dropout backward in its epilogue).

    python tests/_switch_worker.py OUT.npz [bf16|bf16shift|bf16drop]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, half=None):
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import arch, portable_init
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from models.fast_scnn import FastSCNN

    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          arch.portable_state_dict(19, seed=0, variant="bnrand").items()}
    m = FastSCNN(19)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    shape = {"bf16shift": (2, 3, 512, 1024), "bf16drop": (2, 3, 256, 512)}.get(half, (2, 3, 96, 160))
    x = torch.from_numpy(portable_init.input_tensor(3, shape)).to(dev)
    if half == "bf16shift":
        x = x + 4.0
    if half in ("bf16", "bf16shift", "bf16drop"):
        x = x.to(torch.bfloat16)
    t = torch.from_numpy(portable_init.target_tensor(4, (2,) + shape[2:], 19, 0.05)).to(dev)
    res = {}
    exact = half == "bf16shift" and os.environ.get("FSCNN_LTD_FUSED") == "0"
    m._keep_ws = exact
    for i, seed in enumerate((5, 9, 5, 9)):
        m.zero_grad(set_to_none=True)
        m._dropout_seed = seed
        loss = cross_entropy(m(x)[0], t) if i % 2 == 0 else m.forward_loss(x, t)
        loss.backward()
        torch.cuda.synchronize()
        if exact and i == 0:
            res["c0exact0"] = _conv0_dw_exact(m, x).numpy()
        res["loss%d" % i] = np.float32(loss.item())
        res["grad%d" % i] = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu().numpy()
    res["sizes"] = np.array([p.numel() for p in m.parameters()], dtype=np.int64)
    res["names"] = np.array([k for k, _ in m.named_parameters()])
    for k, v in m.state_dict().items():
        if "running" in k:
            res["bn." + k] = v.cpu().numpy()
    np.savez(out, **res)


def _conv0_dw_exact(m, x):
    """conv0's weight gradient in fp64 from the step's STORED tensors (two-launch path: the
    gradient g of conv0's BN output is in the workspace): train-mode BN backward through the
    ReLU mask fmaf(z, scale, shift) > 0, then the stride-2 conv's weight gradient over the bf16
    image (models/fast_scnn.py:153 autograd)."""
    import torch
    from torch.nn.grad import conv2d_weight
    N, _, H, W = x.shape
    H1, W1 = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    g = m.debug_buffer("c0.ga").double().cpu()
    z = m.debug_buffer("c0.z").double().cpu()
    mean = m.debug_buffer("c0.mean").double().cpu().reshape(-1)
    invstd = m.debug_buffer("c0.invstd").double().cpu().reshape(-1)
    sc32 = m.debug_buffer("c0.scale").float().cpu().reshape(-1)
    sh32 = m.debug_buffer("c0.shift").float().cpu().reshape(-1)
    mask = torch.addcmul(sh32, z.float(), sc32) > 0  # the kernels' fmaf(z, scale, shift) > 0
    gm = torch.where(mask, g, torch.zeros_like(g))
    xhat = (z - mean) * invstd
    dz = sc32.double() * (gm - gm.mean(0) - xhat * (gm * xhat).mean(0))
    dz = dz.view(N, H1, W1, 32).permute(0, 3, 1, 2)
    return conv2d_weight(x.double().cpu(), (32, 3, 3, 3), dz, stride=2, padding=0).reshape(-1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
