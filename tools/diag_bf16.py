"""Where does the bf16 train forward leave the emulation's error budget?  GPU side: run the
tests/test_gpu_bf16_train.py case, save the HIP masks (packed) and stage activations to
gpurun_out/diag_bf16.npz.  CPU side (``analyze``): run the fp64 oracle and the bf16 emulation
under those masks and print, per recorded stage, |HIP - fp64| / |emu - fp64|.
    python tools/diag_bf16.py run        (GPU box)
    python tools/diag_bf16.py analyze    (here)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _fscnn_boot  # noqa: E402

_fscnn_boot.load()
from helpers import hip_relu_masks, oracle_bf16_train_emulated, relu_sites  # noqa: E402
from oracle import fast_scnn_ref as ref  # noqa: E402
import test_gpu_bf16_train as T  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out", "diag_bf16.npz")
# (HIP plan unit buffer, oracle record name, channels)
STAGES = [("l2pw", "ltd", 64)] + [("lbp%d" % i, T_name, c) for i, (T_name, c) in enumerate(
    [("global_feature_extractor.bottleneck1.%d" % j, 64) for j in range(3)] +
    [("global_feature_extractor.bottleneck2.%d" % j, 96) for j in range(3)] +
    [("global_feature_extractor.bottleneck3.%d" % j, 128) for j in range(3)])] + \
    [("po", "ppm", 128), ("f", "ffm", 128), ("drop", "drop", 128), ("logits", "logits_lowres", 19)]


def run():
    from models.fast_scnn import FastSCNN
    sd, x, t = T._case()
    m = FastSCNN(T.NC)
    m.load_state_dict(sd)
    m = m.to("cuda").train()
    m._dropout_seed = T.DROP_SEED
    m._keep_ws = True
    out = m(x.to("cuda").to(torch.bfloat16))[0]
    torch.cuda.synchronize()
    with torch.no_grad():
        s64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        _, _, acts = ref.forward(s64, x.double(), T.NC, training=True, dropout_seed=T.DROP_SEED,
                                 record=True)
    masks = hip_relu_masks(m, acts)
    d = {}
    for name, mk in masks.items():
        d["mask:" + name] = np.packbits(mk.numpy().ravel())
    for unit, rec, c in STAGES:
        try:
            if unit in ("f", "logits", "drop"):
                b = m.debug_buffer(unit)
            else:
                b = m.debug_buffer(unit + ".a") if unit != "l2pw" else m.debug_buffer("l2pw.z")
        except Exception as e:  # noqa: BLE001
            print("no buffer", unit, e)
            continue
        d["act:" + rec] = b.float().cpu().numpy()[:, :c]
        if unit == "l2pw":  # lazily applied in training: keep z and the BN table
            d["l2pw.scale"] = m.debug_buffer("l2pw.scale").float().cpu().numpy()
            d["l2pw.shift"] = m.debug_buffer("l2pw.shift").float().cpu().numpy()
    for unit, name in (("flow", "feature_fusion.conv_lower_res.1"),
                       ("fhigh", "feature_fusion.conv_higher_res.1")):
        d["mean:" + name] = m.debug_buffer(unit + ".mean").double().cpu().numpy().ravel()
        d["invstd:" + name] = m.debug_buffer(unit + ".invstd").double().cpu().numpy().ravel()
    # per ReLU site: the HIP pre-activation's per-channel mean over all pixels, and image 0
    for unit, name in relu_sites():
        if unit == "f":
            pre = m.debug_buffer("f").double()
        else:
            pre = m.debug_buffer(unit + ".z").double() * m.debug_buffer(unit + ".scale").double() + \
                m.debug_buffer(unit + ".shift").double()
        N, C, H, W = acts["pre:" + name].shape
        if unit.startswith("ppk"):
            pre = pre.reshape(H, W, N, C).permute(2, 3, 0, 1)
        else:
            pre = pre.reshape(N, H, W, C).permute(0, 3, 1, 2)
        d["pmean:" + name] = pre.mean(dim=(0, 2, 3)).cpu().numpy()
        if unit != "f":
            d["mean:" + name] = m.debug_buffer(unit + ".mean").double().cpu().numpy().ravel()
            d["invstd:" + name] = m.debug_buffer(unit + ".invstd").double().cpu().numpy().ravel()
        d["pimg0:" + name] = pre[0].float().cpu().numpy()
    # self-consistency: each unit's BN statistics against its own stored z (fp64 sums)
    for unit in (["c0", "l1dw", "l1pw", "l2dw", "l2pw"] + ["lb%s%d" % (k, i) for i in range(9) for k in "edp"]
                 + ["po", "fdw", "flow", "fhigh", "c1dw", "c1pw", "c2dw", "c2pw"]):
        z = m.debug_buffer(unit + ".z").double()
        mu, var = z.mean(0), z.var(0, unbiased=False)
        hm = m.debug_buffer(unit + ".mean").double().ravel()
        hi = m.debug_buffer(unit + ".invstd").double().ravel()
        i64 = 1.0 / torch.sqrt(var + 1e-5)
        print("self %-6s M %7d |dmean|/std max %.2e  |dinvstd|/invstd max %.2e" % (
            unit, z.shape[0], ((hm - mu) * i64).abs().max().item(), ((hi - i64) / i64).abs().max().item()))
    np.savez_compressed(OUT, **d)
    print("saved", OUT, len(d))


def analyze():
    d = dict(np.load(OUT))
    sd, x, t = T._case()
    with torch.no_grad():
        s64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        _, _, acts = ref.forward(s64, x.double(), T.NC, training=True, dropout_seed=T.DROP_SEED,
                                 record=True)
    masks = {}
    for _, name in relu_sites():
        ref_shape = acts["pre:" + name].shape
        n = int(np.prod(ref_shape))
        masks[name] = torch.from_numpy(np.unpackbits(d["mask:" + name])[:n].astype(bool)
                                       .reshape(ref_shape))
    ob = ref._Ctx.bn
    stats, estats = {}, {}

    def bn_rec(self, x, prefix):  # the BN input's batch statistics (fp64 and emulated runs)
        if self.training:
            (stats if x.dtype == torch.float64 else estats)[prefix] = (
                x.detach().double().mean(dim=(0, 2, 3)),
                x.detach().double().var(dim=(0, 2, 3), unbiased=False))
        return ob(self, x, prefix)
    ref._Ctx.bn = bn_rec
    try:
        _, _, a64 = oracle_bf16_train_emulated(sd, x, t, T.NC, T.DROP_SEED, emulate=False,
                                               relu_masks=masks, record=True)
        _, _, aem = oracle_bf16_train_emulated(sd, x, t, T.NC, T.DROP_SEED, emulate=True,
                                               relu_masks=masks, record=True, round_blocks=True)
    finally:
        ref._Ctx.bn = ob
    for unit, name in relu_sites() + [("flow", "feature_fusion.conv_lower_res.1"),
                                      ("fhigh", "feature_fusion.conv_higher_res.1")]:
        if "mean:" + name not in d or name not in stats:
            continue
        mu, var = stats[name]
        hm = torch.from_numpy(d["mean:" + name]).double()
        hi = torch.from_numpy(d["invstd:" + name]).double()
        i64 = 1.0 / torch.sqrt(var + 1e-5)
        emu_m, emu_v = estats[name]
        ie = 1.0 / torch.sqrt(emu_v + 1e-5)
        print("bn %-48s dmean/std HIP %.2e emu %.2e | dinvstd/invstd HIP %.2e emu %.2e (norms)" % (
            name, ((hm - mu) * i64).norm().item(), ((emu_m - mu) * i64).norm().item(),
            ((hi - i64) / i64).norm().item(), ((ie - i64) / i64).norm().item()))
    for unit, name in relu_sites():
        if "pmean:" + name not in d:
            continue
        hm = torch.from_numpy(d["pmean:" + name]).double()
        r64 = a64["pre:" + name].detach().double()
        e = aem["pre:" + name].detach().double()
        mh = (hm - r64.mean(dim=(0, 2, 3))).norm().item()
        me = (e.mean(dim=(0, 2, 3)) - r64.mean(dim=(0, 2, 3))).norm().item()
        h0 = torch.from_numpy(d["pimg0:" + name]).double()
        eh, ee = (h0 - r64[0]).norm().item(), (e[0] - r64[0]).norm().item()
        print("pre %-48s img0 err ratio %.2f   channel-mean offset ratio %.2f (%.2e vs %.2e)"
              % (name, eh / max(ee, 1e-30), mh / max(me, 1e-30), mh, me))
    for a_ in (a64, aem):  # the Dropout output (oracle forward: c * keep / (1 - p))
        c_ = a_["cls.dsconv2"].detach()
        keep = ref.dropout_mask(T.DROP_SEED, tuple(c_.shape), 0.1).to(c_.dtype)
        a_["drop"] = c_ * keep / (1.0 - 0.1)
    aem["drop"] = aem["drop"].to(torch.bfloat16).float()  # what the emulated classifier conv reads
    aem["ffm"] = aem["ffm"].to(torch.bfloat16).float()    # what the emulated classifier dw reads
    for unit, rec, c in STAGES:
        if "act:" + rec not in d:
            continue
        h = torch.from_numpy(d["act:" + rec]).double()
        r64 = a64[rec].detach().double()
        if unit == "l2pw":  # the LTD output is applied by its consumers: compare BN+ReLU of z
            h = torch.relu(h * torch.from_numpy(d["l2pw.scale"]).double() +
                           torch.from_numpy(d["l2pw.shift"]).double())
        N, C, H, W = r64.shape
        h = h.reshape(N, H, W, C).permute(0, 3, 1, 2)
        e = aem[rec].detach().double()
        eh, ee = (h - r64).norm().item(), (e - r64).norm().item()
        mh = (h - r64).mean(dim=(0, 2, 3)).norm().item()
        me = (e - r64).mean(dim=(0, 2, 3)).norm().item()
        print("%-45s |HIP-64| %.3e |emu-64| %.3e ratio %.2f  channel-mean offset ratio %.2f (%.2e %.2e)"
              % (rec, eh, ee, eh / max(ee, 1e-30), mh / max(me, 1e-30), mh, me))


if __name__ == "__main__":
    {"run": run, "analyze": analyze}[sys.argv[1]]()
