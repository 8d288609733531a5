#!/usr/bin/env python3
"""Generate golden fixtures by importing the REFERENCE model (survey container only).

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

Imports ``FastSCNN`` from ``/root/reference/models/fast_scnn.py`` (``get_fast_scnn`` is not
importable here: it pulls torchvision through ``data_loader``), loads weights
from the portable counter-based generator, runs it on CPU and writes small ``.npz`` files into
``tests/golden/``.  The fixtures are data only (inputs are regenerated from seeds; expected
outputs are stored).  ``oracle/fast_scnn_ref.py`` is pinned against these by
``tests/test_oracle_golden.py``; the HIP path is then checked against the oracle.
"""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = os.environ.get("FSCNN_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "tests", "golden")

import _fscnn_boot  # noqa: E402

pkg = _fscnn_boot.load()
from fast_scnn_pytorch_amd import arch, portable_init  # noqa: E402
from oracle.fast_scnn_ref import dropout_mask  # noqa: E402


def ref_model(num_classes, aux=False):
    sys.path.insert(0, REF)
    from models.fast_scnn import FastSCNN  # the reference itself
    sys.path.pop(0)
    return FastSCNN(num_classes, aux=aux)


def load_portable(model, num_classes, aux, seed, variant):
    sd = arch.portable_state_dict(num_classes, aux, seed, variant)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return model


def calibrate(model, x):
    """Set running stats to batch stats of ``x`` (momentum 1) so eval activations stay O(1)."""
    moms = {}
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            moms[name] = m.momentum
            m.momentum = 1.0
    model.train()
    drop = [m for m in model.modules() if isinstance(m, torch.nn.Dropout)]
    for d in drop:
        d.p = 0.0
    with torch.no_grad():
        model(x)
    for d in drop:
        d.p = 0.1
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = moms[name]
            m.num_batches_tracked.zero_()
    model.eval()


def bn_buffers(model):
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items()
            if k.endswith("running_mean") or k.endswith("running_var")}


def sample_coords(shape, n, seed):
    tot = int(np.prod(shape))
    u = portable_init.uniform(seed, "coords", n)
    return np.unique(np.minimum((u * tot).astype(np.int64), tot - 1))


def logits_summary(prefix, logits, seed=99):
    """Stats-only golden of full-resolution logits [N,C,H,W]."""
    lg = logits.detach().numpy()
    am = lg.argmax(1).astype(np.uint8)
    idx = sample_coords(lg.shape, 4096, seed)
    srt = np.sort(lg, axis=1)
    return {
        prefix + "argmax": am,
        prefix + "argmax_sha256": np.frombuffer(hashlib.sha256(am.tobytes()).digest(), np.uint8),
        prefix + "hist": np.bincount(am.ravel(), minlength=lg.shape[1]).astype(np.int64),
        prefix + "sample_idx": idx,
        prefix + "sample_val": lg.ravel()[idx].astype(np.float32),
        prefix + "class_mean": lg.mean(axis=(0, 2, 3)).astype(np.float64),
        prefix + "class_min": lg.min(axis=(0, 2, 3)).astype(np.float32),
        prefix + "class_max": lg.max(axis=(0, 2, 3)).astype(np.float32),
        prefix + "min_margin": np.float32((srt[:, -1] - srt[:, -2]).min()),
    }


class _MaskDropout(torch.nn.Module):
    """Replaces the reference's Dropout(0.1) with the portable keep-mask law for train goldens."""

    def __init__(self, seed, p=0.1):
        super().__init__()
        self.seed, self.p = seed, p

    def forward(self, x):
        keep = dropout_mask(self.seed, tuple(x.shape), self.p).to(x.dtype)
        return x * keep / (1.0 - self.p)


def gen_schema():
    out = {}
    for c, aux in ((19, False), (19, True), (2, False)):
        m = ref_model(c, aux)
        sd = m.state_dict()
        tag = "c%d%s" % (c, "_aux" if aux else "")
        out[tag + "_keys"] = np.array(list(sd.keys()))
        out[tag + "_shapes"] = np.array([",".join(str(s) for s in v.shape) for v in sd.values()])
        out[tag + "_params"] = np.array([k for k, _ in m.named_parameters()])
    np.savez_compressed(os.path.join(OUT, "schema.npz"), **out)


def gen_eval(tag, num_classes, shape, variant, calib, record=True, aux=False):
    torch.manual_seed(0)
    m = load_portable(ref_model(num_classes, aux), num_classes, aux, 0, variant).eval()
    out = {"shape": np.array(shape), "num_classes": np.int64(num_classes), "seed_w": np.int64(0),
           "seed_x": np.int64(1), "variant": np.array(variant), "aux": np.int64(aux)}
    if calib:
        xc = torch.from_numpy(portable_init.input_tensor(7, (4,) + tuple(shape[1:]), "calib"))
        calibrate(m, xc)
        out.update({"bn." + k: v for k, v in bn_buffers(m).items()})
    x = torch.from_numpy(portable_init.input_tensor(1, shape))
    acts = {}
    hooks = []
    if record:
        def hook(name):
            def fn(_mod, _inp, outp):
                acts[name] = outp.detach().numpy().copy()
            return fn
        for name in ("learning_to_downsample", "global_feature_extractor.bottleneck1",
                     "global_feature_extractor.bottleneck2", "global_feature_extractor.bottleneck3",
                     "global_feature_extractor.ppm", "feature_fusion", "classifier"):
            hooks.append(m.get_submodule(name).register_forward_hook(hook(name)))
    with torch.no_grad():
        outs = m(x)
    for h in hooks:
        h.remove()
    for k, v in acts.items():
        out["act." + k] = v.astype(np.float32)
    out.update(logits_summary("out0.", outs[0]))
    if aux:
        out.update(logits_summary("out1.", outs[1]))
    np.savez_compressed(os.path.join(OUT, tag + ".npz"), **out)
    print(tag, {k: v.shape for k, v in out.items() if hasattr(v, "shape")}.get("out0.argmax"),
          "min_margin", out["out0.min_margin"])


def sample_tensor(name, t, k=1024):
    a = t.detach().numpy().ravel()
    if a.size <= k:
        return np.arange(a.size), a.astype(np.float32)
    idx = sample_coords(a.shape, k, portable_init._fnv1a64(name) & 0xFFFF)
    return idx, a[idx].astype(np.float32)


def gen_train(tag, num_classes, shape, variant="default", aux=False, drop_seed=1234):
    m = load_portable(ref_model(num_classes, aux), num_classes, aux, 0, variant)
    m.classifier.conv[0] = _MaskDropout(drop_seed)
    if aux:
        m.auxlayer[3] = _MaskDropout(drop_seed + 1)
    m.train()
    x = torch.from_numpy(portable_init.input_tensor(1, shape))
    t = torch.from_numpy(portable_init.target_tensor(3, (shape[0],) + tuple(shape[2:]), num_classes,
                                                     ignore_frac=0.05))
    outs = m(x)
    crit = torch.nn.CrossEntropyLoss(ignore_index=-1)
    loss = crit(outs[0], t)
    if aux:
        loss = loss + 0.4 * crit(outs[1], t)
    loss.backward()
    out = {"shape": np.array(shape), "num_classes": np.int64(num_classes), "seed_w": np.int64(0),
           "seed_x": np.int64(1), "seed_t": np.int64(3), "ignore_frac": np.float64(0.05),
           "drop_seed": np.int64(drop_seed), "variant": np.array(variant), "aux": np.int64(aux),
           "loss": np.float64(loss.item())}
    out.update(logits_summary("out0.", outs[0].detach()))
    for k, p in m.named_parameters():
        idx, val = sample_tensor(k, p.grad)
        out["grad_idx." + k] = idx
        out["grad_val." + k] = val
        out["grad_norm." + k] = np.float64(p.grad.double().norm().item())
    for k, v in m.state_dict().items():
        if "running" in k:
            out["stats." + k] = v.numpy().copy()
    # one SGD step (train.py:195-198: lr 0.01, momentum 0.9, wd 1e-4)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    opt.step()
    for k, p in m.named_parameters():
        idx, val = sample_tensor(k, p.data)
        out["sgd_val." + k] = val
    np.savez_compressed(os.path.join(OUT, tag + ".npz"), **out)
    print(tag, "loss", out["loss"])


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    gen_schema()
    gen_eval("eval_c19_default", 19, (2, 3, 128, 256), "default", calib=False)
    gen_eval("eval_c19_calib", 19, (2, 3, 128, 256), "default", calib=True)
    gen_eval("eval_c19_bnrand_aux", 19, (2, 3, 96, 160), "bnrand", calib=True, aux=True, record=False)
    gen_eval("eval_c2_calib", 2, (2, 3, 96, 128), "default", calib=True)
    gen_train("train_c19", 19, (2, 3, 128, 256))
    gen_train("train_c19_aux", 19, (2, 3, 96, 160), aux=True)
    gen_train("train_c2", 2, (2, 3, 96, 128))
    # stats-only goldens at the literal BASELINE configs (cfg1 768², cfg2 at bs=1, cfg5 at bs=2)
    gen_eval("cfg1_c19_768", 19, (1, 3, 768, 768), "default", calib=True, record=False)
    gen_eval("cfg2_c19_1024x2048", 19, (1, 3, 1024, 2048), "default", calib=True, record=False)
    gen_eval("cfg5_c2_480x640", 2, (2, 3, 480, 640), "default", calib=True, record=False)


if __name__ == "__main__":
    main()
