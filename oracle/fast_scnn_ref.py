"""ORACLE — test infrastructure only, never shipped or measured as the product.

CPU restatement of the reference Fast-SCNN forward (Shinokawa/Fast-SCNN-pytorch,
``models/fast_scnn.py``) written functionally over ``torch.nn.functional`` on CPU tensors and
driven by a plain ``{state_dict key: tensor}`` mapping with the reference key schema
(SURVEY.md Appendix A).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, as the checker.

Pinned against golden vectors produced by importing the reference itself in the survey container
(``tools/gen_golden.py`` → ``tests/golden/*.npz``; checked by ``tests/test_oracle_golden.py``).

Every stage cites the reference line it restates.  Semantics restated exactly (Appendix B):
first conv padding 0, BN eps 1e-5 / momentum 0.1 / biased batch variance for normalisation and
unbiased for the running update, align_corners=True bilinear, AdaptiveAvgPool2d overlapping windows,
PPM concat order [x, f1, f2, f3, f6], LinearBottleneck shortcut iff stride 1 and Cin == Cout,
classifier Dropout(0.1) (here: an explicit keep-mask from ``dropout_mask`` so the HIP path and the
oracle drop the same elements).
"""
import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

# (name, cin, cout, stride) of the 9 LinearBottlenecks — models/fast_scnn.py:170-172,175-180
BOTTLENECKS = [
    ("global_feature_extractor.bottleneck1.0", 64, 64, 2),
    ("global_feature_extractor.bottleneck1.1", 64, 64, 1),
    ("global_feature_extractor.bottleneck1.2", 64, 64, 1),
    ("global_feature_extractor.bottleneck2.0", 64, 96, 2),
    ("global_feature_extractor.bottleneck2.1", 96, 96, 1),
    ("global_feature_extractor.bottleneck2.2", 96, 96, 1),
    ("global_feature_extractor.bottleneck3.0", 96, 128, 1),
    ("global_feature_extractor.bottleneck3.1", 128, 128, 1),
    ("global_feature_extractor.bottleneck3.2", 128, 128, 1),
]


class _Ctx:
    """Holds the parameters, the mode, and collects running-stat updates / intermediates."""

    def __init__(self, sd, training, momentum, record, relu_masks=None):
        self.sd = sd
        self.training = training
        self.momentum = momentum
        self.new_stats = {}
        self.record = record
        self.acts = {}
        self.relu_masks = relu_masks or {}

    def relu(self, x, name):
        """F.relu at the ReLU following BN ``name``.  Test instrumentation: ``relu_masks[name]``
        (a boolean NCHW tensor) replaces the sign test, so a test can evaluate the reference's
        gradients under the mask another implementation took at near-tie pre-activations;
        without it this is exactly F.relu.  record=True keeps the pre-activation."""
        if self.record:
            self.acts["pre:" + name] = x
        m = self.relu_masks.get(name)
        if m is None:
            return F.relu(x)
        return x * m.to(x.dtype)

    def p(self, key):
        return self.sd[key]

    def bn(self, x, prefix):
        """nn.BatchNorm2d (models/fast_scnn.py:56,71,74,87,108,199,203,27)."""
        w, b = self.p(prefix + ".weight"), self.p(prefix + ".bias")
        rm, rv = self.p(prefix + ".running_mean"), self.p(prefix + ".running_var")
        if not self.training:
            return F.batch_norm(x, rm, rv, w, b, False, 0.0, BN_EPS)
        n = x.numel() // x.shape[1]
        if n <= 1:
            # torch raises this for train-mode BN over a single value per channel (SURVEY §0 trap 5)
            raise ValueError("Expected more than 1 value per channel when training, got input size %s"
                             % (list(x.shape),))
        # batch statistics: mean and biased variance for normalisation; the running update uses
        # the unbiased variance (n/(n-1)) with momentum 0.1 — exactly aten's batch_norm.
        rm2, rv2 = rm.detach().clone(), rv.detach().clone()
        y = F.batch_norm(x, rm2, rv2, w, b, True, self.momentum, BN_EPS)
        self.new_stats[prefix + ".running_mean"] = rm2
        self.new_stats[prefix + ".running_var"] = rv2
        self.new_stats[prefix + ".num_batches_tracked"] = self.p(prefix + ".num_batches_tracked") + 1
        return y

    def rec(self, name, x):
        if self.record:
            self.acts[name] = x


def _conv(ctx, x, key, stride=1, padding=0, groups=1, bias=False):
    w = ctx.p(key + ".weight")
    b = ctx.p(key + ".bias") if bias else None
    return F.conv2d(x, w, b, stride=stride, padding=padding, groups=groups)


def _conv_bn_relu(ctx, x, prefix, k, stride):
    """_ConvBNReLU: conv(bias=False, padding=0) → BN → ReLU (models/fast_scnn.py:49-61)."""
    x = _conv(ctx, x, prefix + ".conv.0", stride=stride, padding=0)
    return ctx.relu(ctx.bn(x, prefix + ".conv.1"), prefix + ".conv.1")


def _dsconv(ctx, x, prefix, stride):
    """_DSConv: dw3x3(s, p1) → BN → ReLU → pw → BN → ReLU (models/fast_scnn.py:64-79)."""
    c = x.shape[1]
    x = _conv(ctx, x, prefix + ".conv.0", stride=stride, padding=1, groups=c)
    x = ctx.relu(ctx.bn(x, prefix + ".conv.1"), prefix + ".conv.1")
    x = _conv(ctx, x, prefix + ".conv.3")
    return ctx.relu(ctx.bn(x, prefix + ".conv.4"), prefix + ".conv.4")


def _dwconv(ctx, x, prefix, stride):
    """_DWConv: dw3x3(s, p1) → BN → ReLU (models/fast_scnn.py:82-92)."""
    c = x.shape[1]
    x = _conv(ctx, x, prefix + ".conv.0", stride=stride, padding=1, groups=c)
    return ctx.relu(ctx.bn(x, prefix + ".conv.1"), prefix + ".conv.1")


def _bottleneck(ctx, x, prefix, cin, cout, stride):
    """LinearBottleneck t=6 (models/fast_scnn.py:95-115)."""
    h = _conv_bn_relu(ctx, x, prefix + ".block.0", 1, 1)
    h = _dwconv(ctx, h, prefix + ".block.1", stride)
    h = _conv(ctx, h, prefix + ".block.2")
    h = ctx.bn(h, prefix + ".block.3")
    if stride == 1 and cin == cout:
        h = x + h
    return h


def adaptive_pool_windows(in_size, out_size):
    """AdaptiveAvgPool window [start, end) per output index."""
    return [((i * in_size) // out_size, -((-(i + 1) * in_size) // out_size)) for i in range(out_size)]


def _upsample(x, size):
    """F.interpolate bilinear align_corners=True (models/fast_scnn.py:40,135,212)."""
    return F.interpolate(x, size, mode="bilinear", align_corners=True)


def _ppm(ctx, x, prefix):
    """PyramidPooling (models/fast_scnn.py:118-145): bins 1,2,3,6, concat order [x,f1,f2,f3,f6]."""
    size = x.shape[2:]
    feats = [x]
    for i, k in enumerate((1, 2, 3, 6)):
        p = F.adaptive_avg_pool2d(x, k)
        f = _conv_bn_relu(ctx, p, "%s.conv%d" % (prefix, i + 1), 1, 1)
        feats.append(_upsample(f, size))
    x = torch.cat(feats, dim=1)
    return _conv_bn_relu(ctx, x, prefix + ".out", 1, 1)


def dropout_mask(seed, shape, p):
    """Keep-mask for the classifier Dropout, a pure function of (seed, NCHW linear index).

    The HIP path computes the identical hash (csrc/common.hpp ``dropout_keep``), so train-mode
    parity holds with dropout active.  24-bit uniform from a splitmix64 hash; keep iff u >= p.
    """
    n = int(np.prod(shape))
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = idx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    # keep iff 24-bit uniform u >= p  <=>  (z >> 40) >= ceil(p * 2^24)
    thr = int(np.ceil(np.float64(np.float32(p)) * float(1 << 24)))
    return torch.from_numpy(((z >> np.uint64(40)) >= np.uint64(thr)).reshape(shape))


def forward(sd, x, num_classes, training=False, aux=False, momentum=BN_MOMENTUM,
            dropout_p=0.1, dropout_seed=None, record=False, relu_masks=None):
    """FastSCNN.forward (models/fast_scnn.py:33-46).

    Returns ``(outputs_tuple, new_running_stats, intermediates)``.  In training mode Dropout is
    applied with ``dropout_mask(dropout_seed, ...)`` when ``dropout_seed`` is given, else skipped
    (p treated as 0).  ``sd`` values may be fp32 or fp64 CPU tensors (leaf tensors with
    requires_grad for gradient oracles).  ``relu_masks`` is test instrumentation (``_Ctx.relu``).
    """
    ctx = _Ctx(sd, training, momentum, record, relu_masks)
    size = x.shape[2:]
    # LearningToDownsample (models/fast_scnn.py:148-161)
    h = _conv_bn_relu(ctx, x, "learning_to_downsample.conv", 3, 2)
    ctx.rec("ltd.conv", h)
    h = _dsconv(ctx, h, "learning_to_downsample.dsconv1", 2)
    ctx.rec("ltd.dsconv1", h)
    hr = _dsconv(ctx, h, "learning_to_downsample.dsconv2", 2)
    ctx.rec("ltd", hr)
    # GlobalFeatureExtractor (models/fast_scnn.py:164-187)
    g = hr
    for name, cin, cout, s in BOTTLENECKS:
        g = _bottleneck(ctx, g, name, cin, cout, s)
        ctx.rec(name, g)
    g = _ppm(ctx, g, "global_feature_extractor.ppm")
    ctx.rec("ppm", g)
    # FeatureFusionModule (models/fast_scnn.py:190-218)
    low = _upsample(g, hr.shape[2:])
    low = _dwconv(ctx, low, "feature_fusion.dwconv", 1)
    low = ctx.bn(_conv(ctx, low, "feature_fusion.conv_lower_res.0", bias=True),
                 "feature_fusion.conv_lower_res.1")
    high = ctx.bn(_conv(ctx, hr, "feature_fusion.conv_higher_res.0", bias=True),
                  "feature_fusion.conv_higher_res.1")
    f = ctx.relu(high + low, "feature_fusion")
    ctx.rec("ffm", f)
    # Classifer (models/fast_scnn.py:221-237)
    c = _dsconv(ctx, f, "classifier.dsconv1", 1)
    c = _dsconv(ctx, c, "classifier.dsconv2", 1)
    ctx.rec("cls.dsconv2", c)
    if training and dropout_seed is not None and dropout_p > 0:
        keep = dropout_mask(dropout_seed, tuple(c.shape), dropout_p).to(c.dtype)
        c = c * keep / (1.0 - dropout_p)
    logits = _conv(ctx, c, "classifier.conv.1", bias=True)
    ctx.rec("logits_lowres", logits)
    outs = [_upsample(logits, size)]
    if aux:
        # auxlayer (models/fast_scnn.py:24-31,42-45); its Dropout follows the same mask law with
        # seed+1 when active.
        a = F.conv2d(hr, ctx.p("auxlayer.0.weight"), None, padding=1)
        a = ctx.relu(ctx.bn(a, "auxlayer.1"), "auxlayer.1")
        if training and dropout_seed is not None and dropout_p > 0:
            keep = dropout_mask(dropout_seed + 1, tuple(a.shape), dropout_p).to(a.dtype)
            a = a * keep / (1.0 - dropout_p)
        a = F.conv2d(a, ctx.p("auxlayer.4.weight"), ctx.p("auxlayer.4.bias"))
        outs.append(_upsample(a, size))
    return tuple(outs), ctx.new_stats, ctx.acts


OHEM_CLASS_WEIGHT = [0.8373, 0.918, 0.866, 1.0345, 1.0166, 0.9969, 0.9754, 1.0489, 0.8786, 1.0023,
                     0.9539, 0.9843, 1.1116, 0.9037, 1.0865, 1.0955, 1.0865, 1.1529, 1.0507]


def ohem_target(predict, target, ignore_label=-1, thresh=0.7, min_kept=256):
    """SoftmaxCrossEntropyOHEMLoss.forward's target rebuild (utils/loss.py:151-172) in numpy:
    label probabilities, threshold (k-th smallest when it exceeds thresh), pixels above it set to
    ignore.  Returns (new_target, threshold or None)."""
    n, c, h, w = predict.shape
    input_label = target.numpy().ravel().astype(np.int32)
    x = np.rollaxis(predict.detach().numpy(), 1).reshape((c, -1))
    input_prob = np.exp(x - x.max(axis=0).reshape((1, -1)))
    input_prob /= input_prob.sum(axis=0).reshape((1, -1))
    valid_flag = input_label != ignore_label
    valid_inds = np.where(valid_flag)[0]
    label = input_label[valid_flag]
    num_valid = valid_flag.sum()
    threshold = None
    if min_kept < num_valid and num_valid > 0:
        prob = input_prob[:, valid_flag]
        pred = prob[label, np.arange(len(label), dtype=np.int32)]
        threshold = thresh
        if min_kept > 0:
            index = pred.argsort()
            threshold_index = index[min(len(index), min_kept) - 1]
            if pred[threshold_index] > thresh:
                threshold = pred[threshold_index]
        valid_inds = valid_inds[pred <= threshold]
    label = input_label[valid_inds].copy()
    input_label.fill(ignore_label)
    input_label[valid_inds] = label
    return torch.from_numpy(input_label.reshape(target.shape)).long(), threshold


def ohem_cross_entropy(predict, target, ignore_label=-1, thresh=0.7, min_kept=256,
                       use_weight=True):
    """SoftmaxCrossEntropyOHEMLoss (utils/loss.py:127-176): weighted CE over the rebuilt target."""
    t, _ = ohem_target(predict, target, ignore_label, thresh, min_kept)
    weight = torch.tensor(OHEM_CLASS_WEIGHT, dtype=predict.dtype) if use_weight else None
    return F.cross_entropy(predict, t, weight=weight, ignore_index=ignore_label)


def dice_loss(pred, target, smooth=1e-6):
    """DiceLoss (utils/loss.py:12-39): 1 - (2 sum(p t) + s) / (sum p + sum t + s) with p the
    softmax probability of class 1 (C > 1) or sigmoid(logit) (C == 1)."""
    p = F.softmax(pred, dim=1)[:, 1] if pred.size(1) > 1 else torch.sigmoid(pred.squeeze(1))
    p = p.contiguous().view(-1)
    t = target.contiguous().view(-1).to(p.dtype)
    inter = (p * t).sum()
    return 1 - (2. * inter + smooth) / (p.sum() + t.sum() + smooth)


def focal_dice_loss(pred, target, alpha=0.5, gamma=2.0, dice_weight=0.5, smooth=1e-6):
    """FocalDiceLoss (utils/loss.py:71-100): multi-class logits (:83-86), or one logit channel
    with the sigmoid + binary cross entropy focal term (:87-92)."""
    if pred.size(1) > 1:
        ce = F.cross_entropy(pred, target, reduction="none")
        pt = torch.exp(-ce)
    else:
        prob = torch.sigmoid(pred.squeeze(1))
        tf = target.to(prob.dtype)
        ce = F.binary_cross_entropy(prob, tf, reduction="none")
        pt = torch.where(tf == 1, prob, 1 - prob)
    focal = (alpha * (1 - pt) ** gamma * ce).mean()
    return (1 - dice_weight) * focal + dice_weight * dice_loss(pred, target, smooth)


def to_tensor_normalize(img_hwc_u8, mean, std):
    """transforms.ToTensor() + transforms.Normalize(mean, std) (train.py:104-107): uint8 HWC ->
    fp32 CHW, torchvision's operation order (float().div(255), sub_(mean), div_(std))."""
    t = torch.from_numpy(np.ascontiguousarray(img_hwc_u8)).permute(2, 0, 1).contiguous()
    t = t.float().div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
    return t.sub(m).div(s)


def cityscapes_class_to_index(mask):
    """CitySegmentation._class_to_index (data_loader/cityscapes.py:56-71), the same key / mapping
    tables and np.digitize(right=True) lookup (restated: the reference module imports
    torchvision, which is absent here)."""
    key = np.array([-1, -1, -1, -1, -1, -1, -1, -1, 0, 1, -1, -1, 2, 3, 4, -1, -1, -1, 5, -1, 6,
                    7, 8, 9, 10, 11, 12, 13, 14, 15, -1, -1, 16, 17, 18])
    mapping = np.array(range(-1, len(key) - 1)).astype('int32')
    index = np.digitize(np.asarray(mask).ravel(), mapping, right=True)
    return key[index].reshape(np.asarray(mask).shape)


def seg_counts(pred, label, nclass):
    """SegmentationMetric counters of one batch (utils/metric.py:73-105): numpy int64
    [correct, labeled, inter[C], area_pred[C], area_lab[C]] exactly as batch_pix_accuracy and
    batch_intersection_union compute them (+1 shift, histograms over [1, nclass])."""
    p = np.asarray(pred).astype(np.int64) + 1
    t = np.asarray(label).astype(np.int64) + 1
    labeled = int(np.sum(t > 0))
    correct = int(np.sum((p == t) * (t > 0)))
    p = p * (t > 0).astype(p.dtype)
    inter = p * (p == t)
    hist = lambda v: np.histogram(v, bins=nclass, range=(1, nclass))[0]  # noqa: E731
    return np.concatenate([[correct, labeled], hist(inter), hist(p), hist(t)]).astype(np.int64)


def seg_scores(counts, nclass):
    """SegmentationMetric.get (utils/metric.py:42-54) from accumulated counters."""
    c = np.asarray(counts)
    inter, area_pred, area_lab = c[2:2 + nclass], c[2 + nclass:2 + 2 * nclass], c[2 + 2 * nclass:]
    union = area_pred + area_lab - inter
    pix_acc = 1.0 * c[0] / (np.spacing(1) + c[1])
    iou = 1.0 * inter / (np.spacing(1) + union)
    return pix_acc, iou.mean()


def cross_entropy(logits, target, ignore_index=-1):
    """nn.CrossEntropyLoss(ignore_index=-1), mean over valid pixels (utils/loss.py:103-124)."""
    return F.cross_entropy(logits, target, ignore_index=ignore_index)


def sgd_step(params, grads, bufs, lr, momentum=0.9, weight_decay=1e-4):
    """torch.optim.SGD step (train.py:195-198): d = g + wd*p; buf = m*buf + d (buf=d first); p -= lr*buf."""
    out_p, out_b = {}, {}
    for k, p in params.items():
        d = grads[k] + weight_decay * p
        b = d.clone() if bufs.get(k) is None else momentum * bufs[k] + d
        out_b[k] = b
        out_p[k] = p - lr * b
    return out_p, out_b
