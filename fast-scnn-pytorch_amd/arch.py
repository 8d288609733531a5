"""Canonical Fast-SCNN tensor table: every conv/BN of the network with its state_dict key.

The order is the reference module registration order, so ``named_parameters()`` /
``state_dict()`` of ``fast_scnn.FastSCNN`` match the reference (268 keys
without aux, 276 with aux; 136 / 141 parameter tensors).  The C++ executor
(``csrc/net.cpp``) carries the same table; ``FastSCNN`` checks both agree at construction.

Source of the structure: ``models/fast_scnn.py:20-31`` (top level), ``:153-155`` (LTD),
``:170-173`` (GFE), ``:103-108`` (LinearBottleneck), ``:124-128`` (PPM), ``:196-204`` (FFM),
``:226-231`` (Classifer).
"""

# (prefix, cin, cout) LinearBottleneck instances, t = 6 (models/fast_scnn.py:170-172)
_BOTTLENECKS = [
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

NUM_CLASS = {"citys": 19, "tusimple": 2, "bdd100k": 2, "custom": 2}


def layers(num_classes, aux=False):
    """Ordered primitive list: ('conv', key, cin, cout, k, groups, bias) | ('bn', key, C)."""
    L = []

    def conv(key, cin, cout, k=1, groups=1, bias=False):
        L.append(("conv", key, cin, cout, k, groups, bias))

    def bn(key, c):
        L.append(("bn", key, c))

    def dsconv(pfx, cin, cout):
        conv(pfx + ".conv.0", cin, cin, 3, cin)
        bn(pfx + ".conv.1", cin)
        conv(pfx + ".conv.3", cin, cout)
        bn(pfx + ".conv.4", cout)

    conv("learning_to_downsample.conv.conv.0", 3, 32, 3)
    bn("learning_to_downsample.conv.conv.1", 32)
    dsconv("learning_to_downsample.dsconv1", 32, 48)
    dsconv("learning_to_downsample.dsconv2", 48, 64)
    for pfx, cin, cout, _s in _BOTTLENECKS:
        e = cin * 6
        conv(pfx + ".block.0.conv.0", cin, e)
        bn(pfx + ".block.0.conv.1", e)
        conv(pfx + ".block.1.conv.0", e, e, 3, e)
        bn(pfx + ".block.1.conv.1", e)
        conv(pfx + ".block.2", e, cout)
        bn(pfx + ".block.3", cout)
    for i in range(1, 5):
        conv("global_feature_extractor.ppm.conv%d.conv.0" % i, 128, 32)
        bn("global_feature_extractor.ppm.conv%d.conv.1" % i, 32)
    conv("global_feature_extractor.ppm.out.conv.0", 256, 128)
    bn("global_feature_extractor.ppm.out.conv.1", 128)
    conv("feature_fusion.dwconv.conv.0", 128, 128, 3, 128)
    bn("feature_fusion.dwconv.conv.1", 128)
    conv("feature_fusion.conv_lower_res.0", 128, 128, bias=True)
    bn("feature_fusion.conv_lower_res.1", 128)
    conv("feature_fusion.conv_higher_res.0", 64, 128, bias=True)
    bn("feature_fusion.conv_higher_res.1", 128)
    dsconv("classifier.dsconv1", 128, 128)
    dsconv("classifier.dsconv2", 128, 128)
    conv("classifier.conv.1", 128, num_classes, bias=True)
    if aux:
        conv("auxlayer.0", 64, 32, 3)
        bn("auxlayer.1", 32)
        conv("auxlayer.4", 32, num_classes, bias=True)
    return L


def param_specs(num_classes, aux=False):
    """[(key, shape, kind, fan_in)] in named_parameters() order."""
    out = []
    for op in layers(num_classes, aux):
        if op[0] == "conv":
            _, key, cin, cout, k, groups, bias = op
            fan_in = (cin // groups) * k * k
            out.append((key + ".weight", (cout, cin // groups, k, k), "conv_w", fan_in))
            if bias:
                out.append((key + ".bias", (cout,), "conv_b", fan_in))
        else:
            _, key, c = op
            out.append((key + ".weight", (c,), "bn_w", 0))
            out.append((key + ".bias", (c,), "bn_b", 0))
    return out


def buffer_specs(num_classes, aux=False):
    """[(key, shape, kind)] in named_buffers() order (BN running stats)."""
    out = []
    for op in layers(num_classes, aux):
        if op[0] == "bn":
            _, key, c = op
            out.append((key + ".running_mean", (c,), "bn_rm"))
            out.append((key + ".running_var", (c,), "bn_rv"))
            out.append((key + ".num_batches_tracked", (), "bn_nbt"))
    return out


def state_dict_specs(num_classes, aux=False):
    """{key: (shape, kind, fan_in)} for portable_init.state_dict_arrays, state_dict() order."""
    out = {}
    for op in layers(num_classes, aux):
        if op[0] == "conv":
            _, key, cin, cout, k, groups, bias = op
            fan_in = (cin // groups) * k * k
            out[key + ".weight"] = ((cout, cin // groups, k, k), "conv_w", fan_in)
            if bias:
                out[key + ".bias"] = ((cout,), "conv_b", fan_in)
        else:
            _, key, c = op
            for suf, kind in (("weight", "bn_w"), ("bias", "bn_b"), ("running_mean", "bn_rm"),
                              ("running_var", "bn_rv"), ("num_batches_tracked", "bn_nbt")):
                out[key + "." + suf] = ((c,) if kind != "bn_nbt" else (), kind, 0)
    return out


def portable_state_dict(num_classes, aux=False, seed=0, variant="default"):
    """numpy state_dict from the counter-based generator (see portable_init)."""
    from . import portable_init
    return portable_init.state_dict_arrays(state_dict_specs(num_classes, aux), seed, variant)
