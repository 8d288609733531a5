"""Portable, counter-based parameter and input generator.

Every value is a pure function of (seed, tensor name, element index), computed with splitmix64 in
numpy uint64 arithmetic.  The same weights and inputs can therefore be rebuilt bit-for-bit on the
GPU box without the reference tree and without torch's RNG.

Init laws (``variant``):
  * ``"default"`` mirrors PyTorch's layer defaults used by the reference modules
    (``models/fast_scnn.py:55,70,73,86,107,198,202,230``): conv weight and bias ~ U(±1/sqrt(fan_in)),
    BatchNorm gamma=1, beta=0, running_mean=0, running_var=1, num_batches_tracked=0.
  * ``"bnrand"`` keeps the conv law but randomises BN: gamma~U[0.75,1.25], beta~U[-0.1,0.1],
    running_mean~U[-0.1,0.1], running_var~U[0.5,1.0].  It defeats the bias-dominated-logits trap of
    SURVEY.md §0 only partly; the golden fixtures additionally calibrate running stats.
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _fnv1a64(text):
    h = 0xCBF29CE484222325
    for ch in text.encode("utf-8"):
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(x):
    """Vectorised splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed, name, n):
    """n float64 values in [0, 1) (24-bit resolution, exactly representable in fp32)."""
    key = np.uint64((_fnv1a64(name) ^ (int(seed) * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + key * _GOLDEN
    bits = splitmix64(ctr) >> np.uint64(40)
    return bits.astype(np.float64) * (1.0 / float(1 << 24))


def uniform_range(seed, name, shape, lo, hi):
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform(seed, name, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def input_tensor(seed, shape, name="input"):
    """Synthetic image batch: unit-variance uniform U[-sqrt(3), sqrt(3)) in fp32 (NCHW)."""
    s = np.sqrt(3.0)
    return uniform_range(seed, name, shape, -s, s)


def target_tensor(seed, shape, num_classes, ignore_frac=0.0, name="target"):
    """Synthetic int64 label map; ``ignore_frac`` of pixels set to the ignore label -1."""
    n = int(np.prod(shape))
    u = uniform(seed, name, n)
    t = np.minimum((u * num_classes).astype(np.int64), num_classes - 1)
    if ignore_frac > 0:
        v = uniform(seed, name + ".ignore", n)
        t[v < ignore_frac] = -1
    return t.reshape(shape)


def state_dict_arrays(shapes, seed=0, variant="default"):
    """Build numpy arrays for a state_dict given ``{key: (shape, kind, fan_in)}``.

    ``kind`` is one of conv_w, conv_b, bn_w, bn_b, bn_rm, bn_rv, bn_nbt.
    """
    out = {}
    for key, (shape, kind, fan_in) in shapes.items():
        if kind in ("conv_w", "conv_b"):
            b = 1.0 / np.sqrt(fan_in)
            out[key] = uniform_range(seed, key, shape, -b, b)
        elif kind == "bn_nbt":
            out[key] = np.zeros((), dtype=np.int64)
        elif variant == "default":
            fill = {"bn_w": 1.0, "bn_b": 0.0, "bn_rm": 0.0, "bn_rv": 1.0}[kind]
            out[key] = np.full(shape, fill, dtype=np.float32)
        elif variant == "bnrand":
            lo, hi = {"bn_w": (0.75, 1.25), "bn_b": (-0.1, 0.1), "bn_rm": (-0.1, 0.1),
                      "bn_rv": (0.5, 1.0)}[kind]
            out[key] = uniform_range(seed, key, shape, lo, hi)
        else:
            raise ValueError("unknown init variant %r" % (variant,))
    return out
