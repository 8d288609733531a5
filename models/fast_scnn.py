"""``models.fast_scnn`` shim: the reference module path, backed by the HIP implementation."""
import _fscnn_boot

_pkg = _fscnn_boot.load()
from fast_scnn_pytorch_amd.fast_scnn import (  # noqa: E402,F401
    Classifer, FastSCNN, FeatureFusionModule, GlobalFeatureExtractor, LearningToDownsample,
    LinearBottleneck, PyramidPooling, _ConvBNReLU, _DSConv, _DWConv, get_fast_scnn)

__all__ = ["FastSCNN", "get_fast_scnn"]
