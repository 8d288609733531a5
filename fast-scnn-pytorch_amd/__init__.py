"""fast_scnn_pytorch_amd — MI355X-native (gfx950) Fast-SCNN forward/backward hot path.

Importable as ``fast_scnn_pytorch_amd`` via ``_fscnn_boot.load()`` (the directory name has a
hyphen).  The drop-in module for reference callers is the top-level ``models`` package.

Submodules:
  arch           canonical tensor table (state_dict schema of models/fast_scnn.py)
  portable_init  counter-based weight / input generator (no torch RNG)
  _lib           ctypes binding of the C-ABI library libfastscnn_hip.so (fails loudly if absent)
  fast_scnn      FastSCNN / get_fast_scnn — the reference interface, running on HIP kernels
  loss           fused cross-entropy criterion (HIP)
  optim          fused multi-tensor SGD (HIP)
  ddp            one-process-per-GPU data parallel with bucketed RCCL gradient all-reduce
"""
__all__ = ["FastSCNN", "get_fast_scnn"]


def __getattr__(name):
    if name in ("FastSCNN", "get_fast_scnn"):
        from . import fast_scnn
        return getattr(fast_scnn, name)
    raise AttributeError(name)
