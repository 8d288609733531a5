"""Drop-in replacement for the reference ``models`` package (models/__init__.py:1-3).

``from models.fast_scnn import FastSCNN, get_fast_scnn`` resolves to the MI355X HIP
implementation in ``fast-scnn-pytorch_amd/`` so train.py / eval.py / demo.py run unchanged.
"""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from .fast_scnn import get_fast_scnn  # noqa: E402

__all__ = ["get_fast_scnn"]
