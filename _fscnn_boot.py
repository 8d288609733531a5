"""Bootstrap loader for the ``fast-scnn-pytorch_amd`` package directory.

The package directory name contains a hyphen (it mirrors the upstream repo name), so it cannot be
imported with a plain ``import`` statement.  This module registers it in ``sys.modules`` under the
importable name ``fast_scnn_pytorch_amd`` so that relative imports inside the package work.
"""
import importlib.util
import os
import sys

PKG_NAME = "fast_scnn_pytorch_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fast-scnn-pytorch_amd")


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(PKG_NAME, None)
        raise
    return mod
