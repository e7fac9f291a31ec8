"""Import shim: registers the package directory
``wst-feature-extraction-for-remote-sensing-vegetation-classification-via-machine-learning_amd/``
(whose name is not a Python identifier) as the importable package ``wst_amd``.

    import wst_amd                      # from the repo root (or with the repo on sys.path)
    from wst_amd.numpy import Scattering2D
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "wst-feature-extraction-for-remote-sensing-vegetation-classification-via-machine-learning_amd")

_spec = importlib.util.spec_from_file_location(
    "wst_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules["wst_amd"] = _pkg
_spec.loader.exec_module(_pkg)
