"""wst_amd -- MI355X-native 2-D wavelet scattering transform (drop-in for kymatio's Scattering2D
on the reference's WST feature path).

Import forms mirrored from the reference:
  ``from kymatio.numpy import Scattering2D``  -> ``from wst_amd.numpy import Scattering2D``
  ``from kymatio.torch import Scattering2D``  -> ``from wst_amd.torch import Scattering2D``
  ``from kymatio import Scattering2D`` + ``frontend='numpy'|'torch'`` -> ``wst_amd.Scattering2D``

This directory is the package; the repo-root shim ``wst_amd.py`` registers it under the
importable name ``wst_amd`` (the directory name itself contains hyphens).
"""
from __future__ import annotations

__version__ = "0.1.0"

from .frontend import compute_padding, num_coefficients  # noqa: F401


class Scattering2D:
    """Frontend-dispatching entry point (kymatio 0.3.0 ``frontend/entry.py``): returns a
    numpy (default) or torch frontend instance."""

    def __new__(cls, *args, frontend: str = "numpy", **kwargs):
        fe = str(frontend).lower()
        if fe == "numpy":
            from .numpy import Scattering2D as S
        elif fe == "torch":
            from .torch import Scattering2D as S
        else:
            raise RuntimeError(f"The frontend '{frontend}' is not valid. Must be one of "
                               "'numpy' or 'torch'.")
        return S(*args, **kwargs)
