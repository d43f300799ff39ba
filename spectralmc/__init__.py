"""Import-path alias: ``spectralmc.X`` is ``spectralmc_amd.X``.

Lets code written against the reference package (``from spectralmc.gbm import
BlackScholes`` ...) run unchanged on this implementation: every submodule import under
``spectralmc`` resolves to the same module object under ``spectralmc_amd``.
"""

from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = "spectralmc_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target: str) -> None:
        self._target = target

    def create_module(self, spec):  # noqa: ANN001
        return importlib.import_module(self._target)

    def exec_module(self, module) -> None:  # noqa: ANN001
        return None


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname: str, path=None, target=None):  # noqa: ANN001
        if not fullname.startswith(__name__ + "."):
            return None
        real = _TARGET + fullname[len(__name__):]
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

__version__ = importlib.import_module(_TARGET).__version__
