"""``raydp`` — drop-in import name for ``raydp_amd`` (the reference's package name).

``import raydp`` gives the same API as the reference (``init_spark``, ``stop_spark``,
``raydp.spark``, ``raydp.torch``, ``raydp.utils``, ``raydp.mpi``, ...). Every ``raydp.<sub>``
module IS the corresponding ``raydp_amd.<sub>`` module object (aliased, not copied). When no
real ``ray`` / ``pyspark`` is importable, lightweight ``ray`` and ``pyspark`` facades backed by
this framework are registered so unmodified reference scripts run (see
``raydp_amd/compat``).
"""
import importlib
import importlib.abc
import importlib.util
import sys

import raydp_amd
from raydp_amd import __version__, init_spark, stop_spark


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith("raydp."):
            return None
        real = "raydp_amd." + fullname[len("raydp."):]
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

from raydp_amd import compat as _compat  # noqa: E402

_compat.install()


def __getattr__(name):
    try:
        return importlib.import_module(f"raydp.{name}")
    except ImportError:
        raise AttributeError(name) from None


__all__ = ["init_spark", "stop_spark", "__version__"]
