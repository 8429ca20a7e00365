"""Locate / build / load the in-tree native libraries.

Libraries live next to this file (``raydp_amd/native/lib<name>.so``) so they travel with the
repository snapshot and show up as in-tree ``.so`` loads. CPU libraries are compiled on first
use if absent (g++ is always present); the HIP kernel library is built by
``python -m raydp_amd.native.build`` (hipcc, gfx950) and is *required* on a GPU: the GPU ops
fail loudly instead of falling back to eager PyTorch.
"""
import ctypes
import os
import subprocess
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
_lock = threading.Lock()
_loaded = {}


def lib_path(name: str) -> str:
    return os.path.join(HERE, f"lib{name}.so")


def load(name: str, build_if_missing: bool = True):
    with _lock:
        if name in _loaded:
            return _loaded[name]
        path = lib_path(name)
        if not os.path.exists(path) and build_if_missing:
            from raydp_amd.native import build
            build.build_one(name)
        if not os.path.exists(path):
            raise ImportError(f"native library {path} is not built; run "
                              f"`python -m raydp_amd.native.build`")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL if name == "hipkernels" else 0)
        _loaded[name] = lib
        return lib


def executable(name: str, build_if_missing: bool = True) -> str:
    """Path of an in-tree native executable (built on first use).

    ``RAYDP_NATIVE_BIN_DIR`` points at an alternative build of the services (the sanitizer
    builds of ``scripts/sanitize_runtime.sh``); a binary found there wins."""
    alt = os.environ.get("RAYDP_NATIVE_BIN_DIR")
    if alt and os.path.exists(os.path.join(alt, name)):
        return os.path.join(alt, name)
    from raydp_amd.native import build
    path = build.out_path(name)
    with _lock:
        if build_if_missing and not build._newer(path, build.LIBS[name]["sources"]()):
            build.build_one(name)
    if not os.path.exists(path):
        raise ImportError(f"native executable {path} is not built")
    return path


def is_built(name: str) -> bool:
    return os.path.exists(lib_path(name))
