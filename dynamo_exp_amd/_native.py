"""Loader for the in-tree native extensions.

``_C_kernels`` (HIP, gfx950) must be importable whenever a GPU op runs: GPU
code paths never fall back silently -- if the extension is missing on a box
with a GPU, :func:`kernels` raises.  ``_C_runtime`` (host C++) has pure-Python
fallbacks for CPU-only environments (CI), see ``dynamo_exp_amd.kv.hashing``.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_kernels = None
_kernels_err: Exception | None = None
_runtime = None
_runtime_err: Exception | None = None


def _try_build() -> None:
    if os.environ.get("DX_NO_AUTOBUILD"):
        return
    try:
        from . import build_native

        build_native.build_all()
    except Exception as e:  # pragma: no cover - build env specific
        import sys

        print(f"[dynamo_exp_amd] native build failed: {e}", file=sys.stderr)


def kernels():
    """Return the ``_C_kernels`` module, building it in-tree on first use."""
    global _kernels, _kernels_err
    if _kernels is not None:
        return _kernels
    with _lock:
        if _kernels is not None:
            return _kernels
        import torch  # noqa: F401  -- load torch's HIP runtime before ours (same SONAME)

        try:
            _kernels = importlib.import_module("dynamo_exp_amd._C_kernels")
        except ImportError:
            _try_build()
            try:
                _kernels = importlib.import_module("dynamo_exp_amd._C_kernels")
            except ImportError as e:
                _kernels_err = e
                raise RuntimeError(
                    "dynamo_exp_amd._C_kernels (gfx950 HIP kernels) is not built; run "
                    "`python -m dynamo_exp_amd.build_native`"
                ) from e
    return _kernels


def runtime():
    """Return the ``_C_runtime`` module or None if it cannot be built."""
    global _runtime, _runtime_err
    if _runtime is not None or _runtime_err is not None:
        return _runtime
    with _lock:
        if _runtime is not None or _runtime_err is not None:
            return _runtime
        try:
            _runtime = importlib.import_module("dynamo_exp_amd._C_runtime")
        except ImportError:
            _try_build()
            try:
                _runtime = importlib.import_module("dynamo_exp_amd._C_runtime")
            except ImportError as e:
                _runtime_err = e
                _runtime = None
    return _runtime
