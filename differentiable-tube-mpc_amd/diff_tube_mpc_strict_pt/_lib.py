"""Loader for libdtmpc.so, the HIP (gfx950) implementation of include/dtmpc.h.

There is no fallback: every batched entry point of this package calls the native library, and
loading fails loudly (``NativeLibraryError``) when it is missing.  Build it with
``python differentiable-tube-mpc_amd/build.py`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _abi

LIB_NAME = "libdtmpc.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# DTMPC_LIBRARY names an alternative build of the same ABI (e.g. a kernel variant from
# ``build.py --variant``); it replaces the path, never adds a fallback.
LIB_PATH = os.environ.get("DTMPC_LIBRARY", LIB_PATH)

_lock = threading.Lock()
_lib = None


class NativeLibraryError(RuntimeError):
    """libdtmpc.so is missing, stale or failed a call."""


def load() -> C.CDLL:
    """Load (once) and return the native library with its prototypes bound."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build the HIP extension first "
                "(python differentiable-tube-mpc_amd/build.py)"
            )
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _abi.PROTOTYPES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.dtmpc_abi_version()
        if v != _abi.ABI_VERSION:
            raise NativeLibraryError(f"libdtmpc ABI {v} != expected {_abi.ABI_VERSION}; rebuild")
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != _abi.OK:
        msg = load().dtmpc_last_error().decode(errors="replace")
        if rc == _abi.ERR_BAD_ARG:
            raise ValueError(f"{what}: {msg}")
        raise NativeLibraryError(f"{what} failed ({rc}): {msg}")


def stream_of(t) -> int:
    """Raw hipStream_t of torch's current stream on t's device (0 = default stream)."""
    import torch

    return int(torch.cuda.current_stream(t.device).cuda_stream)
