"""roctx ranges around the engine's layer-level ops (SURVEY §5 tracing aux).

Off by default.  TT2_ROCTX=1 loads ROCm's roctx library and every decorated op pushes a
named range, so `rocprofv3 --marker-trace` (or any roctx consumer) shows the encoder,
decoder, post-net, loss, backward and optimizer spans around the kernels they launch.
Host-side markers: a hipGraph replay runs none of them (they mark the eager / capture
pass), and with the switch off the decorator returns the function unchanged."""
from __future__ import annotations

import ctypes
import functools
import os

_LIBS = ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
         "/opt/rocm/lib/libroctx64.so.4")
_roctx = None


def _load():
    global _roctx
    if _roctx is None:
        for name in _LIBS:
            try:
                lib = ctypes.CDLL(name)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes, lib.roctxRangePushA.restype = [ctypes.c_char_p], ctypes.c_int
            lib.roctxRangePop.argtypes, lib.roctxRangePop.restype = [], ctypes.c_int
            _roctx = lib
            break
        else:
            raise RuntimeError("TT2_ROCTX=1 but no roctx library could be loaded")
    return _roctx


def enabled() -> bool:
    return os.environ.get("TT2_ROCTX", "0") not in ("", "0")


class Range:
    """with Range("name"): ...  (no-op unless TT2_ROCTX=1)"""

    def __init__(self, name: str):
        self.name = name.encode()
        self.on = enabled()

    def __enter__(self):
        if self.on:
            _load().roctxRangePushA(self.name)
        return self

    def __exit__(self, *exc):
        if self.on:
            _load().roctxRangePop()
        return False


def ranged(name: str):
    """Decorator: the call runs inside roctx range `name` when TT2_ROCTX=1 at import time."""

    def deco(fn):
        if not enabled():
            return fn

        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with Range(name):
                return fn(*a, **kw)

        return wrapper

    return deco
