"""Loader for antidote_amd/libantidote_gpu.so (the product C ABI).

Fails loudly: there is no CPU fallback.  If the library is missing, was built
for another ABI, or no gfx950 GPU is present, EngineUnavailable is raised.

PyTorch-ROCm ships its own copy of the HIP runtime (same soname as
/opt/rocm's).  When torch is importable it is imported first, so this
library binds to the runtime torch already loaded and the process holds a
single HIP runtime (device pointers and streams can then be shared with
torch, which bench.py uses for events and torch.distributed).
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AGN_LIB", os.path.join(HERE, "libantidote_gpu.so"))

_lock = threading.Lock()
_lib = None


class EngineUnavailable(RuntimeError):
    """The HIP engine cannot run here (library not built / no MI355X)."""


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


def load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise EngineUnavailable(
                f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            import torch  # noqa: F401  (pin the process's HIP runtime first)
        except Exception:
            pass
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _abi.bind(lib, _abi.PROTOTYPES)
        if lib.agn_abi_version() != _abi.ABI_VERSION:
            raise EngineUnavailable("libantidote_gpu.so ABI mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str = ""):
    if rc != _abi.OK:
        lib = load()
        msg = lib.agn_last_error().decode(errors="replace")
        raise EngineError(rc, f"{what}: {msg}" if what else msg)
    return rc


def env_changed():
    """Tell the library that an AGN_* environment knob changed in this process
    (it caches them: agn_env_reload).  A no-op before the library is loaded."""
    if _lib is not None:
        _lib.agn_env_reload()


def set_knob(name, value):
    """Set (value given) or unset (None) an AGN_* knob for this process and
    pass the change on to the library."""
    if value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = value
    env_changed()
