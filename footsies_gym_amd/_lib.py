"""Loads libfootsies.so (the HIP product path) via ctypes.

There is no CPU fallback: if the library is missing or no MI355X is visible, the
calls fail loudly with :class:`FootsiesError`.
"""
import ctypes as C
import os

from . import _abi

# FOOTSIES_LIB overrides the in-tree library (kernel experiments, tools/kernel_variants.py)
LIB_PATH = os.environ.get("FOOTSIES_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfootsies.so")


class FootsiesGameClosedError(RuntimeError):
    """The reference's FootsiesGameClosedError (exceptions.py:1-2): raised, as there, when an
    environment is used after its game was closed (here: after close())."""


class FootsiesError(RuntimeError):
    """A libfootsies call failed (code + fs_last_error message)."""

    def __init__(self, code, message):
        super().__init__("libfootsies error %d: %s" % (code, message))
        self.code = code


_lib = None


def lib():
    """The loaded library with argtypes/restypes from ``_abi.LIB_FUNCTIONS``."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libfootsies.so is not built (expected at %s); run `python -m footsies_gym_amd.build`"
                              % LIB_PATH)
        # torch first: its HIP runtime (libamdhip64.so.7, bundled with the wheel) is then the one the
        # library's DT_NEEDED entry binds to, so the process holds a single HIP / HSA runtime.  Loaded
        # the other way round, /opt/rocm's runtime comes in first and fs_create's hipGetDeviceCount
        # failed on the MI355X box ("no ROCm-capable device", profiles/r05q_lib_before_torch.log).
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _abi.LIB_FUNCTIONS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.fs_abi_version() != _abi.FS_ABI_VERSION:
            raise ImportError("libfootsies ABI version mismatch")
        _lib = L
    return _lib


def check(rc, handle=None):
    if rc != 0:
        msg = lib().fs_last_error(handle)
        raise FootsiesError(rc, msg.decode() if msg else "")
    return rc
