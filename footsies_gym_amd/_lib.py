"""Loads libfootsies.so (the HIP product path) via ctypes.

There is no CPU fallback: if the library is missing or no MI355X is visible, the
calls fail loudly with :class:`FootsiesError`.
"""
import ctypes as C
import os
import sys

from . import _abi

IN_TREE_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfootsies.so")
# FOOTSIES_LIB overrides the in-tree library (kernel A/B experiments, tools/ab_time.py); lib() says so
# on stderr and `library_info()` reports it, so a swapped library is never silent
LIB_PATH = os.environ.get("FOOTSIES_LIB") or IN_TREE_LIB


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
        # torch first when it is installed: its HIP runtime (libamdhip64.so.7, bundled with the wheel)
        # is then the one the library's DT_NEEDED entry binds to, so the process holds a single HIP /
        # HSA runtime.  Loaded the other way round, /opt/rocm's runtime comes in first and fs_create's
        # hipGetDeviceCount failed on the MI355X box (profiles/r05q_lib_before_torch.log); fs_create
        # now names both images in that case (FS_E_RUNTIME).  Without torch the library binds to
        # /opt/rocm's runtime and the C-ABI works as in tests/native/abi_lockstep.cpp.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if LIB_PATH != IN_TREE_LIB:
            print("footsies_gym_amd: FOOTSIES_LIB overrides the in-tree library: %s" % LIB_PATH, file=sys.stderr)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _abi.LIB_FUNCTIONS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.fs_abi_version() != _abi.FS_ABI_VERSION:
            raise ImportError("libfootsies ABI version mismatch")
        rt, bt = C.c_int(0), C.c_int(0)
        L.fs_runtime_version(C.byref(rt), C.byref(bt))
        # HIP_VERSION = major * 10^7 + minor * 10^5 + patch: the runtime the library bound to must be
        # the major version it was compiled against (a minor mismatch is HIP's supported case)
        if rt.value and rt.value // 10000000 != bt.value // 10000000:
            raise ImportError("libfootsies was built against HIP %d but bound to HIP runtime %d (%s)"
                              % (bt.value, rt.value, runtime_images(L)))
        _lib = L
    return _lib


def runtime_images(L=None):
    """The HIP / HSA runtime images mapped into this process, as fs_runtime_images lists them."""
    buf = C.create_string_buffer(8192)
    (L or lib()).fs_runtime_images(buf, len(buf))
    return buf.value.decode()


def library_info():
    """Which libfootsies.so this process uses and what it is bound to (bench.py reports it)."""
    L = lib()
    rt, bt = C.c_int(0), C.c_int(0)
    L.fs_runtime_version(C.byref(rt), C.byref(bt))
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(IN_TREE_LIB))),
            "override": LIB_PATH != IN_TREE_LIB, "hip_runtime": rt.value, "hip_build": bt.value,
            "runtime_images": runtime_images(L).split()}


def check(rc, handle=None):
    if rc != 0:
        msg = lib().fs_last_error(handle)
        raise FootsiesError(rc, msg.decode() if msg else "")
    return rc
