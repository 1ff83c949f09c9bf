"""footsies_gym_amd -- MI355X-native vectorized FOOTSIES simulator.

The hot path (the per-frame fighter state machine of the reference Unity game,
stepped for N independent arenas) runs in hand-written HIP kernels for gfx950
inside libfootsies.so, reached through a plain C-ABI (include/footsies.h) via
ctypes.  Python-side surfaces:

  FootsiesVectorEnv  gymnasium-style VectorEnv over N arenas (drop-in for N x FootsiesEnv)
  FootsiesEnv        single-arena adapter with the reference FootsiesEnv API
  FootsiesSim        the zero-copy handle (torch device tensors in/out)
  wrappers           vectorized counterparts of the reference's gymnasium wrappers
  moves              the reference's FootsiesMove table (ids, durations, attack frame data)
"""
from ._abi import MOVE_ID_TO_INDEX, MOVE_INDEX_TO_ID, MOVES  # noqa: F401
from ._lib import FootsiesError, FootsiesGameClosedError  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not require torch or a GPU
    if name in ("FootsiesSim", "encode_actions", "decode_actions"):
        from . import simulator
        return getattr(simulator, name)
    if name in ("FootsiesVectorEnv", "FootsiesEnv"):
        from . import vector_env
        return getattr(vector_env, name)
    if name in ("FootsiesActionCombinationsDiscretized", "FootsiesNormalized", "FootsiesFrameSkipped",
                "FootsiesStatistics"):
        from . import wrappers
        return getattr(wrappers, name)
    raise AttributeError(name)


def register():
    """Register FootsiesEnv-v0 / FootsiesVectorEnv-v0 with gymnasium when it is installed
    (the reference registers FootsiesEnv-v0, footsies_gym/__init__.py:3-7)."""
    try:
        from gymnasium.envs.registration import register as _reg
    except Exception:
        return False
    _reg(id="FootsiesEnv-v0", entry_point="footsies_gym_amd.vector_env:FootsiesEnv")
    _reg(id="FootsiesVectorEnv-v0", entry_point="footsies_gym_amd.vector_env:FootsiesVectorEnv")
    return True
