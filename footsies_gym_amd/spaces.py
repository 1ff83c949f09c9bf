"""Observation / action spaces of FootsiesEnv (footsies.py:152-174).

Uses gymnasium.spaces when gymnasium is importable; otherwise a minimal local
stand-in with the same constructor arguments, ``shape``/``dtype`` and
``contains``/``sample`` so code written against the reference keeps working.
"""
import numpy as np

from ._abi import MOVES

try:  # pragma: no cover - depends on the environment
    from gymnasium import spaces as _gs
except Exception:  # gymnasium is not installed in this image
    _gs = None


class _Space:
    def __init__(self, shape, dtype, seed=None):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)


class MultiDiscrete(_Space):
    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        super().__init__(self.nvec.shape, dtype, seed)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x >= 0) & (x < self.nvec)))

    def sample(self):
        return (self._rng.random(self.shape) * self.nvec).astype(self.dtype)


class Box(_Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        shape = shape if shape is not None else np.shape(low)
        super().__init__(shape, dtype, seed)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x >= self.low) & (x <= self.high)))

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)


class MultiBinary(_Space):
    def __init__(self, n, seed=None):
        self.n = n
        super().__init__((n,) if np.isscalar(n) else tuple(n), np.int8, seed)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x == 0) | (x == 1)))

    def sample(self):
        return self._rng.integers(0, 2, self.shape).astype(self.dtype)


class Discrete(_Space):
    def __init__(self, n, seed=None):
        self.n = int(n)
        super().__init__((), np.int64, seed)

    def contains(self, x):
        return 0 <= int(x) < self.n

    def sample(self):
        return int(self._rng.integers(0, self.n))


class Dict(dict):
    def __init__(self, spaces, seed=None):
        super().__init__(spaces)
        self.spaces = self

    def contains(self, x):
        return all(k in x and s.contains(x[k]) for k, s in self.items())

    def sample(self):
        return {k: s.sample() for k, s in self.items()}


if _gs is not None:  # pragma: no cover
    MultiDiscrete, Box, MultiBinary, Discrete, Dict = _gs.MultiDiscrete, _gs.Box, _gs.MultiBinary, _gs.Discrete, _gs.Dict

RELEVANT_MOVES = [m for m in MOVES if m[0] not in ("WIN", "DEAD")]  # footsies.py:153
MAX_MOVE_DURATION = max(m[2] for m in RELEVANT_MOVES)               # footsies.py:154 (55)


def single_observation_space():
    """FootsiesEnv.observation_space (footsies.py:157-168)."""
    n = len(RELEVANT_MOVES)
    return Dict({
        "guard": MultiDiscrete([4, 4]),
        "move": MultiDiscrete([n, n]),
        "move_frame": Box(low=0.0, high=float(MAX_MOVE_DURATION), shape=(2,)),
        "position": Box(low=-4.6, high=4.6, shape=(2,)),
    })


def single_action_space():
    """FootsiesEnv.action_space (footsies.py:171): (left, right, attack)."""
    return MultiBinary(3)


def batch_observation_space(num_envs):
    n = len(RELEVANT_MOVES)
    return Dict({
        "guard": MultiDiscrete(np.full((num_envs, 2), 4)),
        "move": MultiDiscrete(np.full((num_envs, 2), n)),
        "move_frame": Box(low=0.0, high=float(MAX_MOVE_DURATION), shape=(num_envs, 2)),
        "position": Box(low=-4.6, high=4.6, shape=(num_envs, 2)),
    })


def batch_action_space(num_envs):
    return MultiBinary((num_envs, 3))


def normalized_observation_space(normalize_guard=True):
    """FootsiesNormalized.observation_space (normalization.py:24-29)."""
    s = single_observation_space()
    d = {k: s[k] for k in ("guard", "move", "move_frame", "position")}
    if normalize_guard:
        d["guard"] = Box(low=0.0, high=1.0, shape=(2,))
    d["move_frame"] = Box(low=0.0, high=1.0, shape=(2,))
    d["position"] = Box(low=-1.0, high=1.0, shape=(2,))
    return Dict(d)


def frame_skipped_observation_space(wrapped):
    """FootsiesFrameSkipped.observation_space (frame_skip.py:18-33): P2's move_frame only."""
    mf = wrapped["move_frame"]
    return Dict({
        "guard": wrapped["guard"],
        "move": wrapped["move"],
        "move_frame": Box(low=float(mf.low[1]), high=float(mf.high[1]), shape=(1,)),
        "position": wrapped["position"],
    })
