"""Minimal throwaway stand-in for `gymnasium` (not installed here), used ONLY by
tests/golden/make_*.py to import the reference FootsiesEnv and its wrappers in the
build container.  Provides just the names footsies_gym touches, with gymnasium's
documented Wrapper / ActionWrapper / ObservationWrapper delegation semantics."""
from . import spaces  # noqa: F401


class Env:
    metadata = {}

    def reset(self, *, seed=None, options=None):
        return None


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.observation_space = env.observation_space
        self.action_space = env.action_space

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        return self.env.step(action)


class ActionWrapper(Wrapper):
    def step(self, action):
        return self.env.step(self.action(action))


class ObservationWrapper(Wrapper):
    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        return self.observation(obs), reward, terminated, truncated, info
