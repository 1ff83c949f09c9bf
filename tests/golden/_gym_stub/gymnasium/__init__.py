"""Minimal throwaway stand-in for `gymnasium` (not installed here), used ONLY by
tests/golden/make_golden.py to import the reference FootsiesEnv in the build
container.  Provides just the names footsies_gym touches at import/ctor time."""
from . import spaces  # noqa: F401


class Env:
    metadata = {}

    def reset(self, *, seed=None, options=None):
        return None
