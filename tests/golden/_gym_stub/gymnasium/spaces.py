import numpy as np


class Space:
    def __init__(self, *a, **k):
        self.args, self.kwargs = a, k


class Dict(Space):
    def __init__(self, spaces):
        self.spaces = dict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]


class MultiDiscrete(Space):
    pass


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, **k):
        super().__init__(low, high, shape=shape, dtype=dtype, **k)
        shape = shape if shape is not None else np.shape(low)
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)


class MultiBinary(Space):
    pass


class Discrete(Space):
    pass
