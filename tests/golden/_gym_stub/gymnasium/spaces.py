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
    pass


class MultiBinary(Space):
    pass


class Discrete(Space):
    pass
