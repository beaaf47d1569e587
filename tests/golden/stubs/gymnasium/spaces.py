"""Stub spaces (shape/dtype holders) for the golden-vector generator."""


class Space:
    def __init__(self, *a, **k):
        self.args, self.kwargs = a, k


class Dict(Space):
    def __init__(self, spaces=None, **k):
        super().__init__(spaces, **k)
        self.spaces = spaces


class Box(Space):
    pass


class Text(Space):
    pass


class Discrete(Space):
    def __init__(self, n, **k):
        super().__init__(n, **k)
        self.n = n
