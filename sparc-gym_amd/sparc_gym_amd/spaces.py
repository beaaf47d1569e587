"""gymnasium.Env / gymnasium.spaces when gymnasium is importable, else minimal equivalents.

gymnasium is the reference's base (SPaRC_Gym.py:4-5, 44) but is not installed in this image.
The fallback reproduces what the step path's callers use: ``Env.reset(seed=...)`` seeding
``np_random`` exactly as gymnasium.utils.seeding.np_random (Generator(PCG64(SeedSequence(seed)))),
which the seeded puzzle choice at SPaRC_Gym.py:1085 depends on, and ``Discrete(4).sample()``
(Final_Product.py:29).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    import gymnasium as _gym
    from gymnasium import spaces as _spaces
    Env = _gym.Env
    Dict, Box, Text, Discrete = _spaces.Dict, _spaces.Box, _spaces.Text, _spaces.Discrete
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    def np_random(seed=None):
        seed_seq = np.random.SeedSequence(seed)
        return np.random.Generator(np.random.PCG64(seed_seq)), seed_seq.entropy

    class Env:
        metadata = {"render_modes": []}
        _np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random, _ = np_random()
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random, _ = np_random(seed)

        def close(self):
            pass

        @property
        def unwrapped(self):
            return self

    class Space:
        def __init__(self, shape=None, dtype=None, seed=None):
            self.shape, self.dtype = shape, dtype
            self._np_random = None
            if seed is not None:
                self.seed(seed)

        @property
        def np_random(self):
            if self._np_random is None:
                self.seed()
            return self._np_random

        def seed(self, seed=None):
            self._np_random, _ = np_random(seed)
            return [seed]

    class Discrete(Space):
        def __init__(self, n, seed=None, start=0):
            super().__init__((), np.int64, seed)
            self.n, self.start = int(n), int(start)

        def sample(self, mask=None):
            if mask is not None:
                valid = np.flatnonzero(np.asarray(mask, dtype=np.int8))
                return np.int64(self.start + self.np_random.choice(valid)) if len(valid) else np.int64(self.start)
            return np.int64(self.start + self.np_random.integers(self.n))

        def contains(self, x):
            try:
                v = int(x)
            except (TypeError, ValueError):
                return False
            return v == x and self.start <= v < self.start + self.n

        def __repr__(self):
            return f"Discrete({self.n})"

        def __eq__(self, other):
            return isinstance(other, Discrete) and other.n == self.n and other.start == self.start

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            super().__init__(tuple(shape) if shape is not None else np.shape(low), np.dtype(dtype), seed)
            self.low, self.high = low, high

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

    class Dict(Space):
        def __init__(self, spaces=None, seed=None, **kw):
            super().__init__(None, None, seed)
            self.spaces = dict(spaces or {}, **kw)

        def __getitem__(self, k):
            return self.spaces[k]

        def keys(self):
            return self.spaces.keys()

        def __repr__(self):
            return "Dict(" + ", ".join(f"{k!r}: {v}" for k, v in self.spaces.items()) + ")"

    class Text(Space):
        def __init__(self, max_length, min_length=1, charset=None, seed=None):
            super().__init__((), str, seed)
            self.max_length, self.min_length, self.charset = max_length, min_length, charset

        def __repr__(self):
            return f"Text({self.min_length}, {self.max_length})"
