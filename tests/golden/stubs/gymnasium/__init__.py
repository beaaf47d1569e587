"""Minimal stand-in for gymnasium, used ONLY by tests/golden/make_golden.py to import the
reference env in this container (gymnasium is not installed).  Seeding follows
gymnasium.utils.seeding.np_random: Generator(PCG64(SeedSequence(seed)))."""
from . import spaces  # noqa: F401
from .utils import seeding


class Env:
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = seeding.np_random()
        return self._np_random

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = seeding.np_random(seed)


