"""sparc_gym_amd — MI355X-native batched SPaRC puzzle simulator.

Drop-in for tobiTKM/SPaRC-Gym's step path: ``SPaRC_Gym`` mirrors the reference's
``gymnasium.Env`` (SPaRC_Gym/SPaRC_Gym.py:44), ``SPaRCVecEnv`` steps many envs per HIP launch.
The compute runs in hand-written HIP kernels for gfx950 (csrc/) behind the C ABI of
include/sparc_gym_amd.h; there is no CPU fallback.
"""
from . import puzzles, synthetic  # noqa: F401
from .puzzles import PuzzleTable, pack_table, process_puzzles  # noqa: F401

__all__ = ["SPaRC_Gym", "SPaRCVecEnv", "xcd_local_puzzle_index", "process_puzzles", "pack_table", "PuzzleTable",
           "register"]


def __getattr__(name):
    # the env classes need the HIP library; import them lazily so that the host-side loader
    # stays importable for tooling, and fail loudly (ImportError) when the library is missing
    if name == "SPaRC_Gym":
        from .env import SPaRC_Gym
        return SPaRC_Gym
    if name == "SPaRCVecEnv":
        from .vec_env import SPaRCVecEnv
        return SPaRCVecEnv
    if name == "xcd_local_puzzle_index":
        from .vec_env import xcd_local_puzzle_index
        return xcd_local_puzzle_index
    raise AttributeError(name)


def register():
    """Register "SPaRC-Gym" with gymnasium, as SPaRC_Gym/register_env.py:5-8 (if installed)."""
    try:
        from gymnasium.envs.registration import register as _register
    except ImportError:
        return False
    _register(id="SPaRC-Gym", entry_point="sparc_gym_amd.env:SPaRC_Gym")
    return True


register()
