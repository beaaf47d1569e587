"""ctypes binding of include/sparc_gym_amd.h (libsparc_gym_amd.so, built for gfx950).

There is no fallback: if the HIP library is missing or fails to load, importing the env
classes raises.  Build it with ``make -C sparc-gym_amd`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsparc_gym_amd.so")   # the in-tree gfx950 build; no override

SPARC_OK = 0
AUTORESET = {"none": 0, "next_step": 1}

c_void_p, c_int32, c_uint64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64


class SparcConfig(ctypes.Structure):
    _fields_ = [("num_envs", ctypes.c_int32), ("traceback", ctypes.c_int32), ("max_steps", ctypes.c_int32),
                ("autoreset", ctypes.c_int32), ("pitch", ctypes.c_int32), ("words", ctypes.c_int32),
                ("env_offset", ctypes.c_int64)]


class SparcPuzzleTable(ctypes.Structure):
    _fields_ = [("num_puzzles", ctypes.c_int32), ("num_nodes", ctypes.c_int32),
                ("open", c_void_p), ("info", c_void_p), ("trie", c_void_p)]


class SparcStateHost(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("path_len", c_void_p), ("step", c_void_p),
                ("puzzle", c_void_p), ("outcome", c_void_p), ("pending", c_void_p), ("visited", c_void_p)]


class SparcRulesTable(ctypes.Structure):
    _fields_ = [("num_puzzles", ctypes.c_int32), ("num_inst", ctypes.c_int32), ("num_shapes", ctypes.c_int32),
                ("num_offsets", ctypes.c_int32), ("planes", c_void_p), ("inst_first", c_void_p), ("inst", c_void_p),
                ("shape_first", c_void_p), ("shape_area", c_void_p), ("shape_off", c_void_p)]


class SparcEnvRecord(ctypes.Structure):
    """sparc_env_record: one env after sparc_env_step / _reset / _read (one round trip)."""
    _fields_ = [("reward_code", ctypes.c_int8), ("flags", ctypes.c_uint8), ("x", ctypes.c_uint8),
                ("y", ctypes.c_uint8), ("path_len", ctypes.c_uint8), ("outcome", ctypes.c_int8),
                ("pending", ctypes.c_uint8), ("audited", ctypes.c_uint8), ("step", ctypes.c_uint32),
                ("puzzle", ctypes.c_uint32), ("rule_bits", ctypes.c_uint16), ("reserved", ctypes.c_uint16),
                ("host_fits", ctypes.c_uint32), ("fit", ctypes.c_uint64), ("visited", ctypes.c_uint64 * 4),
                ("region", ctypes.c_uint8 * 256)]


assert ctypes.sizeof(SparcEnvRecord) == 320


_SIGS = {
    "sparc_abi_version": ([], c_int32),
    "sparc_last_error": ([c_void_p], ctypes.c_char_p),
    "sparc_create": ([ctypes.c_int, ctypes.POINTER(SparcConfig), ctypes.POINTER(c_void_p)], c_int32),
    "sparc_destroy": ([c_void_p], c_int32),
    "sparc_set_stream": ([c_void_p, c_void_p], c_int32),
    "sparc_use_own_stream": ([c_void_p], c_int32),
    "sparc_sync": ([c_void_p], c_int32),
    "sparc_load_puzzles": ([c_void_p, ctypes.POINTER(SparcPuzzleTable)], c_int32),
    "sparc_reset_host": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_reset_device": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_step_device": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_step_host": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_rollout_device": ([c_void_p, c_int32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p],
                             c_int32),
    "sparc_random_actions_device": ([c_void_p, c_int32, c_uint64, c_uint64, c_void_p], c_int32),
    "sparc_obs_pack_device": ([c_void_p, c_void_p, c_void_p, c_int32, c_int32], c_int32),
    "sparc_step_obs_device": ([c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                               c_void_p, c_void_p], c_int32),
    "sparc_step_gym_device": ([c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
                              c_int32),
    "sparc_rollout_obs_device": ([c_void_p, c_int32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int32, c_int32], c_int32),
    "sparc_rollout_rules_device": ([c_void_p, c_int32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
                                    c_void_p], c_int32),
    "sparc_read_state": ([c_void_p, ctypes.POINTER(SparcStateHost)], c_int32),
    "sparc_env_step": ([c_void_p, c_int32, c_int32, c_int32, ctypes.POINTER(SparcEnvRecord)], c_int32),
    "sparc_env_reset": ([c_void_p, c_int32, ctypes.c_uint32, c_int32, ctypes.POINTER(SparcEnvRecord)], c_int32),
    "sparc_env_read": ([c_void_p, c_int32, c_int32, ctypes.POINTER(SparcEnvRecord)], c_int32),
    "sparc_state_ptr": ([c_void_p, c_int32, ctypes.POINTER(c_void_p)], c_int32),
    "sparc_set_visited_host": ([c_void_p, c_void_p], c_int32),
    "sparc_copy_state_device": ([c_void_p, c_int32, c_void_p], c_int32),
    "sparc_load_rules": ([c_void_p, ctypes.POINTER(SparcRulesTable)], c_int32),
    "sparc_rules_device": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_rules_host": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_rules_finish": ([c_void_p, c_void_p, c_void_p], c_int32),
    "sparc_set_rule_limits": ([c_void_p, ctypes.c_uint32, c_uint64], c_int32),
    "sparc_set_variant": ([c_void_p, c_int32, c_int32], c_int32),
    "sparc_rules_queue_stats": ([c_void_p, c_void_p], c_int32),
    "sparc_comm_unique_id": ([c_void_p], c_int32),
    "sparc_comm_init": ([c_void_p, c_int32, c_int32, c_void_p, ctypes.POINTER(c_void_p)], c_int32),
    "sparc_comm_destroy": ([c_void_p], c_int32),
    "sparc_gather_stats": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int32),
}
COMM_ID_BYTES = 128   # SPARC_COMM_ID_BYTES
EXPORTS = tuple(_SIGS)

_lib = None


class SparcError(RuntimeError):
    pass


def load(path=None, any_abi=False):
    """Load and type the HIP library (cached).  Raises if it is missing: no CPU fallback.

    The product path always loads the in-tree build (``path=None``).  Profiling tools may load
    another build by calling ``load(path)`` themselves before any env is created; later
    ``load()`` calls then return that library.  ``any_abi``: an A/B build of an earlier ABI
    version (the rollout entry points are unchanged; symbols it lacks stay unbound)."""
    global _lib
    if _lib is not None:
        if path is not None and os.path.abspath(path) != _lib._sparc_path:
            raise ImportError(f"libsparc_gym_amd already loaded from {_lib._sparc_path}")
        return _lib
    path = LIB_PATH if path is None else path
    if not os.path.exists(path):
        raise ImportError(f"{path} not found: build the HIP extension (make -C sparc-gym_amd)")
    lib = ctypes.CDLL(path)
    for name, (args, res) in _SIGS.items():
        if any_abi and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    if lib.sparc_abi_version() != 2 and not any_abi:
        raise ImportError("libsparc_gym_amd ABI version mismatch")
    lib._sparc_path = os.path.abspath(path)
    _lib = lib
    return lib


def check(rc, ctx=None):
    if rc != SPARC_OK:
        msg = load().sparc_last_error(ctx)
        msg = msg.decode() if msg else "unknown error"
        if rc == -1:
            raise ValueError(msg)
        raise SparcError(f"sparc error {rc}: {msg}")
