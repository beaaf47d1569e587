"""The C-ABI library loads on the CPU host and exports every symbol include/ declares."""
import ctypes
import os
import re

import pytest

from sparc_gym_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sparc_gym_amd.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:int|const char \*|void)\s*\*?\s*(sparc_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_bound_symbols():
    assert set(declared_symbols()) == set(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.sparc_abi_version() == 2


def test_create_validates_before_touching_a_device():
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    bad = _lib.SparcConfig(0, 0, 100, 0, 7, 1, 0)
    assert lib.sparc_create(0, ctypes.byref(bad), ctypes.byref(ctx)) == -1
    assert b"num_envs" in lib.sparc_last_error(None)
    bad = _lib.SparcConfig(4, 0, 100, 0, 7, 3, 0)
    assert lib.sparc_create(0, ctypes.byref(bad), ctypes.byref(ctx)) == -1
    assert ctx.value is None


def test_null_context_is_an_error_not_a_crash():
    lib = _lib.load()
    assert lib.sparc_step_device(None, None, None, None) != 0
    assert lib.sparc_step_obs_device(None, None, None, None, None, None, 7, 7, None, None) != 0
    assert lib.sparc_rollout_obs_device(None, 4, None, 0, 0, None, None, None, None, None, 7, 7) != 0
    assert lib.sparc_rollout_device(None, 4, None, 0, 0, None, None, None) != 0
    assert lib.sparc_rollout_rules_device(None, 4, None, 0, 0, None, None, None, None) != 0
    assert lib.sparc_set_visited_host(None, None) != 0
    assert lib.sparc_sync(None) != 0
    assert lib.sparc_destroy(None) == 0


def test_comm_entry_points_validate_arguments():
    """The RCCL gather's argument checks run before any RCCL or HIP call."""
    lib = _lib.load()
    comm = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    assert lib.sparc_comm_unique_id(None) == -1
    assert lib.sparc_comm_init(None, 1, 0, uid, ctypes.byref(comm)) == -1
    assert comm.value is None
    assert lib.sparc_gather_stats(None, None, None, None) == -1
    assert lib.sparc_comm_destroy(None) == 0


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        _lib._lib = None
        try:
            _lib.load(str(tmp_path / "nope.so"))
        finally:
            _lib._lib = None


def test_no_environment_variable_selects_a_kernel():
    """Kernel variants (identical results; A/B runs and tests) are chosen only through the debug
    entry point sparc_set_variant: the library reads no environment variable at all (it imports
    neither getenv nor secure_getenv), so a stray variable cannot change the kernel a context
    runs.  sparc_set_variant checks its arguments before touching the context."""
    import shutil
    import subprocess
    nm = shutil.which("nm") or shutil.which("llvm-nm")
    if nm is None:
        pytest.skip("no nm")
    undef = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True,
                           check=True).stdout
    imported = {line.split()[-1].split("@")[0] for line in undef.splitlines() if line.strip()}
    assert not imported & {"getenv", "secure_getenv", "__secure_getenv"}, imported & {"getenv", "secure_getenv"}
    lib = _lib.load()
    assert lib.sparc_set_variant(None, 1, 1) == -1
    src = open(os.path.join(REPO, "sparc-gym_amd", "csrc", "sparc_kernels.hip")).read()
    for name in ("SPARC_IO_CODES", "SPARC_RULE_ROLLOUT", "SPARC_R1R_SHAPE"):
        assert f'"{name}"' not in src
