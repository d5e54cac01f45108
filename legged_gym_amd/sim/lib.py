"""Loader of the product library liblgx.so (HIP, gfx950).

There is deliberately no fallback: if the library or a GPU is missing, `load()` raises.
The CPU oracle under oracle/ is test infrastructure and is never imported from here.
"""
import ctypes as C
import os

from . import abi

_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "liblgx.so")
# an instrumented build of the same sources (tools/phase_clock.sh) may be selected for tuning runs
LIB_PATH = os.environ.get("LGX_LIB_PATH", LIB_PATH)


class LgxError(RuntimeError):
    pass


def load():
    """Load liblgx.so (after torch, so the HIP runtime torch already loaded is shared)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (HIP runtime first: liblgx binds to torch's libamdhip64.so.7)
    if not os.path.exists(LIB_PATH):
        raise LgxError(f"liblgx.so not built ({LIB_PATH}); run `python -c 'import __graft_entry__ as g; g.build()'` "
                       "or `make -C legged_gym_amd/csrc`")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    abi.declare(lib)
    abi.check_layout(lib.lgx_struct_sizes)
    _LIB = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = _LIB.lgx_last_error().decode() if _LIB is not None else ""
        raise LgxError(f"{what} failed ({rc}): {msg}")
