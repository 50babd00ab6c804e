"""The ctypes bindings match the built gfx950 kernel library (CPU: dlopen only, no GPU calls)."""
import ctypes

import pytest

from docagents_amd.ops import kernels as K


def test_every_bound_symbol_is_exported():
    from docagents_amd.ops.build import LIB as path
    if not path.exists():
        pytest.skip("kernel library not built (python -m docagents_amd.ops.build)")
    lib = ctypes.CDLL(str(path))
    missing = [n for n in K._SIGS if not hasattr(lib, n)]
    assert not missing, f"bound in kernels.py but not exported by {path.name}: {missing}"
