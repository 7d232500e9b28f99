"""CPU-side checks of the C-ABI boundary: the library loads and exports every symbol include/vihmc.h
declares, the ctypes structs match the C layout, and creation errors are reported (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "vihmc.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vihmc_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = header_functions()
    for must in ("vihmc_deeponet_plan_create", "vihmc_mlp_plan_create", "vihmc_logp_grad", "vihmc_forward",
                 "vihmc_plan_destroy", "vihmc_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from vihmc import _lib
    L = _lib.lib()
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(header_functions()) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"
    assert L.vihmc_version().decode().startswith("vihmc")


def test_struct_layouts():
    from vihmc import _lib
    assert ctypes.sizeof(_lib.Linear) == 32
    assert ctypes.sizeof(_lib.LikDesc) == 16
    assert _lib.DeepONetDesc.lik.offset % 4 == 0
    assert ctypes.sizeof(_lib.DeepONetDesc) == 4 + 4 + 8 + 8 + 8 + 6 * 4 + 16
    assert ctypes.sizeof(_lib.MLPDesc) == 4 + 4 + 8 + 8 + 6 * 4 + 16


def test_null_arguments_are_errors_not_crashes():
    from vihmc import _lib
    L = _lib.lib()
    rc = L.vihmc_logp_grad(None, None, 1, None, None, None)
    assert rc != 0 and b"null" in L.vihmc_last_error()


def test_engine_refuses_cpu_device():
    from vihmc.engine import DeepONetEngine
    from vihmc.layout import DeepONetSpec
    with pytest.raises(RuntimeError):
        DeepONetEngine(DeepONetSpec(), None, None, None, None, [0], device="cpu")


def test_shipped_library_has_no_diagnostic_switches():
    """Timing-only ablations (FWD_ABL, CB_ABL, BB_ABL) and stamp instrumentation are never in the product
    build: the version string reports them and vihmc._lib refuses such a library."""
    from vihmc import _lib
    assert re.search(r"diag=0(\s|$)", _lib.lib().vihmc_version().decode())
