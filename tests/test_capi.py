"""CPU-side checks of the C ABI: libsra.so loads, exports every symbol that
include/sra.h declares, and rejects bad arguments before touching a GPU."""
from __future__ import annotations

import ctypes

import pytest

import srfl_amd
from srfl_amd import _lib


def test_library_loads_and_exports_header_symbols():
    lib = _lib.load()
    declared = _lib.header_symbols()
    assert "sra_trimmed_mean_f32" in declared
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, "symbols declared in include/sra.h but not exported: %s" % missing
    # every declared symbol has a ctypes signature in the binding
    assert set(declared) <= set(_lib._SIGS), set(declared) - set(_lib._SIGS)


def test_version_and_limits():
    lib = _lib.load()
    assert lib.sra_version() >= 100
    assert lib.sra_max_register_clients() == 128


@pytest.mark.parametrize("fn", ["sra_average_f32", "sra_median_f32"])
def test_null_pointer_rejected_without_gpu(fn):
    with pytest.raises(ValueError):
        _lib.call(fn, None, 4, 4, 4, None, None)


def test_shape_errors_map_to_valueerror():
    dummy = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    with pytest.raises(ValueError, match="ldx"):
        _lib.call("sra_median_f32", dummy, 4, 8, 4, dummy, None)
    with pytest.raises(ValueError, match="b must be"):
        _lib.call("sra_trimmed_mean_f32", dummy, 4, 8, 8, -1, dummy, None)
    assert "b must be" in _lib.last_error()


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.SraLibraryError):
        _lib.load(str(tmp_path / "nope.so"))


def test_package_version():
    assert srfl_amd.__version__


def test_dba_module_needs_a_gpu():
    import numpy as np
    import torch
    from srfl_amd import dba
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = dba.HelperAggregation({"eta": 1})
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        h.median(None, {0: (10, {"w": torch.from_numpy(np.zeros(3, np.float32))})})
