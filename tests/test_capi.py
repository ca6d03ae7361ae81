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


def test_capi_validation_under_asan():
    """The host side of every C-ABI entry point (argument validation,
    workspace sizing, launch set-up) under AddressSanitizer: `make asan`
    builds libsra_asan.so with -fsanitize=address on the host code only
    (device code as usual), and tests/capi_asan_driver.py calls each symbol
    of include/sra.h with null / zero / negative / huge / plausible arguments
    in a subprocess with the ASan runtime preloaded.  Any overflow aborts it."""
    import glob
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "secure-robust-federated-learning_amd", "csrc")
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("no clang ASan runtime in this image")
    subprocess.run(["make", "-C", csrc, "-j8", "asan"], check=True, capture_output=True)
    env = dict(os.environ, LD_PRELOAD=rt[-1], ASAN_OPTIONS="detect_leaks=0",
               SRA_LIB=os.path.join(root, "build", "sra_asan", "libsra_asan.so"))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "capi_asan_driver.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "asan driver:" in r.stdout and "AddressSanitizer" not in r.stderr
