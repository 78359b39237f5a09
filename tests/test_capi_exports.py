"""CPU: the C-ABI library loads and exports every symbol include/*.h declares.

No compute calls here (there is no GPU in the build container)."""
import ctypes
import os
import re

import miotts_amd as m


def _declared_symbols(test_header=False):
    """mio_* names declared in include/*.h: the product headers, or (test_header) the
    test-support library's include/mio_hip_test.h."""
    names = set()
    for fn in sorted(os.listdir(m.INCLUDE_DIR)):
        if not fn.endswith(".h") or (fn == "mio_hip_test.h") != test_header:
            continue
        src = open(os.path.join(m.INCLUDE_DIR, fn), encoding="utf-8").read()
        if 'extern "C"' not in src:
            continue
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for name in re.findall(r"\b(mio_[a-z0-9_]+)\s*\(", src):
            names.add(name)
    return names


def test_library_loads_and_exports_all_declared_symbols():
    L = m.lib().product
    declared = _declared_symbols()
    assert len(declared) >= 10
    missing = [n for n in sorted(declared) if not hasattr(L, n)]
    assert not missing, f"declared but not exported: {missing}"


def test_test_support_symbols_live_in_the_test_library():
    """Synthetic GGUF writers and kernel parity entries (include/mio_hip_test.h) are exported
    by libmiotts_test.so only: the product library carries no test code's entry points."""
    libs = m.lib()
    declared = _declared_symbols(test_header=True)
    assert {"mio_synth_llm_gguf", "mio_hip_debug_matvec", "mio_quantize_rows"} <= declared
    assert libs.test is not None
    missing = [n for n in sorted(declared) if not hasattr(libs.test, n)]
    assert not missing, f"declared but not exported: {missing}"
    # the product library must not define them (the test library is linked against it)
    leaked = [n for n in sorted(declared) if hasattr(ctypes.CDLL(m.LIB_PATH), n)]
    assert not leaked, f"test entry points in libmiotts.so: {leaked}"


def test_error_text_api_without_gpu():
    L = m.lib()
    # a NULL handle is rejected with MIO_ERR_INVALID and an error string, no GPU needed
    rc = L.mio_hip_device_sync(None)
    assert rc == -1
    assert b"null" in L.mio_hip_last_error()
