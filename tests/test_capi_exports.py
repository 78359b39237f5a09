"""CPU: the C-ABI library loads and exports every symbol include/*.h declares.

No compute calls here (there is no GPU in the build container)."""
import ctypes
import os
import re

import miotts_amd as m


def _declared_symbols():
    names = set()
    for fn in sorted(os.listdir(m.INCLUDE_DIR)):
        if not fn.endswith(".h"):
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
    L = m.lib()
    declared = _declared_symbols()
    assert len(declared) >= 10
    missing = [n for n in sorted(declared) if not hasattr(L, n)]
    assert not missing, f"declared but not exported: {missing}"


def test_error_text_api_without_gpu():
    L = m.lib()
    # a NULL handle is rejected with MIO_ERR_INVALID and an error string, no GPU needed
    rc = L.mio_hip_device_sync(None)
    assert rc == -1
    assert b"null" in L.mio_hip_last_error()
