"""CPU test: librestir_amd.so loads (no GPU needed to dlopen it) and exports exactly the entry points
include/restir_c.h declares; product code fails loudly without a device."""
import ctypes
import os
import re

import pytest

from restir_amd import renderer as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "restir_c.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z_0-9]+)\s*\(", hdr)))


def test_header_declares_what_binding_exports():
    assert _declared_symbols() == sorted(R.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(R.LIB_PATH):
        pytest.fail(f"{R.LIB_PATH} missing: run __graft_entry__.build() / make -C restir-embree_amd")
    lib = ctypes.CDLL(R.LIB_PATH)
    for name in _declared_symbols():
        assert hasattr(lib, name), name


def test_no_device_fails_loudly():
    """Without a visible HIP device the product raises instead of falling back to a CPU path."""
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(R.RestirError):
        R.Renderer(8, 8)
