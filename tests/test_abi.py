"""The C-ABI library loads and exports every symbol include/jabd.h declares
(no compute calls: this runs without a GPU)."""
import os
import re

from conftest import ROOT


def _header_functions():
    text = open(os.path.join(ROOT, "include", "jabd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(?:int|int64_t|const char\s*\*)\s+(jabd_\w+)\s*\(", text)
    return sorted(set(names))


def test_header_declares_functions():
    names = _header_functions()
    assert "jabd_batched_nms_f32" in names and "jabd_conv2d_nhwc_f32" in names
    assert len(names) >= 20


def test_library_exports_every_header_symbol():
    from jabd_amd import _lib
    h = _lib.lib()
    for name in _header_functions():
        assert hasattr(h, name), name
    # and the Python binding declares a signature for each one
    assert set(_header_functions()) == set(_lib.SIGNATURES), (
        set(_header_functions()) ^ set(_lib.SIGNATURES))


def test_version_string():
    from jabd_amd import ops
    assert "gfx950" in ops.version()


def test_cpu_tensor_is_rejected():
    import pytest
    import torch
    from jabd_amd import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.nms(torch.zeros(3, 4), torch.zeros(3), 0.3)


def test_struct_mirrors_match_the_library():
    """ctypes mirrors of the argument structs have the C sizes (a field added
    on one side only would shift every later field)."""
    import ctypes
    from jabd_amd._lib import ConvArgs, DwArgs, ExpDwArgs, WindowCopy, lib
    for i, cls in enumerate((ConvArgs, DwArgs, ExpDwArgs, WindowCopy)):
        assert lib().jabd_abi_struct_size(i) == ctypes.sizeof(cls), cls.__name__
