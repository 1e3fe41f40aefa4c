"""libkueue_tas.so loads and exports every symbol include/kueue_tas.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

import kueue_oss_amd
from kueue_oss_amd import native

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADERS = [os.path.join(INCLUDE, "kueue_tas.h"), os.path.join(INCLUDE, "kueue_tas_debug.h")]


def header_functions():
    found = set()
    for h in HEADERS:
        found |= set(re.findall(r"\b(kueue_tas_[a-z_0-9]+)\s*\(", open(h).read()))
    return sorted(found)


def test_header_declares_exported_set():
    assert header_functions() == sorted(native.EXPORTED_SYMBOLS)


def test_library_exports_all_header_symbols():
    lib = kueue_oss_amd.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.kueue_tas_abi_version() == 5


def test_struct_sizes_match_header_layout():
    # kueue_tas_eval_req / _out are passed by pointer across the ABI: pin their sizes.
    lib = kueue_oss_amd.load_library()
    assert lib is not None
    # eval_out: 16 int32 header fields + 2x4 multilayer + 2 reserved = 26 int32
    assert ctypes.sizeof(ctypes.c_int32) * 26 == 104


def test_no_cpu_fallback_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(kueue_oss_amd.NativeLibraryMissing):
        kueue_oss_amd.TASFlavorSnapshot({"levels": ["kubernetes.io/hostname"], "nodes": []})
