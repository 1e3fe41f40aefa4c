import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


import pytest  # noqa: E402

_EMU_SRCS = ("tas_kernels.hip", "tas_device.hip", "tas_host.cpp", "tas_internal.h", "json_reader.h",
             "label_selectors.h", "tas_balanced.h", "tas_pool.h")


@pytest.fixture(scope="session")
def emu_lib():
    """The product sources built against the CPU SIMT emulator (tests/emu):
    kernel logic checked where no GPU is available.  Rebuilt when a source is newer."""
    import subprocess

    from kueue_oss_amd import native

    here = os.path.dirname(os.path.abspath(__file__))
    so = os.path.join(here, "emu", "_build", "libkueue_tas_emu.so")
    srcs = [os.path.join(ROOT, "kueue_oss_amd", "csrc", f) for f in _EMU_SRCS]
    srcs += [os.path.join(here, "emu", f) for f in ("hip_emu.cpp", "build_emu.sh", "hip/hip_runtime.h")]
    srcs.append(os.path.join(ROOT, "include", "kueue_tas.h"))
    srcs.append(os.path.join(ROOT, "include", "kueue_tas_debug.h"))
    import fcntl

    os.makedirs(os.path.join(here, "emu", "_build"), exist_ok=True)
    with open(os.path.join(here, "emu", "_build", ".lock"), "w") as lk:  # one builder across xdist workers
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in srcs):
            subprocess.run([os.path.join(here, "emu", "build_emu.sh")], check=True, capture_output=True)
    return native.load_library(so)
