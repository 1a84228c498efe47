"""pytest configuration.

Markers:
  gpu  -- needs a visible MI355X (gfx950) and the built librsamd.so; these are
          the parity tests proper and call the engine through the C-ABI.
Everything unmarked runs on CPU (oracle pinning, golden fixtures, host-side
matrix logic and argument checks of the C-ABI, gloo multi-process tests).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# A/B runs of the GPU tests against a variant build (make OUT=... KDEFS=...):
# RSAMD_TEST_LIB names the librsamd.so to load instead of the in-tree one.
if os.environ.get("RSAMD_TEST_LIB"):
    from rsamd import _lib as _rs_lib
    _rs_lib.LIB_PATH = os.path.abspath(os.environ["RSAMD_TEST_LIB"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU and the HIP extension")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import c_ref
    c_ref.build()
    return c_ref


@pytest.fixture(scope="session")
def native():
    """The product library; fails loudly when it is not built."""
    from rsamd import _lib
    return _lib.load()


@pytest.fixture(autouse=True)
def bounds_check(request):
    """Against the bounds-checking build (make -C csrc bounds; RSAMD_TEST_LIB
    names lib/bounds/librsamd.so): after every GPU test, no kernel access may
    have fallen outside the buffers its call declared (csrc/bounds.hpp).  A
    no-op with the product library, which does not export rs_bounds_report."""
    yield
    if "gpu" not in request.fixturenames:
        return
    import ctypes as C
    from rsamd import _lib
    lib = _lib.load()
    if not hasattr(lib, "rs_bounds_report"):
        return
    import torch
    torch.cuda.synchronize()
    n, addr, ln, where = C.c_ulonglong(), C.c_ulonglong(), C.c_ulonglong(), C.c_uint()
    lib.rs_bounds_report(C.byref(n), C.byref(addr), C.byref(ln), C.byref(where))
    unit = {1: "kernels.hip", 2: "layout.hip", 9: "host check of a declared range (bounds.hpp)"}.get(
        where.value // 100000, "?")
    assert n.value == 0, (f"{n.value} kernel access(es) outside the call's buffers; first: {ln.value} B at "
                          f"{addr.value:#x}, {unit}:{where.value % 100000}")


@pytest.fixture(scope="session")
def gpu(native):
    """Skip-free GPU gate: a gpu-marked test on a box without a device is an error."""
    n = native.rs_device_count()
    if n < 1:
        pytest.fail("no HIP device visible to librsamd.so (gpu tests need an MI355X)")
    import torch
    assert torch.cuda.is_available(), "torch sees no GPU"
    return torch.device("cuda:0")
