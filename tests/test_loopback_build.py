"""CPU: the loopback build of the library (tests/loopback_rccl, used only by the -m gpu tests that
run the RCCL code path with several ranks on one GPU) exports the same C-ABI as the product
library, does not link RCCL at all, and the product library never names the stand-in."""
import ctypes as C
import os
import subprocess

from sparkucx_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOP_LIB = os.path.join(ROOT, "sparkucx_amd", "libsparkucx_amd_loop.so")


def _dynamic(path):
    return subprocess.run(["readelf", "-dW", path], capture_output=True, text=True,
                          check=True).stdout


def _undefined(path):
    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_loop_build_exports_the_header_and_links_no_rccl():
    lib = C.CDLL(LOOP_LIB)
    missing = [s for s in N.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert hasattr(lib, "sux_loop_ncclSend") and hasattr(lib, "sux_loop_ncclAllGather")
    assert "librccl" not in _dynamic(LOOP_LIB)
    assert not [s for s in _undefined(LOOP_LIB) if s.startswith("nccl")]


def test_product_library_links_rccl_and_not_the_stand_in():
    lib = N.load()
    assert not hasattr(lib, "sux_loop_ncclSend")
    assert "librccl" in _dynamic(N.LIB_PATH)
    assert "ncclSend" in _undefined(N.LIB_PATH)
