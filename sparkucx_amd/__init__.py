"""sparkucx_amd — MI355X-native SparkUCX shuffle data path.

The product is libsparkucx_amd.so (C-ABI in include/sparkucx_amd.h, gfx950 kernels in
csrc/).  This package holds its ctypes binding (native.py) and torch-facing helpers
(shuffle.py) used by tests and bench.py.
"""
from . import native  # noqa: F401

__all__ = ["native"]
