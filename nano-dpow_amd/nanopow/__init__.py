"""nanopow -- MI355X-native Nano proof-of-work engine (drop-in nano-work-server).

``nanopow._lib``   ctypes binding of libnanopow.so (gfx950 HIP kernels, C ABI)
``nanopow.work``   hex/threshold/multiplier rules of the work-server JSON surface
``nanopow.server`` nano-work-server-compatible HTTP JSON server (127.0.0.1:7000)
"""
from ._lib import (CancelToken, Engine, NanoPowError, SearchResult, engine,  # noqa: F401
                   NPOW_OK, NPOW_CANCELLED, NPOW_EXHAUSTED)

__version__ = "0.1.0"
