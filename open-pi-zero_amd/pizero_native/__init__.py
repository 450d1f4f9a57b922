"""MI355X-native execution layer of the Pi0 hot path.

``_lib``  : ctypes binding of libpizero_hip.so (include/pz_abi.h)
``ops``   : torch-tensor front-ends of the C ABI (plumbing only)
``engine``: layer executor for SigLIP + joint model forward/backward/inference
"""

from ._lib import LIB_PATH, NativeError, lib  # noqa: F401
