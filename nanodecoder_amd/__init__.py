"""nanodecoder_amd — MI355X-native (gfx950) engine for NanoDecoder's translate path.

The compute path is ``libnanodec_hip.so`` (hand-written HIP kernels, C-ABI in
``include/nanodec.h``), driven from Python through ctypes.  Submodules import
lazily so that host-only utilities (synthetic data, batching, assembly) work
without the shared library.
"""
__version__ = "0.1.0"
