"""omnifed_amd — MI355X-native gradient-compression codec for OmniFed's hybrid global hop.

Layout:
  csrc/       hand-written HIP kernels (gfx950) + the C ABI (include/omf_codec.h)
  _lib.py     ctypes binding of libomf_codec.so (no CPU fallback)
  codec.py    update-arena plans and device entry points
  hybrid/     drop-in mirror of src/omnifed/hybrid/{compression,communicator}
  ps.py       parameter-server aggregate-after-decode (one GPU) and the RCCL weighted sum
"""

__version__ = "0.1.0"
