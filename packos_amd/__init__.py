"""packos_amd — MI355X-native bulk PackOS encoder/decoder.

Host-side mirror of the reference API (quickwritereader/PackOS) over the C ABI
in include/packos.h, implemented by hand-written HIP kernels for gfx950
(packos_amd/csrc).  Importing this package does not need a GPU; batch calls
do, and they fail loudly when libpackos.so or the GPU is missing.
"""
from . import schema  # noqa: F401
from .schema import *  # noqa: F401,F403

__version__ = "0.1.0"
