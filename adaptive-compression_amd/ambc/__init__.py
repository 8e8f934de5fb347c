"""ambc -- MI355X (gfx950) engine for the per-chunk selection + encode/decode
loop of KalharPandya/adaptive-compression's AdaptiveCompressor.

Python host layer over libambc_hip.so (HIP kernels, C-ABI in include/ambc.h).
"""
from ._lib import AmbcError, AmbcUnavailable, Context, load  # noqa: F401
from .compressor import AdaptiveCompressor, DefaultsWarning, entropy_terms  # noqa: F401
from .methods import (Bzip2Compression, CompressionMethod, DeflateCompression,  # noqa: F401
                      DeltaCompression, DictionaryCompression, HuffmanCompression,
                      LZ4Compression, LZMACompression, NoCompression, RLECompression,
                      ZstdCompression)

__version__ = "0.1.0"
