"""Drop-in module name of the reference's library-codec module."""
from ambc.methods import (HAS_ZSTD, Bzip2Compression, DeflateCompression,  # noqa: F401
                          LZ4Compression, LZMACompression, ZstdCompression, calculate_entropy)

# In the reference HAS_LZ4 says whether LZ4Compression exists, and with it id 9
# is registered (advanced_compression.py:17-23, adaptive_compressor.py:151).
# Here the gfx950 encoder / decoder serve id 9, so the class always exists and
# the flag is True.  Its frames are valid LZ4 frames, which a reference without
# python-lz4 cannot decode.  Files for such a reader are written with
# methods=(1, 3, 4, 5) or AdaptiveCompressor.like_reference().
HAS_LZ4 = True
