"""Drop-in module name of the reference's library-codec module."""
from ambc.methods import (HAS_ZSTD, Bzip2Compression, DeflateCompression,  # noqa: F401
                          LZ4Compression, LZMACompression, ZstdCompression, calculate_entropy)

HAS_LZ4 = True   # served by the gfx950 LZ4 encoder/decoder
