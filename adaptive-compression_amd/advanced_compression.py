"""Drop-in module name of the reference's library-codec module."""
from ambc.methods import (Bzip2Compression, DeflateCompression,  # noqa: F401
                          LZ4Compression, LZMACompression)

HAS_ZSTD = False
HAS_LZ4 = True   # served by the gfx950 LZ4 encoder/decoder
